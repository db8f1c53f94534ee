set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_kernels.py tests/test_gpu_models.py tests/test_gpu_plan.py tests/test_gpu_b256.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_embed_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_embed_tests.log
tail -8 gpurun_out/r3_embed_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3_embed_bench.json 2> gpurun_out/r3_embed_bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r3_embed_bench.err; exit $rc; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r3_embed_bench.json'))
print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'])
for k,v in d['kernels'].items(): print(k, v['avg_us'], v['ms_per_forward'], v.get('achieved'))
print({k:(v.get('value'),v.get('verified')) for k,v in d.get('secondary',{}).items()})
PY
