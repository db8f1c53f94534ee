set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_plan.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_tiny_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_tiny_tests.log
tail -6 gpurun_out/r3_tiny_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config vit_tiny --no-cpu-baseline > gpurun_out/tiny2.json 2> gpurun_out/tiny2.err || exit 1
python -c "
import json;d=json.load(open('gpurun_out/tiny2.json'));print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'], d['roofline']['gemm_ms_per_forward'])
for k,v in d['kernels'].items(): print(k, v['avg_us'], v['ms_per_forward'])
"
