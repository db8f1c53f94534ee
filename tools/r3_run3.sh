set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/valu > gpurun_out/r3_valu.txt 2>&1 || exit 1
cat gpurun_out/r3_valu.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_b256.py tests/test_gpu_plan.py -q --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3c_tests.log
tail -5 gpurun_out/r3c_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || exit 1
cat gpurun_out/r3c_bench.json
