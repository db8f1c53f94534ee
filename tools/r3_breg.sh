set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_breg_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_breg_tests.log
tail -5 gpurun_out/r3_breg_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PGM_DIAGS="old" OUT=r3h_micro bash tools/r3_micro.sh
