set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_api_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_api_tests.log
tail -15 gpurun_out/r3_api_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PGM_DIAGS="${PGM_DIAGS:-}" OUT=${OUT:-r3_micro} bash tools/r3_micro.sh
