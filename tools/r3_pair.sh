set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
NQK_PG_PAIR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_b256.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_pair_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_pair_tests.log
tail -5 gpurun_out/r3_pair_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PGM_ENV="pair:NQK_PG_PAIR=1" OUT=r3e_micro bash tools/r3_micro.sh
