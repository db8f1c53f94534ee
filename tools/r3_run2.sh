set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pgemm.py -q --timeout 120 --timeout-method thread > gpurun_out/r3b_pgtest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3b_pgtest.log
tail -3 gpurun_out/r3b_pgtest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PGM_DIAGS="d3 d4 d31" PGM_ENV="st1:NQK_PG_STAGGER=1;st3:NQK_PG_STAGGER=3" OUT=r3b_micro bash tools/r3_micro.sh
