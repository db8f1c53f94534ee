set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pgemm.py -q --timeout 120 --timeout-method thread > gpurun_out/r3d_pgtest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3d_pgtest.log
tail -3 gpurun_out/r3d_pgtest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PGM_SHAPES=${PGM_SHAPES:-qkv,up} PGM_DIAGS="${PGM_DIAGS:-}" PGM_ENV="${PGM_ENV:-}" OUT=r3d_micro bash tools/r3_micro.sh
