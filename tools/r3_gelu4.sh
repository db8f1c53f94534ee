# interleaved two-pair GELU epilogue (NQK_PG_GELU4=1, main build) vs the pairwise one (g2):
# GEMM + GELU parity tests on the main build, then a same-box bench A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_kernels.py tests/test_gpu_b256.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_gelu4_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_gelu4_tests.log
tail -3 gpurun_out/r3_gelu4_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB_LIBS="g2" bash tools/r3_bench_ab.sh
