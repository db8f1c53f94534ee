set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_attention.py "tests/test_gpu_kernels.py::test_fast_division_exp_erf_exhaustive" "tests/test_gpu_kernels.py::test_gelu_filter_bound_exhaustive" -q --timeout 200 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3l_tests.log
tail -4 gpurun_out/r3l_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AM_LIBS=pk0=tools/diag/libnqk_pk0.so timeout -k 10 120 python -u tools/attn_micro.py > gpurun_out/r3l_attn.txt 2>&1 || exit 1
cat gpurun_out/r3l_attn.txt
export NQK_PG_RESID=1
PGM_DIAGS="head" OUT=r3l_micro bash tools/r3_micro.sh
