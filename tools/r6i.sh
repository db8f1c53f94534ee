# round 6: residual rows in flight in the residual epilogue (RESQ 3 = shipped, 4, 5, 6)
set -u
mkdir -p gpurun_out
PGM_SHAPES=out,down PGM_ROUNDS=4 PGM_LIBS=q4=tools/diag/libnqk_q4.so,q5=tools/diag/libnqk_q5.so,q6=tools/diag/libnqk_q6.so timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/r6i_pg_micro.txt 2>&1 || exit 3
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_kernels.py -k "fused_layernorm or refuses" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r6i_tests.log 2>&1 || exit 4
