# round 6: k_attn16 with interleaved exp pairs (nops 495 -> 70) vs k_attention, bench data; parity
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r6g_tests.log 2>&1 || exit 3
AM_ENV="old:NQK_ATTN16=0" AM_LIBS=w2=tools/diag/libnqk_a16w2.so timeout -k 10 300 python -u tools/attn_real.py > gpurun_out/r6g_attn_real.txt 2>&1 || exit 4
