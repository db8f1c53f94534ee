# round 6: k_attn16 variants on the bench's data (main = QPF 1, MINB 4)
set -u
mkdir -p gpurun_out
NQK_ATTN16=1 AM_ENV="old:NQK_ATTN16=0" AM_LIBS=q0=tools/diag/libnqk_a16q0.so,m5=tools/diag/libnqk_a16m5.so,m6=tools/diag/libnqk_a16m6.so timeout -k 10 300 python -u tools/attn_real.py > gpurun_out/r6d_attn_real.txt 2>&1 || exit 4
