# round 6: does the GELU GEMM's int8 store pattern (16 rows x 64 B per instruction: half lines) cost?
# diagnostic 8192 writes the same bytes as 1 KiB contiguous per instruction (wrong layout, timing only)
set -u
mkdir -p gpurun_out
PGM_SHAPES=up PGM_ROUNDS=5 PGM_LIBS=gline=tools/diag/libnqk_gline.so timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/r6u_pg_micro.txt 2>&1 || exit 3
echo done > gpurun_out/r6u_status.txt
