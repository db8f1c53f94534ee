# round 6: the residual epilogue straight from the accumulator layout (NQK_PG_RDIRECT=1: no LDS
# transposes, all three stages of the next tile issued before the stores): output check against the
# shipped build + kernel timing (pg_micro), then the whole bench interleaved (verified = every row
# against the node loop)
set -u
mkdir -p gpurun_out
PGM_CHECK=1 PGM_SHAPES=out,down PGM_ROUNDS=4 PGM_LIBS=rdir=tools/diag/libnqk_rdir.so timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/r6t_pg_micro.txt 2>&1 || exit 3
if grep -q "DIFF" gpurun_out/r6t_pg_micro.txt; then echo "output differs" > gpurun_out/r6t_status.txt; exit 4; fi
OUT=r6t AB_LIBS="main rdir" AB_REPS=2 AB_BENCH="--steps 30" bash tools/ab.sh || exit 5
echo done > gpurun_out/r6t_status.txt
