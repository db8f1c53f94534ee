#!/bin/bash
# round-4 call B: the exhaustive exp checks, attention variants, LayerNorm quantize A/B, bench A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/b.status
step() { echo "== $1 rc=$2" >> gpurun_out/b.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pgemm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/b_tests.log 2>&1
step tests $?
timeout -k 10 300 env AM_ROUNDS=5 AM_LIBS=apc=tools/diag/libnqk_apc.so,aexp=tools/diag/libnqk_aexp.so,aall=tools/diag/libnqk_aall.so,afull=tools/diag/libnqk_afull.so \
  python -u tools/attn_micro.py > gpurun_out/b_attn_ab.txt 2>&1
step attn_ab $?
timeout -k 10 200 python -u tools/ln_micro.py > gpurun_out/b_ln_ab.txt 2>&1
step ln_ab $?
# the two halves of the dropped tail split measured alone: the whole rounds (M = 341 row
# panels) and the 53 remaining panels (159 tiles, one workgroup each)
for m in 43648 6784; do
  timeout -k 10 200 env GM_M=$m PGM_SHAPES=out,down python -u tools/pg_micro.py > gpurun_out/b_pg_m$m.txt 2>&1
  step pg_m$m $?
done
AB_ENVS="lnexact:NQK_LN_EXACTQ=1" AB_REPS=2 OUT=b bash tools/ab.sh
step ab $?
echo done >> gpurun_out/b.status
