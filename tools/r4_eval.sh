#!/bin/bash
# Round-4 evidence call: the whole GPU test suite, the default bench line, then same-box A/B
# bench runs (the round-3 library tools/diag/libnqk_r3.so; the 1-rank RCCL gather every step,
# NQK_FORCE_COMM=1; the filtered GELU chain instead of the table, NQK_NO_GLUT=1), a rocprofv3
# kernel trace of a short one-stream bench and the FETCH_SIZE / WRITE_SIZE passes
# (tools/gpu_full.sh).  SKIP_TESTS=1 / SKIP_AB=1 skip those parts.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/full.status gpurun_out/r4_ab.txt
step() { echo "== $1 rc=$2" >> gpurun_out/full.status; if [ $2 -ne 0 ]; then exit $2; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  step pytest $?
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
step bench $?
if [ "${SKIP_AB:-0}" != "1" ]; then
  AB_LIBS="main r3" AB_ENVS="comm:NQK_FORCE_COMM=1 noglut:NQK_NO_GLUT=1 lnexact:NQK_LN_EXACTQ=1" AB_REPS=1 OUT=r4 bash tools/ab.sh
  step ab $?
fi
# tail split of the N = 768 GEMMs (pg_launch) and the attention variants (diagnostic builds)
timeout -k 10 300 env PGM_SHAPES=out,up,down PGM_ENV="nosplit:NQK_PG_SPLIT=0" python -u tools/pg_micro.py \
  > gpurun_out/r4_pg_split.txt 2>&1
step pg_split $?
timeout -k 10 300 env AM_LIBS=arot=tools/diag/libnqk_arot.so,acpk=tools/diag/libnqk_acpk.so,apq=tools/diag/libnqk_apq.so,apc=tools/diag/libnqk_apc.so,aboth=tools/diag/libnqk_aboth.so \
  python -u tools/attn_micro.py > gpurun_out/r4_attn_ab.txt 2>&1
step attn_ab $?
SKIP_TESTS=1 SKIP_BENCH=1 bash tools/gpu_full.sh
step gpu_full $?
echo done >> gpurun_out/full.status
