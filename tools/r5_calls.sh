#!/bin/bash
# Round-5 GPU calls, one recipe per call (each ran as one gpurun command: bash tools/r5_calls.sh
# <name>).  Every GPU step runs under its own time limit and the first failure ends the call;
# results go to gpurun_out/ and the ones kept are copied to profiles/r05_*.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STATUS=gpurun_out/r5.status
step() { echo "== $1 rc=$2" >> $STATUS; if [ $2 -ne 0 ]; then exit $2; fi; }

r5_wm2() {
  # 256 x 256-tile k_pg (NQK_PG_WM=2, B shared by the two row halves) against the 128 x 256 form:
  # parity (k_pg vs k_qgemm_big, GELU table vs filtered chain, both forms), the per-shape micro,
  # then whole-bench A/B on the same box
  rm -f $STATUS
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_glut.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/wm2_tests.log 2>&1
  step tests $?
  PGM_ROUNDS=3 timeout -k 10 400 python -u tools/pg_micro.py > gpurun_out/wm2_pg_micro.txt 2>&1
  step pg_micro $?
  AB_ENVS="wm2:NQK_PG_WM=2" AB_REPS=2 OUT=wm2 timeout -k 10 600 bash tools/ab.sh
  step ab $?
  echo done >> $STATUS
}

r5_b() {
  # refactored k_pg build (instantiations split over files), GELU tables of up to 1024 entries on
  # the 256 x 256 form (ViT-Ti's FFN-up), non-blocking RCCL init: parity; hipBLASLt's int8 GEMM
  # at the projection shapes; ViT-Ti with / without its tables; the default bench line
  rm -f $STATUS
  timeout -k 10 900 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_glut.py tests/test_gpu_rccl.py \
    tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/b_tests.log 2>&1
  step tests $?
  timeout -k 10 300 python -u tools/hipblaslt_ref.py > gpurun_out/b_hipblaslt.txt 2>&1
  step hipblaslt $?
  for v in glut noglut; do
    e=""; [ $v = noglut ] && e="NQK_NO_GLUT=1"
    env $e timeout -k 10 300 python -u bench.py --config vit_tiny --no-cpu-baseline --steps 20 > gpurun_out/b_tiny_$v.json 2> gpurun_out/b_tiny_$v.err
    step tiny_$v $?
  done
  timeout -k 10 600 python -u bench.py > gpurun_out/b_bench.json 2> gpurun_out/b_bench.err
  step bench $?
  echo done >> $STATUS
}

"r5_$1"
