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

r5_c() {
  # LayerNorm non-temporal row loads (whole-bench A/B, 3 interleaved reps); the
  # attention's parked cycles (item 2): diagnostic builds without the workgroup barriers (1024), the
  # Q loads (2048), the K / V loads (64), all three (3136), timed on the bench's data in one
  # process, then PMC (wave cycles, parked, issue-stalled) per build, each under its own pass
  rm -f $STATUS
  AB_LIBS="main lnnt" AB_REPS=3 OUT=c timeout -k 10 900 bash tools/ab.sh
  step ab_ln $?
  AM_LIBS=a1024=tools/diag/libnqk_a1024.so,a2048=tools/diag/libnqk_a2048.so,a64=tools/diag/libnqk_a64.so,a3136=tools/diag/libnqk_a3136.so \
    timeout -k 10 300 python -u tools/attn_real.py > gpurun_out/c_attn_real.txt 2>&1
  step attn_real $?
  LIB=numpy-quant_amd/numpy_quant/libnqk.so
  cp $LIB /tmp/libnqk_main.so
  for v in main a1024 a2048 a64; do
    if [ $v = main ]; then cp /tmp/libnqk_main.so $LIB; else cp tools/diag/libnqk_$v.so $LIB; fi
    rm -rf gpurun_out/c_pmc_$v
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS \
      --kernel-trace -d gpurun_out/c_pmc_$v -o run --output-format csv -- python -u tools/attn_real.py > gpurun_out/c_pmc_$v.log 2>&1
    rc=$?
    cp /tmp/libnqk_main.so $LIB
    step pmc_$v $rc
  done
  echo done >> $STATUS
}

r5_d() {
  # persistent attention with wave 3 prefetching the next (image, head) pair (NQK_ATTN_PF, default
  # on): parity, then on the bench's data against the one-pair-per-workgroup form (NQK_ATTN_PF=0)
  # and the V-only prefetch build (pfv), then PMC (parked / issue-stalled cycles) of each
  rm -f $STATUS
  timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_b256.py tests/test_gpu_glut.py tests/test_gpu_fused_kernels.py \
    tests/test_gpu_pgemm.py::test_pg_gemm_vit_tiny_shapes tests/test_gpu_plan.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/d_tests.log 2>&1
  step tests $?
  # K = 192 with the weight panel resident (NQK_PG_RB, default on) vs streamed, ViT-Ti whole bench
  for rep in 1 2; do
    for v in rb norb wn1; do
      e=""; [ $v = norb ] && e="NQK_PG_RB=0"; [ $v = wn1 ] && e="NQK_EMBED_WN1=1"
      env $e timeout -k 10 300 python -u bench.py --config vit_tiny --no-cpu-baseline --steps 20 > gpurun_out/d_tiny_${v}_$rep.json 2> gpurun_out/d_tiny_${v}_$rep.err
      step tiny_$v $?
    done
  done
  AM_LIBS=pfv=tools/diag/libnqk_pfv.so AM_ENV="nopf:NQK_ATTN_PF=0" timeout -k 10 300 python -u tools/attn_real.py \
    > gpurun_out/d_attn_real.txt 2>&1
  step attn_real $?
  for v in pf nopf; do
    e=""; [ $v = nopf ] && e="NQK_ATTN_PF=0"
    rm -rf gpurun_out/d_pmc_$v
    env $e timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS \
      --kernel-trace -d gpurun_out/d_pmc_$v -o run --output-format csv -- python -u tools/attn_real.py > gpurun_out/d_pmc_$v.log 2>&1
    step pmc_$v $?
  done
  AB_ENVS="nopf:NQK_ATTN_PF=0" AB_REPS=2 OUT=d timeout -k 10 600 bash tools/ab.sh
  step ab $?
  echo done >> $STATUS
}

r5_f() {
  # the 256 x 256 form with a 4-deep ring (tools/diag/libnqk_rd4.so, NQK_PG_WM2_RD=4) against the
  # 3-deep one and the 128 x 256 form: parity of the 4-deep build (copied over the main library for
  # its tests), then the per-shape micro (both builds, NQK_PG_WM=1 / 2)
  rm -f $STATUS
  LIB=numpy-quant_amd/numpy_quant/libnqk.so
  cp $LIB /tmp/libnqk_main.so
  cp tools/diag/libnqk_rd4.so $LIB
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_glut.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/f_tests.log 2>&1
  rc=$?
  cp /tmp/libnqk_main.so $LIB
  step tests_rd4 $rc
  PGM_LIBS=rd4=tools/diag/libnqk_rd4.so PGM_ENV="wm2:NQK_PG_WM=2" PGM_SHAPES=qkv,up PGM_ROUNDS=3 \
    timeout -k 10 400 python -u tools/pg_micro.py > gpurun_out/f_pg_micro.txt 2>&1
  step pg_micro $?
  echo done >> $STATUS
}

r5_g() {
  # patch embedding with the XCD-aware tile order (default) vs the plain grid order
  # (NQK_EMBED_NOXCD=1): the embedding parity tests, whole-bench A/B, then FETCH_SIZE of each
  rm -f $STATUS
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_kernels.py -k embed -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/g_tests.log 2>&1
  step tests $?
  AB_ENVS="noxcd:NQK_EMBED_NOXCD=1" AB_REPS=3 OUT=g timeout -k 10 900 bash tools/ab.sh
  step ab $?
  for v in xcd noxcd; do
    e=""; [ $v = noxcd ] && e="NQK_EMBED_NOXCD=1"
    rm -rf gpurun_out/g_pmc_$v
    env $e NQK_SPLIT=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/g_pmc_$v -o run --output-format csv \
      -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/g_pmc_$v.log 2>&1
    step pmc_$v $?
  done
  echo done >> $STATUS
}

r5_h() {
  # stream parts of the fused forward (NQK_STREAMS = 2 default, 3, 4) for ViT-Ti and ViT-Base,
  # whole bench, 2 interleaved reps each
  rm -f $STATUS
  for rep in 1 2; do
    for cfg in vit_tiny vit; do
      for n in 2 3 4; do
        NQK_STREAMS=$n timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary --steps 20 \
          > gpurun_out/h_${cfg}_s${n}_$rep.json 2> gpurun_out/h_${cfg}_s${n}_$rep.err
        step ${cfg}_s$n $?
      done
    done
  done
  echo done >> $STATUS
}

"r5_$1"
