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

r5_i() {
  # LayerNorm (k_ln_quant_lds): packed f32 pairs (NQK_LN_PK) and rows by LDS-DMA into a swizzled
  # image (NQK_LN_DMA), both default on: parity, the kernel micro of all four builds (each checked
  # byte for byte against the main build), then whole-bench A/B against the round-5 build (lnold)
  rm -f $STATUS
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/i_tests.log 2>&1
  step tests $?
  LNM_LIBS=old=tools/diag/libnqk_lnold.so,pk=tools/diag/libnqk_lnpk.so,dma=tools/diag/libnqk_lndma.so LNM_ROUNDS=7 \
    timeout -k 10 300 python -u tools/ln_micro.py > gpurun_out/i_ln_micro.txt 2>&1
  step ln_micro $?
  LNM_LIBS=old=tools/diag/libnqk_lnold.so LN_COLS=192 LNM_ROUNDS=7 timeout -k 10 300 python -u tools/ln_micro.py \
    > gpurun_out/i_ln_micro_tiny.txt 2>&1
  step ln_micro_tiny $?
  AB_LIBS="main lnold" AB_REPS=3 OUT=i timeout -k 10 900 bash tools/ab.sh
  step ab $?
  echo done >> $STATUS
}

r5_j() {
  # LayerNorm workgroup size (NQK_LN_WPB = 1 / 2 / 4 waves; LDS-DMA image for every leaf count):
  # parity of the LN kernels at each size, then the kernel micro for ViT-Base and ViT-Ti rows
  rm -f $STATUS
  for w in 1 2 4; do
    NQK_LN_WPB=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_kernels.py -k ln_quant -x -q --timeout 200 \
      --timeout-method thread > gpurun_out/j_tests_w$w.log 2>&1
    step tests_w$w $?
  done
  for c in 768 192; do
    LNM_LIBS=old=tools/diag/libnqk_lnold.so LNM_ENV="w1:NQK_LN_WPB=1;w2:NQK_LN_WPB=2" LN_COLS=$c LNM_ROUNDS=7 \
      timeout -k 10 300 python -u tools/ln_micro.py > gpurun_out/j_ln_micro_$c.txt 2>&1
    step ln_micro_$c $?
  done
  echo done >> $STATUS
}

r5_k() {
  # persistent double-buffered LayerNorm (NQK_LN_PERS = waves per CU) against the one-shot kernel at
  # 4 and 1 waves per workgroup: parity at each, kernel micro for ViT-Base / ViT-Ti rows, then
  # whole-bench A/B of both configs
  rm -f $STATUS
  for v in NQK_LN_PERS=6 NQK_LN_PERS=3 NQK_LN_WPB=1; do
    env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_kernels.py -k ln_quant -x -q --timeout 200 \
      --timeout-method thread > gpurun_out/k_tests_$v.log 2>&1
    step tests_$v $?
  done
  for c in 768 192; do
    LNM_ENV="w1:NQK_LN_WPB=1;p6:NQK_LN_PERS=6;p4:NQK_LN_PERS=4;p3:NQK_LN_PERS=3" LN_COLS=$c LNM_ROUNDS=7 \
      timeout -k 10 300 python -u tools/ln_micro.py > gpurun_out/k_ln_micro_$c.txt 2>&1
    step ln_micro_$c $?
  done
  for rep in 1 2; do
    for cfg in vit vit_tiny; do
      for v in main w1 p6; do
        e=""; [ $v = w1 ] && e="NQK_LN_WPB=1"; [ $v = p6 ] && e="NQK_LN_PERS=6"
        env $e timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary --steps 20 \
          > gpurun_out/k_${cfg}_${v}_$rep.json 2> gpurun_out/k_${cfg}_${v}_$rep.err
        step ${cfg}_${v} $?
      done
    done
  done
  echo done >> $STATUS
}

r5_l() {
  # k_pg operand delivery: L1 -> L2 read requests and L2 reads / hits per projection shape (the A
  # pieces read 64 of every 128-B line per k step), one --pmc pass per counter block
  rm -f gpurun_out/l_pmc_*
  for pass in tcp tcc; do
    if [ $pass = tcp ]; then c="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
    else c="TCC_READ_sum TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"; fi
    PGM_ROUNDS=1 PGM_REPS=3 timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/l_pmc_$pass -o run --output-format csv \
      -- python -u tools/pg_micro.py > gpurun_out/l_pmc_$pass.log 2>&1
    step pmc_$pass $?
  done
  echo done_l >> $STATUS
}

r5_m() {
  # does k_pg's operand stream pay per L1 -> L2 request?  A pieces as whole 128-B lines (diagnostic
  # 512: same bytes, half the A requests, wrong values) against the shipped pieces (16 rows x 64 B),
  # with the full epilogue and without it (diagnostic 3 / 515), per-shape micro
  rm -f $STATUS
  PGM_LIBS=a512=tools/diag/libnqk_a512.so,d3=tools/diag/libnqk_d3.so,d3a=tools/diag/libnqk_d3a.so PGM_ROUNDS=3 \
    timeout -k 10 400 python -u tools/pg_micro.py > gpurun_out/m_pg_micro.txt 2>&1
  step pg_micro $?
  echo done >> $STATUS
}

r5_n() {
  # LayerNorm defaults: one-shot 4-wave workgroups (main), 1-wave workgroups (w1), persistent with 4
  # waves per CU (p4), whole bench, 3 interleaved reps per config
  rm -f $STATUS
  for rep in 1 2 3; do
    for cfg in vit vit_tiny; do
      for v in main w1 p4; do
        e=""; [ $v = w1 ] && e="NQK_LN_WPB=1"; [ $v = p4 ] && e="NQK_LN_PERS=4"
        env $e timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary --steps 20 \
          > gpurun_out/n_${cfg}_${v}_$rep.json 2> gpurun_out/n_${cfg}_${v}_$rep.err
        step ${cfg}_${v} $?
      done
    done
  done
  echo done >> $STATUS
}

r5_o() {
  # the two batch parts offset so that different kernel kinds run side by side (NQK_STREAM_LAG: part
  # 1 starts a layer after part 0's LN1 / QKV / attention), with k_pg at one workgroup per CU
  # (NQK_PG_WGPC=1: half the register file left for the other part's attention), whole bench
  rm -f $STATUS
  timeout -k 10 300 env NQK_STREAM_LAG=qkv NQK_PG_WGPC=1 python -u -m pytest tests/test_gpu_b256.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/o_tests.log 2>&1
  step tests $?
  for rep in 1 2; do
    for v in main lagqkv lagattn lagln1 wgpc1 lagqkv_wgpc1 lagattn_wgpc1; do
      e=""
      case $v in
        lagqkv) e="NQK_STREAM_LAG=qkv";; lagattn) e="NQK_STREAM_LAG=attn";; lagln1) e="NQK_STREAM_LAG=ln1";;
        wgpc1) e="NQK_PG_WGPC=1";; lagqkv_wgpc1) e="NQK_STREAM_LAG=qkv NQK_PG_WGPC=1";;
        lagattn_wgpc1) e="NQK_STREAM_LAG=attn NQK_PG_WGPC=1";;
      esac
      env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 20 \
        > gpurun_out/o_${v}_$rep.json 2> gpurun_out/o_${v}_$rep.err
      step ${v}_$rep $?
    done
  done
  echo done >> $STATUS
}

r5_p() {
  # attention: the last row tile's 5 real rows by the row-parallel path (NQK_ATTN_TAIL, default on)
  # against the 32-row form (tools/diag/libnqk_notail.so): parity, the kernel on the bench's data
  # (both builds in one process), whole-bench A/B for both configs
  rm -f $STATUS
  timeout -k 10 900 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/p_tests.log 2>&1
  step tests $?
  AM_LIBS=notail=tools/diag/libnqk_notail.so timeout -k 10 300 python -u tools/attn_real.py > gpurun_out/p_attn_real.txt 2>&1
  step attn_real $?
  AB_LIBS="main notail" AB_REPS=3 OUT=p timeout -k 10 900 bash tools/ab.sh
  step ab $?
  LIB=numpy-quant_amd/numpy_quant/libnqk.so
  cp $LIB /tmp/libnqk_main.so
  for rep in 1 2; do
    for v in main notail; do
      if [ $v = main ]; then cp /tmp/libnqk_main.so $LIB; else cp tools/diag/libnqk_notail.so $LIB; fi
      timeout -k 10 300 python -u bench.py --config vit_tiny --no-cpu-baseline --no-secondary --steps 20 \
        > gpurun_out/p_tiny_${v}_$rep.json 2> gpurun_out/p_tiny_${v}_$rep.err
      rc=$?
      cp /tmp/libnqk_main.so $LIB
      step tiny_${v}_$rep $rc
    done
  done
  echo done >> $STATUS
}

r5_q() {
  # the whole forward replayed as one captured hipGraph (bench.py --graph 1: no per-kernel host
  # launches, the two parts' fork / join captured as graph edges) against eager issue, both configs
  rm -f $STATUS
  for rep in 1 2; do
    for cfg in vit vit_tiny; do
      for g in 0 1; do
        timeout -k 10 300 python -u bench.py --config $cfg --graph $g --no-cpu-baseline --no-secondary --steps 20 \
          > gpurun_out/q_${cfg}_g${g}_$rep.json 2> gpurun_out/q_${cfg}_g${g}_$rep.err
        step ${cfg}_g${g}_$rep $?
      done
    done
  done
  echo done >> $STATUS
}

r5_r() {
  # 256 x 256 B-shared tiles (NQK_PG_WM=2) against the shipped 128 x 256 form in the default bench
  # (hipGraph replay, two parts), 3 interleaved reps
  rm -f $STATUS
  AB_ENVS="wm2:NQK_PG_WM=2" AB_REPS=3 OUT=r timeout -k 10 900 bash tools/ab.sh
  step ab $?
  echo done >> $STATUS
}

r5_s() {
  # GELU tables: single-line bucket coordinates (k_pg<PG_GLUT1>, where they fit first) and the
  # (0.885 s, 7.7 s) two-line candidate that keeps ViT-Ti's tables within 512 entries: parity (both
  # table kinds), then ViT-Ti whole bench against the previous candidate set (NQK_GLUT_NO1=1
  # NQK_GLUT_NOWIDE=1), 3 interleaved reps
  rm -f $STATUS
  timeout -k 10 900 python -u -m pytest tests/test_gpu_glut.py tests/test_gpu_b256.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/s_tests.log 2>&1
  step tests $?
  for rep in 1 2 3; do
    for v in main old; do
      e=""; [ $v = old ] && e="NQK_GLUT_NO1=1 NQK_GLUT_NOWIDE=1"
      env $e timeout -k 10 300 python -u bench.py --config vit_tiny --no-cpu-baseline --no-secondary --steps 20 \
        > gpurun_out/s_tiny_${v}_$rep.json 2> gpurun_out/s_tiny_${v}_$rep.err
      step tiny_${v}_$rep $?
    done
  done
  echo done >> $STATUS
}

r5_t() {
  # ViT-Ti's K = 192 GEMMs (QKV, FFN-up + GELU table) at M giving exactly 2 / 2.31 / 3 passes of
  # 128 x 256 tiles over the 512 workgroup slots: how much does the partial last pass cost?
  rm -f $STATUS
  for m in 43648 50432 65536; do
    GM_M=$m PGM_SHAPES=tqkv,tup PGM_ROUNDS=3 timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/t_pg_micro_$m.txt 2>&1
    step micro_$m $?
  done
  echo done >> $STATUS
}

r5_u() {
  # k_pg 64-row tiles at K = 192 (WM = 0, default) against 128-row (NQK_PG_WM0=0): parity (ViT-Ti
  # shapes, GELU tables, the ViT-Ti forward in the plan tests), the kernel micro at M giving 2 /
  # 2.31 / 3 passes of 128-row tiles, then ViT-Ti whole bench, 3 interleaved reps
  rm -f $STATUS
  timeout -k 10 900 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_glut.py tests/test_gpu_plan.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/u_tests.log 2>&1
  step tests $?
  for m in 43648 50432 65536; do
    GM_M=$m PGM_SHAPES=tqkv,tup PGM_ROUNDS=3 PGM_ENV="r128:NQK_PG_WM0=0" timeout -k 10 300 python -u tools/pg_micro.py \
      > gpurun_out/u_pg_micro_$m.txt 2>&1
    step micro_$m $?
  done
  for rep in 1 2 3; do
    for v in main r128; do
      e=""; [ $v = r128 ] && e="NQK_PG_WM0=0"
      env $e timeout -k 10 300 python -u bench.py --config vit_tiny --no-cpu-baseline --no-secondary --steps 20 \
        > gpurun_out/u_tiny_${v}_$rep.json 2> gpurun_out/u_tiny_${v}_$rep.err
      step tiny_${v}_$rep $?
    done
  done
  echo done >> $STATUS
}

r5_v() {
  # the round's final tree: every GPU test, smoke(), a default bench line
  rm -f $STATUS
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/v_tests.log 2>&1
  step tests $?
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1
  step smoke $?
  timeout -k 10 400 python -u bench.py > gpurun_out/v_bench.json 2> gpurun_out/v_bench.err
  step bench $?
  echo done >> $STATUS
}

r5_w() {
  # with the hipGraph replay default: one stream part (NQK_SPLIT=0) and the persistent LayerNorm
  # (NQK_LN_PERS=4) against the shipped two parts / one-shot LN, whole bench, 3 interleaved reps
  rm -f $STATUS
  AB_ENVS="split0:NQK_SPLIT=0 lnp4:NQK_LN_PERS=4" AB_REPS=3 OUT=w timeout -k 10 1100 bash tools/ab.sh
  step ab $?
  echo done >> $STATUS
}

r5_x() {
  # attention: what the V staging alone costs (diagnostic 4096: V loads skipped, K kept; 64: both
  # skipped), the bench's data, one process
  rm -f $STATUS
  AM_LIBS=a4096=tools/diag/libnqk_a4096.so,a64=tools/diag/libnqk_a64.so timeout -k 10 300 python -u tools/attn_real.py \
    > gpurun_out/x_attn_real.txt 2>&1
  step attn_real $?
  echo done >> $STATUS
}

"r5_$1"
