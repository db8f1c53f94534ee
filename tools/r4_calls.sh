#!/bin/bash
# Round-4 GPU calls, one recipe per call (each ran as one gpurun command: bash tools/r4_calls.sh
# <name>; the diagnostic builds a recipe names were made beforehand with tools/pg_diag.sh /
# tools/gemm_diag.sh, and some of their flags were removed once measured); they compose the parity tests, tools/ab.sh (whole-bench A/B), the micro tools and
# rocprofv3 passes.  The evidence each produced is under profiles/r04_*.  Every GPU step runs
# under its own time limit and the first failure ends the call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp

r4_probe() {
  # Round-4 probe (one GPU call): the GELU-table tests, the projection-GEMM timings (k_pg,
  # k_pg with the GELU table, k_pg2, round 2), the MFMA / VALU co-issue microbenchmarks
  # (fill, xwave, valu, overlap2; built beforehand in tools/micro), the counter list, and PMC
  # passes over k_pg vs k_pg2 vs the table epilogue at the QKV and FFN-up shapes
  # (tools/pg_micro.py runs them in one process; the kernel names separate them in the CSV).
  step() { echo "== $1 rc=$2" >> gpurun_out/probe.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  # pytest: rc 1 = failed tests (recorded, the measurements still run); anything else stops
  tstep() { echo "== $1 rc=$2" >> gpurun_out/probe.status; if [ $2 -ne 0 ] && [ $2 -ne 1 ]; then exit $2; fi; }
  rm -f gpurun_out/probe.status
  timeout -k 10 400 python -u -m pytest tests/test_gpu_glut.py "tests/test_gpu_pgemm.py::test_pg_gemm_int4_equals_big_tile" tests/test_gpu_b256.py -v --timeout 200 --timeout-method thread > gpurun_out/glut_tests.log 2>&1
  tstep glut_tests $?
  PGM_LIBS=spread=tools/diag/libnqk_spread.so PGM_ROUNDS=3 timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/pg_micro.txt 2>&1
  step pg_micro $?
  for m in fill xwave valu overlap2; do
    timeout -k 10 150 tools/micro/$m > gpurun_out/micro_$m.txt 2>&1
    step micro_$m $?
  done
  timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
  step counters $?
  export PGM_SHAPES=qkv,up PGM_ROUNDS=1 PGM_REPS=4
  passes=(
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
    "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU"
  )
  i=0
  for p in "${passes[@]}"; do
    i=$((i+1))
    rm -rf gpurun_out/pmc_pg_$i
    timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -d gpurun_out/pmc_pg_$i -o run --output-format csv -- python -u tools/pg_micro.py > gpurun_out/pmc_pg_$i.log 2>&1
    step pmc_pg_$i $?
  done
  echo done >> gpurun_out/probe.status

}

r4_eval() {
  # Round-4 evidence call: the whole GPU test suite, the default bench line, then same-box A/B
  # bench runs (the round-3 library tools/diag/libnqk_r3.so; the 1-rank RCCL gather every step,
  # NQK_FORCE_COMM=1; the filtered GELU chain instead of the table, NQK_NO_GLUT=1), a rocprofv3
  # kernel trace of a short one-stream bench and the FETCH_SIZE / WRITE_SIZE passes
  # (tools/gpu_full.sh).  SKIP_TESTS=1 / SKIP_AB=1 skip those parts.
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

}

r4_b() {
  # round-4 call B: the exhaustive exp checks, attention variants, LayerNorm quantize A/B, bench A/B
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

}

r4_c() {
  # round-4 call C: the whole GPU suite, then whole-bench A/B of the 3-stage-ring patch
  # embedding (k_embed_q3) against the round-3 kernel (NQK_EMBED_RING=0)
  rm -f gpurun_out/c.status
  step() { echo "== $1 rc=$2" >> gpurun_out/c.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/c_tests.log 2>&1
  step tests $?
  AB_ENVS="noring:NQK_EMBED_RING=0" AB_REPS=2 OUT=c bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/c.status

}

r4_d() {
  # round-4 call D: v_cvt_pk_u8_f32 saturation probe; PMC of the whole forward (two SQ passes
  # over a short bench run: attention after its round-4 changes, patch embedding, k_pg incl.
  # SQ_VALU_MFMA_COEXEC_CYCLES)
  rm -f gpurun_out/d.status
  step() { echo "== $1 rc=$2" >> gpurun_out/d.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 60 tools/micro/cvtu8 > gpurun_out/d_cvtu8.txt 2>&1
  step cvtu8 $?
  B="python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    --kernel-trace -d gpurun_out/pmc_d1 -o run --output-format csv -- $B > gpurun_out/pmc_d1.log 2>&1
  step pmc1 $?
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD \
    --kernel-trace -d gpurun_out/pmc_d2 -o run --output-format csv -- $B > gpurun_out/pmc_d2.log 2>&1
  step pmc2 $?
  echo done >> gpurun_out/d.status

}

r4_e() {
  # round-4 call E: parity of the changed kernels (QKV with the saturating convert, the patch
  # embedding's cheaper A conversion and epilogue), QKV micro A/B, whole-bench A/B against the
  # previous commit's build (tools/diag/libnqk_prev.so)
  rm -f gpurun_out/e.status
  step() { echo "== $1 rc=$2" >> gpurun_out/e.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 400 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/e_tests.log 2>&1
  step tests $?
  timeout -k 10 300 env PGM_SHAPES=qkv PGM_ENV="nos8:NQK_PG_NOS8=1" python -u tools/pg_micro.py > gpurun_out/e_pg_qkv.txt 2>&1
  step pg_qkv $?
  AB_LIBS="main prev" AB_REPS=2 OUT=e bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/e.status

}

r4_f() {
  # round-4 call F: the attention kernel on the bench's own data (slow-path counters); the
  # LayerNorm with two row groups per wave: parity, micro A/B, whole-bench A/B (also: the patch
  # embedding with two workgroups per CU, 3 and 4 stream parts)
  rm -f gpurun_out/f.status
  step() { echo "== $1 rc=$2" >> gpurun_out/f.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1
  step tests $?
  timeout -k 10 200 env LNM_ENV="gpw1:NQK_LN_GPW1=1" python -u tools/ln_micro.py > gpurun_out/f_ln_ab.txt 2>&1
  step ln_ab $?
  timeout -k 10 400 env AM_LIBS=astat=tools/diag/libnqk_astat.so,aqdma=tools/diag/libnqk_aqdma.so python -u tools/attn_real.py > gpurun_out/f_attn_real.txt 2>&1
  step attn_real $?
  AB_ENVS="gpw1:NQK_LN_GPW1=1 e2wg:NQK_EMBED_1WG=0 s3:NQK_STREAMS=3 s4:NQK_STREAMS=4" AB_REPS=1 OUT=f bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/f.status

}

r4_g() {
  # round-4 call G: the attention on the bench's own data (slow-path counters, Q by LDS-DMA);
  # whole-bench A/B: patch embedding one vs two workgroups per CU, 3 / 4 stream parts
  rm -f gpurun_out/g.status
  step() { echo "== $1 rc=$2" >> gpurun_out/g.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 400 env AM_LIBS=astat=tools/diag/libnqk_astat.so,aqdma=tools/diag/libnqk_aqdma.so python -u tools/attn_real.py > gpurun_out/g_attn_real.txt 2>&1
  step attn_real $?
  AB_ENVS="e2wg:NQK_EMBED_1WG=0 s3:NQK_STREAMS=3 s4:NQK_STREAMS=4" AB_REPS=1 OUT=g bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/g.status

}

r4_h() {
  # round-4 call H: attention with the per-element P filter margin — parity, timing on the bench's
  # data against the row-wide margin (aprel0) with slow-path counters (astat), whole-bench A/B
  rm -f gpurun_out/h.status
  step() { echo "== $1 rc=$2" >> gpurun_out/h.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_kernels.py tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1
  step tests $?
  timeout -k 10 400 env AM_LIBS=aprel0=tools/diag/libnqk_aprel0.so,astat=tools/diag/libnqk_astat.so python -u tools/attn_real.py > gpurun_out/h_attn_real.txt 2>&1
  step attn_real $?
  AB_LIBS="main aprel0" AB_REPS=2 OUT=h bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/h.status

}

r4_j() {
  # round-4 call J: FFN-down's f32 dequantize from the weights' column L1 bound — parity and
  # whole-bench A/B against the f64 dequantize (NQK_NO_L1=1)
  rm -f gpurun_out/j.status
  step() { echo "== $1 rc=$2" >> gpurun_out/j.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 400 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/j_tests.log 2>&1
  step tests $?
  AB_ENVS="nol1:NQK_NO_L1=1" AB_REPS=2 OUT=j bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/j.status

}

r4_k() {
  # round-4 call K: the QKV filter margin 6.25 / 5.25 units (was 8 / 16): QKV parity, exact-path
  # entries per forward before / after (diagnostic builds over the library), whole-bench A/B
  rm -f gpurun_out/k.status
  step() { echo "== $1 rc=$2" >> gpurun_out/k.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 400 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k_tests.log 2>&1
  step tests $?
  LIB=numpy-quant_amd/numpy_quant/libnqk.so
  cp $LIB /tmp/libnqk_main.so
  for v in slowold slow; do
    cp tools/diag/libnqk_$v.so $LIB
    timeout -k 10 300 python -u tools/pg_slow_rate.py > gpurun_out/k_slow_$v.txt 2>&1
    rc=$?
    cp /tmp/libnqk_main.so $LIB
    step slow_$v $rc
  done
  AB_LIBS="main qold" AB_REPS=2 OUT=k bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/k.status

}

r4_l() {
  # operand-delivery probe: k_pg without its B pieces (-DNQK_PG_DIAG=128), without its A pieces
  # (256), without both (4); wrong results, timings only
  rm -f gpurun_out/l.status
  timeout -k 10 300 env PGM_LIBS=nob=tools/diag/libnqk_nob.so,noa=tools/diag/libnqk_noa.so,noab=tools/diag/libnqk_noab.so PGM_ROUNDS=3 python -u tools/pg_micro.py > gpurun_out/l_pg_operands.txt 2>&1
  echo "== pg_operands rc=$?" >> gpurun_out/l.status
}


r4_m() {
  # round-4 call M: where the attention's time goes on the bench's own data — diagnostic builds
  # (tools/gemm_diag.sh with SRC=nqk_attn, NQK_ATTN_DIAG bits: 1 no V^T staging, 2 no exp,
  # 4 no P quantize, 8 no score MFMAs, 16 no context quantize, 32 no PV MFMAs, 64 no K/V loads,
  # 256 no P exact fallbacks, 512 the clamp-free P path everywhere) timed beside the main build
  rm -f gpurun_out/m.status
  step() { echo "== $1 rc=$2" >> gpurun_out/m.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  L=""
  for n in a1 a2 a4 a8 a16 a32 a64 a256 a512 a768; do L="$L,$n=tools/diag/libnqk_$n.so"; done
  timeout -k 10 400 env AM_LIBS="${L#,}" python -u tools/attn_real.py > gpurun_out/m_attn_real.txt 2>&1
  step attn_real $?
  echo done >> gpurun_out/m.status
}

r4_n() {
  # round-4 call N: the attention's P filter margins from the error bound (4.75 u |r| clamp-free,
  # 4.125 u |tf| clamped, instead of 8 u) and the double-float kpf variant (apkl, 3.125 u):
  # parity, timing and slow-path counts on the bench's data (aold = the previous build,
  # *stat = NQK_ATTN_DIAG 128 counters), whole-bench A/B main vs aold / apkl
  rm -f gpurun_out/n.status
  step() { echo "== $1 rc=$2" >> gpurun_out/n.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_kernels.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/n_tests.log 2>&1
  step tests $?
  timeout -k 10 400 env AM_LIBS=aold=tools/diag/libnqk_aold.so,apkl=tools/diag/libnqk_apkl.so,astat=tools/diag/libnqk_astat.so,aoldstat=tools/diag/libnqk_aoldstat.so,apklstat=tools/diag/libnqk_apklstat.so python -u tools/attn_real.py > gpurun_out/n_attn_real.txt 2>&1
  step attn_real $?
  AB_LIBS="main aold apkl" AB_REPS=2 OUT=n bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/n.status
}

r4_o() {
  # round-4 call O: instruction-cache counters per kernel over one B = 256 forward and the
  # attention timing loop (tools/attn_real.py); the attention kernel's code is 66 KB
  rm -f gpurun_out/o.status
  step() { echo "== $1 rc=$2" >> gpurun_out/o.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  rm -rf gpurun_out/pmc_ic
  timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_ic -o run --output-format csv -- python -u tools/attn_real.py > gpurun_out/o_pmc_ic.log 2>&1
  step pmc_ic $?
  python tools/pmc_kernels.py gpurun_out/pmc_ic --by-grid > gpurun_out/o_pmc_ic.txt 2>&1
  step table $?
  echo done >> gpurun_out/o.status
}

r4_p() {
  # round-4 call P: the attention's P exact fallbacks as one loop per tile over the failed
  # elements (NQK_ATTN_FBL=1, code 66 -> 54 KB) vs per element (afbl0): parity, bench-data timing
  rm -f gpurun_out/p.status
  step() { echo "== $1 rc=$2" >> gpurun_out/p.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_kernels.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/p_tests.log 2>&1
  step tests $?
  timeout -k 10 400 env AM_LIBS=afbl0=tools/diag/libnqk_afbl0.so python -u tools/attn_real.py > gpurun_out/p_attn_real.txt 2>&1
  step attn_real $?
  echo done >> gpurun_out/p.status
}

r4_q() {
  # round-4 call Q: the QKV and GELU-table epilogues without packed f32 instructions
  # (NQK_PG_NOPK=1; MI355X_MICROARCH.md: a v_pk_fma_f32 beside MFMAs costs more than two
  # v_fma_f32): projection-GEMM micro and whole-bench A/B (the bench verifies every row)
  rm -f gpurun_out/q.status
  step() { echo "== $1 rc=$2" >> gpurun_out/q.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 300 env PGM_LIBS=nopk=tools/diag/libnqk_nopk.so PGM_SHAPES=qkv,up PGM_ROUNDS=3 python -u tools/pg_micro.py > gpurun_out/q_pg_micro.txt 2>&1
  step pg_micro $?
  AB_LIBS="main nopk" AB_REPS=2 OUT=q bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/q.status
}

r4_r() {
  # round-4 call R: which k_pg epilogue of the unpacked build (NQK_PG_NOPK=1) differs — the
  # projection-GEMM parity tests with tools/diag/libnqk_nopk.so in place of the library
  # (on the box's copy of the tree only)
  rm -f gpurun_out/r.status
  cp tools/diag/libnqk_nopk.so numpy-quant_amd/numpy_quant/libnqk.so
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_glut.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/r_tests.log 2>&1
  echo "== tests rc=$?" >> gpurun_out/r.status
}

r4_s() {
  # round-4 call S: the QKV epilogue unpacked (NQK_PG_NOPK=1, now the default; the unpacked GELU
  # table epilogue of call Q wrote wrong bytes and is not used) against the packed build (qkvpk),
  # and the residual epilogue unpacked as well (rnopk): parity, micro, whole-bench A/B
  rm -f gpurun_out/s.status
  step() { echo "== $1 rc=$2" >> gpurun_out/s.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 700 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_glut.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s_tests.log 2>&1
  step tests $?
  timeout -k 10 300 env PGM_LIBS=qkvpk=tools/diag/libnqk_qkvpk.so,rnopk=tools/diag/libnqk_rnopk.so PGM_SHAPES=qkv,out,down PGM_ROUNDS=3 python -u tools/pg_micro.py > gpurun_out/s_pg_micro.txt 2>&1
  step pg_micro $?
  AB_LIBS="main qkvpk rnopk" AB_REPS=2 OUT=s bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/s.status
}

r4_t() {
  # round-4 call T: the attention's element pairs as two scalar instructions instead of v_pk_*
  # (NQK_ATTN_UNPK bits: 1 exp, 2 P quantize, 4 score dequantize, 8 context quantize, 15 all;
  # ps0 = NQK_ATTN_PSUM=0, the pairwise sums unpacked): the exhaustive exp test (covers the
  # unpacked exp), parity, timing on the bench's data
  rm -f gpurun_out/t.status
  step() { echo "== $1 rc=$2" >> gpurun_out/t.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_attention.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tests.log 2>&1
  step tests $?
  L=""
  for n in u1 u2 u4 u8 u15 ps0; do L="$L,$n=tools/diag/libnqk_$n.so"; done
  timeout -k 10 400 env AM_LIBS="${L#,}" python -u tools/attn_real.py > gpurun_out/t_attn_real.txt 2>&1
  step attn_real $?
  echo done >> gpurun_out/t.status
}

r4_u() {
  # round-4 call U (run twice: the second time after the "scc" clobber fix in nqk_glut.h, with the
  # main build's table / GEMM tests first): the GELU-table epilogue's f32 pairs unpacked through the vmul2 / vadd2 / vfma2
  # helpers (NQK_PG_GLUT_UNPK=1, tools/diag/libnqk_glutu.so): the table tests with that library in
  # place (box copy only), the FFN-up micro, whole-bench A/B (verified rows)
  rm -f gpurun_out/u.status
  step() { echo "== $1 rc=$2" >> gpurun_out/u.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 600 python -u -m pytest tests/test_gpu_glut.py tests/test_gpu_pgemm.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/u_tests_main.log 2>&1
  step glut_tests_main $?
  cp numpy-quant_amd/numpy_quant/libnqk.so /tmp/libnqk_keep.so
  cp tools/diag/libnqk_glutu.so numpy-quant_amd/numpy_quant/libnqk.so
  timeout -k 10 600 python -u -m pytest tests/test_gpu_glut.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/u_tests.log 2>&1
  rc=$?
  cp /tmp/libnqk_keep.so numpy-quant_amd/numpy_quant/libnqk.so
  step glut_tests_glutu $rc
  timeout -k 10 300 env PGM_LIBS=glutu=tools/diag/libnqk_glutu.so PGM_SHAPES=up PGM_ROUNDS=3 python -u tools/pg_micro.py > gpurun_out/u_pg_micro.txt 2>&1
  step pg_micro $?
  AB_LIBS="main glutu" AB_REPS=2 OUT=u bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/u.status
}

r4_final() {
  # round-4 closing evidence call: the whole GPU test suite, the default bench line, then
  # tools/gpu_full.sh's rocprofv3 kernel trace of a short one-stream bench and the FETCH_SIZE /
  # WRITE_SIZE passes (profiles/r04_final_*)
  rm -f gpurun_out/full.status
  step() { echo "== $1 rc=$2" >> gpurun_out/full.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  step pytest $?
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  step bench $?
  SKIP_TESTS=1 SKIP_BENCH=1 bash tools/gpu_full.sh
  step gpu_full $?
  echo done >> gpurun_out/full.status
}

r4_v() {
  # round-4 call V: the two half-batch streams out of phase (NQK_STREAM_OFFSET: the side stream
  # starts after part 0's embedding, or after a stage of part 0's first layer): parity of the
  # B = 256 forward under each offset, then whole-bench A/B (every row verified)
  rm -f gpurun_out/v.status
  step() { echo "== $1 rc=$2" >> gpurun_out/v.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  for o in embed attn; do
    NQK_STREAM_OFFSET=$o timeout -k 10 400 python -u -m pytest tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/v_tests_$o.log 2>&1
    step tests_$o $?
  done
  AB_ENVS="embed:NQK_STREAM_OFFSET=embed qkv:NQK_STREAM_OFFSET=qkv attn:NQK_STREAM_OFFSET=attn ln2:NQK_STREAM_OFFSET=ln2 up:NQK_STREAM_OFFSET=up" AB_REPS=2 OUT=v bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/v.status
}

r4_w() {
  # round-4 call W: the patch embedding's next-kernel-row image loads issued three k-tiles ahead
  # (NQK_EMBED_PXD=1) instead of one (pxd0): parity (the fused embedding against the im2col
  # path, the B = 256 forward), whole-bench A/B
  rm -f gpurun_out/w.status
  step() { echo "== $1 rc=$2" >> gpurun_out/w.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py tests/test_gpu_l1.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w_tests.log 2>&1
  step tests $?
  AB_LIBS="main pxd0" AB_REPS=3 OUT=w bash tools/ab.sh
  step ab $?
  echo done >> gpurun_out/w.status
}

r4_x() {
  # round-4 call X: sanity of the rebuilt library (same sources): smoke(), the table / GEMM /
  # B = 256 parity tests
  rm -f gpurun_out/x.status
  step() { echo "== $1 rc=$2" >> gpurun_out/x.status; if [ $2 -ne 0 ]; then exit $2; fi; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/x_smoke.log 2>&1
  step smoke $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_glut.py tests/test_gpu_pgemm.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/x_tests.log 2>&1
  step tests $?
  echo done >> gpurun_out/x.status
}

case "${1:-}" in
  probe|eval|b|c|d|e|f|g|h|j|k|l|m|n|o|p|q|r|s|t|u|v|w|x|final) "r4_$1" ;;
  *) echo "usage: tools/r4_calls.sh {probe|eval|b|c|d|e|f|g|h|j|k|l|m|n|o|p|q|r|s|t|u|v|w|x|final}" >&2; exit 2 ;;
esac
