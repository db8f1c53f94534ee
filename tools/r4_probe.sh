#!/bin/bash
# Round-4 probe (one GPU call): the GELU-table tests, the projection-GEMM timings (k_pg,
# k_pg with the GELU table, k_pg2, round 2), the MFMA / VALU co-issue microbenchmarks
# (fill, xwave, valu, overlap2; built beforehand in tools/micro), the counter list, and PMC
# passes over k_pg vs k_pg2 vs the table epilogue at the QKV and FFN-up shapes
# (tools/pg_micro.py runs them in one process; the kernel names separate them in the CSV).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
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
