#!/bin/bash
# round-4 call D: v_cvt_pk_u8_f32 saturation probe; PMC of the whole forward (two SQ passes
# over a short bench run: attention after its round-4 changes, patch embedding, k_pg incl.
# SQ_VALU_MFMA_COEXEC_CYCLES)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
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
