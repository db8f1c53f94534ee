#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own time limit) over a
# command given as arguments, e.g.  GM_ONLY=down:null_epi bash tools/pmc_passes.sh tag python -u tools/gemm_micro.py
# Results: gpurun_out/pmc_<tag>_<pass>/run_counter_collection.csv
set -u
tag=$1; shift
export TMPDIR=/tmp
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-trace -d gpurun_out/pmc_${tag}_$i -o run --output-format csv -- "$@" > gpurun_out/pmc_${tag}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> gpurun_out/pmc_${tag}.status
  if [ $rc -ne 0 ]; then exit $rc; fi
done
