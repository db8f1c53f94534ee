# round 6: PMC of k_attn16 on the bench's data (two passes)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA"
i=0
for p in "$P1" "$P2"; do
  i=$((i+1))
  NQK_ATTN16=1 timeout -s KILL 200 rocprofv3 --pmc $p --kernel-trace -d gpurun_out/pmc_a16_$i -o run --output-format csv -- python -u tools/attn_real.py > gpurun_out/pmc_a16_$i.log 2>&1 || exit 3
done
