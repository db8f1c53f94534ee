#!/bin/bash
# residual GEMMs (attention output, FFN down): big tile, persistent, null epilogue
set -u
mkdir -p gpurun_out
o=gpurun_out/resid.txt
: > $o
for sh in out down; do
  GM_ONLY=$sh:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
  NQK_PROJ_RESID=1 GM_ONLY=$sh:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
  GM_ONLY=$sh:null_epi timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
  GM_M=25216 GM_ONLY=$sh:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
done
