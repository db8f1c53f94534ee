#!/bin/bash
# k_proj epilogue cost split: default vs diagnostic builds (1 = no epilogue stores,
# 2 = trivial epilogue math, 3 = both), QKV and FFN-up + GELU (NQK_PROJ_GELU=1), and the
# k_qgemm_big GELU default for reference.  Output: gpurun_out/pjdiag.txt
set -u
mkdir -p gpurun_out
out=gpurun_out/pjdiag.txt
: > $out
for lib in default pj1 pj2 pj3; do
  if [ $lib = default ]; then L=""; else L=tools/diag/libnqk_$lib.so; fi
  echo "== $lib" >> $out
  GM_LIB=$L GM_ONLY=qkv:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $out 2>&1 || exit 1
  NQK_PROJ_GELU=1 GM_LIB=$L GM_ONLY=up:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $out 2>&1 || exit 1
done
echo "== k_qgemm_big GELU (default library)" >> $out
GM_ONLY=up:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $out 2>&1
