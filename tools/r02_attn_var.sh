#!/bin/bash
# attention timing for the default build and each diagnostic build named
set -u
mkdir -p gpurun_out
rm -f gpurun_out/attn_var.txt
timeout -k 10 60 python -u tools/attn_micro.py >> gpurun_out/attn_var.txt 2>&1 || exit 1
for v in "$@"; do
  echo "== $v" >> gpurun_out/attn_var.txt
  GM_LIB=tools/diag/libnqk_$v.so timeout -k 10 60 python -u tools/attn_micro.py >> gpurun_out/attn_var.txt 2>&1 || exit 1
done
