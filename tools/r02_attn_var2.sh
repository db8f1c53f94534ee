#!/bin/bash
# attention timing: shipped library vs the diagnostic builds named in $LIBS (two rounds)
set -u
mkdir -p gpurun_out
o=gpurun_out/attn_var2.txt
: > $o
for r in 1 2; do
for lib in default ${LIBS:-}; do
  if [ $lib = default ]; then L=""; else L=tools/diag/libnqk_$lib.so; fi
  echo -n "$lib: " >> $o
  GM_LIB=$L timeout -k 10 120 python -u tools/attn_micro.py >> $o 2>&1 || exit 1
done
done
