#!/bin/bash
# PMC passes over one GEMM variant of tools/gemm_micro.py per diagnostic build:
# bash tools/r02_pmc.sh <shape:variant> <lib-name|base> ...
set -u
only=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then unset GM_LIB; else export GM_LIB=tools/diag/libnqk_$v.so; fi
  GM_ONLY=$only bash tools/pmc_passes.sh "${v}_${only/:/_}" python -u tools/gemm_micro.py || exit $?
done
