#!/bin/bash
# Variant builds of libnqk.so for same-box A/B runs (tools/ab.sh AB_LIBS=..., tools/pg_micro.py
# PGM_LIBS=...): each argument name=FILES:FLAGS recompiles the listed sources (comma-separated,
# relative to numpy-quant_amd/csrc) with the extra FLAGS and links tools/diag/libnqk_<name>.so
# from them and the main build's other objects.  e.g.
#   bash tools/diag_build.sh lnnt=nqk_fused.hip:-DNQK_LN_NT=1
set -e
cd "$(dirname "$0")/../numpy-quant_amd/csrc"
make -s -j8
mkdir -p build/diag ../../tools/diag
FL="-O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt"
for arg in "$@"; do
  name="${arg%%=*}"; rest="${arg#*=}"; files="${rest%%:*}"; flags="${rest#*:}"
  for f in ${files//,/ }; do
    /opt/rocm/bin/hipcc $FL $flags -c $f -o build/diag/${f%.hip}_$name.o &
  done
done
wait
for arg in "$@"; do
  name="${arg%%=*}"; rest="${arg#*=}"; files="${rest%%:*}"
  objs=""
  for o in build/*.o; do
    b=$(basename $o .o); keep=1
    for f in ${files//,/ }; do [ "$b" = "${f%.hip}" ] && keep=0; done
    [ $keep = 1 ] && objs+=" $o"
  done
  for f in ${files//,/ }; do objs+=" build/diag/${f%.hip}_$name.o"; done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/diag/libnqk_$name.so $objs \
    -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
done
