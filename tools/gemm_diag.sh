#!/bin/bash
# Diagnostic builds of libnqk.so with compile-time variants of the projection GEMM
# (nqk_fused.hip): NQK_DIAG bits (1 no global loads in the k loop, 2 no LDS fragment reads,
# 4 no barrier, 8 no MFMA) and NQK_TILE_ORDER (1 plain block order, 2 column-panel
# bands).  Arguments are name=FLAGS pairs, e.g. d3="-DNQK_DIAG=3" o1="-DNQK_TILE_ORDER=1";
# each builds tools/diag/libnqk_<name>.so.  SRC=nqk_attn selects the attention source
# (NQK_ATTN_DIAG) instead of nqk_fused.  Results may be garbage; the timings
# (tools/gemm_micro.py with GM_LIB=...) show which resource bounds the loop.
set -e
cd "$(dirname "$0")/../numpy-quant_amd/csrc"
make -s
mkdir -p build/diag ../../tools/diag
for arg in "$@"; do
  name="${arg%%=*}"; flags="${arg#*=}"
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wno-unused-function \
    -Wno-unused-variable --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize \
    $flags -c ${SRC:-nqk_fused}.hip -o build/diag/${SRC:-nqk_fused}_$name.o
  objs=$(ls build/*.o | grep -v ${SRC:-nqk_fused}.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/diag/libnqk_$name.so $objs \
    build/diag/${SRC:-nqk_fused}_$name.o -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
done
