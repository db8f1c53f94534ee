#!/bin/bash
# Diagnostic builds of libnqk.so with compile-time variants of the persistent 16x16x64
# projection GEMM (nqk_pgemm.hip): NQK_PG_DIAG bits (1 no epilogue stores, 2 trivial
# epilogue math, 4 no operand loads, 8 no k-loop barriers, 16 no fragment reads).
# Arguments are name=FLAGS pairs, e.g. d3="-DNQK_PG_DIAG=3"; each builds
# tools/diag/libnqk_<name>.so.  Results may be garbage; the timings (tools/pg_micro.py with
# PGM_LIBS=name=tools/diag/libnqk_name.so,...) show which resource bounds the kernel.
set -e
cd "$(dirname "$0")/../numpy-quant_amd/csrc"
make -s
mkdir -p build/diag ../../tools/diag
for arg in "$@"; do
  name="${arg%%=*}"; flags="${arg#*=}"
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-function \
    -Wno-unused-variable --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt \
    $flags -c nqk_pgemm.hip -o build/diag/nqk_pgemm_$name.o &
done
wait
for arg in "$@"; do
  name="${arg%%=*}"
  objs=$(ls build/*.o | grep -v nqk_pgemm.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/diag/libnqk_$name.so $objs \
    build/diag/nqk_pgemm_$name.o -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
done
