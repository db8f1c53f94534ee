#!/bin/bash
# round-2 projection GEMM check: persistent-kernel parity, then the B=256 GEMM timings
# (tools/gemm_micro.py) of the default build and of any diagnostic builds named
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_kernels.py -x -q -k "persistent" --timeout 120 --timeout-method thread > gpurun_out/proj_test.log 2>&1
rc=$?; echo "test rc=$rc" >> gpurun_out/proj_test.log; [ $rc -ne 0 ] && exit $rc
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="GM_LIB=tools/diag/libnqk_$v.so"; fi
  env $L timeout -k 10 120 python -u tools/gemm_micro.py > gpurun_out/gmd_$v.txt 2>&1 || exit 1
done
