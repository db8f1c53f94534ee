#!/bin/bash
# persistent-GEMM parity, the half-batch GEMM timings, then A/B bench runs
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_kernels.py -x -q -k "persistent" --timeout 120 --timeout-method thread > gpurun_out/proj_test.log 2>&1 || exit 1
GM_M=25216 timeout -k 10 120 python -u tools/gemm_micro.py > gpurun_out/gmd_half.txt 2>&1 || exit 1
bash tools/r02_ab.sh "$@"
