#!/bin/bash
# LayerNorm+quantize: parity tests, then timings of the LDS-transposed and register kernels
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "ln or layernorm or plan" --timeout 120 --timeout-method thread > gpurun_out/ln_test.log 2>&1 || exit 1
timeout -k 10 60 python -u tools/ln_micro.py > gpurun_out/ln_micro.txt 2>&1 || exit 1
NQK_LN_REG=1 timeout -k 10 60 python -u tools/ln_micro.py >> gpurun_out/ln_micro.txt 2>&1 || exit 1
timeout -k 10 60 python -u tools/ln_micro.py >> gpurun_out/ln_micro.txt 2>&1
