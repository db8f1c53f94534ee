#!/bin/bash
# full GPU parity suite, then the B=256 GEMM timings and one bench line
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/gemm_micro.py > gpurun_out/gmd_base.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err
