#!/bin/bash
# fused attention: parity tests, then the B=256 timing
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "attention or attn or plan or b256" --timeout 200 --timeout-method thread > gpurun_out/attn_test.log 2>&1 || exit 1
timeout -k 10 60 python -u tools/attn_micro.py > gpurun_out/attn_micro.txt 2>&1
