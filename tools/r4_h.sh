#!/bin/bash
# round-4 call H: attention with the per-element P filter margin — parity, timing on the bench's
# data against the row-wide margin (aprel0) with slow-path counters (astat), whole-bench A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/h.status
step() { echo "== $1 rc=$2" >> gpurun_out/h.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_kernels.py tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1
step tests $?
timeout -k 10 400 env AM_LIBS=aprel0=tools/diag/libnqk_aprel0.so,astat=tools/diag/libnqk_astat.so python -u tools/attn_real.py > gpurun_out/h_attn_real.txt 2>&1
step attn_real $?
AB_LIBS="main aprel0" AB_REPS=2 OUT=h bash tools/ab.sh
step ab $?
echo done >> gpurun_out/h.status
