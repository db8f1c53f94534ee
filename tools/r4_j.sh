#!/bin/bash
# round-4 call J: FFN-down's f32 dequantize from the weights' column L1 bound — parity and
# whole-bench A/B against the f64 dequantize (NQK_NO_L1=1)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/j.status
step() { echo "== $1 rc=$2" >> gpurun_out/j.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/j_tests.log 2>&1
step tests $?
AB_ENVS="nol1:NQK_NO_L1=1" AB_REPS=2 OUT=j bash tools/ab.sh
step ab $?
echo done >> gpurun_out/j.status
