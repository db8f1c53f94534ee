#!/bin/bash
# round-4 call F: the attention kernel on the bench's own data (slow-path counters); the
# LayerNorm with two row groups per wave: parity, micro A/B, whole-bench A/B (also: the patch
# embedding with two workgroups per CU, 3 and 4 stream parts)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/f.status
step() { echo "== $1 rc=$2" >> gpurun_out/f.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1
step tests $?
timeout -k 10 200 env LNM_ENV="gpw1:NQK_LN_GPW1=1" python -u tools/ln_micro.py > gpurun_out/f_ln_ab.txt 2>&1
step ln_ab $?
timeout -k 10 400 env AM_LIBS=astat=tools/diag/libnqk_astat.so,aqdma=tools/diag/libnqk_aqdma.so python -u tools/attn_real.py > gpurun_out/f_attn_real.txt 2>&1
step attn_real $?
AB_ENVS="gpw1:NQK_LN_GPW1=1 e2wg:NQK_EMBED_1WG=0 s3:NQK_STREAMS=3 s4:NQK_STREAMS=4" AB_REPS=1 OUT=f bash tools/ab.sh
step ab $?
echo done >> gpurun_out/f.status
