#!/bin/bash
# round-4 call E: parity of the changed kernels (QKV with the saturating convert, the patch
# embedding's cheaper A conversion and epilogue), QKV micro A/B, whole-bench A/B against the
# previous commit's build (tools/diag/libnqk_prev.so)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/e.status
step() { echo "== $1 rc=$2" >> gpurun_out/e.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_fused_kernels.py tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/e_tests.log 2>&1
step tests $?
timeout -k 10 300 env PGM_SHAPES=qkv PGM_ENV="nos8:NQK_PG_NOS8=1" python -u tools/pg_micro.py > gpurun_out/e_pg_qkv.txt 2>&1
step pg_qkv $?
AB_LIBS="main prev" AB_REPS=2 OUT=e bash tools/ab.sh
step ab $?
echo done >> gpurun_out/e.status
