# round 6: k_qgemm_big<RESID> with pass 0's residual rows issued before the k loop (NQK_BIG_RPRE=1, the
# main build) against without (tools/diag/libnqk_rpre0.so): parity tests, then ViT-Ti / ViT-Base int4
# benches interleaved
set -u
mkdir -p gpurun_out
OUT=r6v AB_TESTS="tests/test_gpu_fused_kernels.py tests/test_gpu_plan.py" AB_LIBS="main rpre0" AB_REPS=3 AB_BENCH="--config vit_tiny --steps 30" bash tools/ab.sh || exit 3
echo done > gpurun_out/r6v_status.txt
