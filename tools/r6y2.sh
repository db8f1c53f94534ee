# round 6: the opt-in variants at model level — B = 256 fused forwards (test_gpu_b256.py) with the
# 16x16x4 patch embedding (NQK_EMBED_MFMA=16) and five-wave attention workgroups (NQK_ATTN16_NW=5)
set -u
mkdir -p gpurun_out
NQK_EMBED_MFMA=16 NQK_ATTN16_NW=5 timeout -k 10 600 python -u -m pytest tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r6y2_tests.log 2>&1 || exit 3
echo done > gpurun_out/r6y2_status.txt
