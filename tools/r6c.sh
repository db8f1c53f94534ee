# round 6: k_attn16 parity (both kernels on every attention case) + the bench-data timing A/B
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r6c_tests.log 2>&1 || exit 3
AM_ENV="a16:NQK_ATTN16=1" timeout -k 10 300 python -u tools/attn_real.py > gpurun_out/r6c_attn_real.txt 2>&1 || exit 4
