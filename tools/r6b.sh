# round 6: fused LayerNorm (ViT-Ti) parity + same-box A/B of the ViT-Ti bench
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_kernels.py -k "fused_layernorm or refuses" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r6b_tests.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -x -q -rf --timeout 200 --timeout-method thread >> gpurun_out/r6b_tests.log 2>&1 || exit 3
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config vit_tiny --no-cpu-baseline --no-secondary --steps 20 > gpurun_out/r6b_tiny_fused_$i.json 2>/dev/null || exit 4
  NQK_NO_LNFUSE=1 timeout -k 10 200 python -u bench.py --config vit_tiny --no-cpu-baseline --no-secondary --steps 20 > gpurun_out/r6b_tiny_unfused_$i.json 2>/dev/null || exit 5
done
