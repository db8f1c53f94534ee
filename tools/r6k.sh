# round 6: k_attn16 with five waves per workgroup (NQK_ATTN16_NW=5: a workgroup's life 3 row tiles
# instead of 4) against four, ViT-Ti and ViT-Base, interleaved on one box
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6k_tests.log 2>&1 || exit 3
A="--no-cpu-baseline --no-secondary --steps 20 --warmup 3"
for r in 1 2; do
  for nw in 4 5; do
    NQK_ATTN16_NW=$nw timeout -k 10 200 python -u bench.py $A --config vit_tiny > gpurun_out/r6k_tiny_nw${nw}_$r.json 2>gpurun_out/r6k_tiny_nw${nw}_$r.err || exit 4
    NQK_ATTN16_NW=$nw timeout -k 10 200 python -u bench.py $A > gpurun_out/r6k_vit_nw${nw}_$r.json 2>gpurun_out/r6k_vit_nw${nw}_$r.err || exit 5
  done
done
echo done > gpurun_out/r6k_status.txt
