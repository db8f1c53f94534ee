# round 6: full GPU suite + bench (ViT-Ti LN fusion, k_attn16 default) + A/B without k_attn16
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r6e_gpu_tests.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r6e_bench.json 2> gpurun_out/r6e_bench.err || exit 4
NQK_ATTN16=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r6e_bench_noa16.json 2>/dev/null || exit 5
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r6e_bench_2.json 2>/dev/null || exit 6
