# GELU fast-path error per exponent (diagnostic print), then the full evidence call
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k gelu_filter_bound -s -q --timeout 150 --timeout-method thread > gpurun_out/gelu_bound.log 2>&1 || exit 1
tail -3 gpurun_out/gelu_bound.log
bash tools/gpu_full.sh
