# round 6: the BLAS level-2 restatements on the device (sdot at every length, GEMV-T small-m
# kernels, GEMV-N, matrix @ vector) and the model-level tests that route through them
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_api.py tests/test_gpu_models.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r6m_tests.log 2>&1 || exit 3
echo done > gpurun_out/r6m_status.txt
