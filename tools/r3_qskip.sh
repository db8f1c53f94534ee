# QKV exact fallback restricted to the element groups whose filter measure failed (main)
# vs the previous k_pg (hold)
# GEMM / model parity on main, then a same-box bench A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_kernels.py tests/test_gpu_b256.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_qskip_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_qskip_tests.log
tail -3 gpurun_out/r3_qskip_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB_LIBS="hold" bash tools/r3_bench_ab.sh
