set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_plan.py tests/test_gpu_b256.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_attn_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_attn_tests.log
tail -4 gpurun_out/r3_attn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AM_LIBS=old=tools/diag/libnqk_old.so timeout -k 10 200 python -u tools/attn_micro.py
