# interleaved softmax exp / round-pack in the fused attention (main build) vs the previous
# attention source (aold): exhaustive exp selftest + attention / model parity on the main
# build, then a same-box bench A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_attention.py tests/test_gpu_plan.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_attn2x2_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_attn2x2_tests.log
tail -3 gpurun_out/r3_attn2x2_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB_LIBS="aold" bash tools/r3_bench_ab.sh
