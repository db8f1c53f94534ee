set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AM_LIBS=a64=tools/diag/libnqk_a64.so,a8=tools/diag/libnqk_a8.so,a40=tools/diag/libnqk_a40.so timeout -k 10 200 python -u tools/attn_micro.py > gpurun_out/r3_attn_diag3.txt 2>&1 || exit 1
cat gpurun_out/r3_attn_diag3.txt
rm -rf gpurun_out/trace2
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace2 -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/trace2_bench.json 2> gpurun_out/trace2_bench.err || exit 1
echo traced
