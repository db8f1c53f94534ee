# round 6: the patch embedding inside the two-stream step: default bench, the
# bench with nqk_embed_q skipped (tools/embed_diag.py, timing only), 128 x 64 embedding tiles at 3
# workgroups per CU (NQK_EMBED_WN1=1), interleaved; then a kernel trace of the default two-stream bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --no-secondary --steps 20 --warmup 3"
NQK_EMBED_WN1=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_fused_kernels.py -k embed_q -x -q --timeout 120 --timeout-method thread > gpurun_out/r6j_tests.log 2>&1 || exit 3
for r in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r6j_main_$r.json 2>gpurun_out/r6j_main_$r.err || exit 4
  timeout -k 10 200 python -u tools/embed_diag.py $A > gpurun_out/r6j_noembed_$r.json 2>gpurun_out/r6j_noembed_$r.err || exit 5
  NQK_EMBED_WN1=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/r6j_wn1_$r.json 2>gpurun_out/r6j_wn1_$r.err || exit 6
done
rm -rf gpurun_out/r6j_prof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6j_prof -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/r6j_prof.json 2>gpurun_out/r6j_prof.err || exit 7
echo done > gpurun_out/r6j_status.txt
