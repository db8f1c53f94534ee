# round 6: the patch embedding on v_mfma_f32_16x16x4_f32 (NQK_EMBED_MFMA=16) against 32x32x2: parity
# (both forms), the kernel side by side (tools/embed_micro.py), the whole bench interleaved
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_kernels.py -k embed_q -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r6q_tests.log 2>&1 || exit 3
EMB_ENV="m16:NQK_EMBED_MFMA=16;m16wn1:NQK_EMBED_MFMA=16,NQK_EMBED_WN1=1" timeout -k 10 300 python -u tools/embed_micro.py > gpurun_out/r6q_embed_micro.txt 2>&1 || exit 4
A="--no-cpu-baseline --no-secondary --steps 30 --warmup 3"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r6q_main_$r.json 2>gpurun_out/r6q_main_$r.err || exit 5
  NQK_EMBED_MFMA=16 timeout -k 10 200 python -u bench.py $A > gpurun_out/r6q_m16_$r.json 2>gpurun_out/r6q_m16_$r.err || exit 6
done
NQK_EMBED_MFMA=16 timeout -k 10 200 python -u bench.py $A --config vit_tiny > gpurun_out/r6q_tiny_m16.json 2>gpurun_out/r6q_tiny_m16.err || exit 7
timeout -k 10 200 python -u bench.py $A --config vit_tiny > gpurun_out/r6q_tiny_main.json 2>gpurun_out/r6q_tiny_main.err || exit 8
echo done > gpurun_out/r6q_status.txt
