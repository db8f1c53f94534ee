# round 6: where k_embed_q's time goes (diagnostic builds, wrong results: timing only) + the default
# bench with the oracle check of image 0
set -u
mkdir -p gpurun_out
EMB_LIBS=nobar=tools/diag/libnqk_enobar.so,noconv=tools/diag/libnqk_enoconv.so,nost=tools/diag/libnqk_enost.so,all=tools/diag/libnqk_eall.so \
  EMB_ENV="wn1:NQK_EMBED_WN1=1" timeout -k 10 300 python -u tools/embed_micro.py > gpurun_out/r6o_embed_micro.txt 2>&1 || exit 3
timeout -k 10 500 python -u bench.py > gpurun_out/r6o_bench.json 2> gpurun_out/r6o_bench.err || exit 4
echo done > gpurun_out/r6o_status.txt
