#!/bin/bash
# round-4 call G: the attention on the bench's own data (slow-path counters, Q by LDS-DMA);
# whole-bench A/B: patch embedding one vs two workgroups per CU, 3 / 4 stream parts
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/g.status
step() { echo "== $1 rc=$2" >> gpurun_out/g.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 400 env AM_LIBS=astat=tools/diag/libnqk_astat.so,aqdma=tools/diag/libnqk_aqdma.so python -u tools/attn_real.py > gpurun_out/g_attn_real.txt 2>&1
step attn_real $?
AB_ENVS="e2wg:NQK_EMBED_1WG=0 s3:NQK_STREAMS=3 s4:NQK_STREAMS=4" AB_REPS=1 OUT=g bash tools/ab.sh
step ab $?
echo done >> gpurun_out/g.status
