#!/bin/bash
# round-4 call C: the whole GPU suite, then whole-bench A/B of the 3-stage-ring patch
# embedding (k_embed_q3) against the round-3 kernel (NQK_EMBED_RING=0)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/c.status
step() { echo "== $1 rc=$2" >> gpurun_out/c.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/c_tests.log 2>&1
step tests $?
AB_ENVS="noring:NQK_EMBED_RING=0" AB_REPS=2 OUT=c bash tools/ab.sh
step ab $?
echo done >> gpurun_out/c.status
