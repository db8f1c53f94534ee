#!/bin/bash
# parity of the fused GEMM paths + GEMM timings + bench (one GPU call)
set -u
mkdir -p gpurun_out
o=gpurun_out/check2.txt
: > $o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or plan or b256 or persistent" > gpurun_out/check2_tests.log 2>&1 || { echo "tests failed" >> $o; exit 1; }
tail -2 gpurun_out/check2_tests.log >> $o
GM_ONLY=qkv:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
NQK_PROJ_GELU=1 GM_ONLY=up:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
GM_ONLY=up:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
echo "== pj1 (no stores)" >> $o
GM_LIB=tools/diag/libnqk_pj1.so GM_ONLY=qkv:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err || exit 1
NQK_PROJ_GELU=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench2g.json 2> gpurun_out/bench2g.err || exit 1
python - >> $o <<'PY'
import json
for f in ("gpurun_out/bench2.json", "gpurun_out/bench2g.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("verified"), {k: v["avg_us"] for k, v in d.get("kernels", {}).items()})
PY
