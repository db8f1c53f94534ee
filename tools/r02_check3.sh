#!/bin/bash
# parity of the fused GEMM paths, then GEMM timings for the shipped library and the
# diagnostic builds named in $LIBS, then the bench (default and NQK_PROJ_GELU=1)
set -u
mkdir -p gpurun_out
o=gpurun_out/check3.txt
: > $o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or plan or b256 or persistent or gelu" > gpurun_out/check3_tests.log 2>&1 || { echo "tests failed" >> $o; tail -30 gpurun_out/check3_tests.log >> $o; exit 1; }
tail -1 gpurun_out/check3_tests.log >> $o
for lib in default ${LIBS:-}; do
  if [ $lib = default ]; then L=""; else L=tools/diag/libnqk_$lib.so; fi
  echo "== $lib" >> $o
  GM_LIB=$L GM_ONLY=qkv:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
  NQK_PROJ_GELU=1 GM_LIB=$L GM_ONLY=up:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
  GM_LIB=$L GM_ONLY=up:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
done
for lib in default ${ATTN_LIBS:-}; do
  if [ $lib = default ]; then L=""; else L=tools/diag/libnqk_$lib.so; fi
  echo "== attention $lib" >> $o
  GM_LIB=$L timeout -k 10 120 python -u tools/attn_micro.py >> $o 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err || exit 1
NQK_PROJ_GELU=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench3g.json 2> gpurun_out/bench3g.err || exit 1
python - >> $o <<'PY'
import json
for f in ("gpurun_out/bench3.json", "gpurun_out/bench3g.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("verified"), {k: v["avg_us"] for k, v in d.get("kernels", {}).items()})
PY
