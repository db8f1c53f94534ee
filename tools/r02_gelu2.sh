#!/bin/bash
set -u
mkdir -p gpurun_out
o=gpurun_out/gelu2.txt
: > $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or gelu or plan or b256 or vit" > gpurun_out/gelu2_tests.log 2>&1 || { echo "tests failed" >> $o; tail -20 gpurun_out/gelu2_tests.log >> $o; exit 1; }
tail -1 gpurun_out/gelu2_tests.log >> $o
for r in 1 2; do
for lib in default row1; do
  if [ $lib = default ]; then L=""; else L=tools/diag/libnqk_$lib.so; fi
  echo -n "$lib " >> $o
  GM_LIB=$L GM_ONLY=up:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1
done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_g2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['verified'], {k:v['avg_us'] for k,v in d['kernels'].items()})" >> $o
