#!/bin/bash
set -u
mkdir -p gpurun_out
o=gpurun_out/embed.txt
: > $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sgemm or embed or vit or plan or b256 or calibration" > gpurun_out/embed_tests.log 2>&1 || { echo "tests failed" >> $o; tail -20 gpurun_out/embed_tests.log >> $o; exit 1; }
tail -1 gpurun_out/embed_tests.log >> $o
for v in 32 16 32 16; do
  if [ $v = 16 ]; then E="NQK_SGEMM_K16=1"; else E="NQK_X=0"; fi
  env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_e.json 2> gpurun_out/bench_e.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/bench_e.json').read().strip().splitlines()[-1]); print('k$v', d['value'], d['ms_per_step'], d['verified'], d['kernels']['embed_sgemm']['avg_us'])" >> $o
done
