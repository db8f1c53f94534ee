#!/bin/bash
# the fused plan on 2 / 3 / 4 streams: parity (plan + B=256 tests) and bench
set -u
mkdir -p gpurun_out
o=gpurun_out/streams.txt
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sgemm or gemv or embed or vit_graphs" > gpurun_out/sgemm_tests.log 2>&1 || { echo "sgemm tests failed" >> $o; exit 1; }
echo "sgemm: $(tail -1 gpurun_out/sgemm_tests.log)" >> $o
for s in 3 4; do
  NQK_STREAMS=$s timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "plan or b256" > gpurun_out/streams_tests_$s.log 2>&1 || { echo "tests failed at $s streams" >> $o; exit 1; }
  echo "streams $s: $(tail -1 gpurun_out/streams_tests_$s.log)" >> $o
done
for s in 2 3 4 2; do
  NQK_STREAMS=$s timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s$s.json 2> gpurun_out/bench_s$s.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/bench_s$s.json').read().strip().splitlines()[-1]); print('streams $s', d['value'], d['ms_per_step'], d['verified'])" >> $o
done
