#!/bin/bash
set -u
mkdir -p gpurun_out
o=gpurun_out/attn3.txt
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or attn or plan or b256 or vit" > gpurun_out/attn3_tests.log 2>&1 || { echo "tests failed" >> $o; tail -20 gpurun_out/attn3_tests.log >> $o; exit 1; }
tail -1 gpurun_out/attn3_tests.log >> $o
for r in 1 2 3; do timeout -k 10 120 python -u tools/attn_micro.py >> $o 2>&1 || exit 1; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_a3.json 2> gpurun_out/bench_a3.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_a3.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['verified'], {k:v['avg_us'] for k,v in d['kernels'].items()})" >> $o
