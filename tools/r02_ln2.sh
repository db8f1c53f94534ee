#!/bin/bash
# LayerNorm+quantize: parity, then timing at 1 / 2 / 3 / 6 / unlimited workgroups per CU
set -u
mkdir -p gpurun_out
o=gpurun_out/ln2.txt
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ln or layernorm or layer or plan or b256" > gpurun_out/ln2_tests.log 2>&1 || { echo "tests failed" >> $o; tail -20 gpurun_out/ln2_tests.log >> $o; exit 1; }
tail -1 gpurun_out/ln2_tests.log >> $o
for r in 1 2; do
for w in 3 2 4 6 1000; do
  echo -n "wgs/cu $w: " >> $o
  NQK_LN_WGS_PER_CU=$w timeout -k 10 120 python -u tools/ln_micro.py >> $o 2>&1 || exit 1
done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_ln.json 2> gpurun_out/bench_ln.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_ln.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['verified'], {k:v['avg_us'] for k,v in d['kernels'].items()})" >> $o
