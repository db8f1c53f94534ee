#!/bin/bash
set -u
mkdir -p gpurun_out
o=gpurun_out/residf32.txt
: > $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or plan or b256 or vit or persistent or int4" > gpurun_out/residf32_tests.log 2>&1 || { echo "tests failed" >> $o; tail -20 gpurun_out/residf32_tests.log >> $o; exit 1; }
tail -1 gpurun_out/residf32_tests.log >> $o
for r in 1 2; do
for v in f32 f64; do
  if [ $v = f64 ]; then E="NQK_RESID_F64=1"; else E="NQK_X=0"; fi
  for sh in out down; do echo -n "$v " >> $o; env $E GM_ONLY=$sh:fused timeout -k 10 120 python -u tools/gemm_micro.py >> $o 2>&1 || exit 1; done
done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_rf.json 2> gpurun_out/bench_rf.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_rf.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['verified'], {k:v['avg_us'] for k,v in d['kernels'].items()})" >> $o
