#!/bin/bash
# A/B bench runs on one box: bench.py under each environment assignment given
# (e.g. "NQK_NO_PROJ=1" "-"), interleaved twice; "-" = default environment
set -u
mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for v in "$@"; do
    i=$((i+1))
    if [ "$v" = "-" ]; then e=""; else e="$v"; fi
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit 1
    echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print(d['value'], d['ms_per_step'])")" >> gpurun_out/ab.txt
  done
done
