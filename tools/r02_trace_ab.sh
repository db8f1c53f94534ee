#!/bin/bash
# rocprofv3 kernel traces of short bench runs under each environment assignment given
# ("-" = default): gpurun_out/tr_<i>/
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = "-" ]; then e=""; else e="$v"; fi
  rm -rf gpurun_out/tr_$i
  for kv in $e; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr_$i -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tr_$i.log 2>&1 || exit 1
  for kv in $e; do unset "${kv%%=*}"; done
  echo "$i $v" >> gpurun_out/tr_index.txt
done
