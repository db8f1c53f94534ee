#!/bin/bash
# two-stream forward: persistent projection GEMMs on all CUs vs a CU share per stream
set -u
mkdir -p gpurun_out
o=gpurun_out/projcus.txt
: > $o
run() {  # label, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_pc.json 2> gpurun_out/bench_pc.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/bench_pc.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['verified'])" >> $o
}
run default NQK_X=0
run qkv128 NQK_PROJ_CUS=128
run gelu_all NQK_PROJ_GELU=1
run gelu128 NQK_PROJ_GELU=1 NQK_PROJ_CUS=128
run gelu160 NQK_PROJ_GELU=1 NQK_PROJ_CUS=160
run default2 NQK_X=0
run gelu128b NQK_PROJ_GELU=1 NQK_PROJ_CUS=128
