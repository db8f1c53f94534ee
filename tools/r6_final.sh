#!/bin/bash
# Round 6's evidence set, one GPU call: every GPU test, smoke(), the default bench line (with the
# measured CPU baseline), a rocprofv3 kernel trace of a short one-stream bench (NQK_SPLIT=0: every
# launch whole-batch and alone, as bench.py's per-kernel table), and the FETCH_SIZE / WRITE_SIZE
# PMC passes for profiles/pmc_traffic.json (separate runs: TCC slots).  Each step under its own
# time limit; the first failure stops the call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6z}
step() { echo "== $1 rc=$2" >> gpurun_out/${T}_status.txt; if [ $2 -ne 0 ]; then exit $2; fi; }
rm -f gpurun_out/${T}_status.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
step tests $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
step smoke $?
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
step bench $?
rm -rf gpurun_out/${T}_prof
NQK_SPLIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err
step rocprof $?
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/${T}_pmc_$c
  NQK_SPLIT=0 timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/${T}_pmc_$c -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_pmc_$c.log 2>&1
  step pmc_$c $?
done
echo done >> gpurun_out/${T}_status.txt
