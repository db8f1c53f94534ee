#!/bin/bash
# One GPU call for a round's evidence: parity tests, the bench line, a rocprofv3
# kernel-trace of a short bench, and two PMC passes (FETCH_SIZE, WRITE_SIZE) for the
# HBM-traffic summary.  Every GPU step under its own time limit; the first failure stops.
# The profiled runs use NQK_SPLIT=0 (one stream: every launch is a whole-batch launch timed
# alone, matching bench.py's per-kernel breakdown); the bench line itself uses two streams.
# SKIP_TESTS=1 / SKIP_BENCH=1 skip those steps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 rc=$2" >> gpurun_out/full.status; if [ $2 -ne 0 ]; then exit $2; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  step pytest $?
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  step bench $?
fi
export NQK_SPLIT=0
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
step rocprof $?
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
step pmc_fetch $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
step pmc_write $?
