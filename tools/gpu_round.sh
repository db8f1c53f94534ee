#!/bin/bash
# One GPU call: parity tests, then (only if they ran to completion) the bench,
# then (PROFILE=1) a rocprofv3 kernel-trace of a short bench run.
# Each GPU step has its own time limit; a crash/timeout stops the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit 0; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-0}" = "1" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
  rc=$?
  echo "rocprof rc=$rc" >> gpurun_out/prof_bench.err
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${PMC:-0}" = "1" ]; then
  # HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), one
  # stream (whole-batch launches, as bench.py's per-kernel timings)
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_bench_$c
    NQK_SPLIT=0 timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_bench_$c -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc_bench_$c.log 2>&1
    rc=$?
    echo "pmc $c rc=$rc" >> gpurun_out/pmc_bench_$c.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
fi
exit 0
