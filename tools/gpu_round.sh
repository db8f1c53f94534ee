#!/bin/bash
# One GPU call: parity tests, then (only if they ran to completion) the bench.
# Each GPU step has its own time limit; a crash/timeout stops the script.
set -u
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf --timeout 400 ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit 0; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.err
exit $rc
