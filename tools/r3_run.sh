set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pgemm.py -q --timeout 120 --timeout-method thread > gpurun_out/r3a_pgtest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3a_pgtest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r3a_pgtest.log; exit $rc; fi
tail -3 gpurun_out/r3a_pgtest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3a_bench_pg.json 2> gpurun_out/r3a_bench_pg.err || exit 1
NQK_NO_PG=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3a_bench_old.json 2> gpurun_out/r3a_bench_old.err || exit 1
cat gpurun_out/r3a_bench_pg.json gpurun_out/r3a_bench_old.json
