#!/bin/bash
# round-4 call K: the QKV filter margin 6.25 / 5.25 units (was 8 / 16): QKV parity, exact-path
# entries per forward before / after (diagnostic builds over the library), whole-bench A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/k.status
step() { echo "== $1 rc=$2" >> gpurun_out/k.status; if [ $2 -ne 0 ]; then exit $2; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_pgemm.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k_tests.log 2>&1
step tests $?
LIB=numpy-quant_amd/numpy_quant/libnqk.so
cp $LIB /tmp/libnqk_main.so
for v in slowold slow; do
  cp tools/diag/libnqk_$v.so $LIB
  timeout -k 10 300 python -u tools/pg_slow_rate.py > gpurun_out/k_slow_$v.txt 2>&1
  rc=$?
  cp /tmp/libnqk_main.so $LIB
  step slow_$v $rc
done
AB_LIBS="main qold" AB_REPS=2 OUT=k bash tools/ab.sh
step ab $?
echo done >> gpurun_out/k.status
