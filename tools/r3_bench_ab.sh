# same-box A/B of whole bench runs: main build, then each tools/diag/libnqk_<name>.so copied over
# the main library (this box's snapshot only), then main again
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
cp numpy-quant_amd/numpy_quant/libnqk.so /tmp/libnqk_main.so
run() {
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 20 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$1.json'));print('$1', d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
}
run main
for n in ${AB_LIBS}; do
  cp tools/diag/libnqk_$n.so numpy-quant_amd/numpy_quant/libnqk.so
  run $n
done
cp /tmp/libnqk_main.so numpy-quant_amd/numpy_quant/libnqk.so
run main2
