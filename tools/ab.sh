#!/bin/bash
# Same-box A/B driver (one GPU call): parity tests first, then whole-bench runs of several
# builds and / or environment variants interleaved on the same box, then an optional kernel
# microbenchmark.  Replaces round 2 / 3's one-off r02_* / r3_* scripts (git history).
#   AB_TESTS="node ids"          pytest node ids run first; a failure stops the call
#   AB_LIBS="name ..."           builds tools/diag/libnqk_<name>.so (tools/pg_diag.sh), each copied
#                                over the main library for its runs ("main" = the tree's own build)
#   AB_ENVS="name:V=a,W=b ..."   environment variants of the main build
#   AB_REPS=2                    interleaved repetitions of the whole variant list
#   AB_BENCH="--steps 20 ..."    extra bench.py arguments (default: --steps 20)
#   AB_MICRO="pg|attn|ln"        tools/pg_micro.py / attn_micro.py / ln_micro.py afterwards
#                                (their PGM_* / AM_* variables pass through)
#   OUT=tag                      results: gpurun_out/<tag>_*.json, <tag>_ab.txt
# Every GPU step runs under its own time limit; the first failure ends the call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-ab}
fail() { echo "FAILED: $1 rc=$2" >> gpurun_out/${OUT}_ab.txt; exit $2; }
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${AB_TESTS} -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${OUT}_tests.log 2>&1 || fail pytest $?
fi
LIB=numpy-quant_amd/numpy_quant/libnqk.so
cp $LIB /tmp/libnqk_main.so
variants="${AB_LIBS:-main} "
for e in ${AB_ENVS:-}; do variants+="env:$e "; done
i=0
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in $variants; do
    i=$((i+1))
    envs=""
    if [[ $v == env:* ]]; then
      name=${v#env:}; name=${name%%:*}; envs=${v#env:*:}; cp /tmp/libnqk_main.so $LIB
    else
      name=$v
      if [ "$v" = "main" ]; then cp /tmp/libnqk_main.so $LIB; else cp tools/diag/libnqk_$v.so $LIB; fi
    fi
    env ${envs//,/ } timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary ${AB_BENCH:---steps 20} \
      > gpurun_out/${OUT}_${name}_$rep.json 2> gpurun_out/${OUT}_${name}_$rep.err || fail "bench $name" $?
    python3 -c "import json;d=json.load(open('gpurun_out/${OUT}_${name}_$rep.json'));print('$name', d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})" \
      >> gpurun_out/${OUT}_ab.txt
  done
done
cp /tmp/libnqk_main.so $LIB
case "${AB_MICRO:-}" in
  pg) timeout -k 10 300 python -u tools/pg_micro.py > gpurun_out/${OUT}_pg_micro.txt 2>&1 || fail pg_micro $? ;;
  attn) timeout -k 10 300 python -u tools/attn_micro.py > gpurun_out/${OUT}_attn_micro.txt 2>&1 || fail attn_micro $? ;;
  ln) timeout -k 10 300 python -u tools/ln_micro.py > gpurun_out/${OUT}_ln_micro.txt 2>&1 || fail ln_micro $? ;;
esac
echo done >> gpurun_out/${OUT}_ab.txt
