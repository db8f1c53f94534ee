set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=""
for n in ${PGM_DIAGS:-}; do L="$L,$n=tools/diag/libnqk_$n.so"; done
PGM_LIBS="${L#,}" timeout -k 10 ${MICRO_TIMEOUT:-400} python -u tools/pg_micro.py > gpurun_out/${OUT:-r3_micro}.txt 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${OUT:-r3_micro}.txt
cat gpurun_out/${OUT:-r3_micro}.txt
exit $rc
