#!/bin/bash
# retry a gpurun call only while no box / slot was free (exit 3: nothing ran, nothing charged)
log=$1; shift
for i in $(seq 1 ${RETRY_MAX:-40}); do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  echo "attempt $i rc=$rc" >> "$log.attempts"
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 60
done
exit 3
