#!/bin/bash
# Run one gpurun call, re-submitting ONLY when the pod had no free slot
# (gpurun exit 3: nothing ran, nothing charged).  usage: tools/gpurun_wait.sh OUTFILE TIMEOUT CMD...
out=$1; shift; to=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1; rc=$?
  [ $rc -ne 3 ] && break
  sleep 200
done
echo "rc=$rc" >> $out
