#!/bin/bash
# One GPU iteration: pytest (selected files or all -m gpu) then optional bench
# commands; stops at the first fault / abort / timeout (rc not 0 or 1).
# usage: tools/gpu_cycle.sh OUTDIR "PYTEST_ARGS" ["BENCH_ARGS" ...]
out=$1; shift
targs=$1; shift
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest $targs -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1
rc=$?
echo "tests rc=$rc"
tail -3 "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
i=0
for b in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py $b > "$out/bench$i.json" 2> "$out/bench$i.err"
  brc=$?
  echo "bench$i ($b) rc=$brc"
  if [ $brc -ne 0 ]; then tail -5 "$out/bench$i.err"; exit $brc; fi
done
exit 0
