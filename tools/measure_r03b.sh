#!/bin/bash
# Round-3 final measurement, part A: GPU tests, the default bench line (with
# the CPU baseline) and the C1 / C3 / C5 lines.  Part B: tools/measure_r03c.sh.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03f}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 2
for c in c1 c3 c5; do
  timeout -k 10 420 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 3
done
echo done
