#!/bin/bash
# Round-3 measurement pass: GPU tests, the default bench line, C1/C3/C5 lines,
# rocprofv3 kernel statistics of the C2 bench and the C3 loop.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03m}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 2
for c in c1 c3 c5; do
  timeout -k 10 420 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c2 -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_c2_prof.json 2>/dev/null || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c3 -o s --output-format csv -- python3 $R/bench.py --config c3 --no-cpu-baseline --no-compare > $O/bench_c3_prof.json 2>/dev/null || exit 5
echo done
