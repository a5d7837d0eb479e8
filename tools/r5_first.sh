#!/bin/bash
# Round 5, first GPU pass: the whole -m gpu suite, the default C2 bench line,
# then the HBM PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run)
# over the C2 steps.  tools/r5_first.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5a}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
C2="python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-rotating --steps 5 --warmup 2"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/c2f -o p --output-format csv -- $C2 > $O/c2f.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/c2w -o p --output-format csv -- $C2 > $O/c2w.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/c2t -o p --output-format csv -- $C2 > $O/c2t.log 2>&1 || exit 5
find $O -name "*counter_collection.csv" -o -name "*kernel_stats.csv" | sort
