#!/bin/bash
# Round 5 evidence: the default bench line (CPU leg included), one traced run
# of the C2 steps (per-kernel table), the HBM PMC passes (FETCH_SIZE,
# WRITE_SIZE: one counter group per run) and the C3 / C5 / C1 lines.
# tools/r5_final.sh OUT [configs]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5f}
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
cat $O/bench_n1.json
timeout -k 10 60 tools/probe_bin/cv_tune > $O/cv_tune.txt 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp
C2="python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-rotating --steps 20 --warmup 5"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/c2t -o p --output-format csv -- $C2 > $O/c2t.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/c2f -o p --output-format csv -- $C2 > $O/c2f.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/c2w -o p --output-format csv -- $C2 > $O/c2w.log 2>&1 || exit 4
cd $R
for c in ${2:-c3 c5 c1}; do
  timeout -k 10 500 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 5; }
done
ls $O
