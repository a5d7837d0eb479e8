#!/bin/bash
# Round 4: C1 and C5 bench lines, then the C3 bf16 PMC passes (FETCH_SIZE,
# WRITE_SIZE; one counter group per run).  tools/r4_lines.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4l}
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --config c1 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
tail -1 $O/bench_c1.json | cut -c1-300
timeout -k 10 500 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 2; }
tail -1 $O/bench_c5.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
C3="python3 $R/bench.py --config c3 --precision bf16 --no-compare --no-cpu-baseline --no-kernel-table --epochs 1 --warmup-epochs 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/c3f -o p --output-format csv -- $C3 > $O/c3f.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/c3w -o p --output-format csv -- $C3 > $O/c3w.log 2>&1 || exit 4
find $O -name "*counter_collection.csv" | sort
