#!/bin/bash
# Round 4 GPU pass: all GPU tests, the default bench line, the C2 step traces
# (edge tail auto / off), then the GEMM harnesses and the C3 bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
N=${1:-r4p}
O=$R/gpurun_out/$N
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
tail -1 $O/bench_n1.json | cut -c1-200
bash tools/r4_trace.sh $N/tr || exit 4
[ "$2" = "noc3" ] && exit 0
bash tools/r4_c3.sh $N/c3 || exit 5
