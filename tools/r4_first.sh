#!/bin/bash
# Round 4 first GPU pass: the new replay / bench-DP tests, then all GPU tests,
# then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4a}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_graphed.py tests/test_gpu_bench_dp.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/new.log 2>&1; rc=$?
tail -4 $O/new.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
tail -1 $O/bench_n1.json | cut -c1-400
