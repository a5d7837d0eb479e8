#!/bin/bash
# Round 4 GPU pass: the new tests first, then all GPU tests, then the default
# bench line and the same bench with the separate edge-gradient pass (A/B).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4a}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_tail.py tests/test_gpu_graphed.py tests/test_gpu_bench_dp.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/new.log 2>&1; rc=$?
tail -4 $O/new.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
tail -1 $O/bench_n1.json | cut -c1-300
SV2N_EDGE_TAIL=off timeout -k 10 400 python bench.py --no-ref-loop --no-cpu-baseline > $O/bench_n1_tail_off.json 2> $O/bench_n1_tail_off.err || exit 4
tail -1 $O/bench_n1_tail_off.json | cut -c1-300
