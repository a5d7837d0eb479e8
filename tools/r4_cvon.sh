#!/bin/bash
# Round 4: every GPU test with the covariance-layout forward on, then the
# bench and C3 lines with it.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4cvon}
mkdir -p $O
cd $R
export SV2N_COV_VAR_EDGES=on
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -5 $O/bench_n1.err; exit 3; }
tail -1 $O/bench_n1.json | cut -c1-200
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 4; }
tail -1 $O/bench_c3.json | cut -c1-200
