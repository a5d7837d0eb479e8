#!/bin/bash
# Closing check of the committed tree: all GPU tests, smoke(), the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-close}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
tail -1 $O/bench_n1.json | cut -c1-200
