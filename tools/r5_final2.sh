#!/bin/bash
# Round 5 end: the tree as committed — smoke(), the whole -m gpu suite and the
# default bench line.  tools/r5_final2.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5f2}
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 2; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 3; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C2', d['value'], d['ms_per_step'], d['roofline']['frac'])" $O/bench_n1.json
