#!/bin/bash
# Round-3 closing pass: all GPU tests, the default bench line (as the driver runs
# it), and the C3 bench under rocprofv3 kernel statistics.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-s5f}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  timeout -k 10 200 python tools/c3_kernels.py > $O/k_diag$k.txt 2>&1 || exit 4
  timeout -k 10 200 python tools/c3_kernels.py --no-diag > $O/k_nodiag$k.txt 2>&1 || exit 5
  tail -1 $O/k_diag$k.txt; tail -1 $O/k_nodiag$k.txt
done
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 2
tail -1 $O/bench_n1.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c3 -o s --output-format csv -- python3 $R/bench.py --config c3 --no-cpu-baseline --no-compare > $O/bench_c3_prof.json 2>/dev/null || exit 3
echo done
