#!/bin/bash
# Round 4 GPU pass: FIRST (optional) test files verbose, all GPU tests, the
# default bench line, a C2 step trace; "c3" adds the GEMM harnesses and the
# C3 bench line.  tools/r4_pass.sh OUT "FIRST_TESTS" [c3]
set -o pipefail
R=$GRAFT_REPO_ROOT
N=${1:-r4p}
O=$R/gpurun_out/$N
mkdir -p $O
cd $R
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest $2 -m gpu -x -v --timeout 300 --timeout-method thread > $O/first.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" $O/first.log | tail -30; exit 1; }
  tail -1 $O/first.log
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
tail -1 $O/bench_n1.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_tr.json 2>$O/b_tr.err || exit 4
python3 $R/tools/step_table.py $O/st/s_kernel_trace.csv > $O/table.txt || exit 5
cat $O/table.txt | cut -c1-90
cd $R
[ "$3" = "c3" ] || exit 0
bash tools/r4_c3.sh $N/c3 || exit 6
