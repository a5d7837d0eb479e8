#!/bin/bash
# GPU tests (optional), two bench lines and a kernel trace of the C2 bench:
# tools/c2_step_trace.sh OUT [notests]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
if [ "$2" != "notests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b1.json 2> $O/b1.err || exit 2
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b2.json 2> $O/b2.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b3.json 2>/dev/null || exit 4
echo done
