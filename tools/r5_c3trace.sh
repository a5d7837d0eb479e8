#!/bin/bash
# Round 5: kernel trace + stats of the C3 bf16 loop (train steps and the
# one-forward test pass).  tools/r5_c3trace.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5c3t}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o p -- python3 $R/bench.py --config c3 --no-compare --no-cpu-baseline --no-kernel-table --epochs 2 --warmup-epochs 1 > $O/tr.log 2>&1 || exit 1
ls $O/tr
