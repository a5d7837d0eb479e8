#!/bin/bash
# Round 5: in-loop kernel stats of the C3 attention backward per head-split
# setting (SV2N_CANON_BWD_S 0 = default 6 splits, 3), rocprofv3 --kernel-trace --stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5bwds2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for s in 0 3; do
  SV2N_CANON_BWD_S=$s timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$s -o p -- python3 $R/bench.py --config c3 --no-compare --no-cpu-baseline --no-kernel-table --epochs 2 --warmup-epochs 1 > $O/tr$s.log 2>&1 || exit 1
  echo traced $s
done
