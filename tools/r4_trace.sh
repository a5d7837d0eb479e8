#!/bin/bash
# C2 step kernel traces with the edge tail on / off: tools/r4_trace.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4tr}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in auto off; do
  SV2N_EDGE_TAIL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_$v -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_$v.json 2>$O/b_$v.err || exit 4
  python3 $R/tools/step_table.py $O/st_$v/s_kernel_trace.csv > $O/table_$v.txt || exit 5
  tail -1 $O/table_$v.txt
done
