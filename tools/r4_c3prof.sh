#!/bin/bash
# C3 bf16 loop kernel statistics (rocprofv3 --kernel-trace --stats): tools/r4_c3prof.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c3prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k -o k --output-format csv -- \
  python3 $R/bench.py --config c3 --precision bf16 --no-compare --no-cpu-baseline --no-kernel-table --epochs 2 \
  > $O/bench.json 2> $O/bench.err || exit 1
python3 $R/tools/kstats.py $O/k/k_kernel_stats.csv 40 > $O/kstats.txt || exit 2
cat $O/kstats.txt
