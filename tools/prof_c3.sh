#!/bin/bash
# C3 (yaml model, full train loop) kernel statistics and one-epoch trace, bf16
# and f32: rocprofv3 --kernel-trace --stats of bench.py --config c3.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-c3prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for P in bf16 f32; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$P -o k --output-format csv -- \
    python3 $R/bench.py --config c3 --precision $P --no-compare --no-cpu-baseline --epochs 2 \
    > $OUT/bench_$P.json 2> $OUT/bench_$P.err || exit 1
done
