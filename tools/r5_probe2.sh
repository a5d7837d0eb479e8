#!/bin/bash
# Round 5: head-kernel latency probe + rocprofv3 kernel stats of the C3 loop
# after the Waug-less prep.  tools/r5_probe2.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5probe2}
mkdir -p $O
cd $R
timeout -k 10 180 python tools/head_probe.py > $O/head_probe.txt 2>&1 || { tail -20 $O/head_probe.txt; exit 1; }
grep -v amdgpu.ids $O/head_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python3 $R/bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 2; }
echo done
