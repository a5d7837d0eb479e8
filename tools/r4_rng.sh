#!/bin/bash
# Round 4: device dropout generator — its tests first, every GPU test, then
# the C3 bench line and a C3 bf16 kernel trace.  tools/r4_rng.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4rng}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_device_dropout.py tests/test_gpu_train.py tests/test_gpu_head_fuse.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/first.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" $O/first.log | tail -30; exit 1; }
tail -1 $O/first.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 3; }
tail -1 $O/bench_c3.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k -o k --output-format csv -- \
  python3 $R/bench.py --config c3 --precision bf16 --no-compare --no-cpu-baseline --no-kernel-table --epochs 2 \
  > $O/b3.json 2> $O/b3.err || exit 4
python3 $R/tools/kstats.py $O/k/k_kernel_stats.csv 30 > $O/kstats.txt || exit 5
cat $O/kstats.txt
