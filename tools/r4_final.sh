#!/bin/bash
# Round 4 measurement pass: every GPU test, the default bench line (with its
# CPU baseline), a traced C2 step table, the C3 bench line and its kernel
# stats.  tools/r4_final.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4f}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -5 $O/bench_n1.err; exit 3; }
tail -1 $O/bench_n1.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_tr.json 2>$O/b_tr.err || exit 4
python3 $R/tools/step_table.py $O/st/s_kernel_trace.csv > $O/table.txt || exit 5
cut -c1-90 $O/table.txt
cd $R
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 6; }
tail -1 $O/bench_c3.json | cut -c1-300
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/st3 -o s --output-format csv -- python3 $R/bench.py --config c3 --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b3_tr.json 2>$O/b3_tr.err || exit 7
head -14 $O/st3/s_kernel_stats.csv | cut -d, -f2-5 | cut -c1-120
