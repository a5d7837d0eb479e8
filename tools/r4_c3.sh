#!/bin/bash
# Round 4: GEMM harnesses (C3 / C2 shapes), then the C3 bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4c3}
mkdir -p $O
cd $R
bash tools/r4_gemm_exp.sh $(basename $O)/gexp > $O/gexp.log 2>&1 || { tail -20 $O/gexp.log; exit 1; }
grep -v "^$" $O/gexp/gemm_bw.txt | tail -20
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 2; }
tail -1 $O/bench_c3.json | cut -c1-400
