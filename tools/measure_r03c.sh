#!/bin/bash
# Round-3 final measurement, part B: rocprofv3 kernel statistics of the C2,
# C3 and C5 benches, and the FETCH_SIZE / WRITE_SIZE passes (one counter per
# run) of the C2 kernel-table kernels and the C5 layer kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03f}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c2 -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_c2_prof.json 2>/dev/null || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c3 -o s --output-format csv -- python3 $R/bench.py --config c3 --no-cpu-baseline --no-compare > $O/bench_c3_prof.json 2>/dev/null || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o s --output-format csv -- python3 $R/bench.py --config c5 --no-cpu-baseline > $O/bench_c5_prof.json 2>/dev/null || exit 6
RX='k_gemm3d|k_gemm_tt3y|k_edge_|canon'
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc FETCH_SIZE -d $O/c2_fetch -o f --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-graph --steps 3 --warmup 1 > /dev/null 2>&1 || exit 7
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc WRITE_SIZE -d $O/c2_write -o w --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-graph --steps 3 --warmup 1 > /dev/null 2>&1 || exit 8
timeout -s KILL 120 rocprofv3 --kernel-include-regex "fattn|gemm" --pmc FETCH_SIZE -d $O/c5_fetch -o f --output-format csv -- python3 $R/tools/run_c5_steps.py 1024 > $O/c5f.log 2>&1 || exit 9
timeout -s KILL 120 rocprofv3 --kernel-include-regex "fattn|gemm" --pmc WRITE_SIZE -d $O/c5_write -o w --output-format csv -- python3 $R/tools/run_c5_steps.py 1024 > $O/c5w.log 2>&1 || exit 10
echo done
