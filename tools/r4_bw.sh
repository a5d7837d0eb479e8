#!/bin/bash
# bf16 large-tile GEMM check: harness, bf16 GPU tests, C3 bench line.  tools/r4_bw.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4bw}
mkdir -p $O
cd $R
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm_bw_tune.hip -o $O/gemm_bw_tune || exit 1
timeout -k 10 240 $O/gemm_bw_tune > $O/gemm_bw.txt 2>&1 || { cat $O/gemm_bw.txt; exit 2; }
cat $O/gemm_bw.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_operands.py tests/test_gpu_bf16.py tests/test_gpu_fit.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 4; }
tail -1 $O/bench_c3.json | cut -c1-250
