#!/bin/bash
# gemm3 (bf16x3 projection) harness on the C2 / C5 shapes -> gpurun_out/$1/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-g3}
mkdir -p $O
cd $R
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm3_tune.hip -o $O/gemm3_tune || exit 1
timeout -k 10 400 $O/gemm3_tune > $O/gemm3.txt 2>&1; rc=$?
cat $O/gemm3.txt
exit $rc
