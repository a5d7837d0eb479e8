#!/bin/bash
# Round 4 GEMM experiments: the large-tile bf16 GEMM (C3 shapes) and k_gemm3d
# variants (C2 shapes), standalone harnesses.  -> gpurun_out/$1/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-gexp}
mkdir -p $O
cd $R
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm_bw_tune.hip -o $O/gemm_bw_tune || exit 1
timeout -k 10 240 $O/gemm_bw_tune > $O/gemm_bw.txt 2>&1; rc=$?
cat $O/gemm_bw.txt
[ $rc -eq 0 ] || exit 2
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm3_tune.hip -o $O/gemm3_tune || exit 3
timeout -k 10 300 $O/gemm3_tune > $O/gemm3.txt 2>&1; rc=$?
cat $O/gemm3.txt
[ $rc -eq 0 ] || exit 4
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm_tt3y_tune.hip -o $O/tt3y || exit 5
timeout -k 10 240 $O/tt3y > $O/tt3y.txt 2>&1; rc=$?
cat $O/tt3y.txt
exit $rc
