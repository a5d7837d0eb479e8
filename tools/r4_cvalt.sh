#!/bin/bash
# A/B of a covariance-layout forward variant in ab/lib_fwd.so: its tests and the isolated timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4cva}
mkdir -p $O
cd $R
export SV2N_LIB=$R/ab/lib_fwd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_var.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/first.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" $O/first.log | tail -30; exit 1; }
tail -1 $O/first.log
timeout -k 10 120 python tools/cv_probe.py 2>&1 | grep -v amdgpu.ids
unset SV2N_LIB
timeout -k 10 120 python tools/cv_probe.py 2>&1 | grep -v amdgpu.ids
