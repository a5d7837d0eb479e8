#!/bin/bash
# Round 4: covariance-layout kernels — their tests, then the isolated timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4cvq}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_var.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/first.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" $O/first.log | tail -30; exit 1; }
tail -1 $O/first.log
timeout -k 10 120 python tools/cv_probe.py 2>&1 | grep -v amdgpu.ids
