#!/bin/bash
# Round 5 closing verification: the whole -m gpu suite on the release library,
# the bound-checked build over the attention / edge test files (conftest
# asserts zero out-of-extent indices), the reference-loop host probe.
# tools/r5_verify.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5v}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
SV2N_LIB=$R/spotv2net_amd/libsv2n_check.so timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_tiled.py tests/test_gpu_fused.py tests/test_gpu_cov_var.py tests/test_gpu_conv.py \
  tests/test_gpu_hpo_grid.py tests/test_gpu_golden.py tests/test_gpu_parity_full.py tests/test_gpu_edge_tail.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/check_tests.log 2>&1 || { tail -30 $O/check_tests.log; exit 2; }
tail -2 $O/check_tests.log
timeout -k 10 120 python tools/ref_loop_host.py > $O/ref_loop_host.txt 2>&1 || exit 3
timeout -k 10 120 python tools/ref_loop_host.py --fused-adam 1 >> $O/ref_loop_host.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/ref_loop_host.txt
