#!/bin/bash
# Round 5, last pass: the bound-checked build over the attention / edge /
# window / prep test files (conftest asserts zero out-of-extent indices after
# every test), then rocprofv3 kernel stats of the C3 loop.  tools/r5_close3.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5c3}
mkdir -p $O
cd $R
SV2N_LIB=$R/spotv2net_amd/libsv2n_check.so timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_tiled.py tests/test_gpu_fused.py tests/test_gpu_cov_var.py tests/test_gpu_conv.py \
  tests/test_gpu_hpo_grid.py tests/test_gpu_golden.py tests/test_gpu_parity_full.py tests/test_gpu_edge_tail.py \
  tests/test_gpu_window_cv.py tests/test_gpu_gemm.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/check_tests.log 2>&1 || { tail -30 $O/check_tests.log; exit 1; }
tail -2 $O/check_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o p -- python3 $R/bench.py --config c3 --no-compare --no-cpu-baseline --no-kernel-table --epochs 2 --warmup-epochs 1 > $O/tr.log 2>&1 || exit 2
echo traced
