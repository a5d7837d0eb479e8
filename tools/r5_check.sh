#!/bin/bash
# Round 5: the bound-checked build (make CHECK=1 -> libsv2n_check.so) over the
# attention / edge test files (conftest asserts zero out-of-extent indices
# after every test), then the release library's covariance-layout tests, the
# probe and the C2 line.  tools/r5_check.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5chk}
mkdir -p $O
cd $R
SV2N_LIB=$R/spotv2net_amd/libsv2n_check.so timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_tiled.py tests/test_gpu_fused.py tests/test_gpu_cov_var.py tests/test_gpu_conv.py \
  tests/test_gpu_hpo_grid.py tests/test_gpu_golden.py tests/test_gpu_parity_full.py tests/test_gpu_edge_tail.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/check_tests.log 2>&1 || { tail -30 $O/check_tests.log; exit 1; }
tail -2 $O/check_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_var.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 120 python tools/cv_probe.py > $O/probe.txt 2>&1 || exit 3
cat $O/probe.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ref-loop > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python - $O <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/bench.json"))
print("C2", d["value"], "generic", d["value_generic_edges"], "rotating", d["value_rotating"])
print({k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
