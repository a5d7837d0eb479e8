#!/bin/bash
# Round 5: covariance-layout backward A/B (parity tests, probe, C2 line with
# the kernel table).  tools/r5_cvb.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5cvb}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_var.py tests/test_gpu_hpo_grid.py tests/test_gpu_fit.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python tools/cv_probe.py > $O/probe.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ref-loop > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python - $O <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/bench.json"))
print("C2", d["value"], "generic", d["value_generic_edges"], "rotating", d["value_rotating"])
print({k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 5; }
python - $O <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/bench_c3.json"))
print("C3", d["value"], {k: round(v["avg_us"], 1) for k, v in d.get("kernels", {}).items()})
PY
