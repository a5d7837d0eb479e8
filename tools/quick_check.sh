#!/bin/bash
# Quick GPU check after a kernel change: the given test files (default: the
# attention / full-size parity / bf16 / model tests), then the C2 and C3
# bench lines (no CPU baseline).  usage: tools/quick_check.sh TAG [tests...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-quick}
shift
T=${@:-tests/test_gpu_conv.py tests/test_gpu_parity_full.py tests/test_gpu_bf16.py tests/test_gpu_model.py}
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest $T -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 2
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 3
python - $O <<'PY'
import json, sys
for c in ("c2", "c3"):
    for l in open(f"{sys.argv[1]}/bench_{c}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(c, d["value"], d.get("ms_per_step"), d.get("ref_loop_graphs_per_s"),
                  {k: round(v["avg_us"], 1) for k, v in d.get("kernels", {}).items()})
PY
