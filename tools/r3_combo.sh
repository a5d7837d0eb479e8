#!/bin/bash
# One GPU call: attention / fused / parity tests, C2 + C3 bench lines, then the
# C5 fused-backward A/B (product library vs libsv2n_oldbwd.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-combo}
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity_full.py tests/test_gpu_fused.py tests/test_gpu_tiled.py tests/test_gpu_bf16.py tests/test_gpu_model.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 2
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 3
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-ref-loop > $O/new.json 2>$O/new.err || exit 4
SV2N_LIB=$R/spotv2net_amd/libsv2n_oldbwd.so timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-ref-loop > $O/old.json 2>$O/old.err || exit 5
python - $O <<'PY'
import json, sys
for k in ("bench_c2", "bench_c3", "new", "old"):
    for l in open(f"{sys.argv[1]}/{k}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(k, d["value"], d.get("ms_per_step"), d.get("ref_loop_graphs_per_s"),
                  {a: round(b["avg_us"], 1) for a, b in d.get("kernels", {}).items()})
PY
