#!/bin/bash
# C5 A/B: the product library vs an alternative build of the same tree
# (tools/c5_ab.sh OUT [ALT_LIB]; default spotv2net_amd/libsv2n_alt.so), fused tests first.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c5ab}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_tiled.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-ref-loop > $O/new.json 2>$O/new.err || exit 2
SV2N_LIB=$R/${2:-spotv2net_amd/libsv2n_alt.so} timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-ref-loop > $O/old.json 2>$O/old.err || exit 3
python - $O <<'PY'
import json, sys
for k in ("new", "old"):
    for l in open(f"{sys.argv[1]}/{k}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(k, d["value"], d["ms_per_step"], {a: round(b["avg_us"], 1) for a, b in d["kernels"].items()})
PY
