#!/bin/bash
# GPU tests on the product build, then an A/B bench against build_ab/lib_old.so:
# tools/ab_cycle.sh OUT "BENCH_ARGS" ["TEST_ARGS"]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
TESTS=${3:-tests -m gpu}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python bench.py $2 > $O/new$k.json 2>$O/new$k.err || exit 2
  SV2N_LIB=$R/build_ab/lib_old.so timeout -k 10 300 python bench.py $2 > $O/old$k.json 2>$O/old$k.err || exit 3
done
python - $O <<'PY'
import json, sys
for k in ("new1", "old1", "new2", "old2"):
    for l in open(f"{sys.argv[1]}/{k}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(k, d["value"], d["ms_per_step"], {a: round(b["avg_us"], 1) for a, b in d.get("kernels", {}).items()})
PY
