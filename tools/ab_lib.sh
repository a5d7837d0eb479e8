#!/bin/bash
# A/B of two builds of the same tree: tools/ab_lib.sh OUT ALT_LIB "BENCH_ARGS" "TEST_FILES"
# runs the given GPU tests against the alternative library, then bench.py
# alternately with the product library and the alternative (two rounds each).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
ALT=$R/$2
ARGS=$3
TESTS=$4
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  SV2N_LIB=$ALT timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_alt.log 2>&1; rc=$?
  echo "alt tests rc=$rc"; tail -2 $O/tests_alt.log
  [ $rc -eq 0 ] || exit $rc
fi
for k in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/new$k.json 2>$O/new$k.err || exit 2
  SV2N_LIB=$ALT timeout -k 10 300 python bench.py $ARGS > $O/alt$k.json 2>$O/alt$k.err || exit 3
done
python - $O <<'PY'
import json, sys
for k in ("new1", "alt1", "new2", "alt2"):
    for l in open(f"{sys.argv[1]}/{k}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(k, d["value"], d["ms_per_step"], {a: round(b["avg_us"], 1) for a, b in d.get("kernels", {}).items()})
PY
