#!/bin/bash
# C3 bench A/B: GPU tests given, then bench.py --config c3 alternately with the
# product library and build_ab/lib_old.so; prints value, ms/step and the kernel rows.
# usage: tools/ab_c3_bench.sh OUT "TEST_FILES"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest $2 -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-compare > $O/new$k.json 2>$O/new$k.err || exit 2
  SV2N_LIB=$R/build_ab/lib_old.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-compare > $O/old$k.json 2>$O/old$k.err || exit 3
done
python - $O <<'PY'
import json, sys
for k in ("new1", "old1", "new2", "old2"):
    d = json.loads(open(f"{sys.argv[1]}/{k}.json").read().strip().splitlines()[-1])
    print(k, d["value"], d["ms_per_step"], {a: round(b["avg_us"], 1) for a, b in d.get("kernels", {}).items()})
PY
