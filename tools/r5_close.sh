#!/bin/bash
# Round 5 closing pass: the whole -m gpu suite, the C2 line (CPU leg
# included), the C3 line twice (its timed region is ~16 ms: run to run
# spread), C5 and C1.  tools/r5_close.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5c}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 2; }
for c in c3 c3 c5 c1; do
  k=$c; [ -f $O/bench_$c.json ] && k=${c}_2
  timeout -k 10 500 python bench.py --config $c > $O/bench_$k.json 2> $O/bench_$k.err || { tail -20 $O/bench_$k.err; exit 3; }
done
python - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/bench_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["value"], d.get("value_generic_edges"), d.get("value_rotating"), d.get("ref_loop_graphs_per_s"))
PY
