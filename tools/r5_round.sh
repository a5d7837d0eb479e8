#!/bin/bash
# Round 5 check: -m gpu suite, the read-pattern / cv ablation probe, the C2
# bench line (no CPU leg), and the C3 loop.  tools/r5_round.sh OUT [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5r}
mkdir -p $O
cd $R
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
[ -x tools/probe_bin/cv_tune ] && { timeout -k 10 120 tools/probe_bin/cv_tune > $O/cv_tune.txt 2>&1 || exit 2; cat $O/cv_tune.txt; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 4; }
python - $O <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/bench.json"))
print("C2", d["value"], "generic", d["value_generic_edges"], "rotating", d["value_rotating"],
      "ref_loop", d.get("ref_loop_graphs_per_s"), "fwd", d["fwd_graphs_per_s"])
print({k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
c = json.load(open(f"{sys.argv[1]}/bench_c3.json"))
print("C3", c["value"], {k: round(v["avg_us"], 1) for k, v in c["kernels"].items()})
PY
