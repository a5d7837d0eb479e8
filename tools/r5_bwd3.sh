#!/bin/bash
# Round 5: head-mean attention backward capped at 384 workgroups: the
# whole GPU suite, then the C3 line (kernel table) twice.  tools/r5_waug.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5bwd3}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3_$i.json 2> $O/bench_c3_$i.err || { tail -20 $O/bench_c3_$i.err; exit 5; }
python - $O/bench_c3_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("C3", d["value"], d["ms_per_step"], {k: round(v["avg_us"], 1) for k, v in d.get("kernels", {}).items()})
PY
done
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 6; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C1', d['value'], d['ms_per_step'])" $O/bench_c1.json
