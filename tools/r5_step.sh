#!/bin/bash
# Round 5: parity subset + C2 line + traced C2 step (per-kernel table).
# tools/r5_step.sh OUT [pytest files...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5s}
shift
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest ${@:-tests/test_gpu_train.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ref-loop > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
python - $O <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/bench.json"))
print("C2", d["value"], "generic", d["value_generic_edges"], "rotating", d["value_rotating"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o p -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-rotating --steps 20 --warmup 5 > $O/tr.log 2>&1 || exit 3
cd $R && python tools/step_table.py $O/tr/p_kernel_trace.csv > $O/step_table.txt && head -24 $O/step_table.txt
