#!/bin/bash
# Round 5 covariance-layout passes: parity tests, then round-4 vs round-5
# kernels back to back (tools/cv_probe.py) and the C2 bench line with each.
# tools/r5_cv.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5cv}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_var.py tests/test_gpu_hpo_grid.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SV2N_CV_ROUND4=1 timeout -k 10 120 python tools/cv_probe.py > $O/probe_r4.txt 2>&1 || exit 2
timeout -k 10 120 python tools/cv_probe.py > $O/probe_r5.txt 2>&1 || exit 3
cat $O/probe_r4.txt $O/probe_r5.txt
B="python bench.py --no-cpu-baseline --no-ref-loop --steps 50 --warmup 10"
SV2N_CV_ROUND4=1 timeout -k 10 200 $B > $O/bench_r4.json 2> $O/bench_r4.err || exit 4
timeout -k 10 200 $B > $O/bench_r5.json 2> $O/bench_r5.err || exit 5
python - $O <<'PY'
import json, sys
for k in ("r4", "r5"):
    d = json.load(open(f"{sys.argv[1]}/bench_{k}.json"))
    ks = d["kernels"]
    print(k, d["value"], d["value_generic_edges"], d["value_rotating"],
          {n: round(ks[n]["avg_us"], 1) for n in ("edge_logits_fwd_cv", "edge_logits_bwd_cv")})
PY
