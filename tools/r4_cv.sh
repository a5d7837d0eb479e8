#!/bin/bash
# Round 4: covariance-layout edge passes — their tests, every GPU test, then
# bench lines for fwd-only / fwd+bwd / off, a traced step, and C3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4cv}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_var.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/first.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" $O/first.log | tail -30; exit 1; }
tail -1 $O/first.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
run() {  # name fwd bwd
  SV2N_COV_VAR_EDGES=$2 SV2N_COV_VAR_BWD=$3 timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_$1.json 2>> $O/b.err || return 1
  echo "$1 $(python3 -c "import json; d=json.loads(open('$O/b_$1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('value_generic_edges'))")"
}
run fwd on off && run both on on && run off off off || exit 3
cd /tmp && export TMPDIR=/tmp
SV2N_COV_VAR_EDGES=on SV2N_COV_VAR_BWD=on timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/bt.json 2>$O/bt.err || exit 5
python3 $R/tools/step_table.py $O/st/s_kernel_trace.csv > $O/table.txt || exit 6
grep -i "edge\|span" $O/table.txt | cut -c1-80
cd $R
for v in "fwd on off" "both on on" "off off off"; do
  set -- $v
  SV2N_COV_VAR_EDGES=$2 SV2N_COV_VAR_BWD=$3 timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline --no-compare --no-kernel-table > $O/c3_$1.json 2>> $O/c3.err || exit 7
  echo "c3 $1 $(python3 -c "import json; d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
