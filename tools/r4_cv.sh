#!/bin/bash
# Round 4: covariance-layout edge passes — their tests, every GPU test, then
# bench lines and traced steps with SV2N_COV_VAR_EDGES on / off, and C3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4cv}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_var.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/first.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" $O/first.log | tail -30; exit 1; }
tail -1 $O/first.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for v in on off; do
  SV2N_COV_VAR_EDGES=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_$v.json 2>> $O/b.err || exit 3
  echo "$v $(python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
for v in on; do
  SV2N_COV_VAR_EDGES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_$v -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/bt_$v.json 2>$O/bt_$v.err || exit 5
  python3 $R/tools/step_table.py $O/st_$v/s_kernel_trace.csv > $O/table_$v.txt || exit 6
  cut -c1-80 $O/table_$v.txt
done
cd $R
for v in on off; do
  SV2N_COV_VAR_EDGES=$v timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline --no-compare --no-kernel-table > $O/c3_$v.json 2>> $O/c3.err || exit 7
  echo "c3 $v $(python3 -c "import json; d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
