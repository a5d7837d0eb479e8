#!/bin/bash
# A/B: the training step's edge-gradient pass on a side stream beside layer
# 0's weight-gradient GEMM (SV2N_EDGE_BWD_SIDE=on) vs in order: parity tests
# with the switch on, bench lines and traced C2 steps for both, C3 lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4side}
mkdir -p $O
cd $R
SV2N_EDGE_BWD_SIDE=on timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_train.py tests/test_gpu_head_fuse.py tests/test_gpu_graphed.py tests/test_gpu_bf16_operands.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_on.log 2>&1 || { tail -30 $O/tests_on.log; exit 1; }
tail -1 $O/tests_on.log
for v in off on off on; do
  SV2N_EDGE_BWD_SIDE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_$v.json 2>> $O/b.err || exit 2
  echo "$v $(python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
for v in off on; do
  SV2N_EDGE_BWD_SIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_$v -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/bt_$v.json 2>$O/bt_$v.err || exit 5
  python3 $R/tools/step_table.py $O/st_$v/s_kernel_trace.csv > $O/table_$v.txt || exit 6
  echo $v; tail -1 $O/table_$v.txt
done
cd $R
for v in off on; do
  SV2N_EDGE_BWD_SIDE=$v timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline --no-compare --no-kernel-table > $O/c3_$v.json 2>> $O/c3.err || exit 7
  echo "c3 $v $(python3 -c "import json; d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]); print(d['value'])")"
done
