#!/bin/bash
# A/B of the MFMA edge kernels: product library vs ab/lib_d2.so (two tiles in
# flight per wave): GPU tests on both, kernel tables, and traced C2 steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
N=${1:-r4ab}
O=$R/gpurun_out/$N
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
SV2N_LIB=$R/ab/lib_d2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_conv.py tests/test_gpu_edge_tail.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_alt.log 2>&1 || { tail -30 $O/tests_alt.log; exit 3; }
tail -1 $O/tests_alt.log
bash tools/ab_lib.sh $N/ab ab/lib_d2.so "--no-cpu-baseline --no-ref-loop" "" || exit 4
cd /tmp && export TMPDIR=/tmp
for v in prod alt; do
  L=""; [ $v = alt ] && L=$R/ab/lib_d2.so
  SV2N_LIB=$L SV2N_EDGE_TAIL=off timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_$v -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_$v.json 2>$O/b_$v.err || exit 5
  python3 $R/tools/step_table.py $O/st_$v/s_kernel_trace.csv > $O/table_$v.txt || exit 6
  tail -1 $O/table_$v.txt
done
