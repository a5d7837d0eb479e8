#!/bin/bash
# A/B of the MFMA edge backward: product (direct loads) vs ab/lib_lds.so and
# ab/lib_lds3.so (LDS-staged, occupancy 4 / 3): edge parity tests on the alt
# libraries, then traced C2 steps for all three.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4abb}
mkdir -p $O
cd $R
for v in lds lds3; do
  SV2N_LIB=$R/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_conv.py tests/test_gpu_edge_tail.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 3; }
  tail -1 $O/tests_$v.log
done
cd /tmp && export TMPDIR=/tmp
for v in prod lds lds3 prod2; do
  L=""; [ $v = lds ] && L=$R/ab/lib_lds.so; [ $v = lds3 ] && L=$R/ab/lib_lds3.so
  SV2N_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_$v -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop > $O/b_$v.json 2>$O/b_$v.err || exit 5
  python3 $R/tools/step_table.py $O/st_$v/s_kernel_trace.csv > $O/table_$v.txt || exit 6
  echo $v; grep -i edge $O/table_$v.txt; tail -1 $O/table_$v.txt; cat $O/b_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'])"
done
