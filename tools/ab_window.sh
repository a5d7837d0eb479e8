#!/bin/bash
# Window-gather A/B: the GPU tests that cover the device window builder, then
# tools/c3_kernels.py (HIP-event times of the C3 step's non-GEMM launches) and
# the C3 bench line, alternately with the product library and build_ab/lib_old.so.
# usage: tools/ab_window.sh OUT "TEST_FILES"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest $2 -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python tools/c3_kernels.py > $O/k_new$k.txt 2>&1 || exit 2
  SV2N_LIB=$R/build_ab/lib_old.so timeout -k 10 200 python tools/c3_kernels.py > $O/k_old$k.txt 2>&1 || exit 3
  tail -1 $O/k_new$k.txt; tail -1 $O/k_old$k.txt
done
for k in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-compare > $O/c3_new$k.json 2>$O/c3_new$k.err || exit 4
  SV2N_LIB=$R/build_ab/lib_old.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-compare > $O/c3_old$k.json 2>$O/c3_old$k.err || exit 5
  for v in new old; do python -c "
import json; d=json.loads(open('$O/c3_$v$k.json').read().strip().splitlines()[-1]); print('$v$k', d['value'], d['ms_per_step'])"; done
done
