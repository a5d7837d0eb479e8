#!/bin/bash
# Round 5 PMC refresh for C3 (bf16 loop) and C5: FETCH_SIZE and WRITE_SIZE,
# one counter per run (MI355X_MICROARCH.md HBM recipe).  tools/r5_pmc.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C3="python3 $R/bench.py --config c3 --precision bf16 --no-compare --no-cpu-baseline --no-kernel-table --epochs 1 --warmup-epochs 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/c3f -o p --output-format csv -- $C3 > $O/c3f.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/c3w -o p --output-format csv -- $C3 > $O/c3w.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --kernel-include-regex "fattn|gemm" --pmc FETCH_SIZE -d $O/c5f -o p --output-format csv -- python3 $R/tools/run_c5_steps.py 1024 > $O/c5f.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-include-regex "fattn|gemm" --pmc WRITE_SIZE -d $O/c5w -o p --output-format csv -- python3 $R/tools/run_c5_steps.py 1024 > $O/c5w.log 2>&1 || exit 4
find $O -name "*counter_collection.csv" | sort
