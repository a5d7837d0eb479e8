#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (one counter set per run) of the C2 bench
# step over kernels matching a regex, for the product library and, if given,
# SV2N_LIB=ALT: tools/pmc_pair.sh OUT REGEX [ALT_LIB]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
RX=$2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # tag [lib]
  if [ -n "$2" ]; then export SV2N_LIB=$2; else unset SV2N_LIB; fi
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc FETCH_SIZE -d $O/$1_f -o f --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-graph --steps 3 --warmup 1 > /dev/null 2>&1 || return 1
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc WRITE_SIZE -d $O/$1_w -o w --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-graph --steps 3 --warmup 1 > /dev/null 2>&1 || return 1
}
run new "" || exit 5
if [ -n "$3" ]; then run old "$R/$3" || exit 6; fi
echo pmc done
