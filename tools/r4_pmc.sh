#!/bin/bash
# Round 4 PMC passes (one counter group per run, MI355X_MICROARCH.md HBM
# recipe): FETCH_SIZE and WRITE_SIZE over the C2 bench steps and the C3 bf16
# loop, then SQ instruction counters of the C3 weight-gradient GEMM and the C2
# layer-0 GEMMs.  tools/r4_pmc.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C2="python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 5 --warmup 2"
C3="python3 $R/bench.py --config c3 --precision bf16 --no-compare --no-cpu-baseline --no-kernel-table --epochs 1 --warmup-epochs 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/c2f -o p --output-format csv -- $C2 > $O/c2f.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/c2w -o p --output-format csv -- $C2 > $O/c2w.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/c3f -o p --output-format csv -- $C3 > $O/c3f.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/c3w -o p --output-format csv -- $C3 > $O/c3w.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_gemm_bw|k_gemm3d|k_gemm_tt3y" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d $O/sq3 -o p --output-format csv -- $C3 > $O/sq3.log 2>&1 || exit 5
timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_gemm3d|k_gemm_tt3y" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d $O/sq2 -o p --output-format csv -- $C2 > $O/sq2.log 2>&1 || exit 6
find $O -name "*counter_collection.csv" | sort
