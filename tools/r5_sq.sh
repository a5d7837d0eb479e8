#!/bin/bash
# Round 5 SQ counter passes (8 SQ counters per run at most) over the C2 bench
# steps for the projection GEMM and the covariance-layout edge passes: where
# their waves wait.  tools/r5_sq.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C2="python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-rotating --steps 5 --warmup 2"
RX="k_gemm3d|k_gemm_tt3y|k_edge_fwd_cv2|k_edge_bwd_cv2"
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS -d $O/a -o p --output-format csv -- $C2 > $O/a.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU -d $O/b -o p --output-format csv -- $C2 > $O/b.log 2>&1 || exit 2
cd $R && python tools/pmc_sq_summary.py $O/a/p_counter_collection.csv $O/b/p_counter_collection.csv > $O/sq_summary.txt && cat $O/sq_summary.txt
