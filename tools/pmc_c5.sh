# SQ counter pass over the fused C5 attention kernels (eager steps, B=256)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-c5pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-include-regex "fattn" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -d $OUT/sq -o p --output-format csv -- python3 $R/tools/run_c5_steps.py 256 > $OUT/run.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-include-regex "fattn" --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d $OUT/sq2 -o p --output-format csv -- python3 $R/tools/run_c5_steps.py 256 > $OUT/run2.log 2>&1 || exit 2
echo done
