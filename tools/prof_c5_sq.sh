#!/bin/bash
# C5 SQ counter passes over kernels matching a regex: tools/prof_c5_sq.sh OUTDIR [REGEX]
R=$GRAFT_REPO_ROOT
out=$R/$1
rx=${2:-k_fattn_bwd}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
args="--config c5 --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 3 --warmup 1"
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$rx" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS -d $out/sq -o p --output-format csv -- python3 $R/bench.py $args > $out/sq.log 2>&1 || exit 2
timeout -s KILL 180 rocprofv3 --kernel-include-regex "$rx" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $out/sq2 -o p --output-format csv -- python3 $R/bench.py $args > $out/sq2.log 2>&1 || exit 3
echo done
