#!/bin/bash
# C2 train-step kernel trace + two SQ counter passes over kernels matching a
# regex: tools/prof_c2.sh OUTDIR [REGEX]
R=$GRAFT_REPO_ROOT
out=$R/$1
rx=${2:-canon}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $out/tr -o t --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 10 --warmup 3 > $out/tr.json 2> $out/tr.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$rx" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -d $out/sq -o p --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 5 --warmup 2 > $out/sq.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$rx" --pmc SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $out/sq2 -o p --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 5 --warmup 2 > $out/sq2.log 2>&1 || exit 3
echo done
