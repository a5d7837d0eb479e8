#!/bin/bash
# Kernel traces of the C2 train step at several batch sizes (does a kernel's
# time scale with its bytes, or is it a fixed latency?) and one SQ counter
# pass over the n <= 32 attention kernels: tools/probe_batch.sh OUTDIR
R=$GRAFT_REPO_ROOT
out=$R/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for b in 256 512 1024 2048; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $out/b$b -o t --output-format csv -- python3 $R/bench.py --batch $b --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 10 --warmup 3 > $out/b$b.json 2> $out/b$b.err || exit 1
done
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_attn|k_edge" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -d $out/sq -o p --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 5 --warmup 2 > $out/sq.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_attn|k_edge" --pmc SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $out/sq2 -o p --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 5 --warmup 2 > $out/sq2.log 2>&1 || exit 3
echo done
