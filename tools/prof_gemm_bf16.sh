#!/bin/bash
# SQ counters of the C3 bf16 projection GEMM (k_gemm_bf16nt) in bench --config c3
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
args="--config c3 --no-cpu-baseline --no-compare --epochs 1 --warmup-epochs 1"
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_gemm_bf16nt --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS -d $out/sq -o p --output-format csv -- python3 $R/bench.py $args > $out/sq.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_gemm_bf16nt --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $out/sq2 -o p --output-format csv -- python3 $R/bench.py $args > $out/sq2.log 2>&1 || exit 3
echo done
