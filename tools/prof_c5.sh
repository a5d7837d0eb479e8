# rocprofv3 kernel stats of the C5 bench (train + forward) -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-c5prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o s --output-format csv -- python3 $R/bench.py --config c5 --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
