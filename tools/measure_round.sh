set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/final
cd $R && timeout -k 10 420 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final/stats -o s --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/final/bench_prof.json 2>/dev/null || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/final/fetch -o f --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-graph --steps 3 --warmup 1 > /dev/null 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/final/write -o w --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-graph --steps 3 --warmup 1 > /dev/null 2>&1 || exit 4
echo done
