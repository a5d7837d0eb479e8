# bench lines for the non-headline configs (C1, C3, C5) -> gpurun_out/final/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/final
cd $R
for c in c1 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/final/bench_$c.json 2> gpurun_out/final/bench_$c.err || exit 1
done
echo done
