#!/bin/bash
# A/B bench of one environment switch: tools/ab_env.sh OUTDIR VAR "BENCH_ARGS"
# runs bench.py with VAR=1 then VAR=0 (each under its own time limit) and
# stops at the first failure.
out=$1; var=$2; args=$3
mkdir -p "$out"
for v in 1 0; do
  env $var=$v timeout -k 10 300 python bench.py $args > "$out/ab_$v.json" 2> "$out/ab_$v.err" || { echo "bench $var=$v failed"; tail -5 "$out/ab_$v.err"; exit 1; }
  python -c "
import json
d = json.loads(open('$out/ab_$v.json').read().strip().splitlines()[-1])
print('$var=$v', d['value'], d['ms_per_step'], d.get('fwd_graphs_per_s'), d.get('ref_loop_graphs_per_s'))
for k, v in d.get('kernels', {}).items(): print('   ', k, v['avg_us'])"
done
