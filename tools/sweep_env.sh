#!/bin/bash
# bench.py over values of one environment variable:
# tools/sweep_env.sh OUTDIR VAR "v1 v2 ..." "BENCH_ARGS"
out=$1; var=$2; vals=$3; args=$4
mkdir -p "$out"
for v in $vals; do
  env $var=$v timeout -k 10 300 python bench.py $args > "$out/sw_$v.json" 2> "$out/sw_$v.err" || { echo "bench $var=$v failed"; tail -5 "$out/sw_$v.err"; exit 1; }
  python -c "
import json
d = json.loads(open('$out/sw_$v.json').read().strip().splitlines()[-1])
k = d.get('kernels', {})
print('$var=$v', d['value'], d['ms_per_step'], {n: round(x['avg_us'], 1) for n, x in k.items()})"
done
