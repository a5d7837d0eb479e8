#!/bin/bash
# C3 / C1 lines with and without the canonical attention kernels
out=$GRAFT_REPO_ROOT/$1
mkdir -p $out
cd $GRAFT_REPO_ROOT
for v in 1 0; do
  for c in c3 c1; do
    SV2N_ATTN_CANON=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-compare --steps 20 --warmup 5 > $out/$c.$v.json 2> $out/$c.$v.err || { tail -3 $out/$c.$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('$out/$c.$v.json').read().strip().splitlines()[-1]); print('$c canon=$v', d['value'], d.get('fwd_graphs_per_s'), d.get('c3_loop', {}).get('bf16', {}).get('train_graphs_per_s_upper'))"
  done
done
