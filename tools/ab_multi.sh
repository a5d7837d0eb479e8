#!/bin/bash
# A/B/C of several builds: tools/ab_multi.sh OUT "BENCH_ARGS" LIB1 [LIB2 ...]
# (LIB "product" = spotv2net_amd/libsv2n.so); two alternating rounds, then a
# summary line per run (value, ms/step, kernel table avg_us).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
ARGS=$2
shift 2
mkdir -p $O
cd $R
for k in 1 2; do
  i=0
  for L in "$@"; do
    i=$((i+1))
    if [ "$L" = product ]; then
      timeout -k 10 300 python bench.py $ARGS > $O/v$i.$k.json 2>$O/v$i.$k.err || exit 2
    else
      SV2N_LIB=$R/$L timeout -k 10 300 python bench.py $ARGS > $O/v$i.$k.json 2>$O/v$i.$k.err || exit 3
    fi
  done
done
python - $O "$@" <<'PY'
import json, sys
o, libs = sys.argv[1], sys.argv[2:]
for k in (1, 2):
    for i, lib in enumerate(libs, 1):
        for l in open(f"{o}/v{i}.{k}.json"):
            if l.startswith("{"):
                d = json.loads(l)
                print(lib, k, d["value"], d["ms_per_step"],
                      {a: round(b["avg_us"], 1) for a, b in d.get("kernels", {}).items()})
PY
