#!/bin/bash
# A/B of a Python-side change: the tree as is vs a copy of the package with
# one module replaced (the library is shared).
# usage: tools/ab_py.sh OUT MODULE_PATH_IN_PKG OLD_FILE "BENCH_ARGS"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
OLD=/tmp/sv2n_old_$$
rm -rf $OLD && mkdir -p $OLD && cp -r $R/spotv2net_amd $R/bench.py $OLD/ && cp $R/$3 $OLD/spotv2net_amd/$2
for k in 1 2 3; do
  (cd $R && timeout -k 10 300 python bench.py $4 > $O/new$k.json 2>$O/new$k.err) || exit 2
  (cd $OLD && timeout -k 10 300 python bench.py $4 > $O/old$k.json 2>$O/old$k.err) || exit 3
done
rm -rf $OLD
python - $O <<'PY'
import json, sys
for k in ("new1", "old1", "new2", "old2", "new3", "old3"):
    for l in open(f"{sys.argv[1]}/{k}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(k, d["value"], d["ms_per_step"], d.get("ref_loop_graphs_per_s"),
                  d.get("ref_loop_block_layout_graphs_per_s"))
PY
