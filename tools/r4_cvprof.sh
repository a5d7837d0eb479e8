#!/bin/bash
# Round 4: covariance-layout edge passes in isolation, plus SQ counter passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4cvp}
mkdir -p $O
cd $R
timeout -k 10 120 python tools/cv_probe.py > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
cat $O/probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-include-regex "_cv|_mx" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/sq -o p --output-format csv -- python3 $R/tools/cv_probe.py > $O/sq.log 2>&1 || exit 2
python3 - $O <<'PY'
import csv, sys, glob, collections
f = glob.glob(sys.argv[1] + "/sq/*counter_collection.csv")[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
