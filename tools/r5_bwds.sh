#!/bin/bash
# Round 5: A/B of the C3 attention backward's head splits (SV2N_CANON_BWD_S):
# parity subset with a forced split count, then the C3 line per setting.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5bwds}
mkdir -p $O
cd $R
SV2N_CANON_BWD_S=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for s in 0 3 2 0 3; do
  SV2N_CANON_BWD_S=$s timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline > $O/c3_$s.json 2> $O/c3_$s.err || { tail -20 $O/c3_$s.err; exit 2; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('S', sys.argv[2], d['value'], d['kernels']['gat_attn_bwd']['avg_us'])" $O/c3_$s.json $s
done
