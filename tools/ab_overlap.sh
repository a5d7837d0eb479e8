set -o pipefail
mkdir -p gpurun_out/abov
SV2N_OVERLAP_EDGE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity_full.py -x -q --timeout 200 --timeout-method thread > gpurun_out/abov/tests.log 2>&1 || { tail -30 gpurun_out/abov/tests.log; exit 1; }
tail -1 gpurun_out/abov/tests.log
for v in 1 0; do
  SV2N_OVERLAP_EDGE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-ref-loop --no-kernel-table > gpurun_out/abov/b.json 2> gpurun_out/abov/b.err || { tail -5 gpurun_out/abov/b.err; exit 2; }
  python -c "
import json
d=json.loads(open('gpurun_out/abov/b.json').read().splitlines()[-1]); print('overlap $v', d['value'], d['ms_per_step'], d['fwd_graphs_per_s'])"
done
