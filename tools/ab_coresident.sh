set -o pipefail
mkdir -p gpurun_out/cores
for cfg in "SV2N_OVERLAP_EDGE=0" "SV2N_OVERLAP_EDGE=1 SV2N_EDGE_FWD_GRID=256" "SV2N_OVERLAP_EDGE=1 SV2N_EDGE_FWD_GRID=512" "SV2N_OVERLAP_EDGE=0" "SV2N_OVERLAP_EDGE=1 SV2N_EDGE_FWD_GRID=256"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-ref-loop --no-kernel-table > gpurun_out/cores/b.json 2> gpurun_out/cores/b.err || { tail -5 gpurun_out/cores/b.err; exit 2; }
  python -c "
import json
d=json.loads(open('gpurun_out/cores/b.json').read().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['fwd_graphs_per_s'])"
done
SV2N_OVERLAP_EDGE=1 SV2N_EDGE_FWD_GRID=256 bash tools/trace_c2.sh gpurun_out/trco
