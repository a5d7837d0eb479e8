# A/B of library builds on the C2 bench line (diagnostic; round 6)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab}; mkdir -p $O; cd $R
shift
Q="python bench.py --no-cpu-baseline --no-ref-loop --no-rotating"
for v in "$@"; do
  L=$R/spotv2net_amd/libsv2n_$v.so; [ "$v" = main ] && L=$R/spotv2net_amd/libsv2n.so
  SV2N_LIB=$L timeout -k 10 300 $Q > $O/c2_$v.json 2> $O/c2_$v.err || { tail -20 $O/c2_$v.err; exit 1; }
  python -c "
import json,sys; d=json.load(open(sys.argv[1]))
k=d.get('kernels',{})
print(sys.argv[2], d['value'], d.get('value_generic_edges'), d['ms_per_step'], {n: round(v['avg_us'],1) for n,v in k.items() if 'gemm' in n or 'proj' in n or 'wgrad' in n})" $O/c2_$v.json $v
done
