set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c3ab; mkdir -p $O; cd $R
for v in ${C3LIBS:-main}; do
  L=$R/spotv2net_amd/libsv2n_$v.so; [ "$v" = main ] && L=$R/spotv2net_amd/libsv2n.so
  SV2N_LIB=$L timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-kernel-table --no-compare > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'])" $O/c3_$v.json $v
done
