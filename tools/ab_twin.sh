# Same-box A/B of Fit's twin-only x (SV2N_TWIN_ONLY on/off) on BASELINE C3:
# bench lines alternated, then the window gather's kernel time per mode.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/twin; mkdir -p $O; cd $R
export TMPDIR=/tmp
for r in $(seq ${REPS:-4}); do for v in on off; do
  SV2N_TWIN_ONLY=$v timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-kernel-table --no-compare > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || { tail -5 $O/c3_${v}_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'])" $O/c3_${v}_$r.json $v
done; done
for v in on off; do
  SV2N_TWIN_ONLY=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python bench.py --config c3 --no-cpu-baseline --no-kernel-table --no-compare > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
done
