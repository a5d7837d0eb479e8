# Same-box A/B of library builds on the traced C2 step (diagnostic; round 6):
#   bash tools/ab_step.sh OUT lib1 lib2 ...   (lib = main | suffix of libsv2n_<suffix>.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abs}; mkdir -p $O
shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  L=$R/spotv2net_amd/libsv2n_$v.so; [ "$v" = main ] && L=$R/spotv2net_amd/libsv2n.so
  SV2N_LIB=$L timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o p -- \
    python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-rotating --steps 20 \
    --warmup 5 > $O/tr_$v.log 2>&1 || exit 1
  (cd $R && python tools/step_table.py $O/tr_$v/p_kernel_trace.csv > $O/step_$v.txt) || exit 1
  echo "== $v"; head -23 $O/step_$v.txt | tail -22
done
