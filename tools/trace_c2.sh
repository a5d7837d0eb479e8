# C2 train-step kernel trace (no reference loop, no kernel table): tools/trace_c2.sh OUTDIR
R=$GRAFT_REPO_ROOT
out=$R/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $out/tr -o t --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 10 --warmup 3 > $out/tr.json 2> $out/tr.err || exit 1
echo done
