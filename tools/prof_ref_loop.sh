set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3c
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3c/prof -o p --output-format csv -- python3 $R/tools/ref_loop_probe.py --modes free > $R/gpurun_out/r3c/probe.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3c/proftrain -o t --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --steps 50 > $R/gpurun_out/r3c/bench.txt 2>&1 || exit 2
