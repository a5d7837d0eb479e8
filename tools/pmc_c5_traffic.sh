# HBM traffic of the C5 kernels: separate FETCH_SIZE / WRITE_SIZE passes over
# eager C5 steps at B = 1024 (the bench batch) (tools/run_c5_steps.py), then tools/pmc_traffic.py --config c5
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-c5traffic}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-include-regex "fattn|gemm" --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 $R/tools/run_c5_steps.py 1024 > $OUT/f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "fattn|gemm" --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 $R/tools/run_c5_steps.py 1024 > $OUT/w.log 2>&1 || exit 2
echo done
