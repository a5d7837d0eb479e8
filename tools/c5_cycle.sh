set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_tiled.py tests/test_gpu_parity_full.py -q -x --timeout 120 > $O/t.txt 2>&1 || exit 1
cd $R && timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-ref-loop --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit 2
bash $R/tools/prof_c5_sq.sh gpurun_out/$1 k_fattn_bwd || exit 3
