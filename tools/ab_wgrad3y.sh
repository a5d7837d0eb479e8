# tt3y correctness (weight-gradient and train tests) then A/B SV2N_WGRAD3Y on C2 and C5
set -o pipefail
mkdir -p gpurun_out/ab3y
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity_full.py tests/test_gpu_autograd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab3y/tests.log 2>&1 || { tail -30 gpurun_out/ab3y/tests.log; exit 1; }
tail -1 gpurun_out/ab3y/tests.log
bash tools/ab_env.sh gpurun_out/ab3y SV2N_WGRAD3Y "--no-cpu-baseline --no-ref-loop" || exit 2
bash tools/ab_env.sh gpurun_out/ab3y5 SV2N_WGRAD3Y "--config c5 --no-cpu-baseline --no-ref-loop --steps 10 --warmup 3" || exit 3
