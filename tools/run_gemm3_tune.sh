# build + run the bf16x3 GEMM harness on the box -> gpurun_out/tune/
set -o pipefail
mkdir -p gpurun_out/tune
hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude -DSV2N_GEMM_CLOCK tools/gemm3_tune.hip -o gpurun_out/tune/gemm3_tune || exit 1
timeout -k 10 240 gpurun_out/tune/gemm3_tune > gpurun_out/tune/gemm3_tune.txt 2>&1
rc=$?
cat gpurun_out/tune/gemm3_tune.txt
exit $rc
