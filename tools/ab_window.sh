# Same-box A/B of window-gather builds (AB_LIBS, default "libsv2n_ab0 libsv2n"):
# the window tests on the main build, tools/window_micro.py per build, then
# BASELINE C3 bench lines alternated.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wab; mkdir -p $O; cd $R
LIBS=${AB_LIBS:-libsv2n_ab0 libsv2n}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_twin_only.py tests/test_gpu_window_cv.py tests/test_gpu_bf16_operands.py tests/test_gpu_parity_full.py -k "window or twin or gather or Window or cv" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for L in $LIBS; do echo "== $L"; SV2N_LIB=$R/spotv2net_amd/$L.so timeout -k 10 200 python tools/window_micro.py 128 || exit 1; SV2N_LIB=$R/spotv2net_amd/$L.so timeout -k 10 200 python tools/window_micro.py 432 || exit 1; done
for r in $(seq ${REPS:-3}); do for L in $LIBS; do
  SV2N_LIB=$R/spotv2net_amd/$L.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-kernel-table --no-compare > $O/c3_${L}_$r.json 2> $O/c3_${L}_$r.err || { tail -5 $O/c3_${L}_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'])" $O/c3_${L}_$r.json $L
done; done
