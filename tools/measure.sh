#!/bin/bash
# Every GPU measurement behind README / DESIGN numbers, as subcommands (run on
# the GPU box through gpurun; results under gpurun_out/OUT):
#
#   tools/measure.sh tests   OUT [pytest files]  the -m gpu suite (or a subset)
#   tools/measure.sh check   OUT                 bound-checked build (make CHECK=1) over the
#                                                attention / edge / parity tests
#   tools/measure.sh c2      OUT [bench args]    the default bench line (CPU leg included)
#   tools/measure.sh step    OUT                 one traced run of the C2 steps -> per-kernel
#                                                step table (tools/step_table.py)
#   tools/measure.sh pmc     OUT                 FETCH_SIZE / WRITE_SIZE passes (one counter
#                                                group per run) over C2, the C3 bf16 loop and C5
#   tools/measure.sh sq      OUT [kernel regex]  two SQ counter passes (8 SQ counters each)
#                                                over the C2 steps -> tools/pmc_sq_summary.py
#   tools/measure.sh configs OUT [configs]       the c3 / c5 / c1 lines (default all three)
#   tools/measure.sh c3trace OUT                 kernel trace + stats of the C3 bf16 loop
#   tools/measure.sh close   OUT                 tests, c2, step and configs in one call
#
# Same-box A/B of library builds (a build of the same sources with a -D switch,
# loaded through SV2N_LIB; round 6): tools/ab_step.sh OUT lib... (traced C2
# step per build), tools/ab_c3.sh (C3 line per build, C3LIBS="..."),
# tools/ab_run.sh OUT lib... (C2 bench line per build).
#
# Every GPU step has its own time limit and the steps are chained: the first
# failure ends the call (no retries on the box).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cmd=$1
O=$R/gpurun_out/${2:-$cmd}
shift 2 2>/dev/null
mkdir -p "$O"
C2Q="python3 $R/bench.py --no-cpu-baseline --no-kernel-table --no-ref-loop --no-rotating"

tests() {
  cd "$R" && timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; return 1; }
  tail -2 "$O/tests.log"
}

check() {
  cd "$R" && make -s CHECK=1 -j16 || return 1
  SV2N_LIB=$R/spotv2net_amd/libsv2n_check.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_tiled.py tests/test_gpu_fused.py tests/test_gpu_cov_var.py tests/test_gpu_conv.py \
    tests/test_gpu_hpo_grid.py tests/test_gpu_golden.py tests/test_gpu_parity_full.py \
    tests/test_gpu_edge_tail.py tests/test_gpu_window_cv.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$O/check_tests.log" 2>&1 ||
    { tail -30 "$O/check_tests.log"; return 1; }
  tail -2 "$O/check_tests.log"
}

c2() {
  cd "$R" && timeout -k 10 400 python bench.py "$@" > "$O/bench_n1.json" 2> "$O/bench_n1.err" ||
    { tail -20 "$O/bench_n1.err"; return 1; }
  python - "$O/bench_n1.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("C2", d["value"], "generic", d.get("value_generic_edges"), "rotating", d.get("value_rotating"),
      "ref_loop", d.get("ref_loop_graphs_per_s"))
print({k: round(v["avg_us"], 1) for k, v in d.get("kernels", {}).items()})
PY
}

step() {
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr" -o p -- \
    $C2Q --steps 20 --warmup 5 > "$O/tr.log" 2>&1 || return 1
  cd "$R" && python tools/step_table.py "$O/tr/p_kernel_trace.csv" > "$O/step_table.txt" &&
    head -24 "$O/step_table.txt"
}

pmc() {
  cd /tmp && export TMPDIR=/tmp
  local C3="python3 $R/bench.py --config c3 --precision bf16 --no-compare --no-cpu-baseline --no-kernel-table --epochs 1 --warmup-epochs 1"
  local C5="python3 $R/tools/run_c5_steps.py 1024"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/c2_$c" -o p --output-format csv -- \
      $C2Q --steps 20 --warmup 5 > "$O/c2_$c.log" 2>&1 || return 1
    timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/c3_$c" -o p --output-format csv -- $C3 \
      > "$O/c3_$c.log" 2>&1 || return 1
    timeout -s KILL 120 rocprofv3 --kernel-include-regex "fattn|gemm" --pmc $c -d "$O/c5_$c" \
      -o p --output-format csv -- $C5 > "$O/c5_$c.log" 2>&1 || return 1
  done
  find "$O" -name "*counter_collection.csv" | sort
}

sq() {
  local RX=${1:-k_gemm3d|k_gemm_tt3y|k_edge_fwd_cv2|k_edge_bwd_cv2|canon}
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVES SQ_BUSY_CYCLES \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS \
    -d "$O/a" -o p --output-format csv -- $C2Q --steps 5 --warmup 2 > "$O/a.log" 2>&1 || return 1
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT \
    SQ_ACTIVE_INST_VALU -d "$O/b" -o p --output-format csv -- $C2Q --steps 5 --warmup 2 \
    > "$O/b.log" 2>&1 || return 1
  cd "$R" && python tools/pmc_sq_summary.py "$O/a/p_counter_collection.csv" \
    "$O/b/p_counter_collection.csv" > "$O/sq_summary.txt" && cat "$O/sq_summary.txt"
}

configs() {
  cd "$R"
  for c in ${@:-c3 c5 c1}; do
    timeout -k 10 500 python bench.py --config $c > "$O/bench_$c.json" 2> "$O/bench_$c.err" ||
      { tail -20 "$O/bench_$c.err"; return 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], \
d.get('value_full_gather'), d.get('value_generic_edges'))" "$O/bench_$c.json" $c
  done
}

c3trace() {
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr" -o p -- \
    python3 "$R/bench.py" --config c3 --no-compare --no-cpu-baseline --no-kernel-table \
    --epochs 2 --warmup-epochs 1 > "$O/tr.log" 2>&1 || return 1
  ls "$O/tr"
}

close() { tests && c2 && step && configs; }

case $cmd in
  tests|check|c2|step|pmc|sq|configs|c3trace|close) $cmd "$@" ;;
  *) sed -n 2,22p "$0"; exit 2 ;;
esac
