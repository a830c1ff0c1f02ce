#!/bin/bash
# Round-6 GPU-box runs (each step under its own time limit; a timeout / abort /
# segfault stops the script).  Modes:
#   test              GPU test suite + smoke
#   sel  ARGS...      selected GPU tests
#   bench ARGS...     bench.py line
#   benchq ARGS...    bench.py, whole-frame leg only
#   itrace MODE...    rocprofv3 kernel trace of tools/render_modes.py MODE (+ tools/trace_iters.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name, stopping"; exit $rc; fi
  return 0
}
MODE=${1:-all}
shift || true
if [[ $MODE == all || $MODE == test ]]; then
  step pytest_gpu 900 python -u -m pytest tests -q -m gpu --maxfail=200 --timeout 120 --timeout-method thread
  step smoke 300 python __graft_entry__.py smoke
fi
if [[ $MODE == sel ]]; then
  step pytest_sel 900 python -u -m pytest -v -m gpu --maxfail=10 --timeout 300 --timeout-method thread "$@"
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 600 python bench.py --steps 3 --warmup 1 "$@"
fi
if [[ $MODE == benchq ]]; then
  step bench 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tile 0 --other-configs= "$@"
fi
if [[ $MODE == itrace ]]; then
  for m in "$@"; do
    step "itrace_$m" 300 rocprofv3 --kernel-trace -d $OUT/itrace_$m -o run --output-format csv -- python3 tools/render_modes.py $m --frames 3
    f=$(ls $OUT/itrace_$m/*/run_kernel_trace.csv $OUT/itrace_$m/run_kernel_trace.csv 2>/dev/null | head -n 1)
    python3 tools/trace_iters.py "$f" > $OUT/itrace_$m.txt 2>&1 || true
    head -n 12 $OUT/itrace_$m.txt
  done
fi
if [[ $MODE == tailsweep ]]; then
  # fused-tail thresholds: whole frame and the N = 8 / N = 2 row shards
  for t in ${TAILS:-0 32768 131072 524288 4194304}; do
    for m in ${TAIL_MODES:-frame shard8 shard2}; do
      step "tail_${m}_$t" 300 python3 tools/render_modes.py $m --frames 5 --tail $t
    done
  done
fi
if [[ $MODE == ssort ]]; then
  # opaque-shadow queue sort (hipcy_set_shadow_sort): whole frame and the N = 8 row shard
  for m in ${SSORTS:-0 3 5}; do
    for f in frame shard8; do
      step "ssort_${f}_$m" 300 python3 tools/render_modes.py $f --frames 5 --shadow-sort $m
    done
  done
fi
if [[ $MODE == harness ]]; then
  step pytest_harness 900 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_plugin_harness.py "$@"
fi
echo done
