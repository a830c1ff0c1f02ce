#!/bin/bash
# GPU-box check: parity tests, smoke, a short bench and a rocprofv3 kernel trace.
# Every GPU step has its own time limit; a timeout / abort / segfault stops the
# script (no further GPU work), an ordinary test failure does not.
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
  tail -n 25 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name, stopping"; exit $rc; fi
  return 0
}

MODE=${1:-all}
if [[ $MODE == all || $MODE == test ]]; then
  step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu -s --timeout 300 --timeout-method thread
  step smoke 300 python __graft_entry__.py smoke
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench_quick 600 python bench.py --steps 2 --warmup 1 --samples 16 --no-cpu-baseline
  step bench 900 python bench.py --steps 3 --warmup 1 --save gpurun_out/bmw.png
fi
if [[ $MODE == quick ]]; then
  step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
  step bench_w8 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --bvh-width 8
  step bench_w2 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --bvh-width 2
fi
if [[ $MODE == all || $MODE == sort ]]; then
  for m in 3 5; do
    step bench_sort$m 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tile 0 --ray-sort $m
  done
fi
if [[ $MODE == all || $MODE == prof ]]; then
  step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
fi
echo done
