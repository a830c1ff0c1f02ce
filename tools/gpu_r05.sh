#!/bin/bash
# Round-5 GPU-box runs: parity tests, smoke and a bench line (each step under
# its own time limit; a timeout / abort / segfault stops the script).
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
  # selected tests: tools/gpu_r05.sh sel tests/test_x.py ... (-k expressions allowed)
  step pytest_sel 900 python -u -m pytest -v -m gpu --maxfail=10 --timeout 300 --timeout-method thread "$@"
  exit 0
fi
if [[ $MODE == selbench ]]; then
  step pytest_sel 900 python -u -m pytest -v -m gpu --maxfail=10 --timeout 300 --timeout-method thread $SEL
  step bench 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --other-configs= "$@"
  exit 0
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 600 python bench.py --steps 3 --warmup 1 "$@"
fi
if [[ $MODE == benchq ]]; then
  step bench 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tile 0 "$@"
fi
if [[ $MODE == variants ]]; then
  # traversal variants (python -m raytracingproject_amd.build --variant NAME -D... --traversal-only)
  Q="--steps 5 --warmup 1 --no-cpu-baseline --tile 0 --other-configs="
  step bench_default 600 python bench.py $Q "$@"
  for v in ${VARIANTS:-slabfma ww}; do
    step bench_$v 600 env HIPCY_DEVICE_LIB=$PWD/raytracingproject_amd/libhipcycles-$v.so python bench.py $Q "$@"
  done
fi
if [[ $MODE == refill ]]; then
  # lane-refill settings (bench.py --refill ROUNDS MIN_IDLE), "0 16" = off
  Q="--steps 5 --warmup 1 --no-cpu-baseline --other-configs="
  for r in ${REFILLS:-0,16 8,16 16,16 32,16 16,32}; do
    step "bench_refill_${r/,/_}" 600 python bench.py $Q --refill ${r%,*} ${r#*,} "$@"
  done
fi
if [[ $MODE == dbg ]]; then
  # first differing pixels / samples of a parity case: tools/gpu_r05.sh dbg CASE [WIDTH]
  step dbg 300 python tools/dbg_mismatch.py "$@"
fi
if [[ $MODE == configs ]]; then
  # per-kernel breakdown of the other BASELINE configs (one frame each, whole-frame render)
  for c in ${CONFIGS:-classroom_standin}; do
    step "bench_$c" 600 python bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --tile 0 --other-configs= "$@"
  done
fi
if [[ $MODE == sortcmp ]]; then
  # shading-queue sort (ray_sort 8) against unsorted, headline + other configs
  step bench_sort0 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tile 0 "$@"
  step bench_sort8 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tile 0 --ray-sort 8 "$@"
fi
if [[ $MODE == libtest ]]; then
  # parity tests against a variant build: LIB=name tools/gpu_r05.sh libtest -k expr
  step "pytest_lib_$LIB" 600 env HIPCY_DEVICE_LIB=$PWD/raytracingproject_amd/libhipcycles-$LIB.so \
    python -u -m pytest -v -m gpu --maxfail=10 --timeout 300 --timeout-method thread tests/test_gpu_parity.py "$@"
fi
if [[ $MODE == libbench ]]; then
  step "bench_lib_$LIB" 600 env HIPCY_DEVICE_LIB=$PWD/raytracingproject_amd/libhipcycles-$LIB.so \
    python bench.py --steps 5 --warmup 1 --no-cpu-baseline --tile 0 --other-configs= "$@"
fi
if [[ $MODE == micro ]]; then
  # node-fetch microbenchmark (tools/node_fetch_bench.hip), built here
  mkdir -p gpurun_out/bin
  step build_micro 120 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o gpurun_out/bin/node_fetch_bench tools/node_fetch_bench.hip
  step micro 300 gpurun_out/bin/node_fetch_bench
fi
if [[ $MODE == modes ]]; then
  # rocprofv3 kernel traces of the render modes (tools/render_modes.py, tools/trace_gaps.py)
  for m in ${MODES:-frame stream shard8}; do
    step "trace_$m" 300 rocprofv3 --kernel-trace -d $OUT/trace_modes_$m -o run --output-format csv -- python3 tools/render_modes.py $m "$@"
    python3 tools/trace_gaps.py $(ls $OUT/trace_modes_$m/*/run_kernel_trace.csv $OUT/trace_modes_$m/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/gaps_$m.txt 2>&1 || true
    head -14 $OUT/gaps_$m.txt
  done
fi
echo done
