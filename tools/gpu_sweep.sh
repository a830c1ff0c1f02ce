#!/bin/bash
# GPU-box variant sweep: parity tests once, then one short bench per argument
# set (each set is one quoted string).  Stops at the first fatal status.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
if [[ ${SKIP_TESTS:-0} != 1 ]]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
  # any failure stops the sweep: a failing parity test may be a faulting kernel
  if [[ $rc != 0 ]]; then exit $rc; fi
fi
i=0
for args in "$@"; do
  i=$((i+1))
  envs=(); opts=()
  for tok in $args; do
    if [[ $tok == *=* && $tok != --* ]]; then envs+=("$tok"); else opts+=("$tok"); fi
  done
  timeout -k 10 600 env "${envs[@]}" python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline "${opts[@]}" > gpurun_out/sweep_$i.log 2>&1
  rc=$?
  echo "[$args] rc=$rc"
  if [[ $rc != 0 ]]; then tail -n 5 gpurun_out/sweep_$i.log; exit $rc; fi
  grep '"metric"' gpurun_out/sweep_$i.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print('  value %.1f Msps  ms/step %.1f  closest %.1f shade %.1f shadow %.1f  frac %.4f  avg_launch %.3f ms  nodes/ray %.1f tris/ray %.1f' % (d['value'], d['ms_per_step'], d['kernel_ms_per_frame']['k_intersect_closest'], d['kernel_ms_per_frame']['k_shade'], d['kernel_ms_per_frame']['k_intersect_shadow'], r['frac'], r['avg_launch_ms'], r.get('nodes_per_ray', 0), r.get('tris_per_ray', 0)))
" || tail -n 5 gpurun_out/sweep_$i.log
  if fatal $rc; then exit $rc; fi
done
