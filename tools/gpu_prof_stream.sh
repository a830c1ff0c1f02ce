#!/bin/bash
# rocprofv3 kernel statistics of the whole-frame render and of the tile stream
# (bench.py --render stream), same scene and frame count.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
Q="--steps 3 --warmup 1 --no-cpu-baseline --tile 64 --other-configs= --tile-batch 1"
for mode in frame stream; do
  echo "=== $mode"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$mode -o run --output-format csv -- \
    python3 bench.py $Q --render $mode > $OUT/prof_$mode.log 2>&1 || { echo "rc=$? in $mode"; exit 1; }
  tail -n 1 $OUT/prof_$mode.log | cut -c1-200
done
