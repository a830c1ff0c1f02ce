#!/bin/bash
# Round-6 batch 4: light passes and the persistent fused tail / shadow-queue
# sort parity, the fused-tail threshold and shadow-sort sweeps, an iteration
# trace of the N = 8 row shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r06.sh sel tests/test_gpu_parity.py -k "light_passes or fused_tail or shadow_sort or data_passes or cornell_64 or bmw_small" \
  && TAILS="32768 131072 262144 524288" TAIL_MODES="frame shard8" bash tools/gpu_r06.sh tailsweep \
  && bash tools/gpu_r06.sh ssort \
  && bash tools/gpu_r06.sh itrace shard8
