#!/bin/bash
# Round-6 batch 4: the whole GPU suite + smoke (light passes, the _ext shading
# variants, the persistent fused tail, shadow-queue sort, decoupled segments
# in device memory), the bench line with the other configs, the fused-tail
# threshold and shadow-sort sweeps, an iteration trace of the N = 8 row shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r06.sh test \
  && bash tools/gpu_r06.sh bench --other-configs=bmw27_production,classroom_standin,junkshop_standin@1664x832+512x256 \
  && TAILS="32768 131072 262144 524288" TAIL_MODES="frame shard8" bash tools/gpu_r06.sh tailsweep \
  && bash tools/gpu_r06.sh ssort \
  && bash tools/gpu_r06.sh itrace shard8
