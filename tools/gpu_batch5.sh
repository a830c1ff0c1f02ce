#!/bin/bash
# Round-6 batch 5: the whole GPU suite + smoke on the _ext / _vext split, the
# bench line with the other configs, then the lane-pair fused tail experiment.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r06.sh test \
  && bash tools/gpu_r06.sh bench --other-configs=bmw27_production,classroom_standin,junkshop_standin@1664x832+512x256 \
  && bash tools/gpu_pairs.sh
