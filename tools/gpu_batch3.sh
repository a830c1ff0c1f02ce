#!/bin/bash
# Round-6 batch 3: the new parity cases (AOV, voxel, bump-both, decoupled
# volumes, camera inside volume, SSS in fog, shadow catchers, data passes,
# branched path tracing),
# the fused tail, the 8-device harness at the default hold, an iteration
# trace of the N = 8 shard and the bench line with the other configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r06.sh sel tests/test_gpu_parity.py -k "shading_aov or shading_voxel or shading_bump_both or decoupled or camera_inside or fog or shadow_catcher or data_passes or branched or fused_tail or volume_cornell or volume_hetero or sss_disk or sss_cornell" \
  && bash tools/gpu_r06.sh harness -k "share_the_tile_queue" \
  && bash tools/gpu_r06.sh itrace shard8 \
  && bash tools/gpu_r06.sh bench --other-configs=bmw27_production,classroom_standin,junkshop_standin@1664x832+512x256
