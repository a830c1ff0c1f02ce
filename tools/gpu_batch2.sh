#!/bin/bash
# r06 batch 2: the new parity cases (AOV, voxel, bump both, decoupled volumes),
# the multi-device harness, a kernel trace of the N = 8 row shard with the
# fused tail, then the bench line.
set -u
bash tools/gpu_r06.sh sel tests/test_gpu_parity.py -k "shading_aov or shading_voxel or shading_bump_both or decoupled or fused_tail or volume_cornell or volume_hetero" \
  && bash tools/gpu_r06.sh harness -k "share_the_tile_queue" \
  && bash tools/gpu_r06.sh itrace shard8 \
  && bash tools/gpu_r06.sh bench --other-configs=bmw27_production,classroom_standin,junkshop_standin@1664x832+512x256
