#!/bin/bash
# Round-6 shadow-traversal variant: hit leaf children first in the opaque
# any-hit traversal (CY_ANYHIT_LEAF_FIRST; libhipcycles-lf1 against the same
# sources without it, -lf0): parity of the shadow queries and renders, frame
# times, per-kernel averages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lf
export TMPDIR=/tmp
HIPCY_DEVICE_LIB=raytracingproject_amd/libhipcycles-lf1.so timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 120 \
  --timeout-method thread tests/test_gpu_parity.py -k "(shadow_any_hit or (render_matches_reference and bvh4)) and not volume and not fog" \
  > gpurun_out/lf/pytest_lf1.log 2>&1 || { tail -n 20 gpurun_out/lf/pytest_lf1.log; exit 1; }
tail -n 2 gpurun_out/lf/pytest_lf1.log
for lib in lf0 lf1; do
  for m in frame shard8; do
    HIPCY_DEVICE_LIB=raytracingproject_amd/libhipcycles-$lib.so timeout -k 10 240 \
      python3 tools/render_modes.py $m --frames 5 > gpurun_out/lf/${lib}_$m.log 2>&1 || exit 1
    echo "=== $lib $m: $(tail -n 1 gpurun_out/lf/${lib}_$m.log)"
  done
  HIPCY_DEVICE_LIB=raytracingproject_amd/libhipcycles-$lib.so timeout -k 10 240 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/lf/prof_$lib -o run --output-format csv -- \
    python3 tools/render_modes.py frame --frames 3 > gpurun_out/lf/prof_$lib.log 2>&1 || exit 1
done
echo done
