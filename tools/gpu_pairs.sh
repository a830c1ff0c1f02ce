#!/bin/bash
# Round-6 fused tail with lane pairs (CY_TAIL_PAIRS: the path's next ray and
# its light sample's shadow ray traced side by side; libhipcycles-pairs, the
# plain shading objects rebuilt with it): fused-tail parity, then the N = 8
# shard and the whole frame against the default library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pairs
export TMPDIR=/tmp
HIPCY_DEVICE_LIB=raytracingproject_amd/libhipcycles-pairs.so timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 120 \
  --timeout-method thread tests/test_gpu_parity.py -k "fused_tail" > gpurun_out/pairs/pytest_pairs.log 2>&1 \
  || { tail -n 30 gpurun_out/pairs/pytest_pairs.log; exit 1; }
tail -n 2 gpurun_out/pairs/pytest_pairs.log
for lib in default pairs; do
  L=raytracingproject_amd/libhipcycles.so
  [[ $lib == pairs ]] && L=raytracingproject_amd/libhipcycles-pairs.so
  for t in 32768 131072 262144; do
    for m in shard8 frame; do
      HIPCY_DEVICE_LIB=$L timeout -k 10 240 python3 tools/render_modes.py $m --frames 5 --tail $t \
        > gpurun_out/pairs/${lib}_${m}_$t.log 2>&1 || exit 1
      echo "=== $lib $m $t: $(tail -n 1 gpurun_out/pairs/${lib}_${m}_$t.log)"
    done
  done
done
echo done
