#!/bin/bash
# Round-6 shadow-traversal variants (r05 verdict, next #2), each a named leg:
# the opaque-shadow kernel with 21 (default) or 85 wide nodes in LDS
# (CY_LDS_TOP_SHADOW; libhipcycles-shtop21 / -shtop85, the same sources), and
# the shadow-queue direction sort (hipcy_set_shadow_sort 0 / 5): frame time
# of the bench frame, then a kernel trace (per-kernel averages) of each lib.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/shadow
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_sss.py \
  tests/test_nodes.py -k "volume_scene_loads or unimplemented_node" > gpurun_out/shadow/pytest_fixed.log 2>&1 || exit 1
tail -n 2 gpurun_out/shadow/pytest_fixed.log
for lib in shtop21 shtop85; do
  for ss in 0 5; do
    echo "=== $lib sort $ss"
    HIPCY_DEVICE_LIB=raytracingproject_amd/libhipcycles-$lib.so timeout -k 10 240 \
      python3 tools/render_modes.py frame --frames 5 --shadow-sort $ss > gpurun_out/shadow/${lib}_s$ss.log 2>&1 || exit 1
    tail -n 1 gpurun_out/shadow/${lib}_s$ss.log
  done
done
for lib in shtop21 shtop85; do
  HIPCY_DEVICE_LIB=raytracingproject_amd/libhipcycles-$lib.so timeout -k 10 240 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/shadow/prof_$lib -o run --output-format csv -- \
    python3 tools/render_modes.py frame --frames 3 > gpurun_out/shadow/prof_$lib.log 2>&1 || exit 1
  f=$(ls gpurun_out/shadow/prof_$lib/*/run_kernel_stats.csv gpurun_out/shadow/prof_$lib/run_kernel_stats.csv 2>/dev/null | head -n 1)
  echo "=== $lib kernel stats"; head -n 6 "$f" | cut -c1-160
done
# fused-tail kernel at 4 waves per SIMD (libhipcycles-tail4: the plain shading
# objects rebuilt with CY_TAIL_WAVES=4), thresholds 32768 / 131072 / 262144
for t in 32768 131072 262144; do
  for m in shard8 frame; do
    echo "=== tail4 $m $t"
    HIPCY_DEVICE_LIB=raytracingproject_amd/libhipcycles-tail4.so timeout -k 10 240 \
      python3 tools/render_modes.py $m --frames 5 --tail $t > gpurun_out/shadow/tail4_${m}_$t.log 2>&1 || exit 1
    tail -n 1 gpurun_out/shadow/tail4_${m}_$t.log
  done
done
# shading-queue sort (mode 8) on the plain bench scene
for m in frame shard8; do
  echo "=== ray sort 8 $m"
  timeout -k 10 240 python3 tools/render_modes.py $m --frames 5 --ray-sort 8 > gpurun_out/shadow/rsort8_$m.log 2>&1 || exit 1
  tail -n 1 gpurun_out/shadow/rsort8_$m.log
done
echo done
