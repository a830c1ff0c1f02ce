#!/bin/bash
# Traversal-only variant builds (measurement): compiles hipcycles.hip once per
# "name -Ddefine ..." argument, in parallel, and links each with the default
# build's shading objects into raytracingproject_amd/libhipcycles-<name>.so
# ("default" rebuilds the default object and libhipcycles.so itself).
#   tools/build_trav_variants.sh "default" "soa -DCY_LDS_TOP_SOA=1" ...
set -u
cd "$(dirname "$0")/.."
FLAGS=(-O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc -fPIC
       -std=c++17 -Wno-unused-result -Wno-unused-value -Iinclude)
SPECS=("$@")
pids=()
for spec in "${SPECS[@]}"; do
  read -r -a parts <<< "$spec"
  name=${parts[0]}
  mkdir -p "build/device/$name"
  /opt/rocm/bin/hipcc "${FLAGS[@]}" "${parts[@]:1}" -c -o "build/device/$name/hipcycles.o.tmp" \
    raytracingproject_amd/csrc/device/hipcycles.hip > "build/device/$name/build.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
[ $rc -eq 0 ] || { echo "compile failed"; exit 1; }
SHADE=$(ls build/device/default/k_shade_*.o)
for spec in "${SPECS[@]}"; do
  read -r -a parts <<< "$spec"
  name=${parts[0]}
  mv "build/device/$name/hipcycles.o.tmp" "build/device/$name/hipcycles.o"
  out=raytracingproject_amd/libhipcycles-$name.so
  [ "$name" = default ] && out=raytracingproject_amd/libhipcycles.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -fno-gpu-rdc -shared -fPIC -o "$out" "build/device/$name/hipcycles.o" $SHADE
  echo "linked $out"
done
