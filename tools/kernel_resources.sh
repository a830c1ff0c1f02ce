#!/bin/bash
# Per-kernel VGPR / scratch / LDS / occupancy of the device library (compile-time report).
cd "$(dirname "$0")/.."
SRC=${SRC:-raytracingproject_amd/csrc/device/hipcycles.hip}
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-gpu-rdc -std=c++17 -Iinclude "$@" -c --offload-device-only -Rpass-analysis=kernel-resource-usage \
  $SRC -o /tmp/_kres.o 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy|LDS Size" |
  sed -E 's/.*remark: //; s/ \[-Rpass.*//' |
  awk '/Function Name/{if(l)print l; l=$3; next}{l=l"  "$0}END{print l}' | c++filt | sed 's/(CyGlobals.*)//'
