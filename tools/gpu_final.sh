#!/bin/bash
# Round-6 final profile: rocprofv3 kernel trace + stats of the bench run and of
# the instrumented frame, the PMC passes (tools/gpu_prof.sh, each counter group
# in its own run), their reduction into profiles/ (tools/pmc_summary.py), then
# the bench line, which reads the fresh PMC summary for roofline.traffic.  The
# reduced profiles are copied under gpurun_out/final_profiles/ to come back.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final_profiles
bash tools/gpu_prof.sh r06 || exit 1
timeout -k 10 120 python3 tools/pmc_summary.py r06 > gpurun_out/pmc_summary.log 2>&1 || { tail -n 20 gpurun_out/pmc_summary.log; exit 1; }
cp -r profiles/r06 gpurun_out/final_profiles/ && cp profiles/pmc_summary.json gpurun_out/final_profiles/
bash tools/gpu_r06.sh bench --other-configs=bmw27_production,classroom_standin,junkshop_standin@1664x832+512x256
