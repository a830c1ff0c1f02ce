#!/bin/bash
# GPU-box profiling: rocprofv3 kernel trace + stats of bench.py, the same for
# the instrumented frame alone (bench.py --profile-frame: single lane, no
# overlapping kernels), then separate PMC passes over that frame (counters are
# never combined with sys/runtime traces).  Reduce with tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r02}
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --tile 0"}
FARGS=${FRAME_ARGS:-"--profile-frame"}
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  if fatal $rc || [[ $rc != 0 ]]; then echo "FATAL rc=$rc in $name, stopping"; exit $rc; fi
}
if [[ ${SKIP_TRACE:-0} != 1 ]]; then
  step trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace_$TAG -o run --output-format csv -- python3 bench.py $ARGS
fi
step trace_frame 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_frame_$TAG -o run --output-format csv -- python3 bench.py $FARGS
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_INST_LEVEL_VMEM"; do
  name=pmc_$(echo $pmc | cut -d' ' -f1)
  step $name 300 rocprofv3 --pmc $pmc --kernel-trace -d $OUT/${name}_$TAG -o run --output-format csv -- python3 bench.py $FARGS
done
echo done
