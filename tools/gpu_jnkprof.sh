set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/dbg_trace.py gpu shading_bump_paths 23 7 4 > gpurun_out/gpu_trace.txt 2> gpurun_out/gpu_trace.err
echo dbg rc=$?
Q="--config junkshop_standin --width 512 --height 256 --samples 16 --steps 1 --warmup 1 --no-cpu-baseline --other-configs= --tile 0 --scaling-proxy="
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_jnk4 -o run --output-format csv -- python3 bench.py $Q > gpurun_out/jnk4.log 2>&1 || exit $?
echo jnk4 done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_jnk2 -o run --output-format csv -- python3 bench.py $Q --bvh-width 2 > gpurun_out/jnk2.log 2>&1 || exit $?
echo jnk2 done
