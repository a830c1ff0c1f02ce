set -u
mkdir -p gpurun_out
Q="--config classroom_standin --steps 2 --warmup 1 --no-cpu-baseline --tile 0 --scaling-proxy= --other-configs="
timeout -k 10 300 python bench.py $Q > gpurun_out/cls_default.log 2>&1 || exit $?
for v in fixedsvm nolight sssoff; do
  HIPCY_DEVICE_LIB=$PWD/raytracingproject_amd/libhipcycles-$v.so timeout -k 10 300 python bench.py $Q > gpurun_out/cls_$v.log 2>&1 || exit $?
done
echo done
