#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int v) { if (threadIdx.x == 0) printf("device printf %s %08x\n", "tag", v); }
int main() { hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, 0x1234); hipDeviceSynchronize(); printf("host done\n"); return 0; }
