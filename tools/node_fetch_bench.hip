/*
 * node_fetch_bench.hip — measurement tool (not product code): how fast can a
 * CU fetch 128-B BVH nodes whose addresses differ per lane, the access shape of
 * k_intersect_closest (cy_bvhw.h: every lane loads its own node as eight
 * dwordx4 loads from one 128-B line)?
 *
 * Each thread follows a chain of dependent node fetches (the next node index
 * is a hash of the loaded words), like a traversal's descent.  Variants:
 *   0  per lane: 8 x global_load_dwordx4 of the lane's node (the kernel today)
 *   1  cooperative: 8 lanes load one node (16 B each, the whole 128-B line per
 *      8 lanes), 8 instructions fetch the wave's 64 nodes, then the wave
 *      transposes them through LDS (ds_write_b128, ds_read_b128 x 8)
 *   2  per lane: 4 x dwordx4 (a 64-B node)
 *   3  per lane: 8 x dwordx4 with half of the lanes idle (lane utilisation 0.5)
 *   4  cooperative with half of the lanes idle
 * Table sizes: 2 MiB (L2-resident) and 25.6 MB (the BMW stand-in's 4-wide BVH).
 *
 * build: hipcc -O3 --offload-arch=gfx950 -o tools/_build/node_fetch_bench tools/node_fetch_bench.hip
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int BLOCK = 256;
constexpr int CHAIN = 48;

__device__ __forceinline__ unsigned mix(unsigned h)
{
  h ^= h >> 16;
  h *= 0x7feb352dU;
  h ^= h >> 15;
  h *= 0x846ca68bU;
  h ^= h >> 16;
  return h;
}

template<int VAR, int WAVES>
__global__ void __launch_bounds__(BLOCK, WAVES) k_fetch(const float4 *__restrict__ nodes, unsigned n_nodes,
                                                        float *out)
{
  __shared__ float4 stage[(VAR == 1 || VAR == 4) ? BLOCK * 8 : 1];
  const unsigned tid = blockIdx.x * BLOCK + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  unsigned idx = mix(tid) % n_nodes;
  const bool active = (VAR == 3 || VAR == 4) ? (lane & 1) == 0 : true;
  float acc = 0.0f;
  for (int step = 0; step < CHAIN; step++) {
    float4 v[8];
    if constexpr (VAR == 0 || VAR == 3) {
      if (active) {
        const float4 *np = nodes + (size_t)idx * 8;
#pragma unroll
        for (int k = 0; k < 8; k++) {
          v[k] = np[k];
        }
      }
    }
    else if constexpr (VAR == 2) {
      const float4 *np = nodes + (size_t)idx * 8;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        v[k] = np[k];
        v[k + 4] = v[k];
      }
    }
    else {
      /* cooperative: in instruction k lane L fetches part L % 8 of the node of
       * lane 8k + L / 8 */
      float4 *st = stage + wave * 64 * 8;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int owner = 8 * k + (lane >> 3);
        const unsigned oidx = (unsigned)__shfl((int)idx, owner);
        const bool oact = (VAR == 4) ? (owner & 1) == 0 : true;
        if (oact) {
          st[owner * 8 + (lane & 7)] = nodes[(size_t)oidx * 8 + (lane & 7)];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_s_waitcnt(0xc07f); /* lgkmcnt(0) */
      __builtin_amdgcn_wave_barrier();
      if (active) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          v[k] = st[lane * 8 + k];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (active) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        s += v[k].x + v[k].y + v[k].z + v[k].w;
      }
      acc += s;
      idx = mix(__float_as_uint(s) ^ idx ^ (unsigned)step) % n_nodes;
    }
  }
  if (acc == 12345.678f) {
    out[tid] = acc;
  }
}

template<int VAR, int WAVES> static double run(const float4 *nodes, unsigned n, float *out, int blocks)
{
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_fetch<VAR, WAVES>), dim3(blocks), dim3(BLOCK), 0, 0, nodes, n, out);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((k_fetch<VAR, WAVES>), dim3(blocks), dim3(BLOCK), 0, 0, nodes, n, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const double lanes_active = (VAR == 3 || VAR == 4) ? 0.5 : 1.0;
  const double fetches = (double)blocks * BLOCK * CHAIN * lanes_active;
  return fetches / (best * 1e-3); /* node fetches per second */
}

int main()
{
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double clk = 2.4e9;
  printf("device %s, %d CUs\n", p.gcnArchName, cus);
  const unsigned sizes[2] = {16384, 200000};
  float *out;
  CHECK(hipMalloc((void **)&out, sizeof(float) * 64 * 1024 * 1024));
  for (unsigned n : sizes) {
    std::vector<float> h((size_t)n * 32);
    for (size_t i = 0; i < h.size(); i++) {
      h[i] = (float)((i * 2654435761u) % 1000) * 0.001f;
    }
    float4 *nodes;
    CHECK(hipMalloc((void **)&nodes, h.size() * 4));
    CHECK(hipMemcpy(nodes, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const char *names[5] = {"per-lane 8x16B", "cooperative 8 lanes/node + LDS", "per-lane 4x16B (64-B node)",
                            "per-lane 8x16B, half lanes idle", "cooperative, half lanes idle"};
    for (int waves : {4, 8}) {
      /* enough blocks for every wave slot of every CU, x4 for a tail */
      const int blocks = cus * (waves * 4 * 64 / BLOCK) * 4;
      double r[5];
      if (waves == 4) {
        r[0] = run<0, 4>(nodes, n, out, blocks);
        r[1] = run<1, 4>(nodes, n, out, blocks);
        r[2] = run<2, 4>(nodes, n, out, blocks);
        r[3] = run<3, 4>(nodes, n, out, blocks);
        r[4] = run<4, 4>(nodes, n, out, blocks);
      }
      else {
        r[0] = run<0, 8>(nodes, n, out, blocks);
        r[1] = run<1, 8>(nodes, n, out, blocks);
        r[2] = run<2, 8>(nodes, n, out, blocks);
        r[3] = run<3, 8>(nodes, n, out, blocks);
        r[4] = run<4, 8>(nodes, n, out, blocks);
      }
      for (int v = 0; v < 5; v++) {
        printf("table %7.1f MB waves/SIMD %d  %-36s %8.2f G nodes/s  %6.2f cycles/node/CU @2.4GHz\n",
               n * 128.0 / 1e6, waves, names[v], r[v] / 1e9, clk * cus / r[v]);
      }
    }
    CHECK(hipFree(nodes));
  }
  CHECK(hipFree(out));
  return 0;
}
