/*
 * cy_device_common.h — wave-level helpers shared by the wavefront kernels
 * (hipcycles.hip and the per-closure-count shade kernels in k_shade.hip).
 */
#ifndef CY_DEVICE_COMMON_H
#define CY_DEVICE_COMMON_H

#include <hip/hip_runtime.h>

#include "../kernel/cy_integrator.h"

/* Block-aggregated fetch-and-add: every lane with `want` gets a distinct
 * index from *counter, one global atomic per workgroup.  The counters are
 * device-scope atomics shared by all 8 XCDs and serialise at the memory side,
 * so they are claimed per workgroup rather than per wave.  Every thread of the
 * block must call it (it synchronises); lds holds 1 + CY_BLOCK/64 words. */
#define CY_CLAIM_LDS (1 + CY_BLOCK / 64)
__device__ __forceinline__ uint block_claim(uint *counter, bool want, uint *lds)
{
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const unsigned long long mask = __ballot(want);
  if (lane == 0) {
    lds[1 + wave] = (uint)__popcll(mask);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint total = 0;
    for (int w = 0; w < CY_BLOCK / 64; w++) {
      const uint c = lds[1 + w];
      lds[1 + w] = total;
      total += c;
    }
    lds[0] = total ? atomicAdd(counter, total) : 0u;
  }
  __syncthreads();
  const uint idx = lds[0] + lds[1 + wave] + (uint)__popcll(mask & ((1ull << lane) - 1ull));
  __syncthreads();
  return want ? idx : 0xFFFFFFFFu;
}

/* Append the slot of every active lane to a queue (order within the queue is
 * unspecified; results never depend on it). */
__device__ __forceinline__ void queue_push(int *queue, uint *counter, int slot, bool active, uint *lds)
{
  const uint idx = block_claim(counter, active, lds);
  if (active) {
    queue[idx] = slot;
  }
}

__device__ __forceinline__ void stats_add(unsigned long long *dst, uint v)
{
  /* wave reduce then one atomic */
  unsigned long long x = v;
  for (int off = 32; off > 0; off >>= 1) {
    x += __shfl_xor(x, off);
  }
  if ((threadIdx.x & 63) == 0 && x) {
    atomicAdd(dst, x);
  }
}

/* Claim the next work item for every lane with need set (one atomic per
 * workgroup) and start it; samples without a camera ray are recorded as such
 * and the lane claims again.  Returns true when the slot holds a new path.
 * Every thread of the block must call it. */
__device__ __forceinline__ bool slot_refill(const CyGlobals &kg, const CyPathBuffers &b, const CyTile &tile,
                                            int slot, bool need, uint *lds)
{
  uint item = block_claim(tile.work_next, need, lds);
  while (need) {
    if (item >= tile.n_items) {
      return false;
    }
    if (slot_start(&kg, &b, &tile, slot, item)) {
      return true;
    }
    item = atomicAdd(tile.work_next, 1u);
  }
  return false;
}

#endif /* CY_DEVICE_COMMON_H */
