/*
 * cy_device_common.h — wave-level helpers shared by the wavefront kernels
 * (hipcycles.hip and the per-closure-count shade kernels in k_shade.hip).
 */
#ifndef CY_DEVICE_COMMON_H
#define CY_DEVICE_COMMON_H

#include <hip/hip_runtime.h>

#include "../kernel/cy_integrator.h"

__device__ __forceinline__ void queue_push(int *queue, uint *counter, int slot, bool active)
{
  /* wave-aggregated append: one atomic per wave */
  const unsigned long long mask = __ballot(active);
  if (mask == 0) {
    return;
  }
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)mask) - 1;
  uint base = 0;
  if (lane == leader) {
    base = atomicAdd(counter, (uint)__popcll(mask));
  }
  base = __shfl(base, leader);
  if (active) {
    const unsigned long long lower = mask & ((1ull << lane) - 1ull);
    queue[base + __popcll(lower)] = slot;
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

/* Claim the next work item for every lane with need set (one atomic per wave)
 * and start it; samples without a camera ray are recorded as such and the lane
 * claims again.  Returns true when the slot holds a new path. */
__device__ __forceinline__ bool slot_refill(const CyGlobals &kg, const CyPathBuffers &b, const CyTile &tile,
                                            int slot, bool need)
{
  const unsigned long long mask = __ballot(need);
  if (mask == 0) {
    return false;
  }
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)mask) - 1;
  uint base = 0;
  if (lane == leader) {
    base = atomicAdd(tile.work_next, (uint)__popcll(mask));
  }
  base = __shfl(base, leader);
  uint item = base + (uint)__popcll(mask & ((1ull << lane) - 1ull));
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
