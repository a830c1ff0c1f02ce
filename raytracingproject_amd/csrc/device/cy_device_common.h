/*
 * cy_device_common.h — wave-level helpers shared by the wavefront kernels
 * (hipcycles.hip and the per-closure-count shade kernels in k_shade.hip).
 */
#ifndef CY_DEVICE_COMMON_H
#define CY_DEVICE_COMMON_H

#include <hip/hip_runtime.h>

#include "../kernel/cy_integrator.h"

/* XCD-aware work mapping.  Workgroups are dealt round-robin over the 8 XCDs
 * (block b and b + 8 share one, MI355X_MICROARCH.md), each XCD with its own
 * 4 MB L2.  The wavefront queues hold paths in slot order, i.e. neighbouring
 * pixels of one sample next to each other; with the identity mapping every
 * XCD gets every 8th block of 256 paths and its L2 has to hold the BVH nodes
 * of the whole image.  Remapping the `active` leading blocks so that XCD x
 * takes one contiguous eighth of the queue gives each L2 one image region.
 * Blocks at or past `active` (the queue grid is sized for the whole slot pool)
 * keep their index and find no work.  Placement is not guaranteed, so this is
 * for speed only: every index 0 .. active-1 is still taken exactly once.
 * Used by the traversal kernels (BMW frame: closest 45.0 -> 44.5 ms, shadow
 * 23.1 -> 22.9 ms); the shading kernel keeps the identity mapping. */
#ifndef CY_XCD_REMAP
#  define CY_XCD_REMAP 1
#endif
__device__ __forceinline__ int cy_xcd_block(int b, int active)
{
#if CY_XCD_REMAP
  if (b >= active) {
    return b;
  }
  const int q = active >> 3, r = active & 7;
  const int x = b & 7, k = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
#else
  (void)active;
  return b;
#endif
}

/* queue index of this thread: the remapped block of a launch whose first
 * `n_active` threads have work */
__device__ __forceinline__ int cy_queue_index(int n_active)
{
  const int active_blocks = (n_active + (int)blockDim.x - 1) / (int)blockDim.x;
  return cy_xcd_block((int)blockIdx.x, active_blocks) * (int)blockDim.x + (int)threadIdx.x;
}

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
      if (tile.stream) {
        /* the slot goes idle; k_stream_restart hands it work once the host
         * has appended tiles to the lane */
        cy_st(&b.item[slot], CY_NO_ITEM);
      }
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
