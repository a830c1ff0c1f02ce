/*
 * k_trav.h — the traversal kernels' building blocks shared by hipcycles.hip
 * (the wavefront's closest-hit and shadow stages) and k_shade.hip (the fused
 * tail kernel, k_tail_*): the per-workgroup LDS stacks, the scene traversal
 * entry by BVH width / instancing / curve shapes, and the LDS copy of the wide
 * BVH's top nodes.
 */
#ifndef K_TRAV_H
#define K_TRAV_H

#include "cy_device_common.h"
#include "../kernel/cy_bvhw.h"

/* Traversal stack in LDS: BVH2 keeps CY_LDS_STACK node addresses per thread,
 * the wide BVHs CY_LDS_STACKW (node, entry distance) pairs. */
/* Minimum waves per SIMD the traversal kernels are register-allocated for
 * (amdgpu_waves_per_eu); with the LDS stack it sets their occupancy. */
/* hair kernels (the ribbon and thick-curve intersectors) need more registers:
 * at the 96 of five waves they spill; measured on the JNK crop (BVH2 hair):
 * 4 waves (128 VGPRs) 18.6 Msamples/s, 3 waves 16.7 */
#ifndef CY_TRAV_HAIR_WAVES
#  define CY_TRAV_HAIR_WAVES 4
#endif
#define CY_TRAV_WAVES(hair) ((hair) != 0 ? CY_TRAV_HAIR_WAVES : CY_TRAV_MIN_WAVES)
#ifndef CY_TRAV_MIN_WAVES
#  define CY_TRAV_MIN_WAVES 5
#endif

#define CY_STATS_SHARDS 64

/* LDS traversal stacks of one workgroup (one column per thread):
 *   W = 2          BVH2 node addresses, CY_LDS_STACK deep;
 *   W > 2          the wide traversal's ring of CY_LDS_STACKW entries, plus for
 *                  instanced scenes the reference-order top level's BVH2 stack
 *                  (CY_LDS_STACK_TOP deep; cy_path.h bvh2_intersect WI > 2). */
#ifndef CY_LDS_STACK_TOP
#  define CY_LDS_STACK_TOP 8
#endif
/* TOP: the kernel serves the wide BVH's top nodes (2 W float4 each) from
 * LDS, at most NTOP of them (non-instanced scenes; k_intersect_closest,
 * k_intersect_shadow and k_tail, which fill them with lds_fill_top; the host
 * passes the count in kg->bvhw_top).  Other kernels reserve no LDS for them
 * and traverse with n_top = 0. */
template<int W, bool INST, bool TOP = false, int NTOP = CY_LDS_TOP> struct LdsStack {
  CyStackEntry ring[CY_LDS_STACKW * CY_BLOCK];
  int top[(INST ? CY_LDS_STACK_TOP : 1) * CY_BLOCK];
  hc_float4 top_nodes[(!INST && TOP && NTOP > 0) ? NTOP * 2 * W : 1];
};
template<bool INST, bool TOP, int NTOP> struct LdsStack<2, INST, TOP, NTOP> {
  int top[CY_LDS_STACK * CY_BLOCK];
};

/* This thread's ring column of the wide kernels' LDS stack (nullptr for BVH2). */
template<int W, bool INST, bool TOP, int NTOP>
__device__ __forceinline__ CY_LDS CyStackEntry *lds_ring_of(LdsStack<W, INST, TOP, NTOP> *lds)
{
  if constexpr (W > 2) {
    return (CY_LDS CyStackEntry *)(lds->ring + threadIdx.x);
  }
  else {
    return nullptr;
  }
}

/* HAIR (scenes with curves): unaligned nodes and curve leaves of the shapes
 * HAIR selects (1 ribbons, 2 thick curves, 3 both).  Ribbon-only scenes also
 * traverse the wide BVH (W = 4 / 8, cy_bvhw.h); thick curves keep the BVH2. */
template<int W, bool any_hit, bool INST = true, int HAIR = 0, bool TOP = false, int NTOP = CY_LDS_TOP>
__device__ __forceinline__ bool scene_traverse(const CyGlobals *kg, const CyRay *ray, uint visibility,
                                               CyIsect *isect, uint *err, uint *n_nodes, uint *n_leaves,
                                               uint *n_tris, LdsStack<W, INST, TOP, NTOP> *lds, bool *tie = nullptr)
{
  const int t = threadIdx.x;
  if constexpr (W == 2) {
    return bvh2_intersect<any_hit, INST, 2, CY_LDS_STACK, CY_BLOCK, HAIR>(kg, ray, visibility, isect, err, n_nodes,
                                                                         n_leaves, n_tris,
                                                                         (CY_LDS int *)(lds->top + t));
  }
  else if constexpr (INST) {
    /* instanced scene: reference-order top level, wide BVH inside instances */
    return bvh2_intersect<any_hit, true, W, CY_LDS_STACK_TOP, CY_BLOCK, HAIR>(
        kg, ray, visibility, isect, err, n_nodes, n_leaves, n_tris, (CY_LDS int *)(lds->top + t),
        (CY_LDS CyStackEntry *)(lds->ring + t), tie);
  }
  else {
    return bvhw_intersect<W, any_hit, HAIR>(kg, ray, visibility, isect, err, n_nodes, n_leaves, n_tris,
                                            (CY_LDS CyStackEntry *)(lds->ring + t), tie,
                                            (CY_LDS const hc_float4 *)lds->top_nodes,
                                            TOP ? (kg->bvhw_top < NTOP ? kg->bvhw_top : NTOP) : 0);
  }
}

/* Copy the wide BVH's top nodes into the workgroup's LDS (CY_LDS_TOP; every
 * thread of the block calls this before its traversal). */
template<int W, bool INST, bool TOP, int NTOP>
__device__ __forceinline__ void lds_fill_top(const CyGlobals *kg, LdsStack<W, INST, TOP, NTOP> *lds)
{
  if constexpr (W > 2 && !INST && TOP && NTOP > 0) {
    const int n = (kg->bvhw_top < NTOP ? kg->bvhw_top : NTOP) * 2 * W;
    const hc_float4 *src = (const hc_float4 *)kg->bvhw_nodes;
    for (int i = threadIdx.x; i < n; i += CY_BLOCK) {
#  if CY_LDS_TOP_SOA
      /* node i / 2W, float4 i % 2W */
      lds->top_nodes[(i % (2 * W)) * NTOP + i / (2 * W)] = src[i];
#  else
      lds->top_nodes[i] = src[i];
#  endif
    }
    __syncthreads();
  }
}

#endif
