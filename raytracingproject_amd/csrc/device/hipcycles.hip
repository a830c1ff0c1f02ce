/*
 * hipcycles.hip — MI355X (gfx950) Cycles path-tracing device: kernels + C ABI.
 *
 * Host side mirrors CUDADevice (device/cuda/device_cuda_impl.cpp): memory ops,
 * const_copy_to("__data"), named-array binding (global_alloc), render of one
 * RenderTile (CUDADevice::render :1853-1952).  The kernel side is the wavefront
 * integrator of kernel/cy_integrator.h; see DESIGN.md for the data layout.
 */
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "hipcycles.h"
#include "cy_device_common.h"
#include "k_shade.h"
#include "k_trav.h"
#include "../host/cy_bvhw_collapse.h"

/* wide nodes the opaque-shadow kernel serves from LDS (the closest-hit kernel
 * and the fused tail keep CY_LDS_TOP, cy_bvhw.h) */
#ifndef CY_LDS_TOP_SHADOW
#  define CY_LDS_TOP_SHADOW CY_LDS_TOP
#endif

/* PassType bits of the data passes (kernel_types.h:353-364: DEPTH .. MATERIAL_ID) */
#define CY_HOST_DATA_PASSES ((1 << 2) | (1 << 3) | (1 << 4) | (1 << 5) | (1 << 6))
/* the light passes this device writes (PASSMASK(type) = 1 << (type % 32):
 * MIST 0, EMISSION 1, BACKGROUND 2, SHADOW 4, LIGHT 5 (no pass), DIFFUSE_*
 * 6-8, GLOSSY_* 9-11, TRANSMISSION_* 12-14, VOLUME_* 18-19; not AO 3) */
#define CY_HOST_LIGHT_PASSES ((0x7fff & ~(1 << 3)) | (1 << 18) | (1 << 19))

/* ------------------------------------------------------------------------- */
/* Kernels                                                                     */

__global__ void __launch_bounds__(CY_BLOCK) k_accumulate(CyTile tile)
{
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < (int)tile.npix) {
    accumulate_pixel(&tile, p);
  }
}

/* ---------------------------------------------------------------------------
 * Tile streams (hipcy_render_feed).  A lane's work items are numbered over
 * the tiles appended to it; see stream_render for the host side. */

/* chunk b carries on chunk a: the next sample range of the same RenderTile,
 * its items right after a's (stream_fill appends a tile's chunks in a row) */

static __device__ bool stream_chunk_continues(const CyTileDesc &a, const CyTileDesc &b)
{
  /* groups of one tile only (a tile split in sample ranges is never grouped) */
  return a.group_npix == (uint)(a.w * a.h) && b.group_npix == (uint)(b.w * b.h) && a.px_begin == 0 &&
         b.px_begin == 0 && b.buffer == a.buffer && b.x == a.x && b.y == a.y && b.w == a.w && b.h == a.h &&
         b.start_sample == a.start_sample + a.num_samples &&
         b.item_begin == a.item_begin + (uint)(a.w * a.h) * (uint)a.num_samples;
}

/* The records of the lane's completed chunks descs[0 .. gridDim.y-1] added
 * to their render buffers (sample order per pixel, as k_accumulate); one
 * launch per batch of chunks completed together, blockIdx.y the chunk.  A
 * tile split into several chunks of the batch is added by the block row of
 * its first chunk, over all of them in sample order (two rows adding to the
 * same pixels would race and lose samples). */
__global__ void __launch_bounds__(CY_BLOCK) k_accumulate_stream(const CyTileDesc *descs, const hc_float4 *ring,
                                                                uint ring_mask, int pass_stride)
{
  const int y = (int)blockIdx.y;
  CyTileDesc d = descs[y];
  if (y > 0 && stream_chunk_continues(descs[y - 1], d)) {
    return;
  }
  for (int j = y + 1; j < (int)gridDim.y; j++) {
    const CyTileDesc n = descs[j];
    if (!stream_chunk_continues(descs[j - 1], n)) {
      break;
    }
    d.num_samples += n.num_samples;
  }
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < d.w * d.h) {
    accumulate_stream_pixel(d, ring, ring_mask, pass_stride, p);
  }
}

/* Smallest work item held by a live path of the lane (the slots of its next
 * queue): every item below min(this, next unclaimed item) has its record.
 * Reduced per workgroup into CY_MIN_SHARDS words the host takes the minimum of. */
#define CY_MIN_SHARDS 32
__global__ void __launch_bounds__(CY_BLOCK) k_stream_min_live(const int *queue, const uint *count, const uint *items,
                                                              uint *out)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  uint v = 0xFFFFFFFFu;
  if (i < (int)*count) {
    v = cy_ld(&items[queue[i]]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    v = min(v, (uint)__shfl_xor(v, off));
  }
  __shared__ uint red[CY_BLOCK / 64];
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint m = red[0];
    for (int w = 1; w < CY_BLOCK / 64; w++) {
      m = min(m, red[w]);
    }
    if (m != 0xFFFFFFFFu) {
      /* one of CY_MIN_SHARDS words (atomics on one word serialise) */
      atomicMin(out + (blockIdx.x % CY_MIN_SHARDS), m);
    }
  }
}

/* Idle slots of a lane (item CY_NO_ITEM: never started, or no item was left
 * when their path ended) claim the items the host appended since and join
 * the lane's next closest queue. */
__global__ void __launch_bounds__(CY_BLOCK) k_stream_restart(CyGlobals kg, CyPathBuffers b, CyTile tile, int slot_base,
                                                             int n_slots, int *queue_out, uint *count_out)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int slot = slot_base + i;
  const bool idle = i < n_slots && cy_ld(&b.item[slot]) == CY_NO_ITEM;
  __shared__ uint claim[CY_CLAIM_LDS];
  const bool started = slot_refill(kg, b, tile, slot, idle, claim);
  queue_push(queue_out, count_out, slot, started, claim);
}

/* Traversal counters: reduced over the workgroup, then one atomic per counter
 * and workgroup into one of CY_STATS_SHARDS copies (device-scope atomics on a
 * single word serialise at the memory side).  Besides the node / leaf /
 * triangle counts, the loop iterations (nodes + leaves visited) are summed per
 * lane and, as the wave's maximum, per wave: a wave runs as many iterations as
 * its longest ray, so lane_iters / (64 * wave_iters) is the traversal loop's
 * lane utilisation. */
__device__ __forceinline__ void stats_block_add(CyStats *shard, uint n_nodes, uint n_leaves, uint n_tris,
                                                uint n_over)
{
  __shared__ uint red[6];
  if (threadIdx.x < 6) {
    red[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint iters = n_nodes + n_leaves;
  uint v[6] = {n_nodes, n_leaves, n_tris, n_over, iters, iters};
#pragma unroll
  for (int k = 0; k < 6; k++) {
    uint x = v[k];
    for (int off = 32; off > 0; off >>= 1) {
      const uint y = __shfl_xor(x, off);
      x = (k == 5) ? max(x, y) : x + y;
    }
    if ((threadIdx.x & 63) == 0 && x) {
      atomicAdd(&red[k], x);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    CyStats *st = shard + (blockIdx.x % CY_STATS_SHARDS);
    if (red[0]) atomicAdd(&st->nodes, (unsigned long long)red[0]);
    if (red[1]) atomicAdd(&st->leaves, (unsigned long long)red[1]);
    if (red[2]) atomicAdd(&st->tris, (unsigned long long)red[2]);
    if (red[3]) atomicAdd(&st->rays, (unsigned long long)red[3]);
    if (red[4]) atomicAdd(&st->lane_iters, (unsigned long long)red[4]);
    if (red[5]) atomicAdd(&st->wave_iters, (unsigned long long)red[5]);
  }
}

/* ---------------------------------------------------------------------------
 * Iteration budget (hipcy_set_traversal_budget).  A wave runs as many loop
 * iterations as its slowest ray, so a few long traversals keep a wave -- and
 * its slot on the SIMD -- busy with most lanes idle (closest-hit lanes are 45 %
 * utilised on the bench frame, shadow 31 %).  With a budget B a traversal stops
 * after B iterations and is saved as a continuation record; the records are
 * traversed by densely packed continuation launches, which may suspend again
 * into the other buffer, and the last one runs without a budget.  A resumed
 * traversal continues with the same stack, hit and near-tie state, so results
 * are bit-identical.  Used by the non-instanced wide-BVH kernels.
 *
 * Record (SoA, CY_CONT_F4 float4 arrays of `capacity` entries):
 *   0: ray P, t    1: ray D, visibility    2: hit t, u, v, prim
 *   3: cursor code, top | n_ring << 8 | tie << 16, slot, 0
 *   4..7: the LDS ring (8 x (node, entry distance)) */
#define CY_CONT_F4 8
#define CY_CONT_BLOCKS 1280 /* continuation grid: 256 CUs x 5 waves/SIMD x 4 SIMDs / 4 waves per block */
struct CyCont {
  hc_float4 *rec;
  uint *count;
  uint capacity;
};

template<int W>
__device__ __forceinline__ void cont_save(const CyCont &c, uint idx, int slot, const CyRay &ray, uint vis,
                                          const CyIsect &is, const CyTravCursor &cur,
                                          CY_LDS const CyStackEntry *ring)
{
  static_assert(CY_LDS_STACKW == 8, "continuation records hold an 8-entry ring");
  hc_float4 *r = c.rec + idx;
  const size_t cap = c.capacity;
  r[0] = mkf4(ray.P.x, ray.P.y, ray.P.z, ray.t);
  r[cap] = mkf4(ray.D.x, ray.D.y, ray.D.z, as_float(vis));
  r[2 * cap] = mkf4(is.t, is.u, is.v, int_as_float(is.prim));
  r[3 * cap] = mkf4(int_as_float(cur.code), int_as_float(cur.top | (cur.n_ring << 8) | ((int)cur.tie << 16)),
                    int_as_float(slot), cur.code_t);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (cur.n_ring > 0) {
      const CyStackEntry e0 = ring[(2 * k) * CY_BLOCK], e1 = ring[(2 * k + 1) * CY_BLOCK];
      r[(4 + k) * cap] = mkf4(int_as_float(e0.node), e0.t, int_as_float(e1.node), e1.t);
    }
  }
}

template<int W>
__device__ __forceinline__ int cont_load(const CyCont &c, uint idx, CyRay *ray, uint *vis, CyIsect *is,
                                         CyTravCursor *cur, CY_LDS CyStackEntry *ring)
{
  const hc_float4 *r = c.rec + idx;
  const size_t cap = c.capacity;
  const hc_float4 a = r[0], d = r[cap], h = r[2 * cap], q = r[3 * cap];
  ray->P = mk3(a.x, a.y, a.z);
  ray->t = a.w;
  ray->D = mk3(d.x, d.y, d.z);
  *vis = as_uint(d.w);
  is->t = h.x;
  is->u = h.y;
  is->v = h.z;
  is->prim = as_int(h.w);
  is->object = OBJECT_NONE;
  is->type = is->prim != PRIM_NONE ? PRIMITIVE_TRIANGLE : 0;
  cur->code = as_int(q.x);
  cur->code_t = q.w;
  const int packed = as_int(q.y);
  cur->top = packed & 0xFF;
  cur->n_ring = (packed >> 8) & 0xFF;
  cur->tie = ((packed >> 16) & 1) != 0;
  cur->suspended = false;
  if (cur->n_ring > 0) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const hc_float4 e = r[(4 + k) * cap];
      CyStackEntry e0, e1;
      e0.node = as_int(e.x);
      e0.t = e.y;
      e1.node = as_int(e.z);
      e1.t = e.w;
      ring[(2 * k) * CY_BLOCK] = e0;
      ring[(2 * k + 1) * CY_BLOCK] = e1;
    }
  }
  return as_int(q.z);
}

/* A wide traversal of the non-instanced scene from the root (bvhw_intersect)
 * or from a cursor, with the budget. */
template<int W, bool any_hit>
__device__ __forceinline__ void bvhw_run(const CyGlobals *kg, const CyRay *ray, uint visibility, CyIsect *isect,
                                         uint *err, uint *n_nodes, uint *n_leaves, uint *n_tris,
                                         CY_LDS CyStackEntry *ring, bool *tie, int budget, CyTravCursor *cur)
{
  const cfloat3 dir = bvh_clamp_direction(ray->D);
  bvhw_traverse<W, any_hit>(kg, 0, ray->P, dir, rcp3(dir), OBJECT_NONE, visibility, isect, err, n_nodes,
                            n_leaves, n_tris, ring, tie, budget, cur);
}

/* Suspended lanes claim continuation records (all threads of the block call
 * this); a lane that finds the buffer full finishes its traversal now. */
template<int W, bool any_hit>
__device__ __forceinline__ void cont_suspend(const CyGlobals *kg, const CyCont &out, int slot, const CyRay &ray,
                                             uint visibility, CyIsect *isect, uint *err, uint *n_nodes,
                                             uint *n_leaves, uint *n_tris, CY_LDS CyStackEntry *ring, bool *tie,
                                             CyTravCursor *cur, uint *claim)
{
  const uint idx = block_claim(out.count, cur->suspended, claim);
  if (cur->suspended) {
    if (idx < out.capacity) {
      cont_save<W>(out, idx, slot, ray, visibility, *isect, *cur, ring);
    }
    else {
      bvhw_run<W, any_hit>(kg, &ray, visibility, isect, err, n_nodes, n_leaves, n_tris, ring, tie, 0, cur);
    }
  }
}

/* Stage 1: closest hit for every queued path, or (cam_n > 0) for the camera
 * rays of the work items item_base .. item_base + cam_n - 1 held by slots
 * slot_base .. slot_base + cam_n - 1.  One ray per thread: a persistent variant
 * whose lanes take the next ray of a per-workgroup pool when theirs finishes
 * (ray replacement) was measured 2x slower on the BMW stand-in (the refill path
 * with camera-ray generation inside the traversal loop spills at the 80-VGPR
 * budget, and replacement rays break the camera rays' fetch coherence). */
template<bool STATS, int W, bool INST, int HAIR = 0>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_WAVES(HAIR)) k_intersect_closest(CyGlobals kg,
                                                                 CyPathBuffers b,
                                                                 CyTile tile,
                                                                 int cam_n,
                                                                 int slot_base,
                                                                 const int *queue,
                                                                 const uint *counter,
                                                                 uint *err,
                                                                 CyStats *stats)
{
  const int n_active = cam_n > 0 ? cam_n : (int)*counter;
  const int i = cy_queue_index(n_active);
  __shared__ LdsStack<W, INST, true> lds_stack;
  lds_fill_top(&kg, &lds_stack);
  uint n_nodes = 0, n_leaves = 0, n_tris = 0, n_ties = 0;
  const bool active = i < n_active;
  if (active) {
    const int slot = cam_n > 0 ? slot_base + i : queue[i];
    const uint cam_item = cam_n > 0 ? tile.item_base + (uint)i : CY_NO_ITEM;
    CyRay ray;
    uint visibility;
    const bool has_ray = closest_load(&kg, &b, &tile, slot, cam_item, &ray, &visibility);
    CyIsect isect;
    bool hit = false, tie = false;
    if (has_ray && scene_intersect_valid(&ray)) {
      hit = scene_traverse<W, false, INST, HAIR>(&kg, &ray, visibility, &isect, err,
                                                 STATS ? &n_nodes : nullptr, &n_leaves, &n_tris, &lds_stack, &tie);
    }
    if constexpr (W > 2 && HAIR != 0) {
      if (tie) {
        /* hair scenes: the near-tie (or twice-crossed ribbon) ray is re-traced
         * here with the BVH2 in the reference's order (the shading kernels
         * carry no curve intersection) */
        hit = bvh2_intersect<false, INST, 2, 0, CY_BLOCK, HAIR>(&kg, &ray, visibility, &isect, err, nullptr, nullptr,
                                                                 nullptr);
        tie = false;
        if (STATS) {
          n_ties++;
        }
      }
    }
    if constexpr (W > 2 && HAIR == 0) {
      if (tie) {
        /* near-tie (cy_bvhw.h bvhw_traverse): flagged in the stored primitive;
         * the shading stage re-traces the ray with the bound BVH2 in the
         * reference's visiting order (cy_integrator.h shade_path), so the hit
         * is the reference's bit for bit (about 1 ray in 3000 on the bench
         * scene).  There the re-trace does not weigh on this loop's registers. */
        isect.prim |= CY_PRIM_TIE;
        if (STATS) {
          n_ties++;
        }
      }
    }
    closest_store<INST>(&b, slot, has_ray, hit, &isect);
  }
  if (STATS) {
    stats_block_add(stats, n_nodes, n_leaves, n_tris, n_ties);
  }
}

/* Stage 1 with the iteration budget (hipcy_set_traversal_budget; non-instanced
 * wide BVH): as k_intersect_closest, a traversal past `budget` iterations is
 * saved as a continuation record (cont_suspend).  A kernel of its own: the
 * suspend path's registers and barrier must not weigh on k_intersect_closest
 * (folded into one kernel, the unbudgeted frame lost 15 %, 52 vs 45 ms of
 * closest per frame). */
template<bool STATS, int W, bool INST = false>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_MIN_WAVES) k_intersect_closest_budget(CyGlobals kg,
                                                                 CyPathBuffers b,
                                                                 CyTile tile,
                                                                 int cam_n,
                                                                 int slot_base,
                                                                 const int *queue,
                                                                 const uint *counter,
                                                                 uint *err,
                                                                 CyStats *stats,
                                                                 int budget,
                                                                 CyCont cont)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ LdsStack<W, INST> lds_stack;
  uint n_nodes = 0, n_leaves = 0, n_tris = 0, n_ties = 0;
  const bool active = cam_n > 0 ? i < cam_n : i < (int)*counter;
  constexpr bool CAN_SUSPEND = W > 2 && !INST;
  CyTravCursor cur;
  cur.suspended = false;
  CyRay ray;
  uint visibility = 0;
  CyIsect isect;
  isect.prim = PRIM_NONE;
  bool hit = false, tie = false, has_ray = false;
  int slot = 0;
  if (active) {
    slot = cam_n > 0 ? slot_base + i : queue[i];
    const uint cam_item = cam_n > 0 ? tile.item_base + (uint)i : CY_NO_ITEM;
    has_ray = closest_load(&kg, &b, &tile, slot, cam_item, &ray, &visibility);
    if (has_ray && scene_intersect_valid(&ray)) {
      if (CAN_SUSPEND && budget > 0) {
        isect.t = ray.t;
        isect.u = 0.0f;
        isect.v = 0.0f;
        isect.prim = PRIM_NONE;
        isect.object = OBJECT_NONE;
        isect.type = 0;
        cur.code = 0;
        cur.code_t = 0.0f;
        cur.top = 0;
        cur.n_ring = 0;
        cur.tie = false;
        bvhw_run<W, false>(&kg, &ray, visibility, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves, &n_tris,
                           lds_ring_of(&lds_stack), &tie, budget, &cur);
        hit = isect.prim != PRIM_NONE;
      }
      else {
        hit = scene_traverse<W, false, INST>(&kg, &ray, visibility, &isect, err,
                                                   STATS ? &n_nodes : nullptr, &n_leaves, &n_tris, &lds_stack, &tie);
      }
    }
  }
  if constexpr (CAN_SUSPEND) {
    if (budget > 0) {
      __shared__ uint claim[CY_CLAIM_LDS];
      cont_suspend<W, false>(&kg, cont, slot, ray, visibility, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves,
                             &n_tris, lds_ring_of(&lds_stack), &tie, &cur, claim);
      hit = active && has_ray && isect.prim != PRIM_NONE;
    }
  }
  if (active && !cur.suspended) {
    if constexpr (W > 2) {
      if (tie) {
        /* near-tie (cy_bvhw.h bvhw_traverse): flagged in the stored primitive;
         * the shading stage re-traces the ray with the bound BVH2 in the
         * reference's visiting order (cy_integrator.h shade_path), so the hit
         * is the reference's bit for bit (about 1 ray in 3000 on the bench
         * scene).  There the re-trace does not weigh on this loop's registers. */
        isect.prim |= CY_PRIM_TIE;
        if (STATS) {
          n_ties++;
        }
      }
    }
    closest_store<INST>(&b, slot, has_ray, hit, &isect);
  }
  if (STATS) {
    stats_block_add(stats, n_nodes, n_leaves, n_tris, n_ties);
  }
}

/* Stage 1 continuation: suspended closest-hit traversals from `in`, resumed
 * with the budget (suspending again into `out`) or, budget 0, to the end.
 * Grid-stride over the records with a fixed grid. */
template<bool STATS, int W>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_MIN_WAVES) k_closest_continue(CyGlobals kg, CyPathBuffers b,
                                                                                 CyCont in, CyCont out, int budget,
                                                                                 uint *err, CyStats *stats)
{
  __shared__ LdsStack<W, false> lds_stack;
  __shared__ uint claim[CY_CLAIM_LDS];
  CY_LDS CyStackEntry *ring = lds_ring_of(&lds_stack);
  uint n_nodes = 0, n_leaves = 0, n_tris = 0, n_ties = 0;
  const uint n = min(*in.count, in.capacity);
  for (uint base = blockIdx.x * CY_BLOCK; base < n; base += gridDim.x * CY_BLOCK) {
    const uint i = base + threadIdx.x;
    const bool active = i < n;
    CyTravCursor cur;
    cur.suspended = false;
    CyRay ray;
    uint visibility = 0;
    CyIsect isect;
    bool tie = false;
    int slot = 0;
    if (active) {
      slot = cont_load<W>(in, i, &ray, &visibility, &isect, &cur, ring);
      bvhw_run<W, false>(&kg, &ray, visibility, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves, &n_tris, ring,
                         &tie, budget, &cur);
    }
    if (budget > 0) {
      cont_suspend<W, false>(&kg, out, slot, ray, visibility, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves,
                             &n_tris, ring, &tie, &cur, claim);
    }
    if (active && !cur.suspended) {
      if (tie) {
        isect.prim |= CY_PRIM_TIE;
        if (STATS) {
          n_ties++;
        }
      }
      closest_store<false>(&b, slot, true, isect.prim != PRIM_NONE, &isect);
    }
  }
  if (STATS) {
    stats_block_add(stats, n_nodes, n_leaves, n_tris, n_ties);
  }
}

/* Lane refill (hipcy_set_traversal_refill; non-instanced wide BVH without
 * curves).  A wave's rays end after very different numbers of iterations (18
 * loop iterations per wave against 7.3 nodes per ray on the BMW stand-in: lane
 * utilisation 0.45), and a one-ray-per-thread kernel keeps a lane idle from
 * its ray's end to the wave's.  Here waves are persistent: every lane traverses
 * for at most `rounds` iterations (the resumable cursor of the continuation
 * kernels, its LDS ring column kept in place), then lanes whose ray ended store
 * it and -- once at least `min_idle` lanes of the wave are idle -- take the next
 * rays of the queue.  The queue is split into 8 contiguous parts, one per XCD
 * (blockIdx & 7, the dispatch's round-robin; each XCD's L2 then sees one image
 * region, as with cy_xcd_block), handed out in chunks of CY_REFILL_CHUNK by one
 * atomic per wave; a wave whose part is drained moves on to the next part.
 * Each ray's traversal is the same computation split into rounds, so results
 * are bit-identical.  Camera launches first write their rays into the slots
 * (k_camera_rays): generating them inside the loop costs the loop registers. */
#ifndef CY_REFILL_CHUNK
#  define CY_REFILL_CHUNK 256u
#endif
#define CY_REFILL_BLOCKS 1280 /* 256 CUs x 5 waves/SIMD x 4 SIMDs / 4 waves per block */

__global__ void __launch_bounds__(CY_BLOCK) k_camera_rays(CyGlobals kg, CyPathBuffers b, CyTile tile, int cam_n,
                                                          int slot_base)
{
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= cam_n) {
    return;
  }
  CyRay ray;
  uint visibility;
  closest_load(&kg, &b, &tile, slot_base + i, tile.item_base + (uint)i, &ray, &visibility);
  cy_st(&b.ray_P[slot_base + i], mkf4(ray.P.x, ray.P.y, ray.P.z, ray.t));
  cy_st(&b.ray_D[slot_base + i], mkf4(ray.D.x, ray.D.y, ray.D.z, as_float(visibility)));
}

/* The [lo, hi) range of part p of n queue entries. */
__device__ __forceinline__ void refill_part(uint n, uint p, uint *lo, uint *hi)
{
  *lo = (uint)(((unsigned long long)n * p) >> 3);
  *hi = (uint)(((unsigned long long)n * (p + 1)) >> 3);
}

/* Hand out the next queue indices of the wave to its idle lanes (wave-uniform
 * control flow); returns this lane's index or 0xFFFFFFFF. */
__device__ __forceinline__ uint refill_take(uint n, uint *claim, bool idle, uint *part, uint *parts_left,
                                            uint *next, uint *end)
{
  const int lane = threadIdx.x & 63;
  const unsigned long long mask = __ballot(idle);
  const uint rank = (uint)__popcll(mask & ((1ull << lane) - 1ull));
  uint want = (uint)__popcll(mask);
  uint given = 0;
  uint mine = 0xFFFFFFFFu;
  while (want > 0 && *parts_left > 0) {
    if (*next == *end) {
      uint base = 0;
      if (lane == 0) {
        base = atomicAdd(&claim[*part], CY_REFILL_CHUNK);
      }
      base = __shfl(base, 0);
      uint lo, hi;
      refill_part(n, *part, &lo, &hi);
      if (base >= hi - lo) {
        *part = (*part + 1) & 7u;
        (*parts_left)--;
        continue;
      }
      *next = lo + base;
      *end = min(*next + CY_REFILL_CHUNK, hi);
    }
    const uint take = min(*end - *next, want);
    if (idle && rank >= given && rank < given + take) {
      mine = *next + (rank - given);
    }
    given += take;
    want -= take;
    *next += take;
  }
  return mine;
}

template<bool STATS, int W>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_MIN_WAVES) k_closest_refill(CyGlobals kg,
                                                                 CyPathBuffers b,
                                                                 int cam_n,
                                                                 int slot_base,
                                                                 const int *queue,
                                                                 const uint *counter,
                                                                 uint *claim,
                                                                 uint *err,
                                                                 CyStats *stats,
                                                                 int rounds,
                                                                 int min_idle)
{
  const uint n = cam_n > 0 ? (uint)cam_n : *counter;
  __shared__ LdsStack<W, false> lds_stack;
  CY_LDS CyStackEntry *ring = lds_ring_of(&lds_stack);
  uint n_nodes = 0, n_leaves = 0, n_tris = 0, n_ties = 0;
  uint part = blockIdx.x & 7u, parts_left = 8, next = 0, end = 0;
  bool busy = false, tie = false, has_ray = false;
  int slot = 0;
  CyRay ray;
  uint visibility = 0;
  CyIsect isect;
  CyTravCursor cur;
  while (true) {
    const int n_idle = (int)__popcll(__ballot(!busy));
    if (n_idle >= min_idle || n_idle == 64) {
      const uint idx = refill_take(n, claim, !busy, &part, &parts_left, &next, &end);
      if (idx != 0xFFFFFFFFu) {
        slot = cam_n > 0 ? slot_base + (int)idx : queue[idx];
        closest_load(&kg, &b, nullptr, slot, CY_NO_ITEM, &ray, &visibility);
        has_ray = cam_n > 0 ? ray.t != 0.0f : true;
        isect.t = ray.t;
        isect.u = 0.0f;
        isect.v = 0.0f;
        isect.prim = PRIM_NONE;
        isect.object = OBJECT_NONE;
        isect.type = 0;
        cur.code = 0;
        cur.code_t = 0.0f;
        cur.top = 0;
        cur.n_ring = 0;
        cur.tie = false;
        cur.suspended = false;
        tie = false;
        busy = true;
        if (!(has_ray && scene_intersect_valid(&ray))) {
          closest_store<false>(&b, slot, has_ray, false, &isect);
          busy = false;
        }
      }
    }
    if (!__any(busy)) {
      break;
    }
    if (busy) {
      bvhw_run<W, false>(&kg, &ray, visibility, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves, &n_tris, ring,
                         &tie, rounds, &cur);
      if (!cur.suspended) {
        const bool hit = isect.prim != PRIM_NONE;
        if (tie) {
          isect.prim |= CY_PRIM_TIE;
          if (STATS) {
            n_ties++;
          }
        }
        closest_store<false>(&b, slot, true, hit, &isect);
        busy = false;
      }
    }
  }
  if (STATS) {
    stats_block_add(stats, n_nodes, n_leaves, n_tris, n_ties);
  }
}

/* Stage 3 with lane refill: the opaque any-hit traversals of the shadow queue
 * in persistent waves (as k_closest_refill); the occlusion goes to the shadow
 * record's unused w (shadow_D.w, opaque shadows only) and k_shadow_finish then
 * adds the light, finishes paths and refills slots (its slot claims and queue
 * pushes synchronise whole workgroups, which a persistent loop cannot). */
template<bool STATS, int W>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_MIN_WAVES) k_shadow_refill(CyGlobals kg,
                                                                CyPathBuffers b,
                                                                const int *shadow_queue,
                                                                const uint *shadow_count,
                                                                uint *claim,
                                                                uint *err,
                                                                CyStats *stats,
                                                                int rounds,
                                                                int min_idle)
{
  const uint n = *shadow_count;
  __shared__ LdsStack<W, false> lds_stack;
  CY_LDS CyStackEntry *ring = lds_ring_of(&lds_stack);
  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  uint part = blockIdx.x & 7u, parts_left = 8, next = 0, end = 0;
  bool busy = false;
  int slot = 0;
  CyRay ray;
  CyIsect isect;
  CyTravCursor cur;
  while (true) {
    const int n_idle = (int)__popcll(__ballot(!busy));
    if (n_idle >= min_idle || n_idle == 64) {
      const uint idx = refill_take(n, claim, !busy, &part, &parts_left, &next, &end);
      if (idx != 0xFFFFFFFFu) {
        slot = shadow_queue[idx];
        shadow_load(&b, slot, &ray);
        isect.t = ray.t;
        isect.u = 0.0f;
        isect.v = 0.0f;
        isect.prim = PRIM_NONE;
        isect.object = OBJECT_NONE;
        isect.type = 0;
        cur.code = 0;
        cur.code_t = 0.0f;
        cur.top = 0;
        cur.n_ring = 0;
        cur.tie = false;
        cur.suspended = false;
        busy = true;
        if (!scene_intersect_valid(&ray)) {
          ((float *)&b.shadow_D[slot])[3] = 0.0f;
          busy = false;
        }
      }
    }
    if (!__any(busy)) {
      break;
    }
    if (busy) {
      bvhw_run<W, true>(&kg, &ray, PATH_RAY_SHADOW_OPAQUE, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves,
                        &n_tris, ring, nullptr, rounds, &cur);
      if (!cur.suspended) {
        ((float *)&b.shadow_D[slot])[3] = isect.prim != PRIM_NONE ? 1.0f : 0.0f;
        busy = false;
      }
    }
  }
  if (STATS) {
    stats_block_add(stats + CY_STATS_SHARDS, n_nodes, n_leaves, n_tris, 0);
  }
}

__global__ void __launch_bounds__(CY_BLOCK) k_shadow_finish(CyGlobals kg, CyPathBuffers b, CyTile tile,
                                                            const int *shadow_queue, const uint *shadow_count,
                                                            int *queue_out, uint *count_out)
{
  const int n_active = (int)*shadow_count;
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  bool finished = false;
  int slot = 0;
  if (i < n_active) {
    slot = shadow_queue[i];
    finished = shadow_finish(&b, &tile, slot, cy_ld(&b.shadow_D[slot]).w != 0.0f);
  }
  __shared__ uint claim[CY_CLAIM_LDS];
  const bool regen = slot_refill(kg, b, tile, slot, finished, claim);
  queue_push(queue_out, count_out, slot, regen, claim);
}

/* Stage 3: occlusion of the light sample, deferred light add, finish + refill. */
template<bool STATS, int W, bool INST, int HAIR = 0>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_WAVES(HAIR)) k_intersect_shadow(CyGlobals kg,
                                                                CyPathBuffers b,
                                                                CyTile tile,
                                                                const int *shadow_queue,
                                                                const uint *shadow_count,
                                                                int *queue_out,
                                                                uint *count_out,
                                                                uint *err,
                                                                CyStats *stats)
{
  const int n_active = (int)*shadow_count;
  const int i = cy_queue_index(n_active);
  __shared__ LdsStack<W, INST, true, CY_LDS_TOP_SHADOW> lds_stack;
  lds_fill_top(&kg, &lds_stack);
  bool finished = false;
  int slot = 0;
  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  if (i < n_active) {
    slot = shadow_queue[i];
    CyRay ray;
    shadow_load(&b, slot, &ray);
    bool blocked = false;
    if (scene_intersect_valid(&ray)) {
      CyIsect isect;
      blocked = scene_traverse<W, true, INST, HAIR>(&kg, &ray, PATH_RAY_SHADOW_OPAQUE, &isect, err,
                                                    STATS ? &n_nodes : nullptr, &n_leaves, &n_tris, &lds_stack);
    }
    finished = shadow_finish(&b, &tile, slot, blocked);
  }
  __shared__ uint claim[CY_CLAIM_LDS];
  const bool regen = slot_refill(kg, b, tile, slot, finished, claim);
  queue_push(queue_out, count_out, slot, regen, claim);
  if (STATS) {
    stats_block_add(stats + CY_STATS_SHARDS, n_nodes, n_leaves, n_tris, 0);
  }
}


/* Stage 3 with the iteration budget (see k_intersect_closest_budget). */
template<bool STATS, int W, bool INST = false>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_MIN_WAVES) k_intersect_shadow_budget(CyGlobals kg,
                                                                CyPathBuffers b,
                                                                CyTile tile,
                                                                const int *shadow_queue,
                                                                const uint *shadow_count,
                                                                int *queue_out,
                                                                uint *count_out,
                                                                uint *err,
                                                                CyStats *stats,
                                                                int budget,
                                                                CyCont cont)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ LdsStack<W, INST> lds_stack;
  __shared__ uint claim[CY_CLAIM_LDS];
  constexpr bool CAN_SUSPEND = W > 2 && !INST;
  bool finished = false;
  int slot = 0;
  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  const bool active = i < (int)*shadow_count;
  CyTravCursor cur;
  cur.suspended = false;
  CyRay ray;
  CyIsect isect;
  isect.prim = PRIM_NONE;
  bool blocked = false;
  if (active) {
    slot = shadow_queue[i];
    shadow_load(&b, slot, &ray);
    if (scene_intersect_valid(&ray)) {
      if (CAN_SUSPEND && budget > 0) {
        isect.t = ray.t;
        isect.u = 0.0f;
        isect.v = 0.0f;
        isect.prim = PRIM_NONE;
        isect.object = OBJECT_NONE;
        isect.type = 0;
        cur.code = 0;
        cur.code_t = 0.0f;
        cur.top = 0;
        cur.n_ring = 0;
        cur.tie = false;
        bvhw_run<W, true>(&kg, &ray, PATH_RAY_SHADOW_OPAQUE, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves,
                          &n_tris, lds_ring_of(&lds_stack), nullptr, budget, &cur);
        blocked = isect.prim != PRIM_NONE;
      }
      else {
        blocked = scene_traverse<W, true, INST>(&kg, &ray, PATH_RAY_SHADOW_OPAQUE, &isect, err,
                                                      STATS ? &n_nodes : nullptr, &n_leaves, &n_tris, &lds_stack);
      }
    }
  }
  if constexpr (CAN_SUSPEND) {
    if (budget > 0) {
      cont_suspend<W, true>(&kg, cont, slot, ray, PATH_RAY_SHADOW_OPAQUE, &isect, err, STATS ? &n_nodes : nullptr,
                            &n_leaves, &n_tris, lds_ring_of(&lds_stack), nullptr, &cur,
                            claim);
      blocked = active && isect.prim != PRIM_NONE;
    }
  }
  if (active && !cur.suspended) {
    finished = shadow_finish(&b, &tile, slot, blocked);
  }
  const bool regen = slot_refill(kg, b, tile, slot, finished, claim);
  queue_push(queue_out, count_out, slot, regen, claim);
  if (STATS) {
    stats_block_add(stats + CY_STATS_SHARDS, n_nodes, n_leaves, n_tris, 0);
  }
}

/* Stage 3 continuation: suspended shadow traversals, then the same finish,
 * refill and queue push as k_intersect_shadow. */
template<bool STATS, int W>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_MIN_WAVES) k_shadow_continue(CyGlobals kg, CyPathBuffers b,
                                                                                CyTile tile, CyCont in, CyCont out,
                                                                                int budget, int *queue_out,
                                                                                uint *count_out, uint *err,
                                                                                CyStats *stats)
{
  __shared__ LdsStack<W, false> lds_stack;
  __shared__ uint claim[CY_CLAIM_LDS];
  CY_LDS CyStackEntry *ring = lds_ring_of(&lds_stack);
  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  const uint n = min(*in.count, in.capacity);
  for (uint base = blockIdx.x * CY_BLOCK; base < n; base += gridDim.x * CY_BLOCK) {
    const uint i = base + threadIdx.x;
    const bool active = i < n;
    CyTravCursor cur;
    cur.suspended = false;
    CyRay ray;
    uint visibility = 0;
    CyIsect isect;
    int slot = 0;
    bool finished = false;
    if (active) {
      slot = cont_load<W>(in, i, &ray, &visibility, &isect, &cur, ring);
      bvhw_run<W, true>(&kg, &ray, visibility, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves, &n_tris, ring,
                        nullptr, budget, &cur);
    }
    if (budget > 0) {
      cont_suspend<W, true>(&kg, out, slot, ray, visibility, &isect, err, STATS ? &n_nodes : nullptr, &n_leaves,
                            &n_tris, ring, nullptr, &cur, claim);
    }
    if (active && !cur.suspended) {
      finished = shadow_finish(&b, &tile, slot, isect.prim != PRIM_NONE);
    }
    const bool regen = slot_refill(kg, b, tile, slot, finished, claim);
    queue_push(queue_out, count_out, slot, regen, claim);
  }
  if (STATS) {
    stats_block_add(stats + CY_STATS_SHARDS, n_nodes, n_leaves, n_tris, 0);
  }
}

/* Transparent shadows, traversal half (non-instanced scenes): the record-all
 * query of each pending shadow ray (bvh_shadow_all.h; the wide layout's
 * bvhw_shadow_all or the BVH2's) at the traversal kernels' occupancy, leaving
 * the shading kernel below only the occluders' shaders to evaluate.  The
 * outcome goes to the slot's record (CyPathBuffers.shadow_nrec / _hits):
 * blocked, or up to CY_SHADOW_REC_HITS hits sorted by distance; more hits, two
 * at one distance, or a ray the shading kernel ends before its traversal
 * (t = 0, transparent bounces spent) leave CY_SREC_NONE and the shading kernel
 * traverses itself, as before. */
template<int HAIR>
__global__ void __launch_bounds__(CY_BLOCK, CY_TRAV_WAVES(HAIR)) k_shadow_record(CyGlobals kg, CyPathBuffers b,
                                                                                const int *shadow_queue,
                                                                                const uint *shadow_count, uint *err)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int)*shadow_count) {
    return;
  }
  const int slot = shadow_queue[i];
  const uint rec = shadow_record<HAIR>(&kg, &b, slot, err);
  cy_st(&b.shadow_nrec[slot], rec);
}

/* Stage 3 with transparent shadows (KernelIntegrator.transparent_shadows): the
 * record-all occlusion of the light sample with the occluders' shaders
 * evaluated (cy_integrator.h shadow_finish_transparent), then the same finish
 * and refill.  Only scenes with transparent-shadow shaders use it. */
template<bool VOL>
__global__ void __launch_bounds__(CY_BLOCK) k_intersect_shadow_transparent(CyGlobals kg,
                                                                          CyPathBuffers b,
                                                                          CyTile tile,
                                                                          const int *shadow_queue,
                                                                          const uint *shadow_count,
                                                                          int *queue_out,
                                                                          uint *count_out,
                                                                          uint *err)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  bool finished = false;
  int slot = 0;
  if (i < (int)*shadow_count) {
    slot = shadow_queue[i];
    /* shading for transparency keeps no closures (PATH_RAY_SHADOW: none
     * allocated), only the SVM stack */
    float svm[CY_SVM_STACK];
    CyShadeMem mem;
    mem.closure = nullptr;
    mem.svm_stack = svm;
    mem.svm_stride = 1;
    mem.svm_fast = CY_SVM_STACK;
    mem.svm_spill = nullptr;
    finished = shadow_finish_transparent<VOL>(&kg, &b, &tile, slot, mem, err);
  }
  __shared__ uint claim[CY_CLAIM_LDS];
  const bool regen = slot_refill(kg, b, tile, slot, finished, claim);
  queue_push(queue_out, count_out, slot, regen, claim);
}

/* ---------------------------------------------------------------------------
 * Adaptive sampling (kernel_adaptive_sampling.h; launched per RenderTile as
 * CUDADevice::adaptive_sampling_filter / _post, device_cuda_impl.cpp:1779-1851). */
struct CyAdaptiveTile {
  int x, y, w, h, offset, stride;
  float *buffer;
  int pass_stride, aux, sample_count;
};

__device__ __forceinline__ float *adaptive_pixel(const CyAdaptiveTile &t, int x, int y)
{
  return t.buffer + (size_t)(t.offset + x + y * t.stride) * t.pass_stride;
}

/* kernel_do_adaptive_stopping: per-pixel error of the full against the
 * half-sample (aux) estimate; converged pixels get aux.w += 1. */
__global__ void __launch_bounds__(CY_BLOCK) k_adaptive_stopping(CyAdaptiveTile t, int sample, float threshold)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.w * t.h) {
    return;
  }
  float *buffer = adaptive_pixel(t, t.x + i % t.w, t.y + i / t.w);
  const float ix = buffer[0], iy = buffer[1], iz = buffer[2];
  const float *a = buffer + t.aux;
  const float error = (fabsf(ix - a[0]) + fabsf(iy - a[1]) + fabsf(iz - a[2])) /
                      ((float)sample * 0.0001f + sqrtf(ix + iy + iz));
  if (error < threshold * (float)sample) {
    buffer[t.aux + 3] += 1.0f;
  }
}

/* kernel_do_adaptive_filter_x / _y: a pixel next to an unconverged one along
 * the row (column) is marked unconverged too; one thread per row (column),
 * walking it in order as the reference does. */
template<bool ALONG_X> __global__ void __launch_bounds__(CY_BLOCK) k_adaptive_filter(CyAdaptiveTile t)
{
  const int line = blockIdx.x * blockDim.x + threadIdx.x;
  const int n_lines = ALONG_X ? t.h : t.w;
  if (line >= n_lines) {
    return;
  }
  const int n = ALONG_X ? t.w : t.h;
  bool prev = false;
  for (int k = 0; k < n; k++) {
    const int x = ALONG_X ? t.x + k : t.x + line;
    const int y = ALONG_X ? t.y + line : t.y + k;
    float *aux = adaptive_pixel(t, x, y) + t.aux;
    if (aux[3] == 0.0f) {
      if (k > 0 && !prev) {
        float *prev_aux = adaptive_pixel(t, ALONG_X ? x - 1 : x, ALONG_X ? y : y - 1) + t.aux;
        prev_aux[3] = 0.0f;
      }
      prev = true;
    }
    else {
      if (prev) {
        aux[3] = 0.0f;
      }
      prev = false;
    }
  }
}

/* kernel_cuda_adaptive_scale_samples + kernel_adaptive_post_adjust: pixels
 * that stopped early are scaled as if they had taken every sample (combined
 * and aux passes; the device supports no other scaled pass). */
__global__ void __launch_bounds__(CY_BLOCK) k_adaptive_scale(CyAdaptiveTile t, int start_sample, int sample)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.w * t.h) {
    return;
  }
  float *buffer = adaptive_pixel(t, t.x + i % t.w, t.y + i / t.w);
  float mul;
  float *sc = buffer + t.sample_count;
  if (*sc < 0.0f) {
    *sc = -*sc;
    const float lo = (float)start_sample + 1.0f;
    mul = (float)sample / (lo > *sc ? lo : *sc);
    if (mul == 1.0f) {
      return;
    }
  }
  else {
    mul = (float)sample / ((float)sample - 1.0f);
  }
  for (int c = 0; c < 4; c++) {
    buffer[c] *= mul;
    buffer[t.aux + c] *= mul;
  }
}

/* ---------------------------------------------------------------------------
 * Closest-queue sorting (hipcy_set_ray_sort).  A counting sort of the queue by
 * a direction bin, in three launches on the lane's stream: per-block bin
 * histograms (LDS atomics, no device-scope atomics), one exclusive scan of the
 * bin-major histogram, and the scatter.  Within a bin the slots keep their
 * block order up to the order of LDS atomics inside a block, so the rays of
 * neighbouring pixels stay together and share their octant. */
#define CY_SORT_BINS 32

template<int MODE> __device__ __forceinline__ uint ray_sort_key(const hc_float4 d)
{
  const uint oct = (__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 31) << 1) |
                   ((__float_as_uint(d.z) >> 31) << 2);
  if (MODE == 3) {
    return oct;
  }
  const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  const uint major = (ax >= ay && ax >= az) ? 0u : (ay >= az ? 1u : 2u);
  return oct * 4u + major;
}

template<int MODE, bool SHADOW = false>
__global__ void __launch_bounds__(CY_BLOCK) k_sort_count(CyPathBuffers b, const int *queue, const uint *count,
                                                         unsigned char *keys, uint *hist, int nblocks)
{
  constexpr int K = MODE == 3 ? 8 : CY_SORT_BINS;
  __shared__ uint h[K];
  if (threadIdx.x < K) {
    h[threadIdx.x] = 0;
  }
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int)*count) {
    const uint key = ray_sort_key<MODE>(SHADOW ? b.shadow_D[queue[i]] : b.ray_D[queue[i]]);
    keys[i] = (unsigned char)key;
    atomicAdd(&h[key], 1u);
  }
  __syncthreads();
  if (threadIdx.x < K) {
    hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
  }
}

/* Shading-queue sort (hipcy_set_ray_sort mode 8): the same counting sort between
 * the closest-hit and shading launches, keyed by the shader of each path's hit
 * (bin 0: misses and paths without a ray; bin 31: curve hits; otherwise 1 +
 * shader mod 30), so a shading wave runs one SVM program and one closure set
 * instead of interleaving every material of the scene (instruction cache,
 * divergence).  Results are unchanged: every path is shaded by its own slot. */
__global__ void __launch_bounds__(CY_BLOCK) k_shade_sort_count(CyGlobals kg, CyPathBuffers b, const int *queue,
                                                               const uint *count, unsigned char *keys, uint *hist,
                                                               int nblocks)
{
  __shared__ uint h[CY_SORT_BINS];
  if (threadIdx.x < CY_SORT_BINS) {
    h[threadIdx.x] = 0;
  }
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int)*count) {
    const int slot = queue[i];
    const int pw = __float_as_int(b.isect[slot].w);
    uint key = 0;
    if (pw >= 0) {
      const int prim = pw & ~CY_PRIM_TIE;
      if (kg.have_curves && b.isect_type[slot] != PRIMITIVE_TRIANGLE) {
        key = CY_SORT_BINS - 1;
      }
      else {
        key = 1u + ((uint)kg.__tri_shader[kg.__prim_index[prim]] & SHADER_MASK) % (CY_SORT_BINS - 2);
      }
    }
    keys[i] = (unsigned char)key;
    atomicAdd(&h[key], 1u);
  }
  __syncthreads();
  if (threadIdx.x < CY_SORT_BINS) {
    hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
  }
}

/* Exclusive scan of m histogram entries in place, one workgroup (m is at most
 * bins x blocks of a lane, a few hundred thousand words). */
__global__ void __launch_bounds__(1024) k_sort_scan(uint *hist, int m)
{
  __shared__ uint part[1024];
  const int t = threadIdx.x;
  const int per = (m + 1023) / 1024;
  const int b0 = min(m, t * per), b1 = min(m, b0 + per);
  uint s = 0;
  for (int j = b0; j < b1; j++) {
    s += hist[j];
  }
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint run = t ? part[t - 1] : 0u;
  for (int j = b0; j < b1; j++) {
    const uint c = hist[j];
    hist[j] = run;
    run += c;
  }
}

template<int MODE>
__global__ void __launch_bounds__(CY_BLOCK) k_sort_scatter(const int *queue, const uint *count,
                                                           const unsigned char *keys, const uint *offs,
                                                           int nblocks, int *out)
{
  constexpr int K = MODE == 3 ? 8 : CY_SORT_BINS;
  __shared__ uint base[K];
  __shared__ uint h[K];
  if (threadIdx.x < K) {
    base[threadIdx.x] = offs[threadIdx.x * nblocks + blockIdx.x];
    h[threadIdx.x] = 0;
  }
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int)*count) {
    const uint key = keys[i];
    const uint r = atomicAdd(&h[key], 1u);
    out[base[key] + r] = queue[i];
  }
}

template<int W, int HAIR = 0>
__global__ void __launch_bounds__(CY_BLOCK) k_test_intersect(CyGlobals kg, const float *rays, float *out_f, int *out_i, int n, int any_hit, uint *err)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ LdsStack<W, true> lds_stack;
  if (i >= n) {
    return;
  }
  const float *r = rays + 8 * i;
  CyRay ray;
  ray.P = mk3(r[0], r[1], r[2]);
  ray.D = mk3(r[3], r[4], r[5]);
  ray.t = r[6];
  const uint visibility = as_uint(r[7]);
  CyIsect isect;
  isect.t = ray.t;
  isect.u = 0.0f;
  isect.v = 0.0f;
  isect.prim = PRIM_NONE;
  isect.object = OBJECT_NONE;
  isect.type = 0;
  bool hit = false;
  if (scene_intersect_valid(&ray)) {
    /* scene_intersect: shadow visibility means early exit at the first hit
     * (bvh_traversal.h:144-146) */
    if (any_hit || (visibility & PATH_RAY_SHADOW_OPAQUE)) {
      hit = scene_traverse<W, true, true, HAIR>(&kg, &ray, visibility & PATH_RAY_SHADOW_OPAQUE, &isect, err, nullptr,
                                                nullptr, nullptr, &lds_stack);
    }
    else {
      bool tie = false;
      hit = scene_traverse<W, false, true, HAIR>(&kg, &ray, visibility, &isect, err, nullptr, nullptr, nullptr,
                                                 &lds_stack, &tie);
      if (tie) {
        hit = bvh2_intersect<false, true, 2, CY_LDS_STACK, CY_BLOCK, HAIR>(&kg, &ray, visibility, &isect, err,
                                                                           nullptr, nullptr, nullptr);
      }
    }
  }
  out_f[3 * i + 0] = isect.t;
  out_f[3 * i + 1] = isect.u;
  out_f[3 * i + 2] = isect.v;
  out_i[4 * i + 0] = hit ? 1 : 0;
  out_i[4 * i + 1] = isect.prim;
  out_i[4 * i + 2] = isect.object;
  out_i[4 * i + 3] = isect.type;
}

__global__ void k_test_camera(CyGlobals kg, const int *xys, float *out, int n)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) {
    return;
  }
  uint rng_hash;
  CyRay ray;
  camera_sample_ray(&kg, xys[3 * i + 0], xys[3 * i + 1], xys[3 * i + 2], &rng_hash, &ray);
  float *o = out + 8 * i;
  o[0] = ray.P.x;
  o[1] = ray.P.y;
  o[2] = ray.P.z;
  o[3] = ray.D.x;
  o[4] = ray.D.y;
  o[5] = ray.D.z;
  o[6] = ray.t;
  o[7] = as_float(rng_hash);
}

/* SHADER task, SHADER_EVAL_BACKGROUND (kernels/cuda/kernel.cu:195-212
 * kernel_cuda_background): one thread per input pixel, output[x] += world
 * colour.  The SVM stack is private (no closures are kept for
 * PATH_RAY_EMISSION); this task runs once per scene update. */
__global__ void __launch_bounds__(CY_BLOCK) k_background_eval(CyGlobals kg, const hc_uint4 *input, float *output,
                                                               int sx, int sw, uint *err)
{
  const int x = sx + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (x >= sx + sw) {
    return;
  }
  CyClosure closure[1];
  float svm[CY_SVM_STACK];
  CyShadeMem mem;
  mem.closure = closure;
  mem.svm_stack = svm;
  mem.svm_stride = 1;
  mem.svm_fast = CY_SVM_STACK;
  mem.svm_spill = nullptr;
  const hc_uint4 in = input[x];
  const cfloat3 c = background_evaluate(&kg, in.x, in.y, mem, err);
  float *o = output + 4 * (size_t)x;
  o[0] += c.x;
  o[1] += c.y;
  o[2] += c.z;
}

/* SHADER_EVAL_DISPLACE (kernel_cuda_displace, kernels/cuda/kernel.cu:196-205):
 * one thread per input (object, prim, u, v) of the chunk, output += (D, 0). */
__global__ void __launch_bounds__(CY_BLOCK) k_displace_eval(CyGlobals kg, const hc_uint4 *input, float *output,
                                                              int sx, int sw, uint *err)
{
  const int x = sx + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (x >= sx + sw) {
    return;
  }
  float svm[CY_SVM_STACK];
  CyShadeMem mem;
  mem.closure = nullptr;
  mem.svm_stack = svm;
  mem.svm_stride = 1;
  mem.svm_fast = CY_SVM_STACK;
  mem.svm_spill = nullptr;
  const hc_uint4 in = input[x];
  const cfloat3 d = displace_evaluate(&kg, (int)in.x, (int)in.y, as_float(in.z), as_float(in.w), mem, err);
  float *o = output + 4 * (size_t)x;
  o[0] += d.x;
  o[1] += d.y;
  o[2] += d.z;
  o[3] += 0.0f;
}

/* Film convert (kernel/kernel_film.h, kernels/cuda/kernel.cu:156-178): one
 * thread per pixel of the (w x h) rectangle; the parity target is the CPU
 * device, so half output uses its truncating float4_store_half (util_half.h:80-118)
 * rather than CUDA's round-to-nearest __float2half. */
struct CyFilm {
  int pass_stride, display_pass_stride, display_pass_components, display_divide_pass_stride;
  int use_display_exposure, use_display_pass_alpha;
  float exposure;
};

__device__ __forceinline__ ushort film_half(float v, float scale)
{
  float f = v * scale;
  f = (f > 0.0f) ? ((f < 65504.0f) ? f : 65504.0f) : 0.0f;
  const int x = (int)as_uint(f);
  const int absolute = x & 0x7FFFFFFF;
  const int Z = (int)((uint)absolute + 0xC8000000u);
  const int result = (absolute < 0x38800000) ? 0 : Z;
  return (ushort)((result >> 13) & 0x7FFF);
}

template<bool HALF>
__global__ void __launch_bounds__(CY_BLOCK) k_film_convert(CyFilm film, const float *buffer, void *rgba,
                                                            float sample_scale, int sx, int sy, int sw, int sh,
                                                            int offset, int stride)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= sw * sh) {
    return;
  }
  const int x = sx + i % sw, y = sy + i / sw;
  const int index = offset + x + y * stride;
  const bool use_scale = film.display_divide_pass_stride == -1;
  /* film_get_pass_result (kernel_film.h:19-63) */
  float r[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const float *in = buffer + film.display_pass_stride + (size_t)index * film.pass_stride;
  if (film.display_pass_components == 4) {
    const hc_float4 v = *(const hc_float4 *)in;
    r[0] = v.x;
    r[1] = v.y;
    r[2] = v.z;
    r[3] = use_scale ? (film.use_display_pass_alpha ? v.w : 1.0f / sample_scale) : 1.0f;
    if (film.display_divide_pass_stride != -1) {
      /* safe_divide_even_color (util_math.h:525-560) */
      const float *dv = buffer + film.display_divide_pass_stride + (size_t)index * film.pass_stride;
      float q[3];
      for (int c = 0; c < 3; c++) {
        q[c] = (dv[c] != 0.0f) ? r[c] / dv[c] : 0.0f;
      }
      if (dv[0] == 0.0f) {
        if (dv[1] == 0.0f) {
          q[0] = q[2];
          q[1] = q[2];
        }
        else if (dv[2] == 0.0f) {
          q[0] = q[1];
          q[2] = q[1];
        }
        else {
          q[0] = 0.5f * (q[1] + q[2]);
        }
      }
      else if (dv[1] == 0.0f) {
        if (dv[2] == 0.0f) {
          q[1] = q[0];
          q[2] = q[0];
        }
        else {
          q[1] = 0.5f * (q[0] + q[2]);
        }
      }
      else if (dv[2] == 0.0f) {
        q[2] = 0.5f * (q[0] + q[1]);
      }
      r[0] = q[0];
      r[1] = q[1];
      r[2] = q[2];
    }
    if (film.use_display_exposure) {
      r[0] = r[0] * film.exposure;
      r[1] = r[1] * film.exposure;
      r[2] = r[2] * film.exposure;
    }
  }
  else if (film.display_pass_components == 1) {
    r[0] = r[1] = r[2] = in[0];
    r[3] = 1.0f / sample_scale;
  }
  const float scale = use_scale ? sample_scale : 1.0f;
  if (HALF) {
    ushort4 o;
    o.x = film_half(r[0], scale);
    o.y = film_half(r[1], scale);
    o.z = film_half(r[2], scale);
    o.w = film_half(r[3], scale);
    ((ushort4 *)rgba)[index] = o;
  }
  else {
    /* film_map + film_float_to_byte (kernel_film.h:65-92) */
    uchar4 o;
    o.x = (uchar)(saturate(color_linear_to_srgb(r[0] * scale)) * 255.0f);
    o.y = (uchar)(saturate(color_linear_to_srgb(r[1] * scale)) * 255.0f);
    o.z = (uchar)(saturate(color_linear_to_srgb(r[2] * scale)) * 255.0f);
    o.w = (uchar)(saturate(saturate(r[3] * scale)) * 255.0f);
    ((uchar4 *)rgba)[index] = o;
  }
}

/* Kernel instance for (traversal counters, BVH width, instancing). */
struct ClosestK {
  template<bool S, int W, bool I, int H = 0> static constexpr auto fn()
  {
    return k_intersect_closest<S, W, I, H>;
  }
};
struct ShadowK {
  template<bool S, int W, bool I, int H = 0> static constexpr auto fn()
  {
    return k_intersect_shadow<S, W, I, H>;
  }
};
template<class K, bool S, bool I> static auto pick_width(int W, int hair)
{
  /* scenes with curves: the hair node tests; ribbons only on the wide BVH
   * too, thick curves on the BVH2 (their intersection's starting points
   * depend on the bound, cy_bvhw.h) */
  return hair == 1 ? (W == 8 ? K::template fn<S, 8, I, 1>() : W == 4 ? K::template fn<S, 4, I, 1>() :
                                                                     K::template fn<S, 2, I, 1>()) :
         hair == 2 ? K::template fn<S, 2, I, 2>() :
         hair == 3 ? K::template fn<S, 2, I, 3>() :
         W == 8 ? K::template fn<S, 8, I>() :
         W == 4 ? K::template fn<S, 4, I>() :
                  K::template fn<S, 2, I>();
}
template<class K> static auto pick_kernel(bool stats, int W, bool inst, int hair = 0)
{
  return stats ? (inst ? pick_width<K, true, true>(W, hair) : pick_width<K, true, false>(W, hair))
               : (inst ? pick_width<K, false, true>(W, hair) : pick_width<K, false, false>(W, hair));
}

template<int W> static auto pick_closest_cont(bool stats)
{
  return stats ? k_closest_continue<true, W> : k_closest_continue<false, W>;
}
template<int W> static auto pick_shadow_cont(bool stats)
{
  return stats ? k_shadow_continue<true, W> : k_shadow_continue<false, W>;
}

/* ------------------------------------------------------------------------- */
/* Host side                                                                   */

namespace {

std::mutex g_error_mutex;
std::string g_global_error;

struct GlobalBinding {
  uint64_t ptr = 0;
  size_t bytes = 0;
};

}  // namespace


struct hipcy_device {
  int ordinal = 0;
  hipStream_t stream = nullptr;
  std::string error;
  hc_KernelData data_host;
  bool have_data = false;
  hc_KernelData *data_dev = nullptr;
  std::map<std::string, GlobalBinding> globals;
  std::map<uint64_t, size_t> allocations;

  /* wavefront buffers */
  size_t capacity = 0;
  char *pool = nullptr;
  char *vol_pool = nullptr; /* volume stacks of the slots (volume scenes only) */
  CyPathBuffers bufs;
  int *queue[3] = {nullptr, nullptr, nullptr};
  uint *counters = nullptr; /* [3] error word; lane l: [16 + 16 l ...] (see PassLane) */
  /* the slot pool is split into CY_LANES partitions iterated on their own
   * streams, so one partition's kernel tail overlaps the others' work */
  hipStream_t lane_stream[CY_LANES] = {};
  CyStats *stats_dev = nullptr;
  uint *host_counters = nullptr; /* pinned */

  /* closest-queue sorting (hipcy_set_ray_sort): sorted queue, per-ray bin and
   * the per-lane bin x block histogram / scanned offsets */
  int ray_sort = -1; /* -1: automatic (shading-queue sort for the extended shading kernel) */
  int shadow_sort = 0; /* hipcy_set_shadow_sort: 0, 3 or 5 */
  int *sort_queue = nullptr;
  unsigned char *sort_key = nullptr;
  uint *sort_hist = nullptr;
  size_t sort_capacity = 0;

  int profiling = 0; /* bit 0: HIP-event kernel timing, bit 1: traversal counters */

  /* iteration budget of the wide traversal kernels (hipcy_set_traversal_budget):
   * first launch, first continuation; 0 disables.  Per lane two continuation
   * record buffers of cont_capacity entries. */
  int trav_budget[2] = {0, 0};
  int trav_refill[2] = {0, 0};     /* lane refill: iterations per round, idle lanes that trigger a refill */
  /* fused tail (hipcy_set_tail): a lane whose items are all claimed runs its
   * live paths to their ends in one k_tail launch once at most this many are
   * live; 0 disables */
  size_t tail_paths = (size_t)1 << 17;
  uint *refill_claim = nullptr;    /* CY_LANES x 8 per-part chunk counters */
  hc_float4 *cont_rec = nullptr;
  size_t cont_capacity = 0; /* records per buffer */
  size_t cont_lanes = 0;

  /* path slots in flight and the per-sample record buffer of one pass */
  size_t slots_wanted = (size_t)1 << 27;
  size_t record_budget = (size_t)4 << 30; /* bytes of sample records per pass */
  hc_float4 *records = nullptr;
  size_t records_capacity = 0;
  CyTileDesc *tile_descs = nullptr; /* tiles of the current multi-tile pass */
  size_t tile_descs_capacity = 0;
  /* tile streams (hipcy_render_feed): pixel-samples one device holds (in
   * flight + unclaimed; 0 = the slot pool plus as much in reserve), and the
   * lanes' appended tile chunks */
  size_t stream_hold = 0;
  CyTileDesc *stream_desc_dev = nullptr;
  CyTileDesc *stream_desc_host = nullptr; /* pinned */
  uint *min_live_dev = nullptr;           /* per lane CY_MIN_SHARDS words (k_stream_min_live) */
  uint *min_live_host = nullptr;          /* pinned copy */
  CyGlobals kg_stream;

  /* W-wide BVH widened from the bound BVH2 (rebuilt when either BVH2 array,
   * the root or the width changes) */
  int bvh_width = 4;
  int bvh_merge_prims = 0;
  bool bvhw_dirty = true;
  void *bvhw = nullptr;
  size_t bvhw_bytes = 0;
  size_t bvhw_capacity = 0;
  int bvhw_depth = 0;
  int *bvhw_object_root = nullptr; /* inside bvhw, after the nodes */
  int have_instancing = 1;         /* some object without SD_OBJECT_TRANSFORM_APPLIED */
  std::vector<uint32_t> object_flags; /* host copy of __object_flag, taken at bind time */
  std::vector<hc_uint4> svm_nodes;    /* host copy of __svm_nodes, taken at bind time */
  size_t num_shaders = 0;             /* __shaders entries */
  bool shade_tex = false;             /* some shader uses texture / converter / input nodes */
  bool use_volumes = false;           /* KernelIntegrator.use_volumes: the volume shading / shadow kernels */
  bool use_disk_bssrdf = false;       /* disk BSSRDFs: the slots' subsurface indirect-ray records */
  bool sss_pool_vol = false;          /* ... sized with their volume stacks */
  bool use_catcher = false;           /* shadow-catcher objects: the slots' catcher records */
  bool use_branched = false;          /* branched path tracing: the slots' branch records */
  char *br_pool = nullptr;            /* those records and their counters */
  bool use_lightpass = false;         /* light passes: the slots' PathRadiance components */
  bool use_decoupled = false;         /* decoupled volume ray marching: the slots' segment steps */
  int bvhw_top_shadow = 0;            /* wide nodes the opaque-shadow kernel keeps in LDS */
  bool shade_ext = false;             /* the _ext shading variants (catchers, branched, light passes) */
  bool shade_vext = false;            /* the _vext variants (decoupled, camera in a volume, SSS with volumes) */
  char *dec_pool = nullptr;           /* those steps (CY_DECOUPLED_STEPS x CY_DECOUPLED_STEP_BYTES per slot) */
  size_t dec_slots = 0;               /* slots the steps are allocated for */
  char *lp_pool = nullptr;            /* those records (CY_LP_F4 float4 per slot) */
  char *catcher_pool = nullptr;       /* those records (CY_CATCHER_F4 float4 per slot) */
  char *sss_pool = nullptr;           /* those records and their depths */
  bool use_ray_diff = false;          /* a shader reads ray differentials (Bump / *_BUMP_DX / _DY nodes) */
  char *diff_pool = nullptr;          /* the slots' ray and shadow-ray differentials */
  char *srec_pool = nullptr;          /* the slots' transparent-shadow records (k_shadow_record) */
  int shade_closures = 1;             /* closure array of the shading kernel (variant by size) */
  bool features_dirty = true;         /* KernelData or a bound array changed since load_kernels */
  int curve_shapes = 0;               /* curve primitive shapes in __prim_type: 1 ribbon, 2 thick, 3 both */
  bool curve_wide = false;            /* hipcy_set_curve_layout */
  int tri_index_identity = 0;
  hipcy_stats stats;
  std::vector<hipEvent_t> events;

  /* image textures (hipcy_tex_alloc): per SVM slot the device copy of the
   * pixels and its TextureInfo; the table is mirrored into tex_info_dev and
   * bound as __texture_info (CUDADevice::tex_alloc + load_texture_info) */
  std::vector<hc_TextureInfo> tex_info;
  std::vector<void *> tex_mem;
  hc_TextureInfo *tex_info_dev = nullptr;
  size_t tex_info_capacity = 0;
};

static int set_error(hipcy_device *dev, const std::string &msg)
{
  if (dev) {
    if (dev->error.empty()) {
      dev->error = msg;
      fprintf(stderr, "hipcycles: %s\n", msg.c_str());
    }
  }
  else {
    std::lock_guard<std::mutex> lock(g_error_mutex);
    g_global_error = msg;
  }
  return -1;
}

#define HIP_CHECK(dev, call) \
  do { \
    hipError_t _e = (call); \
    if (_e != hipSuccess) { \
      return set_error((dev), std::string(#call) + ": " + hipGetErrorString(_e)); \
    } \
  } while (0)

static int ensure_bvhw(hipcy_device *dev);

/* The W-wide layout serves the scene: triangles, and ribbon curves when
 * hipcy_set_curve_layout asked for it (thick curves keep the bound BVH2:
 * pick_width).  Instanced scenes with curves keep the BVH2 too: no golden case
 * pins ribbons inside instances on the wide layout. */
static bool wide_layout(const hipcy_device *dev)
{
  return dev->bvh_width > 2 &&
         (!dev->data_host.bvh.have_curves ||
          (dev->curve_wide && dev->curve_shapes == 1 && !dev->have_instancing));
}

static bool build_globals(hipcy_device *dev, CyGlobals *kg)
{
  memset(kg, 0, sizeof(*kg));
  kg->data = dev->data_dev;
#define CY_BIND(type, name) \
  { \
    auto it = dev->globals.find(#name); \
    kg->name = (it != dev->globals.end()) ? (const type *)it->second.ptr : nullptr; \
  }
  CY_GLOBAL_ARRAYS(CY_BIND)
#undef CY_BIND
  const bool wide = wide_layout(dev);
  kg->bvhw_nodes = wide ? dev->bvhw : nullptr;
  kg->bvhw_object_root = wide ? dev->bvhw_object_root : nullptr;
  kg->tri_index_identity = wide ? dev->tri_index_identity : 0;
  kg->have_instancing = dev->have_instancing;
  kg->have_curves = dev->data_host.bvh.have_curves ? 1 : 0;
  kg->use_ray_diff = dev->use_ray_diff ? 1 : 0;
  /* LDS copy of the top levels: non-instanced wide BVH only (instanced scenes
   * traverse their top level as the reference's BVH2) */
  const size_t wide_nodes = dev->bvh_width > 2 ? dev->bvhw_bytes / (32 * (size_t)dev->bvh_width) : 0;
  kg->bvhw_top = (wide && !dev->have_instancing) ? (int)std::min<size_t>(CY_LDS_TOP, wide_nodes) : 0;
  dev->bvhw_top_shadow = (wide && !dev->have_instancing) ? (int)std::min<size_t>(CY_LDS_TOP_SHADOW, wide_nodes) : 0;
  kg->bvhw_width = wide ? dev->bvh_width : 0;
  return true;
}

/* Widen the bound BVH2 into the W-wide layout (host collapse of a D2H copy;
 * the arrays are a few tens of MB even for BMW27-class scenes). */
static int ensure_bvhw(hipcy_device *dev)
{
  if (!wide_layout(dev) || !dev->bvhw_dirty) {
    return 0;
  }
  auto nodes = dev->globals.find("__bvh_nodes");
  auto leaves = dev->globals.find("__bvh_leaf_nodes");
  if (leaves == dev->globals.end()) {
    return set_error(dev, "BVH widening: __bvh_leaf_nodes not bound");
  }
  std::vector<float> n2, l2;
  if (nodes != dev->globals.end() && nodes->second.bytes) {
    n2.resize(nodes->second.bytes / 4);
    HIP_CHECK(dev, hipMemcpy(n2.data(), (const void *)nodes->second.ptr, nodes->second.bytes,
                             hipMemcpyDeviceToHost));
  }
  l2.resize(leaves->second.bytes / 4);
  HIP_CHECK(dev, hipMemcpy(l2.data(), (const void *)leaves->second.ptr, leaves->second.bytes,
                           hipMemcpyDeviceToHost));
  cybvhw::Collapser col;
  col.width = dev->bvh_width;
  col.merge_prims = dev->bvh_merge_prims;
  col.allow_curves = dev->data_host.bvh.have_curves != 0;
  col.nodes2 = n2.data();
  col.n_nodes2 = n2.size() / 4;
  col.leaves2 = l2.data();
  col.n_leaves2 = l2.size() / 4;
  /* instance leaves: object of the leaf's primitive slot, and each object's BVH2 root */
  std::vector<uint32_t> pobj, onode;
  auto fetch_u32 = [&](const char *name, std::vector<uint32_t> *v) -> int {
    auto it = dev->globals.find(name);
    if (it != dev->globals.end() && it->second.bytes) {
      v->resize(it->second.bytes / 4);
      HIP_CHECK(dev, hipMemcpy(v->data(), (const void *)it->second.ptr, it->second.bytes, hipMemcpyDeviceToHost));
    }
    return 0;
  };
  if (fetch_u32("__prim_object", &pobj) || fetch_u32("__object_node", &onode)) {
    return -1;
  }
  col.prim_object = pobj.data();
  col.n_prims = pobj.size();
  col.object_node = onode.data();
  col.n_objects = onode.size();
  if (!col.run(dev->data_host.bvh.root)) {
    return set_error(dev, "BVH widening: " + col.error);
  }
  /* wide nodes, then one int per object: the wide root of its own BVH */
  const size_t node_bytes = col.out.size() * 4;
  const size_t bytes = node_bytes + col.object_root.size() * 4;
  if (bytes > dev->bvhw_capacity) {
    if (dev->bvhw) {
      HIP_CHECK(dev, hipFree(dev->bvhw));
      dev->bvhw = nullptr;
    }
    HIP_CHECK(dev, hipMalloc(&dev->bvhw, bytes));
    dev->bvhw_capacity = bytes;
  }
  HIP_CHECK(dev, hipMemcpy(dev->bvhw, col.out.data(), node_bytes, hipMemcpyHostToDevice));
  if (!col.object_root.empty()) {
    HIP_CHECK(dev, hipMemcpy((char *)dev->bvhw + node_bytes, col.object_root.data(), col.object_root.size() * 4,
                             hipMemcpyHostToDevice));
  }
  dev->bvhw_bytes = node_bytes;
  dev->bvhw_object_root = col.object_root.empty() ? nullptr : (int *)((char *)dev->bvhw + node_bytes);
  dev->bvhw_depth = col.max_depth;
  /* triangle-only meshes without motion pack vertices in primitive order */
  dev->tri_index_identity = 0;
  auto ti = dev->globals.find("__prim_tri_index");
  if (ti != dev->globals.end() && ti->second.bytes) {
    std::vector<uint32_t> idx(ti->second.bytes / 4);
    HIP_CHECK(dev, hipMemcpy(idx.data(), (const void *)ti->second.ptr, ti->second.bytes, hipMemcpyDeviceToHost));
    bool ident = true;
    for (size_t i = 0; i < idx.size() && ident; i++) {
      ident = idx[i] == 3u * (uint32_t)i;
    }
    dev->tri_index_identity = ident ? 1 : 0;
  }
  dev->bvhw_dirty = false;
  return 0;
}

static int ensure_capacity(hipcy_device *dev, size_t slots)
{
  if (slots <= dev->capacity) {
    return 0;
  }
  if (dev->pool) {
    hipFree(dev->pool);
    dev->pool = nullptr;
  }
  /* 12 float4 records + 3 ints per slot (queues are separate); the volume
   * stack and records are allocated by ensure_volume_capacity for volume
   * scenes only */
  const size_t rec = 16 * slots;
  const size_t ints = 4 * slots;
  const size_t total = 12 * rec + 3 * ints + 15 * 256;
  HIP_CHECK(dev, hipMalloc((void **)&dev->pool, total));
  char *p = dev->pool;
  auto take = [&](size_t n) {
    char *r = p;
    p += (n + 255) & ~(size_t)255;
    return r;
  };
  dev->bufs.ray_P = (hc_float4 *)take(rec);
  dev->bufs.ray_D = (hc_float4 *)take(rec);
  dev->bufs.isect = (hc_float4 *)take(rec);
  dev->bufs.isect_type = (int *)take(ints);
  dev->bufs.isect_object = (int *)take(ints);
  dev->bufs.state0 = (hc_uint4 *)take(rec);
  dev->bufs.state1 = (hc_uint4 *)take(rec);
  dev->bufs.state2 = (hc_float4 *)take(rec);
  dev->bufs.throughput = (hc_float4 *)take(rec);
  dev->bufs.L = (hc_float4 *)take(rec);
  dev->bufs.shadow_P = (hc_float4 *)take(rec);
  dev->bufs.shadow_D = (hc_float4 *)take(rec);
  dev->bufs.shadow_L = (hc_float4 *)take(rec);
  dev->bufs.shadow_T = (hc_float4 *)take(rec);
  dev->bufs.item = (uint *)take(ints);
  dev->capacity = slots;
  if (dev->dec_pool) {
    hipFree(dev->dec_pool);
    dev->dec_pool = nullptr;
    dev->dec_slots = 0;
  }
  dev->bufs.dec_steps = nullptr;
  if (dev->vol_pool) {
    hipFree(dev->vol_pool);
    dev->vol_pool = nullptr;
  }
  dev->bufs.vol_stack = nullptr;
  dev->bufs.vol_rec = nullptr;
  if (dev->sss_pool) {
    hipFree(dev->sss_pool);
    dev->sss_pool = nullptr;
  }
  if (dev->catcher_pool) {
    hipFree(dev->catcher_pool);
    dev->catcher_pool = nullptr;
  }
  dev->bufs.catcher = nullptr;
  if (dev->br_pool) {
    hipFree(dev->br_pool);
    dev->br_pool = nullptr;
  }
  dev->bufs.br_rec = nullptr;
  dev->bufs.br_count = nullptr;
  if (dev->lp_pool) {
    hipFree(dev->lp_pool);
    dev->lp_pool = nullptr;
  }
  dev->bufs.lp = nullptr;
  dev->bufs.sss_rec = nullptr;
  dev->bufs.sss_vol = nullptr;
  dev->bufs.sss_count = nullptr;
  dev->sss_pool_vol = false;
  if (dev->diff_pool) {
    hipFree(dev->diff_pool);
    dev->diff_pool = nullptr;
  }
  dev->bufs.ray_diff = nullptr;
  dev->bufs.shadow_dP = nullptr;
  if (dev->srec_pool) {
    hipFree(dev->srec_pool);
    dev->srec_pool = nullptr;
  }
  dev->bufs.shadow_hits = nullptr;
  dev->bufs.shadow_nrec = nullptr;
  /* queues live in their own allocation (3 x slots ints) */
  for (int q = 0; q < 3; q++) {
    if (dev->queue[q]) {
      hipFree(dev->queue[q]);
    }
    HIP_CHECK(dev, hipMalloc((void **)&dev->queue[q], ints));
  }
  return 0;
}

/* The per-slot volume stack (CY_VOLUME_STACK / 2 records) and 2 volume
 * records (cy_integrator.h CyPathBuffers.vol_*), for scenes with volumes:
 * 160 B per slot that other scenes do not pay for. */
/* Slots in flight of decoupled volume scenes: each holds its segment's steps
 * (64 KB), 2^18 slots = 16 GB of the 288 GB. */
#define CY_DEC_SLOTS ((size_t)1 << 18)

static size_t slot_limit(const hipcy_device *dev)
{
  return dev->use_decoupled ? CY_DEC_SLOTS : SIZE_MAX;
}

static int ensure_volume_capacity(hipcy_device *dev)
{
  if (dev->use_decoupled && !dev->dec_pool) {
    dev->dec_slots = std::min(dev->capacity, CY_DEC_SLOTS);
    HIP_CHECK(dev, hipMalloc((void **)&dev->dec_pool,
                             dev->dec_slots * (size_t)CY_DECOUPLED_STEPS * CY_DECOUPLED_STEP_BYTES));
  }
  dev->bufs.dec_steps = dev->use_decoupled ? dev->dec_pool : nullptr;
  if (!dev->use_volumes || dev->vol_pool) {
    return 0;
  }
  const size_t rec = 16 * dev->capacity;
  HIP_CHECK(dev, hipMalloc((void **)&dev->vol_pool, (CY_VOLUME_STACK / 2 + 2) * rec));
  dev->bufs.vol_stack = (hc_uint4 *)dev->vol_pool;
  dev->bufs.vol_rec = (hc_uint4 *)(dev->vol_pool + (CY_VOLUME_STACK / 2) * rec);
  return 0;
}

/* The slots' shadow-catcher records (cy_integrator.h CyCatcher, 48 B per
 * slot), for scenes with shadow-catcher objects only. */
static int ensure_catcher_capacity(hipcy_device *dev)
{
  if (dev->use_catcher && !dev->catcher_pool) {
    HIP_CHECK(dev, hipMalloc((void **)&dev->catcher_pool, (size_t)16 * CY_CATCHER_F4 * dev->capacity));
  }
  dev->bufs.catcher = dev->use_catcher ? (hc_float4 *)dev->catcher_pool : nullptr;
  return 0;
}

/* The slots' branch records (cy_integrator.h CY_BR_RECS x CY_BR_REC_F4 float4
 * and two counters per slot, 2.6 KB), for branched path tracing only. */
static int ensure_branch_capacity(hipcy_device *dev)
{
  const size_t recs = (size_t)16 * CY_BR_RECS * CY_BR_REC_F4 * dev->capacity;
  const size_t counts = (size_t)8 * dev->capacity;
  if (dev->use_branched && !dev->br_pool) {
    HIP_CHECK(dev, hipMalloc((void **)&dev->br_pool, recs + counts));
    HIP_CHECK(dev, hipMemset(dev->br_pool + recs, 0, counts));
  }
  dev->bufs.br_rec = dev->use_branched ? (hc_float4 *)dev->br_pool : nullptr;
  dev->bufs.br_count = dev->use_branched ? (uint *)(dev->br_pool + recs) : nullptr;
  return 0;
}

/* The slots' light-pass records (cy_integrator.h CyLightPass, 256 B per
 * slot), for films with light passes only. */
static int ensure_lightpass_capacity(hipcy_device *dev)
{
  if (dev->use_lightpass && !dev->lp_pool) {
    HIP_CHECK(dev, hipMalloc((void **)&dev->lp_pool, (size_t)16 * CY_LP_F4 * dev->capacity));
  }
  dev->bufs.lp = dev->use_lightpass ? (hc_float4 *)dev->lp_pool : nullptr;
  return 0;
}

/* The slots' subsurface indirect-ray records (cy_integrator.h CY_SSS_RECS x
 * CY_SSS_REC_F4 float4 and a depth per slot, 292 B), for scenes with disk
 * BSSRDFs only.  Every path leaves its slot with depth 0, so the depths are
 * cleared once, here. */
static int ensure_sss_capacity(hipcy_device *dev)
{
  const size_t recs = (size_t)16 * CY_SSS_RECS * CY_SSS_REC_F4 * dev->capacity;
  const size_t counts = 4 * dev->capacity;
  /* volume scenes: each record's volume stack and the pending shadow's
   * (CY_SSS_RECS + 1 stacks of CY_VOLUME_STACK / 2 records, 512 B per slot) */
  const bool vol = dev->use_disk_bssrdf && dev->use_volumes;
  const size_t stacks = vol ? (size_t)16 * (CY_SSS_RECS + 1) * (CY_VOLUME_STACK / 2) * dev->capacity : 0;
  if (dev->sss_pool && vol && !dev->sss_pool_vol) {
    /* sized for a scene without volumes (no path is in flight between renders) */
    HIP_CHECK(dev, hipFree(dev->sss_pool));
    dev->sss_pool = nullptr;
  }
  if (dev->use_disk_bssrdf && !dev->sss_pool) {
    HIP_CHECK(dev, hipMalloc((void **)&dev->sss_pool, recs + stacks + counts));
    HIP_CHECK(dev, hipMemset(dev->sss_pool + recs + stacks, 0, counts));
    dev->sss_pool_vol = vol;
  }
  /* other scenes' shading never looks at the records; the depths sit where
   * the pool's own layout put them (a pool sized for a volume scene keeps
   * its stacks when a scene without volumes follows) */
  const size_t pool_stacks = dev->sss_pool_vol ? (size_t)16 * (CY_SSS_RECS + 1) * (CY_VOLUME_STACK / 2) * dev->capacity
                                               : 0;
  dev->bufs.sss_rec = dev->use_disk_bssrdf ? (hc_float4 *)dev->sss_pool : nullptr;
  dev->bufs.sss_vol = vol ? (hc_uint4 *)(dev->sss_pool + recs) : nullptr;
  dev->bufs.sss_count = dev->use_disk_bssrdf ? (uint *)(dev->sss_pool + recs + pool_stacks) : nullptr;
  return 0;
}

/* The slots' ray differentials (CY_RAY_DIFF_F4 float4) and the pending
 * shadow ray's dP (2 float4), 80 B per slot, for scenes whose shaders read
 * differentials only. */
static int ensure_diff_capacity(hipcy_device *dev)
{
  const size_t rays = (size_t)16 * CY_RAY_DIFF_F4 * dev->capacity;
  if (dev->use_ray_diff && !dev->diff_pool) {
    HIP_CHECK(dev, hipMalloc((void **)&dev->diff_pool, rays + (size_t)32 * dev->capacity));
  }
  dev->bufs.ray_diff = dev->use_ray_diff ? (hc_float4 *)dev->diff_pool : nullptr;
  dev->bufs.shadow_dP = dev->use_ray_diff ? (hc_float4 *)(dev->diff_pool + rays) : nullptr;
  return 0;
}

/* The transparent-shadow records of k_shadow_record (CY_SHADOW_REC_HITS
 * float4 and a count per slot, 68 B), for non-instanced scenes with
 * transparent shadows only. */
static int ensure_srec_capacity(hipcy_device *dev)
{
  const bool use = dev->data_host.integrator.transparent_shadows && !dev->have_instancing;
  const size_t hits = (size_t)16 * CY_SHADOW_REC_HITS * dev->capacity;
  if (use && !dev->srec_pool) {
    HIP_CHECK(dev, hipMalloc((void **)&dev->srec_pool, hits + (size_t)4 * dev->capacity));
  }
  dev->bufs.shadow_hits = use ? (hc_float4 *)dev->srec_pool : nullptr;
  dev->bufs.shadow_nrec = use ? (uint *)(dev->srec_pool + hits) : nullptr;
  return 0;
}

extern "C" {

int hipcy_abi_version(void)
{
  return HIPCY_ABI_VERSION;
}

int hipcy_device_count(int *count)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    n = 0;
  }
  *count = n;
  return 0;
}

int hipcy_device_info(int ordinal, char *name, size_t name_len, uint64_t *total_mem)
{
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, ordinal) != hipSuccess) {
    return -1;
  }
  if (name && name_len) {
    snprintf(name, name_len, "%s (%s)", prop.name, prop.gcnArchName);
  }
  if (total_mem) {
    *total_mem = prop.totalGlobalMem;
  }
  return 0;
}

const char *hipcy_global_error(void)
{
  std::lock_guard<std::mutex> lock(g_error_mutex);
  return g_global_error.c_str();
}

hipcy_device *hipcy_create(int ordinal)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || ordinal < 0 || ordinal >= n) {
    set_error(nullptr, "no HIP device with ordinal " + std::to_string(ordinal));
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, ordinal) != hipSuccess) {
    set_error(nullptr, "hipGetDeviceProperties failed");
    return nullptr;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error(nullptr, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
    return nullptr;
  }
  hipcy_device *dev = new hipcy_device();
  dev->ordinal = ordinal;
  hipSetDevice(ordinal);
  for (int l = 0; l < CY_LANES; l++) {
    if (hipStreamCreateWithFlags(&dev->lane_stream[l], hipStreamNonBlocking) != hipSuccess) {
      set_error(nullptr, "device context creation failed (streams)");
      delete dev;
      return nullptr;
    }
  }
  memset(&dev->data_host, 0, sizeof(dev->data_host));
  memset(&dev->stats, 0, sizeof(dev->stats));
  if (hipSetDevice(ordinal) != hipSuccess ||
      hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void **)&dev->data_dev, sizeof(hc_KernelData)) != hipSuccess ||
      hipMalloc((void **)&dev->counters, 16 * 4 * (CY_LANES + 1)) != hipSuccess ||
      hipMalloc((void **)&dev->stats_dev, 2 * CY_STATS_SHARDS * sizeof(CyStats)) != hipSuccess ||
      hipHostMalloc((void **)&dev->host_counters, 16 * 4 * (CY_LANES + 1), hipHostMallocDefault) != hipSuccess) {
    set_error(nullptr, "device context creation failed");
    delete dev;
    return nullptr;
  }
  return dev;
}

void hipcy_destroy(hipcy_device *dev)
{
  if (!dev) {
    return;
  }
  hipSetDevice(dev->ordinal);
  hipStreamSynchronize(dev->stream);
  for (auto &a : dev->allocations) {
    hipFree((void *)a.first);
  }
  for (auto e : dev->events) {
    hipEventDestroy(e);
  }
  if (dev->pool) hipFree(dev->pool);
  if (dev->vol_pool) hipFree(dev->vol_pool);
  if (dev->sss_pool) hipFree(dev->sss_pool);
  if (dev->catcher_pool) hipFree(dev->catcher_pool);
  if (dev->br_pool) hipFree(dev->br_pool);
  if (dev->lp_pool) hipFree(dev->lp_pool);
  if (dev->dec_pool) hipFree(dev->dec_pool);
  if (dev->diff_pool) hipFree(dev->diff_pool);
  if (dev->srec_pool) hipFree(dev->srec_pool);
  if (dev->bvhw) hipFree(dev->bvhw);
  if (dev->records) hipFree(dev->records);
  if (dev->tile_descs) hipFree(dev->tile_descs);
  if (dev->stream_desc_dev) hipFree(dev->stream_desc_dev);
  if (dev->stream_desc_host) hipHostFree(dev->stream_desc_host);
  if (dev->min_live_dev) hipFree(dev->min_live_dev);
  if (dev->min_live_host) hipHostFree(dev->min_live_host);
  for (int q = 0; q < 3; q++) {
    if (dev->queue[q]) hipFree(dev->queue[q]);
  }
  if (dev->cont_rec) hipFree(dev->cont_rec);
  if (dev->refill_claim) hipFree(dev->refill_claim);
  if (dev->sort_queue) hipFree(dev->sort_queue);
  if (dev->sort_key) hipFree(dev->sort_key);
  if (dev->sort_hist) hipFree(dev->sort_hist);
  if (dev->counters) hipFree(dev->counters);
  if (dev->stats_dev) hipFree(dev->stats_dev);
  if (dev->data_dev) hipFree(dev->data_dev);
  for (void *t : dev->tex_mem) {
    if (t) hipFree(t);
  }
  if (dev->tex_info_dev) hipFree(dev->tex_info_dev);
  if (dev->host_counters) hipHostFree(dev->host_counters);
  if (dev->stream) hipStreamDestroy(dev->stream);
  for (int l = 0; l < CY_LANES; l++) {
    if (dev->lane_stream[l]) hipStreamDestroy(dev->lane_stream[l]);
  }
  delete dev;
}

const char *hipcy_error(const hipcy_device *dev)
{
  return dev ? dev->error.c_str() : hipcy_global_error();
}

int hipcy_mem_alloc(hipcy_device *dev, size_t bytes, uint64_t *device_pointer)
{
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  void *p = nullptr;
  HIP_CHECK(dev, hipMalloc(&p, bytes ? bytes : 16));
  dev->allocations[(uint64_t)p] = bytes;
  *device_pointer = (uint64_t)p;
  return 0;
}

int hipcy_mem_free(hipcy_device *dev, uint64_t device_pointer)
{
  auto it = dev->allocations.find(device_pointer);
  if (it == dev->allocations.end()) {
    return set_error(dev, "mem_free of unknown pointer");
  }
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  HIP_CHECK(dev, hipFree((void *)device_pointer));
  dev->allocations.erase(it);
  for (auto g = dev->globals.begin(); g != dev->globals.end();) {
    if (g->second.ptr == device_pointer) {
      g = dev->globals.erase(g);
    }
    else {
      ++g;
    }
  }
  return 0;
}

int hipcy_mem_copy_to(hipcy_device *dev, uint64_t dst, const void *src, size_t bytes)
{
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  HIP_CHECK(dev, hipMemcpyAsync((void *)dst, src, bytes, hipMemcpyHostToDevice, dev->stream));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  /* a bound array rewritten in place: features must be re-checked */
  for (auto &g : dev->globals) {
    if (g.second.ptr == dst) {
      dev->features_dirty = true;
      if (g.first == "__object_flag") {
        dev->object_flags.assign((const uint32_t *)src, (const uint32_t *)src + std::min(bytes, g.second.bytes) / 4);
      }
      if (g.first == "__svm_nodes") {
        /* the program scan of load_kernels reads this copy (node set -> variant) */
        const size_t k = std::min(bytes, g.second.bytes) / sizeof(hc_uint4);
        dev->svm_nodes.assign((const hc_uint4 *)src, (const hc_uint4 *)src + k);
      }
      if (g.first == "__shaders") {
        dev->num_shaders = g.second.bytes / sizeof(hc_KernelShader);
      }
      if (g.first == "__bvh_nodes" || g.first == "__bvh_leaf_nodes" || g.first == "__prim_tri_index" ||
          g.first == "__prim_object" || g.first == "__object_node") {
        dev->bvhw_dirty = true;
      }
    }
  }
  return 0;
}

int hipcy_mem_copy_from(hipcy_device *dev, void *dst, uint64_t src, size_t bytes)
{
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  HIP_CHECK(dev, hipMemcpyAsync(dst, (const void *)src, bytes, hipMemcpyDeviceToHost, dev->stream));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return 0;
}

int hipcy_mem_zero(hipcy_device *dev, uint64_t device_pointer, size_t bytes)
{
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  HIP_CHECK(dev, hipMemsetAsync((void *)device_pointer, 0, bytes, dev->stream));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return 0;
}

int hipcy_const_copy_to(hipcy_device *dev, const char *name, const void *host, size_t size)
{
  if (strcmp(name, "__data") != 0) {
    return set_error(dev, std::string("const_copy_to: unknown constant ") + name);
  }
  if (size != sizeof(hc_KernelData)) {
    return set_error(dev, "const_copy_to: KernelData size " + std::to_string(size) +
                              " != " + std::to_string(sizeof(hc_KernelData)));
  }
  if (!dev->have_data || dev->data_host.bvh.root != ((const hc_KernelData *)host)->bvh.root) {
    dev->bvhw_dirty = true;
  }
  memcpy(&dev->data_host, host, size);
  dev->have_data = true;
  dev->features_dirty = true;
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  HIP_CHECK(dev, hipMemcpyAsync(dev->data_dev, host, size, hipMemcpyHostToDevice, dev->stream));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return 0;
}

/* Mirror the texture table to the device and bind it as __texture_info. */
static int upload_texture_info(hipcy_device *dev)
{
  const size_t n = dev->tex_info.size();
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  if (n > dev->tex_info_capacity) {
    if (dev->tex_info_dev) {
      HIP_CHECK(dev, hipFree(dev->tex_info_dev));
    }
    HIP_CHECK(dev, hipMalloc((void **)&dev->tex_info_dev, n * sizeof(hc_TextureInfo)));
    dev->tex_info_capacity = n;
  }
  if (n) {
    HIP_CHECK(dev, hipMemcpy(dev->tex_info_dev, dev->tex_info.data(), n * sizeof(hc_TextureInfo),
                             hipMemcpyHostToDevice));
  }
  GlobalBinding b;
  b.ptr = (uint64_t)dev->tex_info_dev;
  b.bytes = n * sizeof(hc_TextureInfo);
  dev->globals["__texture_info"] = b;
  dev->features_dirty = true;
  return 0;
}

int hipcy_tex_alloc(hipcy_device *dev, int slot, int data_type, int interpolation, int extension, int width,
                    int height, const void *pixels, size_t bytes)
{
  return hipcy_tex_alloc_3d(dev, slot, data_type, interpolation, extension, width, height, 1, nullptr, pixels, bytes);
}

int hipcy_tex_alloc_3d(hipcy_device *dev, int slot, int data_type, int interpolation, int extension, int width,
                       int height, int depth, const float *transform_3d, const void *pixels, size_t bytes)
{
  if (!dev || slot < 0 || width <= 0 || height <= 0 || depth <= 0 || data_type < 0 || data_type > 7 ||
      interpolation < 0 || interpolation > 3 || extension < 0 || extension > 2) {
    return set_error(dev, "tex_alloc: invalid texture description");
  }
  static const size_t texel_bytes[8] = {16, 4, 8, 4, 1, 2, 8, 2}; /* ImageDataType order */
  if (bytes != texel_bytes[data_type] * (size_t)width * (size_t)height * (size_t)depth) {
    return set_error(dev, "tex_alloc: pixel buffer size does not match the texture description");
  }
  if (hipcy_tex_free(dev, slot) != 0) {
    return -1;
  }
  if ((size_t)slot >= dev->tex_info.size()) {
    dev->tex_info.resize(slot + 1);
    dev->tex_mem.resize(slot + 1, nullptr);
    memset(&dev->tex_info[slot], 0, sizeof(hc_TextureInfo));
  }
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  void *mem = nullptr;
  HIP_CHECK(dev, hipMalloc(&mem, bytes));
  HIP_CHECK(dev, hipMemcpy(mem, pixels, bytes, hipMemcpyHostToDevice));
  dev->tex_mem[slot] = mem;
  hc_TextureInfo &info = dev->tex_info[slot];
  memset(&info, 0, sizeof(info));
  info.data = (uint64_t)mem;
  info.data_type = (uint32_t)data_type;
  info.interpolation = (uint32_t)interpolation;
  info.extension = (uint32_t)extension;
  info.width = (uint32_t)width;
  info.height = (uint32_t)height;
  info.depth = (uint32_t)depth;
  if (transform_3d) {
    /* TextureInfo::transform_3d (util_texture.h:105), rows x, y, z */
    info.use_transform_3d = 1;
    memcpy(&info.transform_3d, transform_3d, 12 * sizeof(float));
  }
  return upload_texture_info(dev);
}

int hipcy_tex_free(hipcy_device *dev, int slot)
{
  if (!dev) {
    return -1;
  }
  if (slot < 0 || (size_t)slot >= dev->tex_mem.size() || !dev->tex_mem[slot]) {
    return 0;
  }
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  HIP_CHECK(dev, hipDeviceSynchronize());
  HIP_CHECK(dev, hipFree(dev->tex_mem[slot]));
  dev->tex_mem[slot] = nullptr;
  memset(&dev->tex_info[slot], 0, sizeof(hc_TextureInfo));
  return upload_texture_info(dev);
}

int hipcy_bind_global(hipcy_device *dev, const char *name, uint64_t device_pointer, size_t bytes)
{
  static const char *known[] = {
#define CY_NAME(type, n) #n,
      CY_GLOBAL_ARRAYS(CY_NAME)
#undef CY_NAME
  };
  bool ok = false;
  for (const char *k : known) {
    if (strcmp(k, name) == 0) {
      ok = true;
    }
  }
  if (!ok) {
    /* Arrays of features this device rejects (curves, motion, attributes...)
     * are accepted but must be empty; hipcy_load_kernels checks features. */
    if (bytes == 0) {
      return 0;
    }
  }
  GlobalBinding b;
  b.ptr = device_pointer;
  b.bytes = bytes;
  dev->globals[name] = b;
  dev->features_dirty = true;
  if (strcmp(name, "__object_flag") == 0) {
    /* the device pointer holds the uploaded array already (global_alloc copies
     * before binding, device_cuda_impl.cpp:1088-1096): keep a host copy for the
     * feature checks of load_kernels, so no render needs a device read-back */
    dev->object_flags.assign(bytes / 4, 0u);
    if (bytes) {
      HIP_CHECK(dev, hipSetDevice(dev->ordinal));
      HIP_CHECK(dev, hipMemcpy(dev->object_flags.data(), (const void *)device_pointer, bytes, hipMemcpyDeviceToHost));
    }
  }
  if (strcmp(name, "__svm_nodes") == 0) {
    /* host copy for the program scan of load_kernels (node set -> kernel variant) */
    dev->svm_nodes.assign(bytes / sizeof(hc_uint4), hc_uint4{});
    if (bytes) {
      HIP_CHECK(dev, hipSetDevice(dev->ordinal));
      HIP_CHECK(dev, hipMemcpy(dev->svm_nodes.data(), (const void *)device_pointer, bytes, hipMemcpyDeviceToHost));
    }
  }
  if (strcmp(name, "__shaders") == 0) {
    dev->num_shaders = bytes / sizeof(hc_KernelShader);
  }
  if (strcmp(name, "__bvh_nodes") == 0 || strcmp(name, "__bvh_leaf_nodes") == 0 ||
      strcmp(name, "__prim_tri_index") == 0 || strcmp(name, "__prim_object") == 0 ||
      strcmp(name, "__object_node") == 0) {
    dev->bvhw_dirty = true;
  }
  return 0;
}

int hipcy_set_bvh_width(hipcy_device *dev, int width)
{
  if (width != 2 && width != 4 && width != 8) {
    return set_error(dev, "set_bvh_width: width must be 2, 4 or 8");
  }
  if (width != dev->bvh_width) {
    dev->bvhw_dirty = true;
  }
  dev->bvh_width = width;
  return 0;
}

int hipcy_set_curve_layout(hipcy_device *dev, int wide)
{
  if (wide != 0 && wide != 1) {
    return set_error(dev, "set_curve_layout: 0 (BVH2) or 1 (wide layout for ribbon scenes)");
  }
  if ((wide != 0) != dev->curve_wide) {
    dev->bvhw_dirty = true;
  }
  dev->curve_wide = wide != 0;
  return 0;
}

int hipcy_set_traversal_budget(hipcy_device *dev, int first, int second)
{
  if (first < 0 || second < 0 || (first == 0) != (second == 0)) {
    return set_error(dev, "set_traversal_budget: budgets must be >= 0, both zero or both positive");
  }
  dev->trav_budget[0] = first;
  dev->trav_budget[1] = second;
  return 0;
}

int hipcy_set_traversal_refill(hipcy_device *dev, int rounds, int min_idle)
{
  if (rounds < 0 || min_idle < 1 || min_idle > 64) {
    return set_error(dev, "set_traversal_refill: rounds >= 0 (0 = off), 1 <= min_idle <= 64");
  }
  dev->trav_refill[0] = rounds;
  dev->trav_refill[1] = min_idle;
  return 0;
}

int hipcy_set_tail(hipcy_device *dev, uint64_t paths)
{
  dev->tail_paths = (size_t)paths;
  return 0;
}

int hipcy_set_shadow_sort(hipcy_device *dev, int mode)
{
  if (mode != 0 && mode != 3 && mode != 5) {
    return set_error(dev, "set_shadow_sort: mode must be 0, 3 or 5");
  }
  dev->shadow_sort = mode;
  return 0;
}

int hipcy_set_ray_sort(hipcy_device *dev, int mode)
{
  if (mode != -1 && mode != 0 && mode != 3 && mode != 5 && mode != 8) {
    return set_error(dev, "set_ray_sort: mode must be -1, 0, 3, 5 or 8");
  }
  dev->ray_sort = mode;
  return 0;
}

int hipcy_set_bvh_leaf_merge(hipcy_device *dev, int max_prims)
{
  if (max_prims < 0 || max_prims > 15) {
    return set_error(dev, "set_bvh_leaf_merge: max_prims must be in [0, 15]");
  }
  if (max_prims != dev->bvh_merge_prims) {
    dev->bvhw_dirty = true;
  }
  dev->bvh_merge_prims = max_prims;
  return 0;
}

uint32_t hipcy_get_bvh_layout_mask(const hipcy_device *)
{
  return 1u; /* BVH_LAYOUT_BVH2 (kernel_types.h:1396-1406) */
}

/* Walk every shader's SVM program (jump table entry -> NODE_END) with the node
 * lengths of svm/svm.h's decoders.  Rejects nodes the HIP interpreter does not
 * implement before any render (the reference compiles only the node groups a
 * scene requests: DeviceRequestedFeatures max_nodes_group / nodes_features,
 * device/device.h:130-200) and reports whether the texture / converter / input
 * nodes are used, which selects the shading-kernel variant. */
static std::string svm_scan(const std::vector<hc_uint4> &prog, size_t num_shaders,
                            const std::vector<void *> &tex_mem, const std::vector<uint32_t> &shader_flags,
                            bool *uses_tex, bool *uses_bssrdf, bool *uses_disk_bssrdf, bool *uses_attr,
                            bool *uses_ray_diff, bool *uses_ies, bool *uses_particles, int *surface_closures,
                            int *volume_closures)
{
  *uses_tex = false;
  *uses_particles = false;
  *uses_ies = false;
  *uses_ray_diff = false;
  *uses_bssrdf = false;
  *uses_disk_bssrdf = false;
  *uses_attr = false;
  /* closures one program can allocate, counted as ShaderGraph::get_num_closures
   * (render/graph.cpp:1130-1161) counts them, except that a phase closure
   * allocates one per evaluation (the reference reserves VOLUME_STACK_SIZE) */
  *surface_closures = 0;
  *volume_closures = 0;
  const size_t n = prog.size();
  /* an image slot the kernel will read must have been allocated (hipcy_tex_alloc):
   * kernel_tex_image_interp indexes __texture_info without a bound check; -1 is
   * the reference's "missing image" id and is never read */
  auto slot_ok = [&](int id) { return id == -1 || (id >= 0 && (size_t)id < tex_mem.size() && tex_mem[id]); };
  if (num_shaders > n) {
    return "jump table larger than the program";
  }
  /* every shader's surface program, and the volume program of shaders with a volume */
  for (size_t pi = 0; pi < 2 * num_shaders; pi++) {
    const size_t sh = pi % num_shaders;
    const bool volume = pi >= num_shaders;
    if (prog[sh].x != NODE_SHADER_JUMP) {
      return "shader " + std::to_string(sh) + ": jump table entry is not NODE_SHADER_JUMP";
    }
    if (volume && !(sh < shader_flags.size() && (shader_flags[sh] & SD_HAS_VOLUME))) {
      continue;
    }
    size_t off = volume ? prog[sh].z : prog[sh].y;
    int closures = 0;
    for (size_t steps = 0;; steps++) {
      if (off >= n || steps > n) {
        return "shader " + std::to_string(sh) + ": program runs past __svm_nodes";
      }
      const hc_uint4 node = prog[off];
      size_t len = 1;
      bool tex = false;
      switch (node.x) {
        case NODE_END:
          len = 0;
          break;
        case NODE_CLOSURE_BSDF: {
          len = 2;
          if (off + 1 >= n) {
            return "closure node: data node past __svm_nodes";
          }
          /* the plain shading kernels carry the basic closure set
           * (cy_types.h CY_CLOSURE_EXT): isotropic GGX / sharp / glass /
           * transparent / Lambert diffuse; anything else selects the full one */
          const uint ctype = node.y & 0xFF;
          closures += (ctype == CLOSURE_BSDF_PRINCIPLED_ID)                                 ? 8 :
                      (ctype == CLOSURE_BSDF_HAIR_PRINCIPLED_ID)                            ? 4 :
                      (ctype >= CLOSURE_BSSRDF_CUBIC_ID && ctype <= CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID) ? 3 :
                      (ctype == CLOSURE_BSDF_SHARP_GLASS_ID || ctype == CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID ||
                       ctype == CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID ||
                       ctype == CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID ||
                       ctype == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID)                 ? 2 :
                                                                                            1;
          const bool rough_diffuse = ctype == CLOSURE_BSDF_DIFFUSE_ID &&
                                     (((node.y >> 8) & 0xFF) != SVM_STACK_INVALID || node.z != 0u);
          const bool tangent = prog[off + 1].y != SVM_STACK_INVALID;
          tex = rough_diffuse || tangent ||
                !(ctype == CLOSURE_BSDF_DIFFUSE_ID || ctype == CLOSURE_BSDF_TRANSPARENT_ID ||
                  ctype == CLOSURE_BSDF_REFLECTION_ID || ctype == CLOSURE_BSDF_MICROFACET_GGX_ID ||
                  ctype == CLOSURE_BSDF_REFRACTION_ID || ctype == CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID ||
                  ctype == CLOSURE_BSDF_SHARP_GLASS_ID || ctype == CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID);
          if (ctype == CLOSURE_BSDF_HAIR_PRINCIPLED_ID) {
            len = 5; /* data node + 3 parameter nodes (the last: the Random attribute) */
            if (off + 4 >= n) {
              return "principled hair BSDF: parameter nodes past __svm_nodes";
            }
            *uses_attr |= prog[off + 4].y != SVM_STACK_INVALID;
          }
          if (ctype == CLOSURE_BSDF_PRINCIPLED_ID) {
            len = 6; /* data node + 4 nodes of principled parameters */
            if (off + 5 >= n) {
              return "principled BSDF: parameter nodes past __svm_nodes";
            }
            /* GGX or multiscatter GGX (specular layer and rough transmission) */
            if (prog[off + 2].y != CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID &&
                prog[off + 2].y != CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID) {
              return "shader " + std::to_string(sh) + ": principled BSDF: unknown distribution " +
                     std::to_string(prog[off + 2].y);
            }
          }
          switch (ctype) {
            case CLOSURE_BSDF_PRINCIPLED_ID:
            case CLOSURE_BSDF_DIFFUSE_ID:
            case CLOSURE_BSDF_TRANSLUCENT_ID:
            case CLOSURE_BSDF_TRANSPARENT_ID:
            case CLOSURE_BSDF_REFLECTION_ID:
            case CLOSURE_BSDF_MICROFACET_GGX_ID:
            case CLOSURE_BSDF_MICROFACET_BECKMANN_ID:
            case CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID:
            case CLOSURE_BSDF_REFRACTION_ID:
            case CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID:
            case CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID:
            case CLOSURE_BSDF_SHARP_GLASS_ID:
            case CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID:
            case CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID:
            case CLOSURE_BSDF_ASHIKHMIN_VELVET_ID:
            case CLOSURE_BSDF_DIFFUSE_TOON_ID:
            case CLOSURE_BSDF_GLOSSY_TOON_ID:
            case CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
            case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID:
            case CLOSURE_BSDF_HAIR_REFLECTION_ID:
            case CLOSURE_BSDF_HAIR_TRANSMISSION_ID:
            case CLOSURE_BSDF_HAIR_PRINCIPLED_ID:
            case CLOSURE_BSSRDF_RANDOM_WALK_ID: /* Subsurface Scattering node */
            case CLOSURE_BSSRDF_CUBIC_ID:
            case CLOSURE_BSSRDF_GAUSSIAN_ID:
            case CLOSURE_BSSRDF_BURLEY_ID: {
              /* a BSSRDF, or a principled BSDF with subsurface (param2: linked
               * or > 0; the method in its second data node's z) */
              const bool principled_sss = ctype == CLOSURE_BSDF_PRINCIPLED_ID &&
                                          (((node.y >> 16) & 0xFF) != SVM_STACK_INVALID || node.w != 0u);
              *uses_bssrdf |= principled_sss || (ctype >= CLOSURE_BSSRDF_CUBIC_ID && ctype <= CLOSURE_BSSRDF_RANDOM_WALK_ID);
              *uses_disk_bssrdf |= (ctype >= CLOSURE_BSSRDF_CUBIC_ID && ctype <= CLOSURE_BSSRDF_BURLEY_ID) ||
                                   (principled_sss && prog[off + 2].z == CLOSURE_BSSRDF_PRINCIPLED_ID);
              break;
            }
            default:
              return "shader " + std::to_string(sh) + ": closure type " + std::to_string(ctype) +
                     " is not implemented";
          }
          break;
        }
        case NODE_VALUE_V:
          len = 2;
          break;
        case NODE_CLOSURE_VOLUME:
          closures += ((node.y & 0xFF) == CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID) ? 1 : 0;
          tex = true; /* volumes run in the extended shading kernels */
          break;
        case NODE_PRINCIPLED_VOLUME:
          len = 3; /* value node, attribute node */
          if (off + 2 >= n) {
            return "principled volume: parameter nodes past __svm_nodes";
          }
          if (((node.z >> 16) & 0xFF) != SVM_STACK_INVALID || __builtin_bit_cast(float, prog[off + 1].w) > 0.0f) {
            return "shader " + std::to_string(sh) + ": principled volume blackbody emission is not implemented";
          }
          closures += 1;
          tex = true;
          break;
        case NODE_CLOSURE_HOLDOUT: /* svm_closure.h:1043-1057 */
          closures += 1;
          tex = true;
          break;
        case NODE_TEXTURE_MAPPING: /* three matrix rows */
          len = 4;
          tex = true;
          break;
        case NODE_MIN_MAX: /* min and max rows */
          len = 3;
          tex = true;
          break;
        case NODE_PARTICLE_INFO:
          *uses_particles = true;
          tex = true;
          break;
        case NODE_HAIR_INFO:
          tex = true;
          break;
        case NODE_CLOSURE_EMISSION:
        case NODE_CLOSURE_BACKGROUND:
        case NODE_CLOSURE_SET_WEIGHT:
        case NODE_CLOSURE_WEIGHT:
        case NODE_EMISSION_WEIGHT:
        case NODE_MIX_CLOSURE:
        case NODE_JUMP_IF_ZERO:
        case NODE_JUMP_IF_ONE:
        case NODE_VALUE_F:
        case NODE_FRESNEL:
        case NODE_LAYER_WEIGHT:
          break;
        case NODE_MATH:
          tex = true;
          break;
        case NODE_VECTOR_MATH:
          len = (node.y == 20) ? 2 : 1; /* WRAP: extra node */
          tex = true;
          break;
        case NODE_TEX_COORD_BUMP_DX:
        case NODE_TEX_COORD_BUMP_DY:
          *uses_ray_diff = true;
          /* fall through */
        case NODE_TEX_COORD:
          len = (node.y == 1 && node.w != 0) ? 4 : 1; /* OBJECT with a transform */
          tex = true;
          break;
        case NODE_SET_BUMP:
          *uses_ray_diff = true;
          tex = true;
          break;
        case NODE_ENTER_BUMP_EVAL: /* displacement method "both": the undisplaced position */
          *uses_ray_diff = true;
          *uses_attr = true;
          tex = true;
          break;
        case NODE_LEAVE_BUMP_EVAL:
          tex = true;
          break;
        case NODE_AOV_START: /* svm_aov.h: AOV outputs of the camera path's hits */
        case NODE_AOV_COLOR:
        case NODE_AOV_VALUE:
          tex = true;
          break;
        case NODE_TEX_VOXEL: /* Point Density: a 3D texture; world space carries a transform */
          len = ((node.z >> 24) & 0xFF) == 1u ? 4 : 1;
          if (off + len > n) {
            return "voxel texture: transform nodes past __svm_nodes";
          }
          if (!slot_ok((int)node.y) || (int)node.y == -1) {
            return "shader " + std::to_string(sh) + ": voxel texture slot " + std::to_string((int)node.y) +
                   " was never allocated (tex_alloc_3d)";
          }
          *uses_attr |= ((node.z >> 24) & 0xFF) == 0u;
          tex = true;
          break;
        case NODE_VECTOR_DISPLACEMENT: /* height / vector displacement inside a bump program */
          len = 2;
          tex = true;
          break;
        case NODE_DISPLACEMENT:
        case NODE_CLOSURE_SET_NORMAL: /* the bump program of displacement method "bump" */
        case NODE_AMBIENT_OCCLUSION:
        case NODE_BEVEL:
          tex = true;
          break;
        case NODE_WIREFRAME:
          *uses_ray_diff |= (node.w & 0xFF) != 0 || ((node.w >> 8) & 0xFF) != 0; /* pixel size / bump forms */
          tex = true;
          break;
        case NODE_RGB_RAMP:
          if (off + 1 >= n) {
            return "rgb ramp: table size node past __svm_nodes";
          }
          len = 2 + (size_t)prog[off + 1].x;
          tex = true;
          break;
        case NODE_MIX:
        case NODE_SEPARATE_HSV:
        case NODE_COMBINE_HSV:
        case NODE_CLAMP:
          len = 2;
          tex = true;
          break;
        case NODE_MAP_RANGE:
          len = 3;
          tex = true;
          break;
        case NODE_TEX_IMAGE:
          len = 1 + (size_t)(((int)node.y > 0) ? (int)node.y : 0); /* UDIM tile nodes */
          if (off + len > n) {
            return "image texture: UDIM tile nodes past __svm_nodes";
          }
          if ((int)node.y <= 0) {
            if (!slot_ok(-(int)node.y)) {
              return "shader " + std::to_string(sh) + ": image texture slot " + std::to_string(-(int)node.y) +
                     " was never allocated (tex_alloc)";
            }
          }
          else {
            for (size_t k = 1; k < len; k++) {
              /* tile node: (tile, slot, tile, slot); an unused pair has tile -1 */
              const hc_uint4 tn = prog[off + k];
              if (((int)tn.x != -1 && !slot_ok((int)tn.y)) || ((int)tn.z != -1 && !slot_ok((int)tn.w))) {
                return "shader " + std::to_string(sh) + ": UDIM tile image slot was never allocated (tex_alloc)";
              }
            }
          }
          tex = true;
          break;
        case NODE_TEX_ENVIRONMENT:
          if (!slot_ok((int)node.y)) {
            return "shader " + std::to_string(sh) + ": environment texture slot " + std::to_string((int)node.y) +
                   " was never allocated (tex_alloc)";
          }
          tex = true;
          break;
        case NODE_WAVELENGTH:
        case NODE_BLACKBODY:
          tex = true;
          break;
        case NODE_IES:
          *uses_ies = true;
          tex = true;
          break;
        case NODE_TEX_SKY: /* 8 parameter nodes, Nishita 3 (with its texture slot) */
          len = (node.w == 2u) ? 4 : 9;
          if (off + len > n) {
            return "sky texture: parameter nodes past __svm_nodes";
          }
          if (node.w == 2u && !slot_ok((int)prog[off + 3].z)) {
            return "shader " + std::to_string(sh) + ": sky texture slot " + std::to_string((int)prog[off + 3].z) +
                   " was never allocated (tex_alloc)";
          }
          tex = true;
          break;
        case NODE_TEX_NOISE:
        case NODE_TEX_WAVE:
        case NODE_TEX_MUSGRAVE:
        case NODE_TEX_VORONOI:
          len = 3; /* two parameter nodes */
          tex = true;
          break;
        case NODE_TEX_MAGIC:
          len = 2;
          tex = true;
          break;
        case NODE_TEX_BRICK:
          len = 4;
          tex = true;
          break;
        case NODE_ATTR_BUMP_DX:
        case NODE_ATTR_BUMP_DY:
        case NODE_VERTEX_COLOR_BUMP_DX:
        case NODE_VERTEX_COLOR_BUMP_DY:
          *uses_ray_diff = true;
          /* fall through */
        case NODE_ATTR:
        case NODE_VERTEX_COLOR:
        case NODE_TANGENT:
          *uses_attr = true;
          tex = true;
          break;
        case NODE_NORMAL_MAP:
          *uses_attr |= (node.y >> 24) == 0u; /* tangent space reads the UV tangent attributes */
          tex = true;
          break;
        case NODE_OBJECT_INFO:
        case NODE_CAMERA:
        case NODE_VECTOR_ROTATE:
        case NODE_VECTOR_TRANSFORM:
          tex = true;
          break;
        case NODE_NORMAL:
          len = 2; /* direction node */
          tex = true;
          break;
        case NODE_RGB_CURVES:
        case NODE_VECTOR_CURVES:
          if (off + 1 >= n) {
            return "curves: table size node past __svm_nodes";
          }
          len = 2 + (size_t)prog[off + 1].x;
          tex = true;
          break;
        case NODE_GEOMETRY_BUMP_DX:
        case NODE_GEOMETRY_BUMP_DY:
          *uses_ray_diff = true;
          /* fall through */
        case NODE_GEOMETRY:
          *uses_attr |= node.y == 2u; /* Tangent: primitive_tangent reads the generated coordinates */
          tex = true;
          break;
        case NODE_TEX_WHITE_NOISE:
        case NODE_CONVERT:
        case NODE_HSV:
        case NODE_GAMMA:
        case NODE_BRIGHTCONTRAST:
        case NODE_LIGHT_PATH:
        case NODE_MAPPING:
        case NODE_TEX_GRADIENT:
        case NODE_TEX_CHECKER:
        case NODE_LIGHT_FALLOFF:
        case NODE_INVERT:
        case NODE_SEPARATE_VECTOR:
        case NODE_COMBINE_VECTOR:
          tex = true;
          break;
        default:
          return "shader " + std::to_string(sh) + ": SVM node " + std::to_string(node.x) + " is not implemented";
      }
      *uses_tex |= tex;
      if (len == 0) {
        int *m = volume ? volume_closures : surface_closures;
        *m = std::max(*m, closures);
        break;
      }
      off += len;
    }
  }
  return "";
}

int hipcy_load_kernels(hipcy_device *dev)
{
  if (!dev->have_data) {
    return set_error(dev, "load_kernels: KernelData not uploaded");
  }
  const hc_KernelData &d = dev->data_host;
  std::string why;
  if (d.cam.type < 0 || d.cam.type > 2) why = "unknown camera type";
  else if (d.cam.type == 2 && (d.cam.panorama_type < 0 || d.cam.panorama_type > 3)) why = "unknown panorama type";
  else if (d.cam.shuttertime != -1.0f || d.cam.num_motion_steps) why = "motion blur";
  else if (d.cam.interocular_offset != 0.0f) why = "stereo";
  else if (d.integrator.sampling_pattern != 0) why = "only the Sobol pattern";
  else if (d.integrator.use_volumes && !d.integrator.transparent_shadows)
    why = "volumes without transparent shadows (shader.cpp:529-536 sets them for every volume shader)";
  else if (d.integrator.transparent_shadows && d.integrator.transparent_max_bounce > CY_SHADOW_MAX_HITS)
    why = "transparent shadows deeper than " + std::to_string(CY_SHADOW_MAX_HITS) + " bounces";
  else if (d.integrator.transparent_shadows &&
           (d.integrator.max_bounce > 255 || d.integrator.transparent_max_bounce > 255))
    why = "transparent shadows with more than 255 bounces";
  else if (d.integrator.use_ambient_occlusion) why = "ambient occlusion";
  else if (d.integrator.adaptive_stop_per_sample)
    why = "adaptive_stop_per_sample (a CPU-device setting; this device filters at adaptive_step samples)";
  else if (d.background.portal_weight > 0.0f || d.background.num_portals) why = "light portals";
  else if (d.background.sun_weight > 0.0f) why = "sky texture sun sampling";
  else if (d.integrator.max_closures > CY_DEVICE_MAX_CLOSURE && !d.integrator.use_volumes)
    why = "max_closures > " + std::to_string(CY_DEVICE_MAX_CLOSURE);
  else if (d.bvh.have_motion || d.bvh.use_bvh_steps) why = "motion blur (motion triangles / curves)";
  else if (d.bvh.have_curves && (d.bvh.curve_subdivisions < 1 || d.bvh.curve_subdivisions > 16))
    why = "curve_subdivisions outside 1..16";
  else if (d.bvh.bvh_layout != 1) why = "bvh_layout must be BVH2";
  else if (d.film.use_light_pass && (d.film.light_pass_flag & ~CY_HOST_LIGHT_PASSES) != 0)
    why = "light passes other than mist, emission, background, shadow and the diffuse / glossy / transmission / "
          "volume direct, indirect and colour passes (no AO pass)";
  else if ((d.film.pass_flag & 2) == 0 || (d.film.pass_flag & ~(2 | CY_HOST_DATA_PASSES | (1 << 11) | (1 << 12) |
                                                                  (1 << 13) | (1 << 14))) != 0 ||
           d.film.pass_combined != 0)
    why = "only the combined pass (+ depth, normal, UV, object / material index, AOV color / value, adaptive aux "
          "buffer / sample count)";
  else if (d.film.pass_denoising_data || d.film.cryptomatte_passes)
    why = "denoising / cryptomatte passes";
  else if (d.film.pass_adaptive_aux_buffer && (d.integrator.adaptive_step <= 0 ||
                                              (d.integrator.adaptive_step & (d.integrator.adaptive_step - 1))))
    why = "adaptive_step must be a power of two";
  else if (d.background.map_weight > 0.0f &&
           (d.background.map_res_x <= 0 || d.background.map_res_y <= 0 ||
            dev->globals.find("__light_background_marginal_cdf") == dev->globals.end() ||
            dev->globals.find("__light_background_conditional_cdf") == dev->globals.end() ||
            dev->globals["__light_background_marginal_cdf"].bytes < (size_t)(d.background.map_res_y + 1) * 8 ||
            dev->globals["__light_background_conditional_cdf"].bytes <
                (size_t)(d.background.map_res_x + 1) * d.background.map_res_y * 8))
    why = "background map CDFs not bound at the map resolution";
  if (!why.empty()) {
    return set_error(dev, "load_kernels: unsupported scene feature: " + why);
  }
  const char *required[] = {"__bvh_nodes", "__bvh_leaf_nodes", "__prim_tri_verts", "__prim_tri_index",
                            "__prim_visibility", "__prim_index", "__prim_object", "__object_flag",
                            "__tri_shader", "__tri_vindex", "__svm_nodes", "__shaders",
                            "__lookup_table", "__sample_pattern_lut"};
  for (const char *r : required) {
    if (dev->globals.find(r) == dev->globals.end()) {
      return set_error(dev, std::string("load_kernels: array not bound: ") + r);
    }
  }
  dev->curve_shapes = 0;
  if (d.bvh.have_curves) {
    for (const char *r : {"__curves", "__curve_keys", "__prim_type"}) {
      if (dev->globals.find(r) == dev->globals.end()) {
        return set_error(dev, std::string("load_kernels: scene with curves, array not bound: ") + r);
      }
    }
    /* which curve shapes occur (selects the hair kernels: the thick
     * intersector alone sets their register budget) */
    const GlobalBinding &pt = dev->globals["__prim_type"];
    std::vector<uint32_t> types(pt.bytes / 4);
    if (!types.empty()) {
      HIP_CHECK(dev, hipSetDevice(dev->ordinal));
      HIP_CHECK(dev, hipMemcpy(types.data(), (const void *)pt.ptr, pt.bytes, hipMemcpyDeviceToHost));
    }
    for (uint32_t t : types) {
      if (t & (CY_PRIMITIVE_CURVE_RIBBON | CY_PRIMITIVE_MOTION_CURVE_RIBBON)) {
        dev->curve_shapes |= 1;
      }
      else if (t & (CY_PRIMITIVE_CURVE_THICK | CY_PRIMITIVE_MOTION_CURVE_THICK)) {
        dev->curve_shapes |= 2;
      }
    }
    if (dev->curve_shapes == 0) {
      dev->curve_shapes = 3;
    }
  }
  std::vector<uint32_t> shader_flags(dev->num_shaders, 0u);
  if (dev->num_shaders) {
    std::vector<hc_KernelShader> ks(dev->num_shaders);
    HIP_CHECK(dev, hipSetDevice(dev->ordinal));
    HIP_CHECK(dev, hipMemcpy(ks.data(), (const void *)dev->globals["__shaders"].ptr,
                             dev->num_shaders * sizeof(hc_KernelShader), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ks.size(); i++) {
      shader_flags[i] = (uint32_t)ks[i].flags;
    }
  }
  bool uses_bssrdf = false, uses_disk_bssrdf = false, uses_attr = false, uses_ray_diff = false, uses_ies = false;
  bool uses_particles = false;
  int surface_closures = 0, volume_closures = 0;
  why = svm_scan(dev->svm_nodes, dev->num_shaders, dev->tex_mem, shader_flags, &dev->shade_tex, &uses_bssrdf,
                 &uses_disk_bssrdf, &uses_attr, &uses_ray_diff, &uses_ies, &uses_particles, &surface_closures,
                 &volume_closures);
  if (why.empty() && uses_particles && dev->globals.find("__particles") == dev->globals.end()) {
    /* ParticleSystemManager::device_update_particles (particles.cpp:61-105) */
    why = "particle info node without the __particles table bound";
  }
  if (why.empty() && uses_ies && dev->globals.find("__ies") == dev->globals.end()) {
    /* LightManager::device_update_ies (light.cpp:1080-1125) */
    why = "IES texture without the __ies table bound";
  }
  if (why.empty() && uses_attr && dev->globals.find("__attributes_map") == dev->globals.end()) {
    /* the attribute nodes look attributes up through the objects' maps
     * (GeometryManager::device_update_attributes, geometry.cpp:379-474) */
    why = "attribute / texture coordinate (UV, Generated) / vertex color nodes without __attributes_map";
  }
  if (!why.empty()) {
    return set_error(dev, "load_kernels: unsupported shader: " + why);
  }
  /* the data passes (depth, normal, UV, object / material index) are written
   * by the extended shading kernels */
  if (d.film.pass_flag & CY_HOST_DATA_PASSES) {
    dev->shade_tex = true;
  }
  /* kernel_path_shader_apply (kernel_path.h:254-283): shadow-catcher objects
   * take the extended shading kernels (the catcher's part of PathRadiance per
   * slot, the all-lights connection behind a catcher) */
  dev->use_catcher = false;
  for (uint32_t f : dev->object_flags) {
    dev->use_catcher |= (f & SD_OBJECT_SHADOW_CATCHER) != 0;
  }
  if (dev->use_catcher) {
    if (d.integrator.use_volumes) {
      return set_error(dev, "load_kernels: unsupported scene feature: shadow catcher objects in a scene with volumes");
    }
    if (uses_bssrdf) {
      return set_error(dev, "load_kernels: unsupported scene feature: shadow catcher objects with subsurface "
                            "scattering");
    }
    dev->shade_tex = true;
  }
  /* kernel_branched_path_integrate (kernel_path_branched.h): the extended
   * shading kernels, each camera hit's indirect samples (and the camera ray
   * through transparency) waiting in CY_BR_RECS records per slot; not with
   * volumes, BSSRDFs or shadow catchers */
  dev->use_branched = d.integrator.branched != 0;
  if (dev->use_branched) {
    const int samples = std::max(d.integrator.diffuse_samples,
                                 std::max(d.integrator.glossy_samples, d.integrator.transmission_samples));
    if (d.integrator.use_volumes) {
      return set_error(dev, "load_kernels: unsupported scene feature: branched path tracing with volumes");
    }
    if (uses_bssrdf) {
      return set_error(dev, "load_kernels: unsupported scene feature: branched path tracing with subsurface "
                            "scattering");
    }
    if (dev->use_catcher) {
      return set_error(dev, "load_kernels: unsupported scene feature: branched path tracing with shadow catchers");
    }
    if ((size_t)d.integrator.max_closures * (size_t)std::max(samples, 1) + 1 > (size_t)CY_BR_RECS + 1) {
      return set_error(dev, "load_kernels: branched path tracing with up to " +
                                std::to_string(d.integrator.max_closures) + " closures x " + std::to_string(samples) +
                                " samples: more waiting paths than the device's " + std::to_string(CY_BR_RECS) +
                                " per slot");
    }
    dev->shade_tex = true;
  }
  /* kernel_write_light_passes (kernel_passes.h:285-337): the extended shading
   * kernels keep the path's PathRadiance components in a record per slot;
   * not with volumes, BSSRDFs, shadow catchers or branched path tracing */
  dev->use_lightpass = d.film.use_light_pass != 0;
  if (dev->use_lightpass) {
    const char *with = d.integrator.use_volumes ? "volumes"
                       : uses_bssrdf            ? "subsurface scattering"
                       : dev->use_catcher       ? "shadow catchers"
                       : dev->use_branched      ? "branched path tracing"
                                                : nullptr;
    if (with) {
      return set_error(dev, std::string("load_kernels: unsupported scene feature: light passes with ") + with);
    }
    dev->shade_tex = true;
  }
  dev->shade_ext = dev->use_catcher || dev->use_branched || dev->use_lightpass;
  dev->use_volumes = d.integrator.use_volumes != 0;
  dev->use_decoupled = dev->use_volumes && d.integrator.volume_decoupled != 0;
  /* every volume scene takes the _vext variants: the _vol build (the volume
   * extras compiled out, CY_VOLUME_EXT = 0) rendered volume_cornell,
   * volume_hetero, shading_voxel and the JNK crop wrong on the GPU while its
   * host emulation matched, so it is not built */
  dev->shade_vext = dev->use_volumes;
  dev->use_disk_bssrdf = uses_disk_bssrdf;
  dev->use_ray_diff = uses_ray_diff;
  dev->shade_closures = d.integrator.max_closures;
  if (dev->use_volumes) {
    /* the volume stack of a path holds the world and every volume object it
     * is inside of (plus the terminator) */
    size_t volume_objects = 0;
    bool volume_attributes = false;
    for (uint32_t f : dev->object_flags) {
      volume_objects += (f & SD_OBJECT_HAS_VOLUME) ? 1 : 0;
      volume_attributes |= (f & SD_OBJECT_HAS_VOLUME_ATTRIBUTES) != 0;
    }
    /* the volume stack's shaders evaluate into one closure array (merged
     * when their phase closures are equal): a bound on what a shading
     * point allocates selects the array (the reference's max_closures
     * reserves VOLUME_STACK_SIZE per volume closure, never reached here) */
    const int bound = std::max(std::min(surface_closures, (int)d.integrator.max_closures),
                               (int)(volume_objects + 1) * volume_closures);
    dev->shade_closures = std::max(bound, 1);
    if (bound > CY_DEVICE_MAX_CLOSURE) {
      why = "volume scene needing " + std::to_string(bound) + " closures > " + std::to_string(CY_DEVICE_MAX_CLOSURE);
    }
    else if (volume_objects + 2 > CY_VOLUME_STACK) {
      why = "more than " + std::to_string(CY_VOLUME_STACK - 2) + " volume objects (the device's volume stack)";
    }
    else if (volume_attributes) {
      why = "volume attributes (voxel grids)";
    }
    else if (volume_objects && dev->globals.find("__object_volume_step") == dev->globals.end()) {
      why = "volume objects without __object_volume_step";
    }
    if (!why.empty()) {
      return set_error(dev, "load_kernels: unsupported scene feature: " + why);
    }
    dev->shade_tex = true;
  }
  /* instanced geometry present? (selects the traversal kernels with instance
   * leaves and the instance paths of shading) */
  dev->have_instancing = 0;
  for (uint32_t f : dev->object_flags) {
    if (!(f & SD_OBJECT_TRANSFORM_APPLIED)) {
      dev->have_instancing = 1;
    }
  }
  /* scene-preparation step of the device: widen the BVH now, not in the first render */
  if (ensure_bvhw(dev) != 0) {
    return -1;
  }
  dev->features_dirty = false;
  return 0;
}

int hipcy_set_profiling(hipcy_device *dev, int flags)
{
  dev->profiling = flags;
  return 0;
}

int hipcy_get_stats(const hipcy_device *dev, hipcy_stats *out)
{
  *out = dev->stats;
  return 0;
}

int hipcy_synchronize(hipcy_device *dev)
{
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return dev->error.empty() ? 0 : -1;
}

static hipEvent_t get_event(hipcy_device *dev, size_t i)
{
  while (dev->events.size() <= i) {
    hipEvent_t e;
    hipEventCreate(&e);
    dev->events.push_back(e);
  }
  return dev->events[i];
}

static int check_device_error(hipcy_device *dev)
{
  uint err = dev->host_counters[3];
  if (err) {
    const uint code = err >> 24, detail = err & 0xFFFFFF;
    static const char *names[] = {"none", "unsupported SVM node", "unsupported closure",
                                  "SVM stack offset beyond HIP stack", "BVH stack overflow",
                                  "unsupported primitive", "unsupported scene feature"};
    return set_error(dev, std::string("kernel error: ") + (code < 7 ? names[code] : "?") + " (" +
                              std::to_string(detail) + ")");
  }
  return 0;
}

static int path_trace(hipcy_device *dev, const hipcy_work_tile *tiles, int n_tiles, int y_step);

int hipcy_path_trace(hipcy_device *dev, const hipcy_work_tile *t)
{
  return path_trace(dev, t, 1, 1);
}

int hipcy_path_trace_rows(hipcy_device *dev, const hipcy_work_tile *t, int y_step)
{
  return path_trace(dev, t, 1, y_step < 1 ? 1 : y_step);
}

int hipcy_path_trace_tiles(hipcy_device *dev, const hipcy_work_tile *tiles, int n_tiles)
{
  return path_trace(dev, tiles, n_tiles, 1);
}

static int ensure_records(hipcy_device *dev, size_t n)
{
  if (n <= dev->records_capacity) {
    return 0;
  }
  if (dev->records) {
    HIP_CHECK(dev, hipFree(dev->records));
    dev->records = nullptr;
  }
  HIP_CHECK(dev, hipMalloc((void **)&dev->records, n * sizeof(hc_float4)));
  dev->records_capacity = n;
  return 0;
}

struct EvQuad {
  hipEvent_t a, b, c, d;
};

/* One partition of the slot pool with its own stream, queues and counters. */
struct PassLane {
  hipStream_t s;
  int index;
  int slot_base;
  int cam_n; /* > 0 until the lane's camera launch is enqueued */
  uint *cnt;  /* device: [0..2] queue counts, [4] next item */
  uint *hcnt; /* pinned host copy */
  int *q[3];
  int qa, qb;
  uint n_active;
  CyTile tile;
  hipEvent_t done;
  bool stream = false;  /* tile stream lane */
  bool min_live = false; /* tile stream: also reduce the live paths' smallest item */
  bool tail = false;     /* the lane's fused tail (k_tail) is enqueued: its last launch */
};

/* The queue sort in effect: the requested mode, or (automatic, -1) the
 * shading-queue sort when the scene runs the extended shading kernel without
 * curves -- measured: production-material BMW 272 -> 423, CLS 93 -> 116
 * Msamples/s, while the plain kernel's scenes lose by it (BMW 1241 -> 1207,
 * BBS 245 -> 187) and the hair scene is flat (profiles/r04/sort_*.json). */
static int effective_sort(const hipcy_device *dev)
{
  if (dev->ray_sort >= 0) {
    return dev->ray_sort;
  }
  return (dev->shade_tex && !dev->data_host.bvh.have_curves) ? 8 : 0;
}

/* One iteration of a lane: closest -> shade -> shadow.  The lane's first
 * iteration is its camera launch (cam_n > 0): slot slot_base + i starts work
 * item item_base + i, and the closest and shade kernels generate its camera
 * ray themselves (no slot initialisation pass). */
static int lane_iterate(hipcy_device *dev, const CyGlobals &kg, PassLane &ln, int W, size_t *ev,
                        std::vector<EvQuad> *quads)
{
  const bool prof = (dev->profiling & 1) != 0;
  const bool counters = (dev->profiling & 2) != 0;
  hipStream_t s = ln.s;
  uint *err = dev->counters + 3;
  const int qa = ln.qa, qb = ln.qb, qs = 2;
  const int cam_n = ln.cam_n;
  ln.cam_n = 0;
  dev->stats.iterations++;
  dev->stats.closest_rays += ln.n_active;
  HIP_CHECK(dev, hipMemsetAsync(ln.cnt + qb, 0, 4, s));
  HIP_CHECK(dev, hipMemsetAsync(ln.cnt + qs, 0, 4, s));
  dim3 grid((ln.n_active + CY_BLOCK - 1) / CY_BLOCK), block(CY_BLOCK);
  /* bounce iterations: bin the closest queue by ray direction (counting sort
   * into sort_queue); closest and shade then read the sorted queue */
  const int *queue_in = ln.q[qa];
  /* sort buffers exist only where a pass sized them (path_trace_pass) */
  const int sort = (dev->sort_queue && dev->sort_capacity >= dev->capacity) ? effective_sort(dev) : 0;
  if ((sort == 3 || sort == 5) && cam_n == 0 && ln.n_active >= 4 * CY_BLOCK) {
    const int nblocks = (int)grid.x;
    const int K = sort == 3 ? 8 : CY_SORT_BINS;
    uint *hist = dev->sort_hist + (size_t)CY_SORT_BINS * (ln.slot_base / CY_BLOCK + ln.index);
    unsigned char *keys = dev->sort_key + ln.slot_base;
    int *sorted = dev->sort_queue + ln.slot_base;
    hipLaunchKernelGGL(sort == 3 ? k_sort_count<3> : k_sort_count<5>, grid, block, 0, s, dev->bufs,
                       ln.q[qa], ln.cnt + qa, keys, hist, nblocks);
    hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, hist, K * nblocks);
    hipLaunchKernelGGL(sort == 3 ? k_sort_scatter<3> : k_sort_scatter<5>, grid, block, 0, s, ln.q[qa],
                       ln.cnt + qa, keys, hist, nblocks, sorted);
    queue_in = sorted;
  }
  EvQuad p;
  if (prof) {
    p.a = get_event(dev, (*ev)++);
    p.b = get_event(dev, (*ev)++);
    p.c = get_event(dev, (*ev)++);
    p.d = get_event(dev, (*ev)++);
    HIP_CHECK(dev, hipEventRecord(p.a, s));
  }
  /* iteration budget: non-instanced wide BVH only (the kernels' CAN_SUSPEND) */
  const bool budget = dev->trav_budget[0] > 0 && W > 2 && !kg.have_instancing && !kg.have_curves && dev->cont_rec;
  CyCont ca = {}, cb = {};
  if (budget) {
    const size_t cap = dev->cont_capacity;
    ca.rec = dev->cont_rec + (size_t)(2 * ln.index) * CY_CONT_F4 * cap;
    cb.rec = ca.rec + CY_CONT_F4 * cap;
    ca.capacity = cb.capacity = (uint)cap;
    ca.count = ln.cnt + 8;
    cb.count = ln.cnt + 9;
  }
  /* closest, then (budget) the continuations: A -> B with the second budget,
   * B to the end */
  auto continuations = [&](bool shadow) -> int {
    HIP_CHECK(dev, hipMemsetAsync(cb.count, 0, 4, s));
    for (int k = 0; k < 2; k++) {
      const CyCont &in = k == 0 ? ca : cb;
      const CyCont &out = k == 0 ? cb : ca;
      const int bud = k == 0 ? dev->trav_budget[1] : 0;
      if (!shadow) {
        auto kfn = W == 8 ? pick_closest_cont<8>(counters) : pick_closest_cont<4>(counters);
        hipLaunchKernelGGL(kfn, dim3(CY_CONT_BLOCKS), block, 0, s, kg, dev->bufs, in, out, bud, err, dev->stats_dev);
      }
      else {
        auto kfn = W == 8 ? pick_shadow_cont<8>(counters) : pick_shadow_cont<4>(counters);
        hipLaunchKernelGGL(kfn, dim3(CY_CONT_BLOCKS), block, 0, s, kg, dev->bufs, ln.tile, in, out, bud, ln.q[qb],
                           ln.cnt + qb, err, dev->stats_dev);
      }
    }
    return 0;
  };
  {
    if (budget) {
      HIP_CHECK(dev, hipMemsetAsync(ca.count, 0, 4, s));
    }
    if (budget) {
      auto kfn = counters ? (W == 8 ? k_intersect_closest_budget<true, 8> : k_intersect_closest_budget<true, 4>)
                          : (W == 8 ? k_intersect_closest_budget<false, 8> : k_intersect_closest_budget<false, 4>);
      hipLaunchKernelGGL(kfn, grid, block, 0, s, kg, dev->bufs, ln.tile, cam_n, ln.slot_base, queue_in,
                         ln.cnt + qa, err, dev->stats_dev, dev->trav_budget[0], ca);
      if (continuations(false) != 0) {
        return -1;
      }
    }
    else if (dev->trav_refill[0] > 0 && W > 2 && !kg.have_instancing && !kg.have_curves) {
      /* persistent waves with lane refill (k_closest_refill) */
      if (!dev->refill_claim) {
        HIP_CHECK(dev, hipMalloc((void **)&dev->refill_claim, (size_t)CY_LANES * 8 * sizeof(uint)));
      }
      uint *claim = dev->refill_claim + 8 * ln.index;
      HIP_CHECK(dev, hipMemsetAsync(claim, 0, 8 * sizeof(uint), s));
      if (cam_n > 0) {
        hipLaunchKernelGGL(k_camera_rays, dim3((cam_n + CY_BLOCK - 1) / CY_BLOCK), block, 0, s, kg, dev->bufs,
                           ln.tile, cam_n, ln.slot_base);
      }
      auto kfn = counters ? (W == 8 ? k_closest_refill<true, 8> : k_closest_refill<true, 4>)
                          : (W == 8 ? k_closest_refill<false, 8> : k_closest_refill<false, 4>);
      hipLaunchKernelGGL(kfn, dim3(std::min<uint>(CY_REFILL_BLOCKS, grid.x)), block, 0, s, kg, dev->bufs, cam_n,
                         ln.slot_base, queue_in, ln.cnt + qa, claim, err, dev->stats_dev, dev->trav_refill[0],
                         dev->trav_refill[1]);
    }
    else {
      auto kfn = pick_kernel<ClosestK>(counters, W, kg.have_instancing != 0, dev->curve_shapes);
      hipLaunchKernelGGL(kfn, grid, block, 0, s, kg, dev->bufs, ln.tile, cam_n, ln.slot_base, queue_in,
                         ln.cnt + qa, err, dev->stats_dev);
    }
  }
  if (prof) {
    HIP_CHECK(dev, hipEventRecord(p.b, s));
  }
  const int *shade_queue = queue_in;
  if (sort == 8 && cam_n == 0 && ln.n_active >= 4 * CY_BLOCK) {
    /* shading-queue sort by the hit's shader (k_shade_sort_count) */
    const int nblocks = (int)grid.x;
    uint *hist = dev->sort_hist + (size_t)CY_SORT_BINS * (ln.slot_base / CY_BLOCK + ln.index);
    unsigned char *keys = dev->sort_key + ln.slot_base;
    int *sorted = dev->sort_queue + ln.slot_base;
    hipLaunchKernelGGL(k_shade_sort_count, grid, block, 0, s, kg, dev->bufs, queue_in, ln.cnt + qa, keys, hist,
                       nblocks);
    hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, hist, CY_SORT_BINS * nblocks);
    hipLaunchKernelGGL(k_sort_scatter<5>, grid, block, 0, s, queue_in, ln.cnt + qa, keys, hist, nblocks, sorted);
    shade_queue = sorted;
  }
  cy_launch_shade(dev->shade_closures, dev->shade_tex, dev->use_volumes, dev->shade_ext, dev->shade_vext, grid,
                  block, s, kg,
                  dev->bufs, ln.tile, cam_n,
                  ln.slot_base, shade_queue, ln.cnt + qa, ln.q[qb], ln.cnt + qb, ln.q[qs], ln.cnt + qs, err);
  if (prof) {
    HIP_CHECK(dev, hipEventRecord(p.c, s));
  }
  if (dev->data_host.integrator.transparent_shadows) {
    if (dev->bufs.shadow_nrec) {
      const int hair = kg.have_curves ? dev->curve_shapes : 0;
      auto krec = hair == 0 ? k_shadow_record<0> : hair == 1 ? k_shadow_record<1> :
                  hair == 2 ? k_shadow_record<2> : k_shadow_record<3>;
      hipLaunchKernelGGL(krec, grid, block, 0, s, kg, dev->bufs, ln.q[qs], ln.cnt + qs, err);
    }
    auto kfn = dev->use_volumes ? k_intersect_shadow_transparent<true> : k_intersect_shadow_transparent<false>;
    hipLaunchKernelGGL(kfn, grid, block, 0, s, kg, dev->bufs, ln.tile, ln.q[qs], ln.cnt + qs, ln.q[qb], ln.cnt + qb,
                       err);
  }
  else {
    if (budget) {
      HIP_CHECK(dev, hipMemsetAsync(ca.count, 0, 4, s));
    }
    if (budget) {
      auto kfn = counters ? (W == 8 ? k_intersect_shadow_budget<true, 8> : k_intersect_shadow_budget<true, 4>)
                          : (W == 8 ? k_intersect_shadow_budget<false, 8> : k_intersect_shadow_budget<false, 4>);
      hipLaunchKernelGGL(kfn, grid, block, 0, s, kg, dev->bufs, ln.tile, ln.q[qs], ln.cnt + qs, ln.q[qb],
                         ln.cnt + qb, err, dev->stats_dev, dev->trav_budget[0], ca);
      if (continuations(true) != 0) {
        return -1;
      }
    }
    else if (dev->trav_refill[0] > 0 && W > 2 && !kg.have_instancing && !kg.have_curves) {
      uint *claim = dev->refill_claim + 8 * ln.index;
      HIP_CHECK(dev, hipMemsetAsync(claim, 0, 8 * sizeof(uint), s));
      auto kfn = counters ? (W == 8 ? k_shadow_refill<true, 8> : k_shadow_refill<true, 4>)
                          : (W == 8 ? k_shadow_refill<false, 8> : k_shadow_refill<false, 4>);
      hipLaunchKernelGGL(kfn, dim3(std::min<uint>(CY_REFILL_BLOCKS, grid.x)), block, 0, s, kg, dev->bufs, ln.q[qs],
                         ln.cnt + qs, claim, err, dev->stats_dev, dev->trav_refill[0], dev->trav_refill[1]);
      hipLaunchKernelGGL(k_shadow_finish, grid, block, 0, s, kg, dev->bufs, ln.tile, ln.q[qs], ln.cnt + qs,
                         ln.q[qb], ln.cnt + qb);
    }
    else {
      const int *shadow_queue = ln.q[qs];
      if (dev->shadow_sort && dev->sort_queue && dev->sort_capacity >= dev->capacity &&
          ln.n_active >= 4 * CY_BLOCK) {
        /* shadow-queue sort (hipcy_set_shadow_sort): the sort buffers are free
         * again once shading has read the closest queue (same stream) */
        const int nblocks = (int)grid.x;
        const int K = dev->shadow_sort == 3 ? 8 : CY_SORT_BINS;
        uint *hist = dev->sort_hist + (size_t)CY_SORT_BINS * (ln.slot_base / CY_BLOCK + ln.index);
        unsigned char *keys = dev->sort_key + ln.slot_base;
        int *sorted = dev->sort_queue + ln.slot_base;
        auto kcount = dev->shadow_sort == 3 ? k_sort_count<3, true> : k_sort_count<5, true>;
        hipLaunchKernelGGL(kcount, grid, block, 0, s, dev->bufs, ln.q[qs], ln.cnt + qs, keys, hist, nblocks);
        hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, hist, K * nblocks);
        hipLaunchKernelGGL(dev->shadow_sort == 3 ? k_sort_scatter<3> : k_sort_scatter<5>, grid, block, 0, s, ln.q[qs],
                           ln.cnt + qs, keys, hist, nblocks, sorted);
        shadow_queue = sorted;
      }
      auto kfn = pick_kernel<ShadowK>(counters, W, kg.have_instancing != 0, dev->curve_shapes);
      CyGlobals kgs = kg; /* its own count of LDS-resident top nodes (CY_LDS_TOP_SHADOW) */
      kgs.bvhw_top = std::min(kg.bvhw_top > 0 ? dev->bvhw_top_shadow : 0, dev->bvhw_top_shadow);
      hipLaunchKernelGGL(kfn, grid, block, 0, s, kgs, dev->bufs, ln.tile, shadow_queue, ln.cnt + qs, ln.q[qb],
                         ln.cnt + qb, err, dev->stats_dev);
    }
  }
  if (prof) {
    HIP_CHECK(dev, hipEventRecord(p.d, s));
    quads->push_back(p);
  }
  if (ln.stream && ln.min_live) {
    /* tile streams: the smallest item still held by a live path (min_live
     * shards) and the next unclaimed item (cnt[4]) tell the host which tiles
     * are done */
    uint *shards = dev->min_live_dev + CY_MIN_SHARDS * ln.index;
    HIP_CHECK(dev, hipMemsetAsync(shards, 0xFF, CY_MIN_SHARDS * 4, s));
    hipLaunchKernelGGL(k_stream_min_live, grid, block, 0, s, ln.q[qb], ln.cnt + qb, dev->bufs.item, shards);
    HIP_CHECK(dev, hipMemcpyAsync(dev->min_live_host + CY_MIN_SHARDS * ln.index, shards, CY_MIN_SHARDS * 4,
                                  hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(dev, hipGetLastError());
  /* the queue counts and the next unclaimed item (cnt[4]) */
  HIP_CHECK(dev, hipMemcpyAsync(ln.hcnt, ln.cnt, 20, hipMemcpyDeviceToHost, s));
  /* the kernels' error word, read with the lane's counts */
  HIP_CHECK(dev, hipMemcpyAsync(ln.hcnt + 6, err, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(dev, hipEventRecord(ln.done, s));
  return 0;
}

/* Whether the pass may end its lanes with the fused tail kernel (k_shade.hip
 * k_tail_*): the plain shading variants, triangle scenes with opaque shadows,
 * no traversal budget / lane refill, no per-kernel timing. */
static bool tail_allowed(const hipcy_device *dev, const CyGlobals &kg)
{
  return dev->tail_paths > 0 && dev->profiling == 0 && !kg.have_curves &&
         !dev->data_host.integrator.transparent_shadows && dev->trav_budget[0] == 0 && dev->trav_refill[0] == 0 &&
         !dev->shade_tex && !dev->use_volumes && dev->shade_closures <= 8;
}

/* The lane's last launch: its live paths (queue qa) run to their ends in one
 * k_tail launch; the rays it traced come back in cnt[13] / cnt[14]. */
static int lane_tail(hipcy_device *dev, const CyGlobals &kg, PassLane &ln, int W)
{
  hipStream_t s = ln.s;
  uint *err = dev->counters + 3;
  dev->stats.iterations++;
  HIP_CHECK(dev, hipMemsetAsync(ln.cnt + 13, 0, 12, s)); /* ray counts and the take-next counter */
  const dim3 grid((ln.n_active + CY_BLOCK - 1) / CY_BLOCK), block(CY_BLOCK);
  if (!cy_launch_tail(dev->shade_closures, dev->shade_tex, dev->use_volumes, W, kg.have_instancing != 0, grid, block,
                      s, kg, dev->bufs, ln.tile, ln.q[ln.qa], ln.cnt + ln.qa, ln.cnt + 13, err)) {
    return set_error(dev, "path_trace: no tail kernel for this shading variant");
  }
  HIP_CHECK(dev, hipGetLastError());
  HIP_CHECK(dev, hipMemcpyAsync(ln.hcnt, ln.cnt, 16 * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(dev, hipMemcpyAsync(ln.hcnt + 6, err, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(dev, hipEventRecord(ln.done, s));
  ln.tail = true;
  return 0;
}

/* Queue-sort buffers (hipcy_set_ray_sort) sized to the slot pool: called after
 * ensure_capacity by every entry that iterates lanes (path_trace_pass and the
 * tile stream), so the automatic shading-queue sort runs on both. */
static int ensure_sort(hipcy_device *dev)
{
  if ((effective_sort(dev) || dev->shadow_sort) && dev->sort_capacity < dev->capacity) {
    const size_t cap = dev->capacity;
    if (dev->sort_queue) HIP_CHECK(dev, hipFree(dev->sort_queue));
    if (dev->sort_key) HIP_CHECK(dev, hipFree(dev->sort_key));
    if (dev->sort_hist) HIP_CHECK(dev, hipFree(dev->sort_hist));
    dev->sort_queue = nullptr;
    dev->sort_key = nullptr;
    dev->sort_hist = nullptr;
    dev->sort_capacity = 0;
    HIP_CHECK(dev, hipMalloc((void **)&dev->sort_queue, cap * sizeof(int)));
    HIP_CHECK(dev, hipMalloc((void **)&dev->sort_key, cap));
    /* lane l's histogram starts at CY_SORT_BINS * (slot_base / CY_BLOCK + l) */
    HIP_CHECK(dev, hipMalloc((void **)&dev->sort_hist,
                             (size_t)CY_SORT_BINS * (cap / CY_BLOCK + CY_LANES + 1) * sizeof(uint)));
    dev->sort_capacity = cap;
  }
  return 0;
}

/* One pass over samples [tile.start_sample, tile.end_sample) of the tile: the
 * items are split into CY_LANES contiguous ranges, each iterated by its own
 * slot partition on its own stream; the host enqueues one iteration of every
 * active lane, then waits for their queue counts. */
static int path_trace_pass(hipcy_device *dev, const CyGlobals &kg, CyTile tile, int W, size_t *ev,
                           std::vector<EvQuad> *quads)
{
  const size_t n_slots = std::min<size_t>(std::min<size_t>(tile.n_items, dev->capacity), slot_limit(dev));
  /* per-kernel event timing (profiling bit 0) needs kernels that do not
   * overlap: one lane then */
  const int max_lanes = (dev->profiling & 1) ? 1 : CY_LANES;
  const int lanes = (int)std::max<size_t>(1, std::min<size_t>(max_lanes, n_slots / (4 * CY_BLOCK)));
  tile.samples_out = dev->records;
  if (ensure_sort(dev) != 0) {
    return -1;
  }
  if (dev->trav_budget[0] > 0 && W > 2 && !kg.have_instancing && !kg.have_curves) {
    /* continuation records: per lane two buffers of a quarter of the lane's
     * slots; HIPCY_CONT_CAPACITY overrides the size (tests force the
     * buffer-full path, where a suspended traversal finishes in place) */
    size_t cap = std::max<size_t>(65536, (n_slots / lanes + 3) / 4);
    if (const char *env = getenv("HIPCY_CONT_CAPACITY")) {
      cap = std::max<size_t>(1, (size_t)strtoull(env, nullptr, 10));
    }
    if (cap != dev->cont_capacity || lanes > (int)dev->cont_lanes) {
      if (dev->cont_rec) {
        HIP_CHECK(dev, hipFree(dev->cont_rec));
        dev->cont_rec = nullptr;
      }
      dev->cont_capacity = 0;
      HIP_CHECK(dev, hipMalloc((void **)&dev->cont_rec, (size_t)2 * CY_LANES * CY_CONT_F4 * cap * sizeof(hc_float4)));
      dev->cont_capacity = cap;
      dev->cont_lanes = CY_LANES;
    }
  }
  PassLane ln[CY_LANES];
  /* the main stream's pending work (buffer zeroing, uploads) precedes the lanes */
  hipEvent_t start = get_event(dev, (*ev)++);
  HIP_CHECK(dev, hipEventRecord(start, dev->stream));
  for (int l = 0; l < lanes; l++) {
    PassLane &L = ln[l];
    L.index = l;
    L.s = dev->lane_stream[l];
    HIP_CHECK(dev, hipStreamWaitEvent(L.s, start, 0));
    L.slot_base = (int)(n_slots * l / lanes);
    const int lane_slots = (int)(n_slots * (l + 1) / lanes) - L.slot_base;
    L.cnt = dev->counters + 16 * (l + 1);
    L.hcnt = dev->host_counters + 16 * (l + 1);
    L.qa = 0;
    L.qb = 1;
    L.done = get_event(dev, (*ev)++);
    L.tile = tile;
    const uint begin = (uint)((uint64_t)tile.n_items * l / lanes);
    L.tile.n_items = (uint)((uint64_t)tile.n_items * (l + 1) / lanes);
    L.tile.work_next = L.cnt + 4;
    L.tile.item_base = begin;
    /* camera launch: one item per slot of the lane */
    L.cam_n = (int)std::min<uint>((uint)lane_slots, L.tile.n_items - begin);
    L.n_active = (uint)L.cam_n;
    for (int q = 0; q < 3; q++) {
      L.q[q] = dev->queue[q] + L.slot_base;
    }
    L.hcnt[4] = begin + (uint)L.cam_n;
    HIP_CHECK(dev, hipMemsetAsync(L.cnt, 0, 12, L.s));
    HIP_CHECK(dev, hipMemcpyAsync(L.cnt + 4, L.hcnt + 4, 4, hipMemcpyHostToDevice, L.s));
  }
  /* lanes in submission order: the oldest lane's iteration is waited for,
   * and its next one enqueued at once, while the other lanes run */
  int fifo[CY_LANES];
  int head = 0, n_fifo = 0;
  for (int l = 0; l < lanes; l++) {
    if (ln[l].n_active > 0) {
      if (lane_iterate(dev, kg, ln[l], W, ev, quads) != 0) {
        return -1;
      }
      fifo[(head + n_fifo++) % CY_LANES] = l;
    }
  }
  dev->host_counters[3] = 0;
  const bool tail_ok = tail_allowed(dev, kg);
  while (n_fifo > 0) {
    PassLane &L = ln[fifo[head]];
    head = (head + 1) % CY_LANES;
    n_fifo--;
    HIP_CHECK(dev, hipEventSynchronize(L.done));
    if (L.tail) {
      /* the fused tail ran every remaining path of the lane to its end */
      dev->stats.closest_rays += L.hcnt[13];
      dev->stats.shadow_rays += L.hcnt[14];
      if (L.hcnt[6]) {
        dev->host_counters[3] = L.hcnt[6];
        break;
      }
      continue;
    }
    dev->stats.shadow_rays += L.hcnt[2];
    L.n_active = L.hcnt[L.qb];
    std::swap(L.qa, L.qb);
    if (L.hcnt[6]) {
      dev->host_counters[3] = L.hcnt[6];
      break;
    }
    if (L.n_active > 0) {
      /* every item of the lane claimed and few paths left: the fused tail */
      const bool tail = tail_ok && L.n_active <= dev->tail_paths && L.hcnt[4] >= L.tile.n_items;
      if ((tail ? lane_tail(dev, kg, L, W) : lane_iterate(dev, kg, L, W, ev, quads)) != 0) {
        return -1;
      }
      fifo[(head + n_fifo++) % CY_LANES] = L.index;
    }
  }
  /* all lanes finished: accumulate on the main stream after them */
  for (int l = 0; l < lanes; l++) {
    HIP_CHECK(dev, hipEventRecord(ln[l].done, ln[l].s));
    HIP_CHECK(dev, hipStreamWaitEvent(dev->stream, ln[l].done, 0));
  }
  const int npix = (int)tile.npix;
  hipLaunchKernelGGL(k_accumulate, dim3((unsigned)((npix + CY_BLOCK - 1) / CY_BLOCK)), dim3(CY_BLOCK), 0,
                     dev->stream, tile);
  HIP_CHECK(dev, hipGetLastError());
  return 0;
}

static int path_trace(hipcy_device *dev, const hipcy_work_tile *tiles, int n_tiles, int y_step)
{
  if (!dev->error.empty()) {
    return -1;
  }
  if (n_tiles < 1 || (n_tiles > 1 && y_step != 1)) {
    return set_error(dev, "path_trace: invalid tile set");
  }
  const hipcy_work_tile *t = &tiles[0];
  for (int k = 1; k < n_tiles; k++) {
    if (tiles[k].start_sample != t->start_sample || tiles[k].num_samples != t->num_samples) {
      return set_error(dev, "path_trace_tiles: all tiles of a pass must render the same sample range");
    }
  }
  /* re-validate only after the scene changed (Scene::device_update) */
  if (dev->features_dirty && hipcy_load_kernels(dev) != 0) {
    return -1;
  }
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  /* pixels of the pass, numbered tile by tile */
  std::vector<CyTileDesc> descs;
  size_t npix = 0;
  for (int k = 0; k < n_tiles; k++) {
    const hipcy_work_tile &tk = tiles[k];
    if (tk.w < 0 || tk.h < 0 || (tk.w * tk.h > 0 && !tk.buffer)) {
      return set_error(dev, "path_trace: invalid tile");
    }
    if ((size_t)tk.w * tk.h == 0) {
      continue;
    }
    CyTileDesc d;
    d.x = tk.x;
    d.y = tk.y;
    d.w = tk.w;
    d.h = tk.h;
    d.offset = tk.offset;
    d.stride = tk.stride;
    d.buffer = (float *)tk.buffer;
    d.px_begin = (uint)npix;
    d.start_sample = tk.start_sample;
    d.item_begin = 0;
    d.num_samples = tk.num_samples;
    d.group_npix = 0; /* tile streams only */
    d.group_first = 0;
    descs.push_back(d);
    npix += (size_t)tk.w * tk.h;
  }
  if (npix == 0 || t->num_samples <= 0) {
    return 0;
  }
  if (npix > 0xFFFFFFFFull) {
    return set_error(dev, "path_trace: tile set too large for 32-bit work items");
  }
  if (descs.size() > 1) {
    const size_t bytes = descs.size() * sizeof(CyTileDesc);
    if (bytes > dev->tile_descs_capacity) {
      if (dev->tile_descs) {
        HIP_CHECK(dev, hipFree(dev->tile_descs));
        dev->tile_descs = nullptr;
      }
      HIP_CHECK(dev, hipMalloc((void **)&dev->tile_descs, bytes));
      dev->tile_descs_capacity = bytes;
    }
    HIP_CHECK(dev, hipMemcpyAsync(dev->tile_descs, descs.data(), bytes, hipMemcpyHostToDevice, dev->stream));
  }
  /* samples per pass: as many as the record budget holds for these pixels */
  size_t per_pass = std::max<size_t>(
      1, std::min<size_t>((size_t)t->num_samples, dev->record_budget / (npix * sizeof(hc_float4))));
  /* adaptive sampling: passes of adaptive_step samples (AdaptiveSampling::
   * align_static_samples, device_task.cpp:147-163, of a step that size), so
   * the stopping / filter kernels run at every need_filter sample, as the
   * CPU device does them per sample */
  const hc_KernelFilm &film = dev->data_host.film;
  const hc_KernelIntegrator &integ = dev->data_host.integrator;
  const bool adaptive = film.pass_adaptive_aux_buffer != 0;
  if (adaptive) {
    if (y_step != 1) {
      return set_error(dev, "path_trace_rows: adaptive sampling needs whole tiles (shard by tiles)");
    }
    const size_t step = (size_t)integ.adaptive_step;
    if (per_pass >= step) {
      per_pass = step;
    }
    else {
      while (step % per_pass != 0) {
        per_pass--;
      }
    }
  }
  if (npix * per_pass > 0xFFFFFFFFull) {
    return set_error(dev, "path_trace: tile too large for 32-bit work items");
  }
  const size_t items = npix * per_pass;
  if (ensure_capacity(dev, std::min(items, dev->slots_wanted)) != 0 || ensure_volume_capacity(dev) != 0 ||
      ensure_sss_capacity(dev) != 0 || ensure_catcher_capacity(dev) != 0 || ensure_branch_capacity(dev) != 0 || ensure_lightpass_capacity(dev) != 0 || ensure_diff_capacity(dev) != 0 ||
      ensure_srec_capacity(dev) != 0 ||
      ensure_records(dev, items) != 0 || ensure_bvhw(dev) != 0) {
    return -1;
  }
  CyGlobals kg;
  build_globals(dev, &kg);
  const int W = kg.bvhw_nodes ? dev->bvh_width : 2;

  memset(&dev->stats, 0, sizeof(dev->stats));
  dev->stats.bvh_width = W;
  dev->stats.bvh_depth = W > 2 ? dev->bvhw_depth : 0;
  {
    auto it = dev->globals.find("__bvh_nodes");
    dev->stats.bvh_bytes = W > 2 ? dev->bvhw_bytes : (it != dev->globals.end() ? it->second.bytes : 0);
  }
  hipStream_t s = dev->stream;
  HIP_CHECK(dev, hipMemsetAsync(dev->counters, 0, 16 * 4 * (CY_LANES + 1), s));
  HIP_CHECK(dev, hipMemsetAsync(dev->stats_dev, 0, 2 * CY_STATS_SHARDS * sizeof(CyStats), s));
  size_t ev = 0;
  hipEvent_t t_begin = get_event(dev, ev++);
  HIP_CHECK(dev, hipEventRecord(t_begin, s));
  std::vector<EvQuad> quads;

  for (int s0 = t->start_sample; s0 < t->start_sample + t->num_samples; s0 += (int)per_pass) {
    CyTile tile;
    const CyTileDesc &d0 = descs[0];
    tile.x = d0.x;
    tile.y = d0.y;
    tile.w = d0.w;
    tile.h = d0.h;
    tile.y_step = y_step;
    tile.start_sample = s0;
    tile.end_sample = std::min(s0 + (int)per_pass, t->start_sample + t->num_samples);
    tile.offset = d0.offset;
    tile.stride = d0.stride;
    tile.buffer = d0.buffer;
    tile.pass_stride = dev->data_host.film.pass_stride;
    tile.npix = (uint)npix;
    tile.n_tiles = (int)descs.size();
    tile.descs = descs.size() > 1 ? dev->tile_descs : nullptr;
    tile.n_items = (uint)(npix * (size_t)(tile.end_sample - tile.start_sample));
    tile.aux_offset = film.pass_adaptive_aux_buffer;
    tile.sample_count_offset = film.pass_sample_count;
    tile.write_aux = (film.pass_adaptive_aux_buffer && integ.adaptive_threshold > 0.0f) ? 1 : 0;
    if (path_trace_pass(dev, kg, tile, W, &ev, &quads) != 0) {
      return -1;
    }
    if (dev->host_counters[3]) {
      break;
    }
    /* CUDADevice::render: filter_sample = sample + num_samples - 1, then
     * AdaptiveSampling::need_filter (device_task.cpp:184-192) */
    const int filter_sample = tile.end_sample - 1;
    if (adaptive && filter_sample > integ.adaptive_min_samples &&
        (filter_sample & (integ.adaptive_step - 1)) == (integ.adaptive_step - 1)) {
      for (const CyTileDesc &d : descs) {
        const CyAdaptiveTile at = {d.x, d.y, d.w, d.h, d.offset, d.stride, d.buffer,
                                   tile.pass_stride, film.pass_adaptive_aux_buffer, film.pass_sample_count};
        hipLaunchKernelGGL(k_adaptive_stopping, dim3((unsigned)((d.w * d.h + CY_BLOCK - 1) / CY_BLOCK)),
                           dim3(CY_BLOCK), 0, s, at, filter_sample, integ.adaptive_threshold);
        hipLaunchKernelGGL(k_adaptive_filter<true>, dim3((unsigned)((d.h + 63) / 64)), dim3(64), 0, s, at);
        hipLaunchKernelGGL(k_adaptive_filter<false>, dim3((unsigned)((d.w + 63) / 64)), dim3(64), 0, s, at);
      }
      HIP_CHECK(dev, hipGetLastError());
    }
  }
  /* CUDADevice::adaptive_sampling_post: rescale pixels that stopped early */
  if (adaptive && film.pass_sample_count && !dev->host_counters[3]) {
    const int end_sample = t->start_sample + t->num_samples;
    for (const CyTileDesc &d : descs) {
      const CyAdaptiveTile at = {d.x, d.y, d.w, d.h, d.offset, d.stride, d.buffer,
                                 (int)film.pass_stride, film.pass_adaptive_aux_buffer, film.pass_sample_count};
      hipLaunchKernelGGL(k_adaptive_scale, dim3((unsigned)((d.w * d.h + CY_BLOCK - 1) / CY_BLOCK)), dim3(CY_BLOCK),
                         0, s, at, t->start_sample, end_sample);
    }
    HIP_CHECK(dev, hipGetLastError());
  }
  hipEvent_t t_end = get_event(dev, ev++);
  HIP_CHECK(dev, hipEventRecord(t_end, s));
  HIP_CHECK(dev, hipMemcpyAsync(dev->host_counters, dev->counters, 16, hipMemcpyDeviceToHost, s));
  HIP_CHECK(dev, hipStreamSynchronize(s));
  float ms = 0.0f;
  hipEventElapsedTime(&ms, t_begin, t_end);
  dev->stats.total_ms = ms;
  if (dev->profiling & 1) {
    double closest = 0.0, shadow = 0.0, shade = 0.0;
    for (auto &p : quads) {
      float a = 0, b = 0, c = 0;
      hipEventElapsedTime(&a, p.a, p.b);
      hipEventElapsedTime(&b, p.b, p.c);
      hipEventElapsedTime(&c, p.c, p.d);
      closest += a;
      shade += b;
      shadow += c;
    }
    dev->stats.intersect_ms = closest + shadow;
    dev->stats.closest_ms = closest;
    dev->stats.shade_ms = shade;
    dev->stats.closest_launches = quads.size();
    dev->stats.shadow_ms = shadow;
    dev->stats.shadow_launches = quads.size();
  }
  if (dev->profiling & 2) {
    std::vector<CyStats> shards(2 * CY_STATS_SHARDS);
    HIP_CHECK(dev, hipMemcpy(shards.data(), dev->stats_dev, shards.size() * sizeof(CyStats), hipMemcpyDeviceToHost));
    CyStats st[2] = {};
    for (int k = 0; k < 2; k++) {
      for (int j = 0; j < CY_STATS_SHARDS; j++) {
        const CyStats &x = shards[k * CY_STATS_SHARDS + j];
        st[k].nodes += x.nodes;
        st[k].leaves += x.leaves;
        st[k].tris += x.tris;
        st[k].rays += x.rays;
        st[k].lane_iters += x.lane_iters;
        st[k].wave_iters += x.wave_iters;
      }
    }
    dev->stats.inner_nodes = st[0].nodes + st[1].nodes;
    dev->stats.leaves = st[0].leaves + st[1].leaves;
    dev->stats.triangles = st[0].tris + st[1].tris;
    dev->stats.closest_nodes = st[0].nodes;
    dev->stats.closest_leaves = st[0].leaves;
    dev->stats.closest_tris = st[0].tris;
    dev->stats.tie_rays = st[0].rays;
    dev->stats.closest_lane_iters = st[0].lane_iters;
    dev->stats.closest_wave_iters = st[0].wave_iters;
    dev->stats.shadow_nodes = st[1].nodes;
    dev->stats.shadow_tris = st[1].tris;
    dev->stats.shadow_lane_iters = st[1].lane_iters;
    dev->stats.shadow_wave_iters = st[1].wave_iters;
  }
  return check_device_error(dev);
}

/* ---------------------------------------------------------------------------
 * Tile streams: hipcy_render_feed (the RENDER task's acquire_tile loop of
 * CUDADevice::thread_run, device_cuda_impl.cpp:2342-2391, with tiles fed to a
 * running wavefront instead of one render per tile).
 *
 * Each lane keeps its own list of appended tile chunks (a RenderTile, or a
 * sample range of one when the tile alone would overflow the lane's record
 * ring) and numbers their work items consecutively.  After every lane
 * iteration the host knows the lane's next unclaimed item and the smallest
 * item a live path still holds (k_stream_min_live); every chunk below both is
 * complete, so its records are added to its buffer (k_accumulate_stream, on the
 * lane's stream, in chunk order) and the RenderTile is released once that has
 * run.  The host appends tiles whenever a lane's unclaimed items fall below
 * its slot count, so the pool stays full across tile borders and no device
 * holds more than `hold` pixel-samples of the shared queue: with several
 * devices on one TileManager each keeps taking tiles as fast as it finishes
 * them.  Slots whose path ended while the lane had no item left go idle and
 * are restarted (k_stream_restart) once tiles arrive.
 * ------------------------------------------------------------------------- */
struct FeedTile {
  hipcy_work_tile t;
  uint64_t tag;
  int next_sample;       /* first sample not yet appended to a lane */
  bool released = false; /* handed back through feed->release */
};

/* A group of tiles appended to a lane together with one sample range: its
 * items are numbered sample-major over the group's pixels (CyTileDesc
 * group_npix), as a whole-frame pass numbers its items, so the rays in flight
 * spread over all of the group's tiles instead of piling onto one 64x64 tile
 * (a single tile's samples one after the other made the camera launch 45 %
 * slower: every CU fetched the same few BVH nodes and triangles).  A tile
 * too large for the record ring is split in sample ranges, each a group of
 * one. */
struct StreamChunk {
  uint item_begin, item_end;
  size_t desc_begin, desc_end; /* the group's tile descriptors */
  int start_sample, num_samples;
  uint npix;    /* pixels of the group (its items per sample) */
  bool open;    /* still taking tiles (descriptors not yet uploaded) */
  bool grouped; /* whole tiles: more may join */
};

struct StreamLane {
  PassLane ln;
  int lane_slots = 0;
  hc_float4 *ring = nullptr;
  uint ring_cap = 0;
  CyTileDesc *desc_dev = nullptr;
  CyTileDesc *desc_host = nullptr; /* pinned, append-only within a session */
  int desc_cap = 0;
  size_t n_descs = 0;   /* descriptors written to desc_host */
  size_t uploaded = 0;  /* descriptors copied to desc_dev (closed groups only) */
  std::vector<int> desc_feed;   /* per descriptor: its FeedTile */
  std::vector<char> desc_last;  /* per descriptor: the RenderTile's last samples */
  std::vector<StreamChunk> chunks;
  size_t done_chunks = 0; /* chunks whose accumulation is enqueued */
  size_t lo_chunk = 0;    /* first chunk that can still hand out items */
  uint n_items = 0;
  uint work_next = 0;
  uint ring_head = 0;
  int cur_feed = -1; /* RenderTile partly appended to this lane */
  bool closed = false;
  std::vector<int> release; /* RenderTiles whose last accumulation is enqueued */
};

#define CY_STREAM_DESCS 16384
#define CY_STREAM_ITEM_CAP 0xE0000000u /* 32-bit items; claims past the end overshoot by < 2^28 */

struct StreamState {
  hipcy_device *dev;
  const hipcy_tile_feed *feed;
  std::vector<FeedTile> tiles;
  size_t released = 0;
  bool feed_empty = false;
  std::vector<int> carry; /* RenderTiles left partly appended by closed lanes */
};

static bool feed_cancelled(const StreamState &st)
{
  return st.feed->cancelled && st.feed->cancelled(st.feed->user);
}

static void feed_release_tile(StreamState &st, size_t f)
{
  FeedTile &F = st.tiles[f];
  if (!F.released) {
    F.released = true;
    st.feed->release(st.feed->user, &F.t, F.tag);
    st.released++;
  }
}

/* Error exit of a tile stream: every acquired tile goes back to the queue's
 * owner, as CUDADevice::thread_run releases each tile it acquired whatever its
 * render did (device_cuda_impl.cpp:2361-2388).  The device's sticky error is
 * set before this runs, so the caller's release callback can tell these tiles
 * from finished ones (hipcy_error is non-empty). */
static void feed_release_all(StreamState &st)
{
  hipcy_device *dev = st.dev;
  /* no kernel may still write a buffer that is handed back */
  for (int l = 0; l < CY_LANES; l++) {
    if (dev->lane_stream[l]) {
      hipStreamSynchronize(dev->lane_stream[l]);
    }
  }
  hipStreamSynchronize(dev->stream);
  for (size_t f = 0; f < st.tiles.size(); f++) {
    feed_release_tile(st, f);
  }
}

/* Close the lane's open group: its descriptors get the group's pixel count and
 * every descriptor not yet on the device is copied there in one transfer. */
static int stream_close(hipcy_device *dev, StreamLane &S)
{
  if (!S.chunks.empty() && S.chunks.back().open) {
    StreamChunk &g = S.chunks.back();
    for (size_t k = g.desc_begin; k < g.desc_end; k++) {
      S.desc_host[k].group_npix = g.npix;
    }
    g.open = false;
  }
  if (S.n_descs > S.uploaded) {
    HIP_CHECK(dev, hipMemcpyAsync(S.desc_dev + S.uploaded, S.desc_host + S.uploaded,
                                  (S.n_descs - S.uploaded) * sizeof(CyTileDesc), hipMemcpyHostToDevice, S.ln.s));
    S.uploaded = S.n_descs;
  }
  return 0;
}

/* Append tiles to the lane until it holds `target` unclaimed items (or the
 * queue, the ring or the lane's numbering runs out): whole tiles with the
 * sample range of the lane's open group join it.  one_chunk: at most one tile
 * (the initial round-robin fill); keep_open: leave the group open for the next
 * call (closed otherwise, so its items can be handed out). */
static int stream_fill(StreamState &st, StreamLane &S, uint target, bool one_chunk, bool keep_open = false)
{
  hipcy_device *dev = st.dev;
  uint unclaimed = S.n_items - std::min(S.work_next, S.n_items);
  while (!S.closed && unclaimed < target) {
    if (S.cur_feed < 0) {
      if (!st.carry.empty()) {
        S.cur_feed = st.carry.front();
        st.carry.erase(st.carry.begin());
      }
      else {
        if (st.feed_empty || feed_cancelled(st)) {
          st.feed_empty = true;
          break;
        }
        FeedTile f;
        memset(&f.t, 0, sizeof(f.t));
        f.tag = 0;
        if (!st.feed->acquire(st.feed->user, &f.t, &f.tag)) {
          st.feed_empty = true;
          break;
        }
        f.next_sample = f.t.start_sample;
        st.tiles.push_back(f);
        if (f.t.w < 0 || f.t.h < 0 || (f.t.w * f.t.h > 0 && f.t.num_samples > 0 && !f.t.buffer)) {
          return set_error(dev, "render_feed: invalid tile");
        }
        if ((size_t)f.t.w * f.t.h == 0 || f.t.num_samples <= 0) {
          /* nothing to render: released at once */
          feed_release_tile(st, st.tiles.size() - 1);
          continue;
        }
        S.cur_feed = (int)st.tiles.size() - 1;
      }
    }
    FeedTile &F = st.tiles[S.cur_feed];
    const uint npix = (uint)(F.t.w * F.t.h);
    if ((size_t)npix * 2 > S.ring_cap) {
      return set_error(dev, "render_feed: tile of " + std::to_string(npix) +
                                " pixels does not fit the record ring (raise hipcy_set_slots record_bytes)");
    }
    const int remaining = F.t.start_sample + F.t.num_samples - F.next_sample;
    const int chunk_s = std::min(remaining, (int)std::max<uint>(1u, (S.ring_cap / 4) / npix));
    const uint items = npix * (uint)chunk_s;
    const bool whole = chunk_s == remaining && F.next_sample == F.t.start_sample;
    StreamChunk *g = (!S.chunks.empty() && S.chunks.back().open) ? &S.chunks.back() : nullptr;
    const bool join = whole && g && g->grouped && g->start_sample == F.next_sample && g->num_samples == chunk_s &&
                      (uint64_t)g->npix + npix <= S.ring_cap;
    if ((uint64_t)S.n_items + items > CY_STREAM_ITEM_CAP || (int)S.n_descs >= S.desc_cap) {
      S.closed = true;
      break;
    }
    if ((uint64_t)S.n_items + items - S.ring_head > S.ring_cap) {
      break; /* ring full until older tiles complete */
    }
    if (g && !join && stream_close(dev, S) != 0) {
      return -1;
    }
    const size_t k = S.n_descs;
    CyTileDesc d;
    d.x = F.t.x;
    d.y = F.t.y;
    d.w = F.t.w;
    d.h = F.t.h;
    d.offset = F.t.offset;
    d.stride = F.t.stride;
    d.buffer = (float *)F.t.buffer;
    d.start_sample = F.next_sample;
    d.num_samples = chunk_s;
    d.group_npix = npix; /* the group's, set when it closes */
    if (join) {
      d.item_begin = g->item_begin;
      d.px_begin = g->npix;
      d.group_first = (uint)g->desc_begin;
      g->npix += npix;
      g->item_end += items;
      g->desc_end = k + 1;
    }
    else {
      d.item_begin = S.n_items;
      d.px_begin = 0;
      d.group_first = (uint)k;
      StreamChunk c;
      c.item_begin = S.n_items;
      c.item_end = S.n_items + items;
      c.desc_begin = k;
      c.desc_end = k + 1;
      c.start_sample = F.next_sample;
      c.num_samples = chunk_s;
      c.npix = npix;
      c.open = true;
      c.grouped = whole;
      S.chunks.push_back(c);
    }
    S.desc_host[k] = d;
    S.n_descs = k + 1;
    S.desc_feed.push_back(S.cur_feed);
    S.desc_last.push_back(chunk_s == remaining ? 1 : 0);
    S.n_items += items;
    unclaimed += items;
    F.next_sample += chunk_s;
    if (chunk_s == remaining) {
      S.cur_feed = -1;
    }
    if (one_chunk) {
      break;
    }
  }
  if (!keep_open && stream_close(dev, S) != 0) {
    return -1;
  }
  return 0;
}

/* The lane's chunks below `bound` are complete: enqueue their accumulation. */
static int stream_complete(StreamState &st, StreamLane &S, uint bound)
{
  hipcy_device *dev = st.dev;
  const int pass_stride = dev->data_host.film.pass_stride;
  const size_t first = S.done_chunks < S.chunks.size() ? S.chunks[S.done_chunks].desc_begin : 0;
  size_t last = first;
  int max_pix = 0;
  while (S.done_chunks < S.chunks.size() && !S.chunks[S.done_chunks].open &&
         S.chunks[S.done_chunks].item_end <= bound) {
    const StreamChunk &c = S.chunks[S.done_chunks];
    for (size_t k = c.desc_begin; k < c.desc_end; k++) {
      max_pix = std::max(max_pix, S.desc_host[k].w * S.desc_host[k].h);
      if (S.desc_last[k]) {
        S.release.push_back(S.desc_feed[k]);
      }
    }
    last = c.desc_end;
    S.done_chunks++;
  }
  if (last > first) {
    /* the completed groups' descriptors are consecutive in the lane's array */
    hipLaunchKernelGGL(k_accumulate_stream, dim3((unsigned)((max_pix + CY_BLOCK - 1) / CY_BLOCK), (unsigned)(last - first)),
                       dim3(CY_BLOCK), 0, S.ln.s, (const CyTileDesc *)(S.desc_dev + first), (const hc_float4 *)S.ring,
                       S.ring_cap - 1, pass_stride);
  }
  HIP_CHECK(dev, hipGetLastError());
  S.ring_head = S.done_chunks < S.chunks.size() ? S.chunks[S.done_chunks].item_begin : S.n_items;
  return 0;
}

static void stream_release(StreamState &st, StreamLane &S)
{
  for (int f : S.release) {
    feed_release_tile(st, (size_t)f);
  }
  S.release.clear();
}

/* Hand the lane's new items to its idle slots and refresh the tile view the
 * kernels get; n_live = the lane's live paths after its last iteration. */
static int stream_restart(StreamState &st, StreamLane &S, uint n_live)
{
  hipcy_device *dev = st.dev;
  PassLane &L = S.ln;
  while (S.lo_chunk < S.chunks.size() && S.chunks[S.lo_chunk].item_end <= S.work_next) {
    S.lo_chunk++;
  }
  L.tile.n_items = S.n_items;
  L.tile.n_tiles = (int)S.uploaded;
  L.tile.desc_lo = S.lo_chunk < S.chunks.size() ? (uint)S.chunks[S.lo_chunk].desc_begin
                                                : (uint)(S.uploaded ? S.uploaded - 1 : 0);
  const uint avail = S.n_items - S.work_next;
  uint n_active = n_live;
  if (n_live < (uint)S.lane_slots && avail > 0) {
    hipLaunchKernelGGL(k_stream_restart, dim3((unsigned)((S.lane_slots + CY_BLOCK - 1) / CY_BLOCK)), dim3(CY_BLOCK), 0,
                       L.s, st.dev->kg_stream, dev->bufs, L.tile, L.slot_base, S.lane_slots, L.q[L.qa], L.cnt + L.qa);
    HIP_CHECK(dev, hipGetLastError());
    n_active = (uint)std::min<uint64_t>((uint64_t)S.lane_slots, (uint64_t)n_live + avail);
  }
  L.n_active = n_active;
  return 0;
}

/* The slot pool of a tile stream (and the per-slot extras the scene needs). */
static int stream_pool(hipcy_device *dev, size_t slots)
{
  if (ensure_capacity(dev, slots) != 0 || ensure_volume_capacity(dev) != 0 || ensure_sss_capacity(dev) != 0 ||
      ensure_catcher_capacity(dev) != 0 || ensure_branch_capacity(dev) != 0 || ensure_lightpass_capacity(dev) != 0 || ensure_diff_capacity(dev) != 0 || ensure_srec_capacity(dev) != 0 || ensure_sort(dev) != 0) {
    return -1;
  }
  return 0;
}

static int stream_session(StreamState &st, const CyGlobals &kg, int W, size_t lane_slots, uint ring_cap,
                          size_t *ev)
{
  hipcy_device *dev = st.dev;
  const int lanes = CY_LANES;
  StreamLane lane[CY_LANES];
  for (int l = 0; l < lanes; l++) {
    StreamLane &S = lane[l];
    PassLane &L = S.ln;
    L.index = l;
    L.s = dev->lane_stream[l];
    L.cnt = dev->counters + 16 * (l + 1);
    L.hcnt = dev->host_counters + 16 * (l + 1);
    L.qa = 0;
    L.qb = 1;
    L.done = get_event(dev, (*ev)++);
    L.stream = true;
    S.ring = dev->records + (size_t)ring_cap * l;
    S.ring_cap = ring_cap;
    S.desc_dev = dev->stream_desc_dev + (size_t)CY_STREAM_DESCS * l;
    S.desc_host = dev->stream_desc_host + (size_t)CY_STREAM_DESCS * l;
    S.desc_cap = CY_STREAM_DESCS;
    CyTile &t = L.tile;
    t = CyTile();
    t.y_step = 1;
    t.pass_stride = dev->data_host.film.pass_stride;
    t.stream = 1;
    t.ring_mask = ring_cap - 1;
    t.samples_out = S.ring;
    t.descs = S.desc_dev;
    t.work_next = L.cnt + 4;
    t.item_base = 0;
    t.aux_offset = 0;
    t.sample_count_offset = 0;
    t.write_aux = 0;
    t.npix = 1;
  }
  /* initial fill, round robin one tile at a time: each lane wants its slots'
   * worth of camera rays plus as many in reserve; a lane's tiles form one
   * group (so every lane's rays in flight cover tiles all over the queue) */
  for (bool more = true; more;) {
    more = false;
    for (int l = 0; l < lanes; l++) {
      StreamLane &S = lane[l];
      const size_t before = S.n_descs;
      if (stream_fill(st, S, 2 * (uint)lane_slots, true, true) != 0) {
        return -1;
      }
      more |= S.n_descs > before;
    }
  }
  for (int l = 0; l < lanes; l++) {
    if (stream_close(dev, lane[l]) != 0) {
      return -1;
    }
  }
  if (st.feed_empty && st.carry.empty()) {
    /* the whole queue is in the lanes: no lane needs more slots than items */
    size_t most = 0;
    for (int l = 0; l < lanes; l++) {
      most = std::max<size_t>(most, lane[l].n_items);
    }
    most = std::max<size_t>((most + CY_BLOCK - 1) / CY_BLOCK * CY_BLOCK, 4 * CY_BLOCK);
    lane_slots = std::min(lane_slots, most);
  }
  if (stream_pool(dev, lane_slots * lanes) != 0) {
    return -1;
  }
  /* idle marks: every slot of the pool starts without an item */
  HIP_CHECK(dev, hipMemsetAsync(dev->bufs.item, 0xFF, lane_slots * lanes * sizeof(uint), dev->stream));
  HIP_CHECK(dev, hipMemsetAsync(dev->counters, 0, 16 * 4 * (CY_LANES + 1), dev->stream));
  hipEvent_t start = get_event(dev, (*ev)++);
  HIP_CHECK(dev, hipEventRecord(start, dev->stream));
  for (int l = 0; l < lanes; l++) {
    StreamLane &S = lane[l];
    PassLane &L = S.ln;
    HIP_CHECK(dev, hipStreamWaitEvent(L.s, start, 0));
    L.slot_base = (int)(lane_slots * l);
    for (int q = 0; q < 3; q++) {
      L.q[q] = dev->queue[q] + L.slot_base;
    }
    S.lane_slots = (int)lane_slots;
  }
  for (int l = 0; l < lanes; l++) {
    StreamLane &S = lane[l];
    PassLane &L = S.ln;
    L.cam_n = (int)std::min<uint>((uint)lane_slots, S.n_items);
    L.n_active = (uint)L.cam_n;
    S.work_next = (uint)L.cam_n;
    L.tile.n_items = S.n_items;
    L.tile.n_tiles = (int)S.uploaded;
    L.tile.desc_lo = 0;
    L.hcnt[4] = S.work_next;
    HIP_CHECK(dev, hipMemcpyAsync(L.cnt + 4, L.hcnt + 4, 4, hipMemcpyHostToDevice, L.s));
  }
  /* lanes in submission order (as path_trace_pass): the oldest lane is
   * waited for, its finished tiles accumulated, tiles appended and idle slots
   * restarted, and its next iteration enqueued while the others run */
  int fifo[CY_LANES];
  int head = 0, n_fifo = 0;
  bool queued[CY_LANES] = {};
  auto submit = [&](int l) -> int {
    /* a group is complete only once no live path holds one of its items: with
     * one incomplete group that is when the lane has no live path, which the
     * counts tell; the smallest live item (k_stream_min_live, a pass over the
     * queue) is needed only with two or more */
    lane[l].ln.min_live = lane[l].chunks.size() > lane[l].done_chunks + 1;
    if (lane_iterate(dev, kg, lane[l].ln, W, ev, nullptr) != 0) {
      return -1;
    }
    fifo[(head + n_fifo++) % CY_LANES] = l;
    queued[l] = true;
    return 0;
  };
  for (int l = 0; l < lanes; l++) {
    if (lane[l].ln.n_active > 0 && submit(l) != 0) {
      return -1;
    }
  }
  dev->host_counters[3] = 0;
  while (n_fifo > 0) {
    const int l = fifo[head];
    head = (head + 1) % CY_LANES;
    n_fifo--;
    queued[l] = false;
    StreamLane &S = lane[l];
    PassLane &L = S.ln;
    HIP_CHECK(dev, hipEventSynchronize(L.done));
    if (L.hcnt[6]) {
      dev->host_counters[3] = L.hcnt[6];
      break;
    }
    /* the accumulations enqueued before this iteration have run */
    stream_release(st, S);
    dev->stats.shadow_rays += L.hcnt[2];
    const uint n_live = L.hcnt[L.qb];
    uint wn = L.hcnt[4];
    uint live_min = n_live > 0 ? 0u : 0xFFFFFFFFu;
    if (L.min_live) {
      live_min = 0xFFFFFFFFu;
      for (int k = 0; k < CY_MIN_SHARDS; k++) {
        live_min = std::min(live_min, dev->min_live_host[CY_MIN_SHARDS * l + k]);
      }
    }
    if (wn > S.n_items) {
      /* claims past the end: put the counter back so appended items are
       * handed out from the first one */
      wn = S.n_items;
      L.hcnt[12] = wn;
      HIP_CHECK(dev, hipMemcpyAsync(L.cnt + 4, L.hcnt + 12, 4, hipMemcpyHostToDevice, L.s));
    }
    S.work_next = wn;
    if (stream_complete(st, S, std::min(live_min, wn)) != 0) {
      return -1;
    }
    std::swap(L.qa, L.qb);
    if (stream_fill(st, S, (uint)lane_slots, false) != 0 || stream_restart(st, S, n_live) != 0) {
      return -1;
    }
    if (L.n_active > 0 && submit(l) != 0) {
      return -1;
    }
    /* an idle lane takes tiles again while the queue has some */
    for (int k = 0; k < lanes; k++) {
      StreamLane &I = lane[k];
      if (queued[k] || I.ln.n_active > 0 || I.closed || (st.feed_empty && st.carry.empty())) {
        continue;
      }
      if (stream_fill(st, I, (uint)lane_slots, false) != 0 || stream_restart(st, I, 0) != 0) {
        return -1;
      }
      if (I.ln.n_active > 0 && submit(k) != 0) {
        return -1;
      }
    }
  }
  /* drained: every chunk is complete; run the last accumulations, then release */
  for (int l = 0; l < lanes; l++) {
    StreamLane &S = lane[l];
    if (!dev->host_counters[3] && stream_complete(st, S, S.n_items) != 0) {
      return -1;
    }
    HIP_CHECK(dev, hipStreamSynchronize(S.ln.s));
    if (dev->host_counters[3]) {
      S.release.clear();
      continue;
    }
    stream_release(st, S);
    if (S.cur_feed >= 0) {
      st.carry.push_back(S.cur_feed); /* closed lane: the rest of this RenderTile goes on in the next session */
    }
  }
  return 0;
}

/* Adaptive sampling filters each RenderTile between sample steps: those
 * scenes are rendered one acquired tile per device pass, as CUDADevice does. */
static int feed_per_tile(StreamState &st)
{
  hipcy_device *dev = st.dev;
  while (!feed_cancelled(st)) {
    FeedTile f;
    memset(&f.t, 0, sizeof(f.t));
    f.tag = 0;
    if (!st.feed->acquire(st.feed->user, &f.t, &f.tag)) {
      break;
    }
    f.next_sample = f.t.start_sample;
    st.tiles.push_back(f);
    if (path_trace(dev, &st.tiles.back().t, 1, 1) != 0 || hipcy_synchronize(dev) != 0) {
      return -1;
    }
    feed_release_tile(st, st.tiles.size() - 1);
  }
  return 0;
}

int hipcy_set_stream_hold(hipcy_device *dev, uint64_t pixel_samples)
{
  dev->stream_hold = pixel_samples ? (size_t)pixel_samples : dev->stream_hold;
  return 0;
}

int hipcy_render_feed(hipcy_device *dev, const hipcy_tile_feed *feed)
{
  if (!dev->error.empty()) {
    return -1;
  }
  if (!feed || !feed->acquire || !feed->release) {
    return set_error(dev, "render_feed: acquire and release callbacks are required");
  }
  if (dev->features_dirty && hipcy_load_kernels(dev) != 0) {
    return -1;
  }
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  StreamState st;
  st.dev = dev;
  st.feed = feed;
  if (dev->data_host.film.pass_adaptive_aux_buffer) {
    if (feed_per_tile(st) != 0) {
      feed_release_all(st);
      return -1;
    }
    return 0;
  }
  const int lanes = CY_LANES;
  const size_t hold = feed->hold ? (size_t)feed->hold
                                  : dev->stream_hold ? dev->stream_hold : 2 * dev->slots_wanted;
  /* half of a lane's share in flight, half in reserve */
  size_t lane_slots = std::min(dev->slots_wanted / lanes, std::max<size_t>(hold / (2 * lanes), 4 * CY_BLOCK));
  lane_slots = std::min(lane_slots, slot_limit(dev) / lanes);
  lane_slots = (lane_slots + CY_BLOCK - 1) / CY_BLOCK * CY_BLOCK;
  /* per-lane record ring: the largest power of two the record budget holds */
  uint ring_cap = 1u << 12;
  while ((size_t)ring_cap * 2 * sizeof(hc_float4) * lanes <= dev->record_budget && ring_cap < (1u << 30)) {
    ring_cap <<= 1;
  }
  /* the slot pool is sized by each session once its first tiles are in
   * (stream_pool) */
  if (ensure_records(dev, (size_t)ring_cap * lanes) != 0 || ensure_bvhw(dev) != 0) {
    return -1;
  }
  if (!dev->stream_desc_dev) {
    HIP_CHECK(dev, hipMalloc((void **)&dev->stream_desc_dev, sizeof(CyTileDesc) * CY_STREAM_DESCS * CY_LANES));
    HIP_CHECK(dev, hipHostMalloc((void **)&dev->stream_desc_host, sizeof(CyTileDesc) * CY_STREAM_DESCS * CY_LANES,
                                 hipHostMallocDefault));
    HIP_CHECK(dev, hipMalloc((void **)&dev->min_live_dev, CY_MIN_SHARDS * CY_LANES * 4));
    HIP_CHECK(dev, hipHostMalloc((void **)&dev->min_live_host, CY_MIN_SHARDS * CY_LANES * 4, hipHostMallocDefault));
  }
  CyGlobals kg;
  build_globals(dev, &kg);
  dev->kg_stream = kg;
  const int W = kg.bvhw_nodes ? dev->bvh_width : 2;
  memset(&dev->stats, 0, sizeof(dev->stats));
  dev->stats.bvh_width = W;
  HIP_CHECK(dev, hipMemsetAsync(dev->stats_dev, 0, 2 * CY_STATS_SHARDS * sizeof(CyStats), dev->stream));
  /* per-kernel event timing needs one lane without overlap: not in streams */
  const int prof = dev->profiling;
  dev->profiling &= ~1;
  size_t ev = 0;
  hipEvent_t t_begin = get_event(dev, ev++);
  HIP_CHECK(dev, hipEventRecord(t_begin, dev->stream));
  int rc = 0;
  do {
    /* a session ends when every lane drained; another starts only when a lane
     * ran out of item numbers or tile slots while the queue still had tiles */
    rc = stream_session(st, kg, W, lane_slots, ring_cap, &ev);
  } while (rc == 0 && !dev->host_counters[3] && (!st.feed_empty || !st.carry.empty()));
  dev->profiling = prof;
  if (rc != 0) {
    feed_release_all(st);
    return -1;
  }
  hipEvent_t t_end = get_event(dev, ev++);
  HIP_CHECK(dev, hipEventRecord(t_end, dev->stream));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  float ms = 0.0f;
  hipEventElapsedTime(&ms, t_begin, t_end);
  dev->stats.total_ms = ms;
  if (check_device_error(dev) != 0) {
    feed_release_all(st);
    return -1;
  }
  return 0;
}

int hipcy_set_slots(hipcy_device *dev, uint64_t slots, uint64_t record_bytes)
{
  if (slots) {
    dev->slots_wanted = (size_t)slots;
  }
  if (record_bytes) {
    dev->record_budget = (size_t)record_bytes;
  }
  return 0;
}

int hipcy_intersect(hipcy_device *dev, uint64_t rays, uint64_t out_f, uint64_t out_i, int n, int any_hit)
{
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  if (ensure_bvhw(dev) != 0) {
    return -1;
  }
  CyGlobals kg;
  build_globals(dev, &kg);
  HIP_CHECK(dev, hipMemsetAsync(dev->counters, 0, 64, dev->stream));
  const int W = kg.bvhw_nodes ? dev->bvh_width : 2;
  auto ktest = kg.have_curves ? (W == 8 ? k_test_intersect<8, 1> : W == 4 ? k_test_intersect<4, 1> : k_test_intersect<2, 3>) :
               W == 8 ? k_test_intersect<8> : W == 4 ? k_test_intersect<4> : k_test_intersect<2>;
  hipLaunchKernelGGL(ktest,
                     dim3((n + CY_BLOCK - 1) / CY_BLOCK), dim3(CY_BLOCK), 0, dev->stream, kg,
                     (const float *)rays, (float *)out_f, (int *)out_i, n, any_hit, dev->counters + 3);
  HIP_CHECK(dev, hipGetLastError());
  HIP_CHECK(dev, hipMemcpyAsync(dev->host_counters, dev->counters, 16, hipMemcpyDeviceToHost, dev->stream));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return check_device_error(dev);
}

int hipcy_camera_rays(hipcy_device *dev, uint64_t xys, uint64_t out, int n)
{
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  CyGlobals kg;
  build_globals(dev, &kg);
  hipLaunchKernelGGL(k_test_camera, dim3((n + 255) / 256), dim3(256), 0, dev->stream, kg,
                     (const int *)xys, (float *)out, n);
  HIP_CHECK(dev, hipGetLastError());
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return 0;
}

int hipcy_film_convert(hipcy_device *dev, uint64_t buffer, uint64_t rgba_byte, uint64_t rgba_half,
                       float sample_scale, int x, int y, int w, int h, int offset, int stride)
{
  if (!dev->error.empty()) {
    return -1;
  }
  if (!dev->have_data) {
    return set_error(dev, "film_convert: KernelData not uploaded");
  }
  if (!buffer || (!rgba_byte && !rgba_half) || w < 0 || h < 0) {
    return set_error(dev, "film_convert: invalid arguments");
  }
  if (w == 0 || h == 0) {
    return 0;
  }
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  const hc_KernelData &d = dev->data_host;
  CyFilm film;
  film.pass_stride = d.film.pass_stride;
  film.display_pass_stride = d.film.display_pass_stride;
  film.display_pass_components = d.film.display_pass_components;
  film.display_divide_pass_stride = d.film.display_divide_pass_stride;
  film.use_display_exposure = d.film.use_display_exposure;
  film.use_display_pass_alpha = d.film.use_display_pass_alpha;
  film.exposure = d.film.exposure;
  const long n = (long)w * h;
  dim3 grid((unsigned)((n + CY_BLOCK - 1) / CY_BLOCK)), block(CY_BLOCK);
  if (rgba_half) {
    hipLaunchKernelGGL(k_film_convert<true>, grid, block, 0, dev->stream, film, (const float *)buffer,
                       (void *)rgba_half, sample_scale, x, y, w, h, offset, stride);
  }
  else {
    hipLaunchKernelGGL(k_film_convert<false>, grid, block, 0, dev->stream, film, (const float *)buffer,
                       (void *)rgba_byte, sample_scale, x, y, w, h, offset, stride);
  }
  HIP_CHECK(dev, hipGetLastError());
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return 0;
}

int hipcy_shader_eval(hipcy_device *dev, int eval_type, uint64_t input, uint64_t output, int shader_x,
                      int shader_w, int offset, int num_samples)
{
  (void)offset; /* passed to kernel_cuda_background, unused by kernel_background_evaluate */
  if (!dev->error.empty()) {
    return -1;
  }
  if (eval_type != HIPCY_SHADER_EVAL_BACKGROUND && eval_type != HIPCY_SHADER_EVAL_DISPLACE) {
    return set_error(dev, "shader_eval: eval_type must be SHADER_EVAL_DISPLACE or SHADER_EVAL_BACKGROUND");
  }
  if (!dev->have_data) {
    return set_error(dev, "shader_eval: KernelData not uploaded");
  }
  if (!input || !output || shader_x < 0 || shader_w < 0 || num_samples < 0) {
    return set_error(dev, "shader_eval: invalid arguments");
  }
  if (dev->globals.find("__svm_nodes") == dev->globals.end() ||
      dev->globals.find("__shaders") == dev->globals.end()) {
    return set_error(dev, "shader_eval: __svm_nodes / __shaders not bound");
  }
  if (shader_w == 0) {
    return 0;
  }
  HIP_CHECK(dev, hipSetDevice(dev->ordinal));
  CyGlobals kg;
  build_globals(dev, &kg);
  uint *err = dev->counters + 3;
  HIP_CHECK(dev, hipMemsetAsync(err, 0, 4, dev->stream));
  /* CUDADevice::shader (device_cuda_impl.cpp:2019-2093): chunks of 65536, once per sample */
  const int chunk = 65536;
  for (int sample = 0; sample < num_samples; sample++) {
    for (int x = shader_x; x < shader_x + shader_w; x += chunk) {
      const int w = std::min(chunk, shader_x + shader_w - x);
      hipLaunchKernelGGL(eval_type == HIPCY_SHADER_EVAL_DISPLACE ? k_displace_eval : k_background_eval,
                         dim3((w + CY_BLOCK - 1) / CY_BLOCK), dim3(CY_BLOCK), 0, dev->stream, kg,
                         (const hc_uint4 *)input, (float *)output, x, w, err);
      HIP_CHECK(dev, hipGetLastError());
    }
  }
  HIP_CHECK(dev, hipMemcpyAsync(dev->host_counters + 3, err, 4, hipMemcpyDeviceToHost, dev->stream));
  HIP_CHECK(dev, hipStreamSynchronize(dev->stream));
  return check_device_error(dev);
}

}  // extern "C"
