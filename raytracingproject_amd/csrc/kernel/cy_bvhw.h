/*
 * cy_bvhw.h — closest-hit and opaque any-hit traversal of the device's W-wide
 * BVH (W = 4 or 8, layout: csrc/host/cy_bvhw_collapse.h).
 *
 * Same query as bvh2_intersect (bvh/bvh_traversal.h:34-227) with the same
 * direction clamp, the same slab arithmetic on the same (exact) child boxes,
 * the same ray_triangle_intersect on the same primitive arrays and the same
 * visibility tests, so every primitive the BVH2 traversal accepts is also
 * reached here; only the visiting order differs, and with it the winner
 * between primitives whose hit distances agree to the last ulp
 * (tests/test_bvh_wide.py bounds that).
 *
 * Per wide node the W child boxes are tested, the hit children sorted by entry
 * distance with a small sorting network, the nearest visited next and the rest
 * pushed far-to-near with their entry distance (a popped entry farther than the
 * current hit is skipped).  Leaf children are stack entries too, so triangles
 * are tested in near-to-far order.  The newest CY_LDS_STACKW stack entries
 * live in an LDS ring (below).
 *
 * Instancing: instanced scenes traverse the top level as the reference does
 * (cy_path.h bvh2_intersect with WI = W: same visiting order, so the same
 * sequence of bvh_instance_push/pop roundings of t) and each instance with its
 * object's wide BVH (bvhw_traverse from bvhw_object_root).  A fully wide
 * two-level traversal (instances in the wide top level) was measured first:
 * its other order of entering instances changes t in the last ulp for about
 * 0.1 % of camera rays, and renders then drift from the reference.
 */
#ifndef CY_BVHW_H
#define CY_BVHW_H

#include "cy_path.h"

#ifndef CY_LDS_STACKW
#  define CY_LDS_STACKW 8
#endif
/* child code bit of an oriented-box node (hair scenes; cy_bvhw_collapse.h) */
#define CY_BVHW_OBB (1u << 30)
#define CY_BVHW_STACK 96
/* request the next triangle's vertices before testing the current one */
#ifndef CY_TRI_PREFETCH
#  define CY_TRI_PREFETCH 1
#endif

/* Traversal stack of (child code, entry distance) pairs.  The newest
 * CY_LDS_STACKW entries live in a ring in LDS: entry k of thread t is the
 * 8-byte CyStackEntry at ring[k * CY_BLOCK + t] (one ds_write_b64 /
 * ds_read_b64 per push / pop, conflict-free for 64 consecutive lanes).  When
 * the ring is full its oldest entry moves to a private overflow array and comes
 * back only after the ring has drained, so only rays keeping more than
 * CY_LDS_STACKW entries pending ever touch scratch.
 *
 * The ring position and counts are plain locals of the traversal function
 * (never members of an object whose address is taken), and the overflow arrays
 * are separate allocas: the compiler keeps the counters in registers and only
 * the dynamically indexed overflow arrays live in scratch. */
#if (CY_LDS_STACKW & (CY_LDS_STACKW - 1)) != 0
#  error "CY_LDS_STACKW must be a power of two"
#endif
#define CY_OVER_STACK (CY_BVHW_STACK - CY_LDS_STACKW)
#if defined(__HIP_DEVICE_COMPILE__)
#  define CY_RING_STRIDE CY_BLOCK
#else
#  define CY_RING_STRIDE 1
#endif

/* returns false when the stack is full (CY_BVHW_STACK entries) */
#define CY_STACK_PUSH(c_, t_) \
  ([&]() -> bool { \
    if (n_ring == CY_LDS_STACKW) { \
      if (n_over == CY_OVER_STACK) { \
        return false; \
      } \
      const CyStackEntry old = ring[top * CY_RING_STRIDE]; \
      over_node[n_over] = old.node; \
      over_t[n_over] = old.t; \
      n_over++; \
      n_ring--; \
    } \
    CyStackEntry e_; \
    e_.node = (c_); \
    e_.t = (t_); \
    ring[top * CY_RING_STRIDE] = e_; \
    top = (top + 1) & (CY_LDS_STACKW - 1); \
    n_ring++; \
    return true; \
  }())

/* Slab-test min / max.  The reference's min / max ((a < b) ? a : b,
 * util_math.h:122-167) and the hardware's v_min_f32 / v_max_f32 (min3 / max3)
 * agree on every operand the slab test produces except the sign of a zero
 * result: the operands are products of finite differences and finite inverse
 * directions (bvh_clamp_direction bounds |idir| by 1.2e24), so never NaN, and
 * min(-0, +0) may return either zero.  Every later use of these values is a
 * comparison (hit = tmax >= tmin, the child sort, the stack's cull against the
 * current hit, the leaf-box entry check) or a copy into one, for which -0 and
 * +0 are equal, so the traversal decides exactly as the reference's arithmetic
 * does.  0 selects the reference's form (measurement switch).
 * Exception: scene_intersect_valid, like the reference's (bvh/bvh.h), tests
 * only P.x and D.x for finiteness, so a ray whose P.y, P.z, D.y or D.z is NaN
 * or infinite is still traversed.  Its slab operands can be NaN, where
 * fminf / fmaxf drop the NaN and the reference's ternaries keep it, so the wide
 * traversal may open other boxes than the reference and the hit it reports is
 * outside the bit-exactness claim.  Such a ray comes only from a path state
 * that is already non-finite; no golden case produces one. */
#ifndef CY_FAST_MINMAX
#  define CY_FAST_MINMAX 1
#endif
#if CY_FAST_MINMAX
CY_FN float slab_min(float a, float b)
{
  return __builtin_fminf(a, b);
}
CY_FN float slab_max(float a, float b)
{
  return __builtin_fmaxf(a, b);
}
#else
CY_FN float slab_min(float a, float b)
{
  return cmin(a, b);
}
CY_FN float slab_max(float a, float b)
{
  return cmax(a, b);
}
#endif

CY_FN hc_uint4 as_uint4(hc_float4 f)
{
  hc_uint4 u;
  u.x = as_uint(f.x);
  u.y = as_uint(f.y);
  u.z = as_uint(f.z);
  u.w = as_uint(f.w);
  return u;
}

CY_FN void bvhw_cswap(float &ta, int &ca, float &tb, int &cb)
{
  const bool sw = tb < ta;
  const float t0 = sw ? tb : ta;
  const float t1 = sw ? ta : tb;
  const int c0 = sw ? cb : ca;
  const int c1 = sw ? ca : cb;
  ta = t0;
  tb = t1;
  ca = c0;
  cb = c1;
}

/* ascending sort of (entry distance, child code); misses carry +inf */
template<int W> CY_FN void bvhw_sort(float (&t)[W], int (&c)[W])
{
  if constexpr (W == 4) {
    bvhw_cswap(t[0], c[0], t[1], c[1]);
    bvhw_cswap(t[2], c[2], t[3], c[3]);
    bvhw_cswap(t[0], c[0], t[2], c[2]);
    bvhw_cswap(t[1], c[1], t[3], c[3]);
    bvhw_cswap(t[1], c[1], t[2], c[2]);
  }
  else {
    /* Batcher odd-even merge sort, 19 comparators */
    bvhw_cswap(t[0], c[0], t[1], c[1]);
    bvhw_cswap(t[2], c[2], t[3], c[3]);
    bvhw_cswap(t[4], c[4], t[5], c[5]);
    bvhw_cswap(t[6], c[6], t[7], c[7]);
    bvhw_cswap(t[0], c[0], t[2], c[2]);
    bvhw_cswap(t[1], c[1], t[3], c[3]);
    bvhw_cswap(t[4], c[4], t[6], c[6]);
    bvhw_cswap(t[5], c[5], t[7], c[7]);
    bvhw_cswap(t[1], c[1], t[2], c[2]);
    bvhw_cswap(t[5], c[5], t[6], c[6]);
    bvhw_cswap(t[0], c[0], t[4], c[4]);
    bvhw_cswap(t[1], c[1], t[5], c[5]);
    bvhw_cswap(t[2], c[2], t[6], c[6]);
    bvhw_cswap(t[3], c[3], t[7], c[7]);
    bvhw_cswap(t[2], c[2], t[4], c[4]);
    bvhw_cswap(t[3], c[3], t[5], c[5]);
    bvhw_cswap(t[1], c[1], t[2], c[2]);
    bvhw_cswap(t[3], c[3], t[4], c[4]);
    bvhw_cswap(t[5], c[5], t[6], c[6]);
  }
}

/* Slab test in FMA form (measurement switch): (lo - P) * idir as
 * fma(lo, idir, -P * idir) with P * idir hoisted per ray, one operation per
 * plane instead of two.  Its rounding differs from the reference's form by at
 * most 2^-24 |P idir| (the hoisted product) plus 3 ulp of the result, so the
 * interval is widened by 2^-21 (|P.x idir.x| + |P.y idir.y| + |P.z idir.z|)
 * and 2^-20 relative: every box the exact test accepts is still accepted
 * (boxes only decide which triangles are tested; the triangle test and the
 * near-tie re-trace decide the hit). */
#ifndef CY_SLAB_FMA
#  define CY_SLAB_FMA 0
#endif

/* Top levels of the wide BVH served from LDS: the collapse numbers wide nodes
 * breadth first (cy_bvhw_collapse.h), so nodes 0 .. CY_LDS_TOP-1 are the root
 * and the levels below it (W = 4: 1 + 4 + 16 = 21 nodes for two levels below
 * the root, 85 for three).  The traversal kernels copy them into LDS once per
 * workgroup (hipcycles.hip lds_fill_top) and every visit of one of them reads
 * LDS instead of issuing eight 16-B global loads to a 128-B line.  0 = off. */
#ifndef CY_LDS_TOP
#  define CY_LDS_TOP 21
#endif
/* LDS image layout of the top nodes: 0 node after node (float4 k of node n at
 * n * 2W + k), 1 float4-major (at k * CY_LDS_TOP + n), so lanes reading the
 * same float4 of different nodes hit different banks */
#ifndef CY_LDS_TOP_SOA
#  define CY_LDS_TOP_SOA 0
#endif

/* opaque any-hit without the child sort (measurement switch) */
#ifndef CY_ANYHIT_NOSORT
#  define CY_ANYHIT_NOSORT 0
#endif
/* opaque any-hit with the hit leaf children first (measurement switch): a
 * shadow ray ends at any occluder, so the order of the children only decides
 * how soon one is found, never the result */
#ifndef CY_ANYHIT_LEAF_FIRST
#  define CY_ANYHIT_LEAF_FIRST 0
#endif

/* Near-tie window of the exact closest hit: hits within 2^-20 (about 8 ulps)
 * of the best distance are kept as candidates and resolved in the reference's
 * order at the end (bvhw_traverse). */
/* 0: no near-tie detection (visiting-order ties resolved as they fall; for
 * measuring its cost only) */
#ifndef CY_EXACT_TIES
#  define CY_EXACT_TIES 1
#endif
/* tuning switches of the near-tie detection (measurement builds only) */
#ifndef CY_TIE_BOX_WIDEN
#  define CY_TIE_BOX_WIDEN 1
#endif
#ifndef CY_TIE_EXACT_OK
#  define CY_TIE_EXACT_OK 1
#endif

/* Traversal of the wide BVH from node `root` with the ray already in the space
 * of that BVH (P, dir, idir; `object` = the instance it belongs to or
 * OBJECT_NONE) and the current hit in *isect (its t bounds the query).  Hits
 * found update *isect.  Returns true when it found a hit (for any_hit: at the
 * first one).  The BVH holds no instance leaves: instanced scenes traverse their
 * top level in reference order (cy_path.h bvh2_intersect, WI > 2) and call this
 * per instance.
 *
 * Exact closest hit.  The reference visits triangles in its BVH2 order and
 * accepts each one whose distance passes T <= t * den against the current t
 * (util_math_intersect.h:178), so when several triangles lie at (nearly) the
 * same distance -- shared edges, fan centres, coplanar faces -- the survivor
 * depends on that order, on rounding, and on which of their boxes the
 * reference's current t still admits.  Here hits are collected against the best
 * distance widened by CY_TIE_EPS (boxes and stack entries culled against the
 * same bound, so no such hit is missed) and *tie is set when two hits, or a hit
 * and the incoming one, fall inside one window.  Only then can the order
 * matter: that ray is re-traced with the reference-order BVH2 traversal
 * (cy_integrator.h shade_path; about 1 ray in 3000 on the bench scene).  Hits
 * beyond the window lose in either order. */
template<int W, bool any_hit, int HAIR>
CY_FN bool bvhw_traverse(const CyGlobals *kg,
                         int root,
                         cfloat3 P,
                         cfloat3 dir,
                         cfloat3 idir,
                         int object,
                         uint visibility,
                         CyIsect *isect,
                         uint *err,
                         uint *cnt_nodes,
                         uint *cnt_leaves,
                         uint *cnt_tris,
                         CY_LDS CyStackEntry *lds_ring,
                         bool *tie_out,
                         int budget,
                         CyTravCursor *cur,
                         CY_LDS const hc_float4 *top_nodes,
                         int n_top)
{
  /* ring column of this thread (device) or a local array (host) */
#if defined(__HIP_DEVICE_COMPILE__)
  CY_LDS CyStackEntry *ring = lds_ring;
#else
  CyStackEntry host_ring[CY_LDS_STACKW];
  CyStackEntry *ring = host_ring;
  (void)lds_ring;
#endif
  int top = cur ? cur->top : 0;       /* ring slot of the next push */
  int n_ring = cur ? cur->n_ring : 0; /* valid ring entries (0 .. CY_LDS_STACKW) */
  int n_over = 0;                     /* entries in the overflow arrays */
  int over_node[CY_OVER_STACK];
  float over_t[CY_OVER_STACK];
  bool found_hit = false;

  bool tie = cur ? cur->tie : false; /* two hits inside the window of the current best */
  /* a hit accepted in front of its own leaf's box entry by more than the tie
   * window: the triangle test's rounding (sliver triangles) put it clearly
   * closer than the box that holds it, so the reference, whose culling bound
   * is not widened, may have culled that box against a hit between the two --
   * resolved by the reference-order re-trace like a near-tie (sticky).  A hit
   * within the window of its box entry (every hit on an axis-aligned face can
   * round an ulp below its flat box) needs no flag: a competing hit between
   * the two lies inside the tie window and sets `tie` */
  bool bad = cur ? cur->tie : false;
  int iters = 0;
  /* culling bound: the best distance widened by the tie window (recomputed
   * where used rather than kept in a register) */
#define CY_T_CULL ((any_hit || !CY_EXACT_TIES) ? isect->t : isect->t * (1.0f + CY_TIE_EPS))
#define CY_T_BOX ((any_hit || !CY_EXACT_TIES || !CY_TIE_BOX_WIDEN) ? isect->t : isect->t * (1.0f + CY_TIE_EPS))

  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  const hc_float4 *nodes = (const hc_float4 *)kg->bvhw_nodes;
#if CY_SLAB_FMA
  const float pix = P.x * idir.x, piy = P.y * idir.y, piz = P.z * idir.z;
  const float ewide = (fabsf(pix) + fabsf(piy) + fabsf(piz)) * 0x1p-21f;
#endif
  constexpr int Q = W / 4; /* float4 per array */
  int code = cur ? cur->code : root;
  float code_t = cur ? cur->code_t : 0.0f; /* entry distance of `code`'s box */
  if (cur) {
    cur->suspended = false;
  }

  while (true) {
    if constexpr (HAIR != 0) {
      if (code >= 0 && (code & (int)CY_BVHW_OBB)) {
        /* oriented-box node (cy_bvhw_collapse.h emit_obb): the reference's
         * unaligned two-child test (bvh_nodes.h:79-135) on its own transforms */
        n_nodes++;
        const int idx = code & ~(int)CY_BVHW_OBB;
        hc_float4 nd[7];
#if defined(__HIP_DEVICE_COMPILE__) && CY_LDS_TOP > 0 && !CY_LDS_TOP_SOA
        if (idx < n_top) {
          CY_LDS const hc_float4 *lp = top_nodes + (size_t)idx * (8 * Q);
#  pragma unroll
          for (int k = 0; k < 7; k++) {
            nd[k] = lp[k];
          }
        }
        else
#endif
        {
          const hc_float4 *np = nodes + (size_t)idx * (8 * Q);
#pragma unroll
          for (int k = 0; k < 7; k++) {
            nd[k] = np[k];
          }
        }
        const hc_uint4 h = as_uint4(nd[0]);
        const float t = CY_T_BOX;
        float d0, d1;
        const bool hit0 = (h.x & visibility) && bvh_obb_intersect(nd[1], nd[2], nd[3], P, dir, t, &d0);
        const bool hit1 = (h.y & visibility) && bvh_obb_intersect(nd[4], nd[5], nd[6], P, dir, t, &d1);
        if (hit0 && hit1) {
          /* nearer child next, the other pushed (bvh_traversal.h:104-125) */
          const bool first1 = d1 < d0;
          if (!CY_STACK_PUSH(first1 ? (int)h.z : (int)h.w, first1 ? d0 : d1)) {
            cy_set_error(err, CY_ERR_BVH_STACK, W);
            return found_hit;
          }
          code = first1 ? (int)h.w : (int)h.z;
          code_t = first1 ? d1 : d0;
          continue;
        }
        if (hit0 || hit1) {
          code = hit0 ? (int)h.z : (int)h.w;
          code_t = hit0 ? d0 : d1;
          continue;
        }
        goto pop;
      }
    }
    if (cur && budget > 0) {
      /* out of iterations: stop before processing `code` (never with entries
       * in the private overflow arrays, which do not outlive this call) */
      if (iters >= budget && n_over == 0) {
        cur->code = code;
        cur->code_t = code_t;
        cur->top = top;
        cur->n_ring = n_ring;
        cur->tie = tie || bad;
        cur->suspended = true;
        break;
      }
      iters++;
    }
    if (code >= 0) {
      /* inner node: test the W child boxes */
      n_nodes++;
      const hc_float4 *np = nodes + (size_t)code * (8 * Q);
      hc_float4 nd[8 * Q];
#if defined(__HIP_DEVICE_COMPILE__) && CY_LDS_TOP > 0
      if (code < n_top) {
#  if CY_LDS_TOP_SOA
        CY_LDS const hc_float4 *lp = top_nodes + code;
#    pragma unroll
        for (int k = 0; k < 8 * Q; k++) {
          nd[k] = lp[k * CY_LDS_TOP];
        }
#  else
        CY_LDS const hc_float4 *lp = top_nodes + (size_t)code * (8 * Q);
#    pragma unroll
        for (int k = 0; k < 8 * Q; k++) {
          nd[k] = lp[k];
        }
#  endif
      }
      else
#endif
      {
#pragma unroll
        for (int k = 0; k < 8 * Q; k++) {
          nd[k] = np[k];
        }
      }
      float tn[W];
      int cc[W];
      const float t = CY_T_BOX;
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const hc_float4 lx = nd[0 * Q + q], hx = nd[1 * Q + q];
        const hc_float4 ly = nd[2 * Q + q], hy = nd[3 * Q + q];
        const hc_float4 lz = nd[4 * Q + q], hz = nd[5 * Q + q];
        const hc_uint4 ch = as_uint4(nd[6 * Q + q]);
        const hc_uint4 mt = as_uint4(nd[7 * Q + q]);
        const float alx[4] = {lx.x, lx.y, lx.z, lx.w}, ahx[4] = {hx.x, hx.y, hx.z, hx.w};
        const float aly[4] = {ly.x, ly.y, ly.z, ly.w}, ahy[4] = {hy.x, hy.y, hy.z, hy.w};
        const float alz[4] = {lz.x, lz.y, lz.z, lz.w}, ahz[4] = {hz.x, hz.y, hz.z, hz.w};
        const uint ach[4] = {ch.x, ch.y, ch.z, ch.w}, amt[4] = {mt.x, mt.y, mt.z, mt.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
#if CY_SLAB_FMA
          const float clox = __builtin_fmaf(alx[j], idir.x, -pix);
          const float chix = __builtin_fmaf(ahx[j], idir.x, -pix);
          const float cloy = __builtin_fmaf(aly[j], idir.y, -piy);
          const float chiy = __builtin_fmaf(ahy[j], idir.y, -piy);
          const float cloz = __builtin_fmaf(alz[j], idir.z, -piz);
          const float chiz = __builtin_fmaf(ahz[j], idir.z, -piz);
          const float cmn = max4(0.0f, cmin(clox, chix), cmin(cloy, chiy), cmin(cloz, chiz)) * (1.0f - 0x1p-20f) -
                            ewide;
          const float cmx = (min4(t, cmax(clox, chix), cmax(cloy, chiy), cmax(cloz, chiz)) + ewide) *
                            (1.0f + 0x1p-20f);
#else
          const float clox = (alx[j] - P.x) * idir.x;
          const float chix = (ahx[j] - P.x) * idir.x;
          const float cloy = (aly[j] - P.y) * idir.y;
          const float chiy = (ahy[j] - P.y) * idir.y;
          const float cloz = (alz[j] - P.z) * idir.z;
          const float chiz = (ahz[j] - P.z) * idir.z;
          const float cmn = slab_max(slab_max(0.0f, slab_min(clox, chix)),
                                     slab_max(slab_min(cloy, chiy), slab_min(cloz, chiz)));
          const float cmx = slab_min(slab_min(t, slab_max(clox, chix)),
                                     slab_min(slab_max(cloy, chiy), slab_max(cloz, chiz)));
#endif
          const bool hit = (cmx >= cmn) && (amt[j] & 0x0FFFFFFFu & visibility);
          const int s = 4 * q + j;
          /* the node stores final codes: inner >= 0, leaf ~(first << 4 | count) */
          cc[s] = (int)ach[j];
          tn[s] = hit ? cmn : CY_INF;
        }
      }
      if (any_hit && CY_ANYHIT_NOSORT) {
        /* any hit ends the query, so the children need no distance order:
         * the first hit child is visited next, the others pushed as found */
        int next = 0;
        bool have_next = false;
#pragma unroll
        for (int s = 0; s < W; s++) {
          if (tn[s] != CY_INF) {
            if (!have_next) {
              next = cc[s];
              have_next = true;
            }
            else if (!CY_STACK_PUSH(cc[s], tn[s])) {
              cy_set_error(err, CY_ERR_BVH_STACK, W);
              return found_hit;
            }
          }
        }
        if (!have_next) {
          goto pop;
        }
        code = next;
        continue;
      }
      if (any_hit && CY_ANYHIT_LEAF_FIRST) {
#pragma unroll
        for (int s = 0; s < W; s++) {
          tn[s] = (tn[s] != CY_INF && cc[s] < 0) ? -1.0f : tn[s];
        }
      }
      bvhw_sort<W>(tn, cc);
      if (tn[0] == CY_INF) {
        goto pop;
      }
      {
        /* push the hit children after the nearest, far to near: make room in
         * the ring first (its oldest entries move to the overflow arrays, as
         * one push at a time would move them; rare), then write them */
        int npush = 0;
#pragma unroll
        for (int s = 1; s < W; s++) {
          npush += tn[s] != CY_INF ? 1 : 0;
        }
        if (n_ring + npush > CY_LDS_STACKW) {
          while (n_ring + npush > CY_LDS_STACKW) {
            if (n_over == CY_OVER_STACK) {
              cy_set_error(err, CY_ERR_BVH_STACK, W);
              return found_hit;
            }
            const CyStackEntry old = ring[((top - n_ring) & (CY_LDS_STACKW - 1)) * CY_RING_STRIDE];
            over_node[n_over] = old.node;
            over_t[n_over] = old.t;
            n_over++;
            n_ring--;
          }
        }
#pragma unroll
        for (int s = W - 1; s >= 1; s--) {
          if (tn[s] != CY_INF) {
            CyStackEntry e_;
            e_.node = cc[s];
            e_.t = tn[s];
            ring[top * CY_RING_STRIDE] = e_;
            top = (top + 1) & (CY_LDS_STACKW - 1);
          }
        }
        n_ring += npush;
      }
      code = cc[0];
      code_t = tn[0];
      continue;
    }
    else {
      /* leaf: contiguous primitive range; the next triangle's vertices are
       * requested before the current one is tested */
      n_leaves++;
      const int packed = ~code;
      int prim_addr = packed >> 4;
      if ((packed & 15) == 0) {
        cy_set_error(err, CY_ERR_FEATURE, 1); /* instance leaf: traversed by bvh2_intersect<.., WI> */
        return found_hit;
      }
      const int prim_end = prim_addr + (packed & 15);
      if constexpr (HAIR != 0) {
        /* hair scenes: a leaf holds one primitive type (the BVH2's leaves,
         * unmerged); ribbon segments here (HAIR = 1: thick curves keep the
         * BVH2, see hipcycles.hip pick_width) */
        if (kg->__prim_type[prim_addr] & PRIMITIVE_ALL_CURVE) {
          for (; prim_addr < prim_end; prim_addr++) {
            n_tris++;
            const uint ctype = kg->__prim_type[prim_addr];
            if (!(ctype & (CY_PRIMITIVE_CURVE_RIBBON | CY_PRIMITIVE_MOTION_CURVE_RIBBON))) {
              cy_set_error(err, CY_ERR_PRIMITIVE, ctype);
              return found_hit;
            }
            if (!(kg->__prim_visibility[prim_addr] & visibility)) {
              continue;
            }
            cy_c4 curve[4];
            curve_segment_keys(kg, (int)kg->__prim_index[prim_addr], (int)CY_PRIMITIVE_UNPACK_SEGMENT(ctype), curve);
            float tt, uu, vv, tmin;
            if (any_hit) {
              /* the reference's ribbon test at the ray's own bound */
              if (ribbon_intersect_steps<false>(P, dir, KD->bvh.curve_subdivisions, curve, isect->t, &tt, &uu, &vv,
                                                &tmin)) {
                isect->prim = prim_addr;
                isect->object = object;
                isect->type = (int)ctype;
                isect->u = uu;
                isect->v = vv;
                isect->t = tt;
                found_hit = true;
                goto ray_done;
              }
              continue;
            }
            /* every step of the ribbon: with one step hit the result is that
             * hit whatever bound it is tested against, like a triangle's; a
             * ribbon crossed twice returns its first step's hit below the
             * bound, which depends on the bound the reference's visiting
             * order gives it -- such a ray is re-traced in that order unless
             * all of its crossings lie beyond the tie window (sticky) */
            const int steps = ribbon_intersect_steps<true>(P, dir, KD->bvh.curve_subdivisions, curve, CY_FLT_MAX, &tt,
                                                           &uu, &vv, &tmin);
            if (steps == 0 || !(tmin <= CY_T_CULL)) {
              continue;
            }
            if (steps > 1) {
              bad |= CY_EXACT_TIES != 0;
              if (!(tt <= isect->t)) {
                continue;
              }
            }
            else {
              tie = CY_EXACT_TIES && !(tt < isect->t * (1.0f - CY_TIE_EPS)) && isect->prim != PRIM_NONE;
              bad |= CY_EXACT_TIES && tt <= isect->t && tt * (1.0f + CY_TIE_EPS) < code_t;
              if (!(tt <= isect->t)) {
                continue; /* inside the window only: the reference's bound rejects it */
              }
            }
            isect->prim = prim_addr;
            isect->object = object;
            isect->type = (int)ctype;
            isect->u = uu;
            isect->v = vv;
            isect->t = tt;
            found_hit = true;
          }
          goto pop;
        }
      }
      const bool ident = kg->tri_index_identity != 0;
      uint vi = ident ? 3u * (uint)prim_addr : kg->__prim_tri_index[prim_addr];
      hc_float4 v0 = kg->__prim_tri_verts[vi], v1 = kg->__prim_tri_verts[vi + 1], v2 = kg->__prim_tri_verts[vi + 2];
      for (; prim_addr < prim_end; prim_addr++) {
        n_tris++;
        hc_float4 w0 = v0, w1 = v1, w2 = v2;
        if (CY_TRI_PREFETCH && prim_addr + 1 < prim_end) {
          vi = ident ? 3u * (uint)(prim_addr + 1) : kg->__prim_tri_index[prim_addr + 1];
          w0 = kg->__prim_tri_verts[vi];
          w1 = kg->__prim_tri_verts[vi + 1];
          w2 = kg->__prim_tri_verts[vi + 2];
        }
        float tt, uu, vv;
        bool exact_ok;
        if (ray_triangle_intersect2(P, dir, CY_T_CULL, isect->t, f4to3(v0), f4to3(v1), f4to3(v2), &uu, &vv, &tt,
                                    &exact_ok) &&
            (kg->__prim_visibility[prim_addr] & visibility)) {
          if (any_hit) {
            isect->prim = prim_addr;
            isect->object = object;
            isect->type = PRIMITIVE_TRIANGLE;
            isect->u = uu;
            isect->v = vv;
            isect->t = tt;
            found_hit = true;
            goto ray_done;
          }
          /* a second hit at (nearly) the distance of the current one -- of this
           * call or the incoming hit -- makes the result depend on the visiting
           * order: flag the ray; a hit clearly below the current one clears it */
          tie = CY_EXACT_TIES && !(tt < isect->t * (1.0f - CY_TIE_EPS)) && isect->prim != PRIM_NONE;
          bad |= CY_EXACT_TIES && exact_ok && tt * (1.0f + CY_TIE_EPS) < code_t;
          if (exact_ok || !CY_TIE_EXACT_OK) {
            /* the reference's acceptance test at the exact bound */
            isect->prim = prim_addr;
            isect->object = object;
            isect->type = PRIMITIVE_TRIANGLE;
            isect->u = uu;
            isect->v = vv;
            isect->t = tt;
            found_hit = true;
          }
        }
        if (CY_TRI_PREFETCH) {
          v0 = w0;
          v1 = w1;
          v2 = w2;
        }
        else if (prim_addr + 1 < prim_end) {
          vi = ident ? 3u * (uint)(prim_addr + 1) : kg->__prim_tri_index[prim_addr + 1];
          v0 = kg->__prim_tri_verts[vi];
          v1 = kg->__prim_tri_verts[vi + 1];
          v2 = kg->__prim_tri_verts[vi + 2];
        }
      }
    }
  pop:
    {
      bool found = false;
      while (n_ring > 0 || n_over > 0) {
        if (n_ring == 0) {
          /* ring drained: move the newest overflow entries back into it (rare;
           * pops then always read LDS, never a pointer that may be private) */
          const int k = n_over < CY_LDS_STACKW ? n_over : CY_LDS_STACKW;
          for (int j = n_over - k; j < n_over; j++) {
            CyStackEntry e_;
            e_.node = over_node[j];
            e_.t = over_t[j];
            ring[top * CY_RING_STRIDE] = e_;
            top = (top + 1) & (CY_LDS_STACKW - 1);
          }
          n_over -= k;
          n_ring = k;
        }
        top = (top - 1) & (CY_LDS_STACKW - 1);
        n_ring--;
        const CyStackEntry e = ring[top * CY_RING_STRIDE];
        code = e.node;
        code_t = e.t;
        if (e.t <= CY_T_BOX) {
          found = true;
          break;
        }
      }
      if (!found) {
        goto ray_done;
      }
    }
    continue;
  ray_done:
    break;
  }

#undef CY_T_CULL
#undef CY_T_BOX
  if (tie_out && (tie || bad)) {
    *tie_out = true;
  }
  if (cnt_nodes) {
    *cnt_nodes += n_nodes;
    *cnt_leaves += n_leaves;
    *cnt_tris += n_tris;
  }
  return found_hit;
}

/* While-while traversal with postponed leaves (Aila & Laine, "Understanding
 * the Efficiency of Ray Traversal on GPUs", HPG 2009), measurement switch.
 * bvhw_traverse handles one node OR one leaf per iteration, so a wave whose
 * lanes are split between inner nodes and leaves runs both bodies every
 * iteration.  Here a lane that meets a leaf parks it and keeps descending
 * inner nodes until every lane of the wave holds a leaf (or has run out of
 * nodes); then the parked leaves are tested together.  Same boxes, culling
 * bounds, triangle test and near-tie bookkeeping as bvhw_traverse; only the
 * order in which leaves are tested changes, which the near-tie window already
 * makes irrelevant to the result. */
#ifndef CY_WHILE_WHILE
#  define CY_WHILE_WHILE 0
#endif

CY_FN bool cy_wave_all(bool p)
{
#if defined(__HIP_DEVICE_COMPILE__)
  return __all(p ? 1 : 0) != 0;
#else
  return p;
#endif
}

template<int W, bool any_hit>
CY_FN bool bvhw_traverse_ww(const CyGlobals *kg,
                            cfloat3 P,
                            cfloat3 dir,
                            cfloat3 idir,
                            uint visibility,
                            CyIsect *isect,
                            uint *err,
                            uint *cnt_nodes,
                            uint *cnt_leaves,
                            uint *cnt_tris,
                            CY_LDS CyStackEntry *lds_ring,
                            bool *tie_out)
{
#if defined(__HIP_DEVICE_COMPILE__)
  CY_LDS CyStackEntry *ring = lds_ring;
#else
  CyStackEntry host_ring[CY_LDS_STACKW];
  CyStackEntry *ring = host_ring;
  (void)lds_ring;
#endif
  int top = 0, n_ring = 0, n_over = 0;
  int over_node[CY_OVER_STACK];
  float over_t[CY_OVER_STACK];
  bool found_hit = false, tie = false;
#define CY_T_CULL ((any_hit || !CY_EXACT_TIES) ? isect->t : isect->t * (1.0f + CY_TIE_EPS))
#define CY_T_BOX ((any_hit || !CY_EXACT_TIES || !CY_TIE_BOX_WIDEN) ? isect->t : isect->t * (1.0f + CY_TIE_EPS))
  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  const hc_float4 *nodes = (const hc_float4 *)kg->bvhw_nodes;
  constexpr int Q = W / 4;

  int code = 0; /* next node or leaf to visit (root) */
  float code_t = 0.0f, leaf_t = 0.0f; /* their boxes' entry distances (see bvhw_traverse `bad`) */
  bool bad = false;
  bool have_code = true;
  int leaf = 0; /* parked leaf */
  bool have_leaf = false;

  /* pops the nearest pending entry that the current hit does not cull */
  auto pop = [&]() -> bool {
    while (n_ring > 0 || n_over > 0) {
      if (n_ring == 0) {
        const int k = n_over < CY_LDS_STACKW ? n_over : CY_LDS_STACKW;
        for (int j = n_over - k; j < n_over; j++) {
          CyStackEntry e_;
          e_.node = over_node[j];
          e_.t = over_t[j];
          ring[top * CY_RING_STRIDE] = e_;
          top = (top + 1) & (CY_LDS_STACKW - 1);
        }
        n_over -= k;
        n_ring = k;
      }
      top = (top - 1) & (CY_LDS_STACKW - 1);
      n_ring--;
      const CyStackEntry e = ring[top * CY_RING_STRIDE];
      if (e.t <= CY_T_BOX) {
        code = e.node;
        code_t = e.t;
        return true;
      }
    }
    return false;
  };

  while (have_code || have_leaf) {
    /* inner phase: descend until every lane holds a leaf or has no nodes left */
    while (!cy_wave_all(have_leaf || !have_code)) {
      if (!have_code || (code < 0 && have_leaf)) {
        continue; /* waits for the wave */
      }
      if (code < 0) {
        leaf = code;
        leaf_t = code_t;
        have_leaf = true;
        have_code = pop();
        continue;
      }
      n_nodes++;
      const hc_float4 *np = nodes + (size_t)code * (8 * Q);
      float tn[W];
      int cc[W];
      const float t = CY_T_BOX;
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const hc_float4 lx = np[0 * Q + q], hx = np[1 * Q + q];
        const hc_float4 ly = np[2 * Q + q], hy = np[3 * Q + q];
        const hc_float4 lz = np[4 * Q + q], hz = np[5 * Q + q];
        const hc_uint4 ch = ((const hc_uint4 *)np)[6 * Q + q];
        const hc_uint4 mt = ((const hc_uint4 *)np)[7 * Q + q];
        const float alx[4] = {lx.x, lx.y, lx.z, lx.w}, ahx[4] = {hx.x, hx.y, hx.z, hx.w};
        const float aly[4] = {ly.x, ly.y, ly.z, ly.w}, ahy[4] = {hy.x, hy.y, hy.z, hy.w};
        const float alz[4] = {lz.x, lz.y, lz.z, lz.w}, ahz[4] = {hz.x, hz.y, hz.z, hz.w};
        const uint ach[4] = {ch.x, ch.y, ch.z, ch.w}, amt[4] = {mt.x, mt.y, mt.z, mt.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const float clox = (alx[j] - P.x) * idir.x;
          const float chix = (ahx[j] - P.x) * idir.x;
          const float cloy = (aly[j] - P.y) * idir.y;
          const float chiy = (ahy[j] - P.y) * idir.y;
          const float cloz = (alz[j] - P.z) * idir.z;
          const float chiz = (ahz[j] - P.z) * idir.z;
          const float cmn = max4(0.0f, cmin(clox, chix), cmin(cloy, chiy), cmin(cloz, chiz));
          const float cmx = min4(t, cmax(clox, chix), cmax(cloy, chiy), cmax(cloz, chiz));
          const bool hit = (cmx >= cmn) && (amt[j] & 0x0FFFFFFFu & visibility);
          const int s = 4 * q + j;
          cc[s] = (int)ach[j];
          tn[s] = hit ? cmn : CY_INF;
        }
      }
      bvhw_sort<W>(tn, cc);
      if (tn[0] == CY_INF) {
        have_code = pop();
        continue;
      }
#pragma unroll
      for (int s = W - 1; s >= 1; s--) {
        if (tn[s] != CY_INF) {
          if (!CY_STACK_PUSH(cc[s], tn[s])) {
            cy_set_error(err, CY_ERR_BVH_STACK, W);
            have_code = false;
            have_leaf = false;
            goto out;
          }
        }
      }
      code = cc[0];
      code_t = tn[0];
    }

    /* leaf phase: the parked leaves of the wave together */
    if (have_leaf) {
      have_leaf = false;
      n_leaves++;
      const int packed = ~leaf;
      int prim_addr = packed >> 4;
      if ((packed & 15) == 0) {
        cy_set_error(err, CY_ERR_FEATURE, 1);
        goto out;
      }
      const int prim_end = prim_addr + (packed & 15);
      const bool ident = kg->tri_index_identity != 0;
      uint vi = ident ? 3u * (uint)prim_addr : kg->__prim_tri_index[prim_addr];
      hc_float4 v0 = kg->__prim_tri_verts[vi], v1 = kg->__prim_tri_verts[vi + 1], v2 = kg->__prim_tri_verts[vi + 2];
      for (; prim_addr < prim_end; prim_addr++) {
        n_tris++;
        hc_float4 w0 = v0, w1 = v1, w2 = v2;
        if (prim_addr + 1 < prim_end) {
          vi = ident ? 3u * (uint)(prim_addr + 1) : kg->__prim_tri_index[prim_addr + 1];
          w0 = kg->__prim_tri_verts[vi];
          w1 = kg->__prim_tri_verts[vi + 1];
          w2 = kg->__prim_tri_verts[vi + 2];
        }
        float tt, uu, vv;
        bool exact_ok;
        if (ray_triangle_intersect2(P, dir, CY_T_CULL, isect->t, f4to3(v0), f4to3(v1), f4to3(v2), &uu, &vv, &tt,
                                    &exact_ok) &&
            (kg->__prim_visibility[prim_addr] & visibility)) {
          if (any_hit) {
            isect->prim = prim_addr;
            isect->object = OBJECT_NONE;
            isect->type = PRIMITIVE_TRIANGLE;
            isect->u = uu;
            isect->v = vv;
            isect->t = tt;
            found_hit = true;
            have_code = false;
            break;
          }
          tie = CY_EXACT_TIES && !(tt < isect->t * (1.0f - CY_TIE_EPS)) && isect->prim != PRIM_NONE;
          bad |= CY_EXACT_TIES && exact_ok && tt * (1.0f + CY_TIE_EPS) < leaf_t;
          if (exact_ok || !CY_TIE_EXACT_OK) {
            isect->prim = prim_addr;
            isect->object = OBJECT_NONE;
            isect->type = PRIMITIVE_TRIANGLE;
            isect->u = uu;
            isect->v = vv;
            isect->t = tt;
            found_hit = true;
          }
        }
        v0 = w0;
        v1 = w1;
        v2 = w2;
      }
    }
  }
out:
#undef CY_T_CULL
#undef CY_T_BOX
  if (tie_out && (tie || bad)) {
    *tie_out = true;
  }
  if (cnt_nodes) {
    *cnt_nodes += n_nodes;
    *cnt_leaves += n_leaves;
    *cnt_tris += n_tris;
  }
  return found_hit;
}

/* Closest hit (any_hit == false) or opaque-shadow any hit over a scene without
 * instances with the wide BVH: scene_intersect (bvh/bvh.h:154-237). */
template<int W, bool any_hit, int HAIR = 0>
CY_FN bool bvhw_intersect(const CyGlobals *kg,
                          const CyRay *ray,
                          uint visibility,
                          CyIsect *isect,
                          uint *err,
                          uint *cnt_nodes,
                          uint *cnt_leaves,
                          uint *cnt_tris,
                          CY_LDS CyStackEntry *lds_ring = nullptr,
                          bool *tie = nullptr,
                          CY_LDS const hc_float4 *top_nodes = nullptr,
                          int n_top = 0)
{
  isect->t = ray->t;
  isect->u = 0.0f;
  isect->v = 0.0f;
  isect->prim = PRIM_NONE;
  isect->object = OBJECT_NONE;
  isect->type = 0;
  const cfloat3 dir = bvh_clamp_direction(ray->D);
#if CY_WHILE_WHILE
  bvhw_traverse_ww<W, any_hit>(kg, ray->P, dir, rcp3(dir), visibility, isect, err, cnt_nodes, cnt_leaves, cnt_tris,
                               lds_ring, tie);
#else
  bvhw_traverse<W, any_hit, HAIR>(kg, 0, ray->P, dir, rcp3(dir), OBJECT_NONE, visibility, isect, err, cnt_nodes,
                                  cnt_leaves, cnt_tris, lds_ring, tie, 0, nullptr, top_nodes, n_top);
#endif
  return isect->prim != PRIM_NONE;
}

#endif /* CY_BVHW_H */
