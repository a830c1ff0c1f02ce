/*
 * cy_bvh8.h — closest-hit and opaque any-hit traversal of the device's 8-wide
 * quantized BVH (layout: csrc/host/cy_bvh8_collapse.h).
 *
 * Same query as bvh2_intersect (bvh/bvh_traversal.h:34-227): identical
 * direction clamp, slab arithmetic on decoded (conservative) child boxes,
 * ray_triangle_intersect on the same primitive arrays and the same visibility
 * tests, so every triangle the BVH2 traversal accepts is also reached here.
 * Only the visiting order differs, which decides between primitives whose hit
 * distances agree to a few ulp (tests/test_bvh8.py bounds that).
 *
 * Per wide node one 128-B line is read: 64 B of header + quantized bounds, the
 * 8 child boxes are tested, then 64 B of child words / visibility.  Leaf
 * children that are hit are intersected right away in octant order; inner
 * children are visited near-to-far by the octant slot order, the nearest next
 * and the rest pushed with their entry distance (popped entries farther than
 * the current hit are skipped).  The stack lives in LDS (one column per
 * thread) for its first CY_LDS_STACK8 entries.
 */
#ifndef CY_BVH8_H
#define CY_BVH8_H

#include "cy_path.h"

#ifndef CY_LDS_STACK8
#  define CY_LDS_STACK8 16
#endif
#define CY_BVH8_STACK 128

struct CyStack8 {
  int *lds_node; /* &lds_base[threadIdx.x] or nullptr */
  float *lds_t;
  int spill_node[CY_BVH8_STACK];
  float spill_t[CY_BVH8_STACK];
  CY_MFN void set(int i, int node, float t)
  {
    if (lds_node && i < CY_LDS_STACK8) {
      lds_node[i * CY_BLOCK] = node;
      lds_t[i * CY_BLOCK] = t;
    }
    else {
      spill_node[i] = node;
      spill_t[i] = t;
    }
  }
  CY_MFN void get(int i, int *node, float *t) const
  {
    if (lds_node && i < CY_LDS_STACK8) {
      *node = lds_node[i * CY_BLOCK];
      *t = lds_t[i * CY_BLOCK];
    }
    else {
      *node = spill_node[i];
      *t = spill_t[i];
    }
  }
};

CY_FN uint bvh8_byte(uint w, int k)
{
  return (w >> (8 * k)) & 0xFFu;
}

/* slot-ordered bit mask -> k-ordered (k = slot ^ c): a fixed bit permutation */
CY_FN uint bvh8_permute(uint m, uint c)
{
  if (c & 1u) m = ((m & 0x55u) << 1) | ((m & 0xAAu) >> 1);
  if (c & 2u) m = ((m & 0x33u) << 2) | ((m & 0xCCu) >> 2);
  if (c & 4u) m = ((m & 0x0Fu) << 4) | ((m & 0xF0u) >> 4);
  return m;
}

CY_FN uint bvh8_select(const uint (&a)[8], int i)
{
  uint r = a[0];
#pragma unroll
  for (int j = 1; j < 8; j++) {
    r = (i == j) ? a[j] : r;
  }
  return r;
}

CY_FN float bvh8_selectf(const float (&a)[8], int i)
{
  float r = a[0];
#pragma unroll
  for (int j = 1; j < 8; j++) {
    r = (i == j) ? a[j] : r;
  }
  return r;
}

CY_FN int bvh8_lowest(uint m)
{
  return find_first_set(m) - 1;
}

CY_FN int bvh8_highest(uint m)
{
  return 31 - __builtin_clz(m);
}

template<bool any_hit>
CY_FN bool bvh8_intersect(const CyGlobals *kg,
                          const CyRay *ray,
                          uint visibility,
                          CyIsect *isect,
                          uint *err,
                          uint *cnt_nodes,
                          uint *cnt_leaves,
                          uint *cnt_tris,
                          int *lds_stack = nullptr)
{
  CyStack8 stack;
  stack.lds_node = lds_stack;
  stack.lds_t = lds_stack ? (float *)(lds_stack + CY_LDS_STACK8 * CY_BLOCK) : nullptr;
  int sp = 0;

  const cfloat3 P = ray->P;
  const cfloat3 dir = bvh_clamp_direction(ray->D);
  const cfloat3 idir = rcp3(dir);
  const uint oct = (dir.x < 0.0f ? 1u : 0u) | (dir.y < 0.0f ? 2u : 0u) | (dir.z < 0.0f ? 4u : 0u);
  const uint c = 7u ^ oct;

  isect->t = ray->t;
  isect->u = 0.0f;
  isect->v = 0.0f;
  isect->prim = PRIM_NONE;
  isect->object = OBJECT_NONE;
  isect->type = 0;

  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  const hc_uint4 *nodes = kg->bvh8_nodes;
  int node = 0;

  while (true) {
    n_nodes++;
    const hc_uint4 *np = nodes + (size_t)node * 8;
    const hc_uint4 h0 = np[0];
    const hc_uint4 bx = np[1];
    const hc_uint4 by = np[2];
    const hc_uint4 bz = np[3];
    const float ox = as_float(h0.x), oy = as_float(h0.y), oz = as_float(h0.z);
    const float sx = as_float((h0.w & 0xFFu) << 23);
    const float sy = as_float(((h0.w >> 8) & 0xFFu) << 23);
    const float sz = as_float(((h0.w >> 16) & 0xFFu) << 23);
    const float t = isect->t;
    float tmin[8];
    uint box_hits = 0;
#pragma unroll
    for (int s = 0; s < 8; s++) {
      const uint wlo = (s < 4) ? 0 : 1;
      const int sh = s & 3;
      const float lox = ox + (float)bvh8_byte(wlo ? bx.y : bx.x, sh) * sx;
      const float hix = ox + (float)bvh8_byte(wlo ? bx.w : bx.z, sh) * sx;
      const float loy = oy + (float)bvh8_byte(wlo ? by.y : by.x, sh) * sy;
      const float hiy = oy + (float)bvh8_byte(wlo ? by.w : by.z, sh) * sy;
      const float loz = oz + (float)bvh8_byte(wlo ? bz.y : bz.x, sh) * sz;
      const float hiz = oz + (float)bvh8_byte(wlo ? bz.w : bz.z, sh) * sz;
      const float clox = (lox - P.x) * idir.x;
      const float chix = (hix - P.x) * idir.x;
      const float cloy = (loy - P.y) * idir.y;
      const float chiy = (hiy - P.y) * idir.y;
      const float cloz = (loz - P.z) * idir.z;
      const float chiz = (hiz - P.z) * idir.z;
      const float cmn = max4(0.0f, cmin(clox, chix), cmin(cloy, chiy), cmin(cloz, chiz));
      const float cmx = min4(t, cmax(clox, chix), cmax(cloy, chiy), cmax(cloz, chiz));
      tmin[s] = cmn;
      box_hits |= (cmx >= cmn) ? (1u << s) : 0u;
    }

    uint leaf_k = 0, inner_k = 0;
    uint child[8], meta[8];
    if (box_hits) {
      const hc_uint4 c0 = np[4];
      const hc_uint4 c1 = np[5];
      const hc_uint4 v0 = np[6];
      const hc_uint4 v1 = np[7];
      child[0] = c0.x; child[1] = c0.y; child[2] = c0.z; child[3] = c0.w;
      child[4] = c1.x; child[5] = c1.y; child[6] = c1.z; child[7] = c1.w;
      meta[0] = v0.x; meta[1] = v0.y; meta[2] = v0.z; meta[3] = v0.w;
      meta[4] = v1.x; meta[5] = v1.y; meta[6] = v1.z; meta[7] = v1.w;
      uint leaf_s = 0, inner_s = 0;
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const bool h = ((box_hits >> s) & 1u) && (meta[s] & 0x0FFFFFFFu & visibility);
        const bool is_leaf = (int)child[s] < 0;
        leaf_s |= (h && is_leaf) ? (1u << s) : 0u;
        inner_s |= (h && !is_leaf) ? (1u << s) : 0u;
      }
      leaf_k = bvh8_permute(leaf_s, c);
      inner_k = bvh8_permute(inner_s, c);
    }

    /* leaf children, near to far */
    while (leaf_k) {
      const int k = bvh8_lowest(leaf_k);
      leaf_k &= leaf_k - 1u;
      const int s = k ^ (int)c;
      n_leaves++;
      int prim_addr = ~(int)bvh8_select(child, s);
      const int prim_end = prim_addr + (int)(bvh8_select(meta, s) >> 28);
      for (; prim_addr < prim_end; prim_addr++) {
        n_tris++;
        const uint tri_vindex = kg->__prim_tri_index[prim_addr];
        const hc_float4 *tv = kg->__prim_tri_verts + tri_vindex;
        float tt, uu, vv;
        if (ray_triangle_intersect(P, dir, isect->t, f4to3(tv[0]), f4to3(tv[1]), f4to3(tv[2]), &uu, &vv, &tt)) {
          if (kg->__prim_visibility[prim_addr] & visibility) {
            isect->prim = prim_addr;
            isect->object = OBJECT_NONE;
            isect->type = PRIMITIVE_TRIANGLE;
            isect->u = uu;
            isect->v = vv;
            isect->t = tt;
            if (any_hit) {
              if (cnt_nodes) {
                *cnt_nodes += n_nodes;
                *cnt_leaves += n_leaves;
                *cnt_tris += n_tris;
              }
              return true;
            }
          }
        }
      }
    }

    if (inner_k) {
      /* push all but the nearest, farthest first */
      const int k0 = bvh8_lowest(inner_k);
      uint rest = inner_k & (inner_k - 1u);
      while (rest) {
        const int k = bvh8_highest(rest);
        rest &= ~(1u << k);
        const int s = k ^ (int)c;
        if (sp >= CY_BVH8_STACK) {
          cy_set_error(err, CY_ERR_BVH_STACK, 8);
          return false;
        }
        stack.set(sp++, (int)bvh8_select(child, s), bvh8_selectf(tmin, s));
      }
      node = (int)bvh8_select(child, k0 ^ (int)c);
      continue;
    }

    /* pop the next entry still in front of the current hit */
    bool found = false;
    while (sp > 0) {
      float et;
      stack.get(--sp, &node, &et);
      if (et <= isect->t) {
        found = true;
        break;
      }
    }
    if (!found) {
      break;
    }
  }

  if (cnt_nodes) {
    *cnt_nodes += n_nodes;
    *cnt_leaves += n_leaves;
    *cnt_tris += n_tris;
  }
  return (isect->prim != PRIM_NONE);
}

#endif /* CY_BVH8_H */
