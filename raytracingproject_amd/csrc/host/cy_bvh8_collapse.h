/*
 * cy_bvh8_collapse.h — widen the host's packed BVH2 into the device's 8-wide
 * quantized BVH (host C++, header-only; used by the device library when the
 * BVH arrays are bound, and by the CPU tests).
 *
 * The host keeps building Cycles' BVH2 (bvh/bvh2.cpp pack_aligned_node /
 * pack_leaf: 4 float4 per inner node, 1 float4 per leaf, leaf address ~i) and
 * binds it as __bvh_nodes / __bvh_leaf_nodes; get_bvh_layout_mask() stays
 * BVH_LAYOUT_BVH2.  This is the widening step the reference does for its
 * 4/8-wide CPU layouts in BVH::pack_nodes / widen_children_nodes
 * (bvh/bvh.cpp:149-176), done here on the BVH2 the device was handed, so the
 * primitive arrays and primitive indices are untouched.
 *
 * Collapse: starting at the BVH2 root, a wide node takes the two children of a
 * BVH2 node and repeatedly opens the inner child of largest surface area until
 * it holds 8 children or only leaves.  Every BVH2 leaf (<= 8 triangles in a
 * contiguous primitive range) becomes a leaf child.
 *
 * Node (CY_BVH8_NODE_UINT4 = 8 x uint4 = 128 B, one HBM/L2 line):
 *   u0 : origin.xyz (float), w = ex | ey << 8 | ez << 16 (biased exponents
 *        of the per-axis scale 2^(e-127))
 *   u1 : x bounds: bytes qlo[0..7] (x, y), qhi[0..7] (z, w)
 *   u2 : y bounds, u3 : z bounds (same packing)
 *   u4, u5 : child words, slot 0..7: >= 0 inner child node index, < 0 leaf
 *            ~first_primitive
 *   u6, u7 : per-slot visibility (low 28 bits, the BVH2 node's child visibility)
 *            | primitive count << 28 for leaves; 0 = empty slot
 * Decoded bounds lo = origin + (float)q * scale are computed with the same
 * float operations on host and device; the builder adjusts q until every
 * decoded box contains the exact BVH2 child box, so the slab test of a wide
 * child passes whenever the reference BVH2 test of that child passes.
 *
 * Slots are assigned per node so that slot s holds the child whose centroid
 * offset best matches the octant with sign bits s; a ray whose direction has
 * sign bits o visits hit children in order k = 0..7 of slot k ^ (7 ^ o)
 * (near-to-far without sorting).
 */
#ifndef CY_BVH8_COLLAPSE_H
#define CY_BVH8_COLLAPSE_H

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#define CY_BVH8_NODE_UINT4 8

namespace cybvh8 {

struct Box {
  float lo[3], hi[3];
};

struct Ref {
  int addr; /* BVH2 address: >= 0 inner node (float4 units), < 0 leaf ~index */
  Box box;
  uint32_t vis;
};

static inline uint32_t f2u(float f)
{
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

static inline float u2f(uint32_t u)
{
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static inline float area(const Box &b)
{
  const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  return dx * dy + dy * dz + dz * dx;
}

/* decode exactly as the device does (no contraction: built with -ffp-contract=off) */
static inline float decode(float origin, uint32_t q, float scale)
{
  volatile float qs = (float)q * scale;
  return origin + qs;
}

struct Collapser {
  const float *nodes2;    /* __bvh_nodes as floats (4 per float4) */
  size_t n_nodes2;        /* float4 count */
  const float *leaves2;   /* __bvh_leaf_nodes */
  size_t n_leaves2;
  std::vector<uint32_t> out; /* 32 uint32 per wide node */
  std::string error;
  int max_depth = 0;

  void children(int addr, Ref c[2])
  {
    const float *n = nodes2 + 4 * (size_t)addr;
    uint32_t w[4];
    memcpy(w, n, 16);
    for (int k = 0; k < 2; k++) {
      c[k].vis = w[k];
      c[k].addr = (int)w[2 + k];
      c[k].box.lo[0] = n[4 + k];
      c[k].box.hi[0] = n[4 + 2 + k];
      c[k].box.lo[1] = n[8 + k];
      c[k].box.hi[1] = n[8 + 2 + k];
      c[k].box.lo[2] = n[12 + k];
      c[k].box.hi[2] = n[12 + 2 + k];
    }
  }

  bool leaf_range(int addr, int *start, int *count, uint32_t *vis)
  {
    const size_t li = (size_t)(-addr - 1);
    if (li >= n_leaves2) {
      error = "leaf index out of range";
      return false;
    }
    uint32_t w[4];
    memcpy(w, leaves2 + 4 * li, 16);
    const int s = (int)w[0], e = (int)w[1];
    if (s < 0) {
      error = "instanced BVH leaves are not supported";
      return false;
    }
    if ((w[3] & 1u) == 0u) { /* PRIMITIVE_TRIANGLE = 1 */
      error = "only triangle leaves are supported";
      return false;
    }
    if (e - s < 1 || e - s > 15) {
      error = "leaf with " + std::to_string(e - s) + " primitives";
      return false;
    }
    *start = s;
    *count = e - s;
    *vis = w[2];
    return true;
  }

  /* Quantize one axis: choose exponent, then per-child q with containment. */
  bool quantize_axis(float plo, float phi, const Ref *ch, int n, int axis, uint8_t *qlo, uint8_t *qhi,
                     uint32_t *ebias)
  {
    const float extent = phi - plo;
    int e = -100;
    if (extent > 0.0f) {
      e = (int)std::ceil(std::log2((double)extent / 255.0));
    }
    if (e < -126) {
      e = -126;
    }
    for (; e < 127; e++) {
      const float scale = u2f((uint32_t)(e + 127) << 23);
      bool ok = true;
      for (int i = 0; i < n && ok; i++) {
        const float clo = ch[i].box.lo[axis], chi = ch[i].box.hi[axis];
        double fl = std::floor(((double)clo - (double)plo) / (double)scale);
        long q = fl < 0 ? 0 : (long)fl;
        if (q > 255) q = 255;
        while (q > 0 && decode(plo, (uint32_t)q, scale) > clo) q--;
        if (decode(plo, (uint32_t)q, scale) > clo) {
          ok = false;
          break;
        }
        double fh = std::ceil(((double)chi - (double)plo) / (double)scale);
        long r = fh < 0 ? 0 : (long)fh;
        if (r < q) r = q;
        while (r <= 255 && decode(plo, (uint32_t)r, scale) < chi) r++;
        if (r > 255) {
          ok = false;
          break;
        }
        qlo[i] = (uint8_t)q;
        qhi[i] = (uint8_t)r;
      }
      if (ok) {
        *ebias = (uint32_t)(e + 127);
        return true;
      }
    }
    error = "quantization failed";
    return false;
  }

  bool emit(size_t idx, Ref *ch, int n, std::vector<std::pair<size_t, Ref>> *pending)
  {
    Box pb = ch[0].box;
    for (int i = 1; i < n; i++) {
      for (int a = 0; a < 3; a++) {
        pb.lo[a] = fminf(pb.lo[a], ch[i].box.lo[a]);
        pb.hi[a] = fmaxf(pb.hi[a], ch[i].box.hi[a]);
      }
    }
    /* octant slot assignment (greedy over child/slot scores) */
    float pc[3];
    for (int a = 0; a < 3; a++) pc[a] = 0.5f * (pb.lo[a] + pb.hi[a]);
    int slot_of[8];
    bool used_slot[8] = {false}, used_child[8] = {false};
    for (int round = 0; round < n; round++) {
      float best = -FLT_MAX;
      int bc = -1, bs = -1;
      for (int i = 0; i < n; i++) {
        if (used_child[i]) continue;
        for (int s = 0; s < 8; s++) {
          if (used_slot[s]) continue;
          float score = 0.0f;
          for (int a = 0; a < 3; a++) {
            const float off = 0.5f * (ch[i].box.lo[a] + ch[i].box.hi[a]) - pc[a];
            score += ((s >> a) & 1) ? -off : off;
          }
          if (score > best) {
            best = score;
            bc = i;
            bs = s;
          }
        }
      }
      used_child[bc] = true;
      used_slot[bs] = true;
      slot_of[bc] = bs;
    }
    uint8_t qlo[3][8], qhi[3][8];
    uint32_t eb[3];
    for (int a = 0; a < 3; a++) {
      if (!quantize_axis(pb.lo[a], pb.hi[a], ch, n, a, qlo[a], qhi[a], &eb[a])) {
        return false;
      }
    }
    uint32_t w[32];
    memset(w, 0, sizeof(w));
    w[0] = f2u(pb.lo[0]);
    w[1] = f2u(pb.lo[1]);
    w[2] = f2u(pb.lo[2]);
    w[3] = eb[0] | (eb[1] << 8) | (eb[2] << 16);
    uint8_t *bytes = reinterpret_cast<uint8_t *>(w);
    for (int i = 0; i < n; i++) {
      const int s = slot_of[i];
      for (int a = 0; a < 3; a++) {
        bytes[16 * (1 + a) + s] = qlo[a][i];
        bytes[16 * (1 + a) + 8 + s] = qhi[a][i];
      }
      const uint32_t vis = ch[i].vis & 0x0FFFFFFFu;
      if (vis == 0u) {
        continue; /* invisible to every ray kind: leave the slot empty */
      }
      if (ch[i].addr < 0) {
        int start, count;
        uint32_t lvis;
        if (!leaf_range(ch[i].addr, &start, &count, &lvis)) {
          return false;
        }
        w[16 + s] = (uint32_t)(~start);
        w[24 + s] = vis | ((uint32_t)count << 28);
      }
      else {
        const size_t child = out.size() / 32;
        out.resize(out.size() + 32, 0u);
        w[16 + s] = (uint32_t)child;
        w[24 + s] = vis;
        pending->push_back(std::make_pair(child, ch[i]));
      }
    }
    memcpy(&out[idx * 32], w, sizeof(w));
    return true;
  }

  bool open(const Ref &r, Ref ch[8], int *n)
  {
    children(r.addr, ch);
    *n = 2;
    while (*n < 8) {
      int best = -1;
      float ba = -1.0f;
      for (int i = 0; i < *n; i++) {
        if (ch[i].addr >= 0 && (ch[i].vis & 0x0FFFFFFFu) && area(ch[i].box) > ba) {
          ba = area(ch[i].box);
          best = i;
        }
      }
      if (best < 0) {
        break;
      }
      Ref two[2];
      children(ch[best].addr, two);
      ch[best] = two[0];
      ch[(*n)++] = two[1];
    }
    return true;
  }

  /* root: BVH2 root address (KernelBVH.root) */
  bool run(int root)
  {
    out.clear();
    out.resize(32, 0u);
    std::vector<std::pair<size_t, Ref>> pending, next;
    Ref ch[8];
    int n = 0;
    if (root < 0) {
      /* single-leaf scene: one wide node holding the leaf (unbounded box) */
      int start, count;
      uint32_t vis;
      if (!leaf_range(root, &start, &count, &vis)) {
        return false;
      }
      ch[0].addr = root;
      ch[0].vis = vis;
      for (int a = 0; a < 3; a++) {
        ch[0].box.lo[a] = -FLT_MAX;
        ch[0].box.hi[a] = FLT_MAX;
      }
      /* unbounded box: origin -FLT_MAX, scale 2^127 decodes to [-FLT_MAX, inf] */
      uint32_t *w = &out[0];
      w[0] = w[1] = w[2] = f2u(-FLT_MAX);
      w[3] = 254u | (254u << 8) | (254u << 16);
      uint8_t *bytes = reinterpret_cast<uint8_t *>(w);
      for (int a = 0; a < 3; a++) {
        bytes[16 * (1 + a) + 0] = 0;
        bytes[16 * (1 + a) + 8] = 255;
      }
      w[16] = (uint32_t)(~start);
      w[24] = (vis & 0x0FFFFFFFu) | ((uint32_t)count << 28);
      return true;
    }
    Ref r;
    r.addr = root;
    r.vis = 0xFFFFFFFFu;
    open(r, ch, &n);
    if (!emit(0, ch, n, &pending)) {
      return false;
    }
    int depth = 1;
    while (!pending.empty()) {
      next.clear();
      for (auto &p : pending) {
        open(p.second, ch, &n);
        if (!emit(p.first, ch, n, &next)) {
          return false;
        }
      }
      pending.swap(next);
      depth++;
    }
    max_depth = depth;
    return true;
  }
};

}  // namespace cybvh8

#endif
