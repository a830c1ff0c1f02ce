/*
 * cy_bvhw_collapse.h — widen the host's packed BVH2 into the device's W-wide
 * BVH (W = 4 or 8; host C++, header-only; used by the device library when the
 * BVH arrays are bound, and by the CPU tests through tools/host_emu.cpp).
 *
 * The host keeps building Cycles' BVH2 (bvh/bvh2.cpp pack_aligned_node /
 * pack_leaf: 4 float4 per inner node, 1 float4 per leaf, leaf address ~i) and
 * binds it as __bvh_nodes / __bvh_leaf_nodes; get_bvh_layout_mask() stays
 * BVH_LAYOUT_BVH2.  This is the widening step the reference does for its
 * 4/8-wide CPU layouts in BVH::pack_nodes / widen_children_nodes
 * (bvh/bvh.cpp:149-176), done on the BVH2 the device was handed, so the
 * primitive arrays and primitive indices are untouched.
 *
 * Collapse: a wide node starts from the two children of a BVH2 node and
 * repeatedly opens the inner child of largest surface area until it holds W
 * children or only leaves.  A BVH2 leaf becomes a leaf child (its primitive
 * range); an inner BVH2 subtree whose leaves hold at most `merge_prims`
 * primitives in one contiguous range also becomes a single leaf child.
 *
 * Node (32*W bytes: 128 B for W = 4, one L2 line; 256 B for W = 8), arrays of
 * W 32-bit words:  lo.x  hi.x  lo.y  hi.y  lo.z  hi.z  child  meta
 *   bounds : the exact BVH2 child boxes (float), so the slab test of a wide
 *            child is bit-for-bit the reference's test of that BVH2 child
 *            (bvh/bvh_nodes.h:31-80);
 *   child  : >= 0 inner child node index, < 0 leaf ~(first_primitive << 4 |
 *            count) (instance leaf: ~(object << 4), count 0), the code the
 *            traversal pushes as it is;
 *   meta   : child visibility (low 28 bits, as the BVH2 node stored it) |
 *            primitive count << 28 for leaves (0 for an instance); 0 = empty slot.
 * Instanced geometry (two-level BVH, bvh/bvh.cpp:323-520): each object BVH
 * root __object_node[object] is collapsed once into its own wide subtree;
 * object_root[object] is its wide root.
 *
 * Curves (allow_curves): the hair BVH2 stores the children of an *unaligned*
 * node as oriented boxes (bvh2.cpp:133-163 pack_unaligned_node: visibility |
 * PATH_RAY_NODE_UNALIGNED, the two children, per child the transform taking
 * its box to the unit cube; 7 float4).  Each child's transform is absolute
 * (world space to its unit cube), but a child's oriented box need not lie
 * inside its parent's, so unaligned nodes are not widened: each is copied as
 * an oriented two-child *OBB node* (code CY_BVHW_OBB | index) whose
 * transforms are the reference's own, and the traversal applies the
 * reference's oriented slab test to them on every unaligned node of a path.
 * Wide nodes open only aligned BVH2 nodes (an aligned child's box lies inside
 * its parent's, so skipping it culls nothing the reference keeps); an
 * unaligned child stays a wide child (the box its aligned parent stores) and
 * becomes an OBB node below it.  Curve leaves keep their primitive ranges (merging is off: a
 * merged leaf could mix types); the traversal reads the primitive type.
 */
#ifndef CY_BVHW_COLLAPSE_H
#define CY_BVHW_COLLAPSE_H

#include <cfloat>
#include <cstdint>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace cybvhw {

/* child code of an OBB node: its node index with this bit set (codes of wide
 * inner nodes stay below it, leaf codes are negative) */
static constexpr uint32_t OBB_CODE = 1u << 30;
static constexpr uint32_t NODE_UNALIGNED = 1u << 13; /* PATH_RAY_NODE_UNALIGNED */

struct Ref {
  int addr; /* BVH2 address: >= 0 inner node (float4 units), < 0 leaf ~index */
  float lo[3], hi[3];
  uint32_t vis;
};

static inline float area(const Ref &b)
{
  const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  return dx * dy + dy * dz + dz * dx;
}

struct Collapser {
  int width = 4;
  int merge_prims = 0; /* subtrees with <= this many contiguous primitives become one leaf */
  const float *nodes2 = nullptr; /* __bvh_nodes as floats (4 per float4) */
  size_t n_nodes2 = 0;           /* float4 count */
  const float *leaves2 = nullptr;
  size_t n_leaves2 = 0;
  const uint32_t *prim_object = nullptr; /* __prim_object (instance leaves) */
  size_t n_prims = 0;
  const uint32_t *object_node = nullptr; /* __object_node: BVH2 root of each object's own BVH */
  size_t n_objects = 0;
  std::vector<int> object_root; /* per object: wide root of its BVH, -1 if not instanced */
  std::vector<uint32_t> out; /* 8 * width words per wide node */
  std::string error;
  int max_depth = 0;
  std::vector<int> sub_start, sub_count; /* per BVH2 inner node (index addr/4): contiguous range or -1 */
  bool allow_curves = false; /* hair BVH2: unaligned nodes become OBB nodes, curve leaves, no merging */
  size_t n_obb = 0;          /* OBB nodes emitted */

  bool unaligned(int addr) const
  {
    if (!allow_curves || addr < 0 || (size_t)addr >= n_nodes2) {
      return false;
    }
    uint32_t w0;
    memcpy(&w0, nodes2 + 4 * (size_t)addr, 4);
    return (w0 & NODE_UNALIGNED) != 0;
  }

  size_t words() const
  {
    return 8 * (size_t)width;
  }

  void children(int addr, Ref c[2]) const
  {
    const float *n = nodes2 + 4 * (size_t)addr;
    uint32_t w[4];
    memcpy(w, n, 16);
    for (int k = 0; k < 2; k++) {
      c[k].vis = w[k];
      c[k].addr = (int)w[2 + k];
      c[k].lo[0] = n[4 + k];
      c[k].hi[0] = n[4 + 2 + k];
      c[k].lo[1] = n[8 + k];
      c[k].hi[1] = n[8 + 2 + k];
      c[k].lo[2] = n[12 + k];
      c[k].hi[2] = n[12 + 2 + k];
    }
  }

  bool leaf_range(int addr, int *start, int *count)
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
      /* object instance leaf (bvh2.cpp pack_leaf: ~slot, 0): code it as a
       * count-0 leaf whose index is the object */
      const size_t slot = (size_t)(~s);
      if (!prim_object || slot >= n_prims) {
        error = "instance leaf without __prim_object";
        return false;
      }
      const uint32_t ob = prim_object[slot];
      if (!object_node || ob >= n_objects || ob >= (1u << 27)) {
        error = "instance leaf object out of range";
        return false;
      }
      instances.push_back((int)ob);
      *start = (int)ob;
      *count = 0;
      return true;
    }
    /* PRIMITIVE_TRIANGLE = 1; curves: PRIMITIVE_ALL_CURVE = bits 2..5 */
    if ((w[3] & 1u) == 0u && !(allow_curves && (w[3] & 0x3Cu))) {
      error = allow_curves ? "leaf of an unsupported primitive type" : "only triangle leaves are supported";
      return false;
    }
    if (e - s < 1 || e - s > 15) {
      error = "leaf with " + std::to_string(e - s) + " primitives";
      return false;
    }
    *start = s;
    *count = e - s;
    return true;
  }

  /* contiguous primitive range of a BVH2 subtree (memoised), or count -1 */
  bool subtree_range(int addr, int *start, int *count)
  {
    if (addr < 0) {
      return leaf_range(addr, start, count);
    }
    const size_t i = (size_t)addr / 4;
    if (sub_count[i] != -2) {
      *start = sub_start[i];
      *count = sub_count[i];
      return true;
    }
    Ref c[2];
    children(addr, c);
    int s0, n0, s1, n1;
    if (!subtree_range(c[0].addr, &s0, &n0) || !subtree_range(c[1].addr, &s1, &n1)) {
      return false;
    }
    int s = -1, n = -1;
    if (n0 > 0 && n1 > 0 && (c[0].vis & 0x0FFFFFFFu) == (c[1].vis & 0x0FFFFFFFu)) {
      if (s0 + n0 == s1) {
        s = s0;
        n = n0 + n1;
      }
      else if (s1 + n1 == s0) {
        s = s1;
        n = n0 + n1;
      }
    }
    if (n > 15) {
      n = -1;
    }
    sub_start[i] = s;
    sub_count[i] = n;
    *start = s;
    *count = n;
    return true;
  }

  bool mergeable(const Ref &r, int *start, int *count)
  {
    if (r.addr < 0) {
      return leaf_range(r.addr, start, count);
    }
    if (merge_prims <= 0 || allow_curves) {
      return false;
    }
    int s, n;
    if (!subtree_range(r.addr, &s, &n)) {
      return false;
    }
    if (n > 0 && n <= merge_prims) {
      *start = s;
      *count = n;
      return true;
    }
    return false;
  }

  bool open(const Ref &r, Ref *ch, int *n)
  {
    children(r.addr, ch);
    *n = 2;
    while (*n < width) {
      int best = -1;
      float ba = -1.0f;
      for (int i = 0; i < *n; i++) {
        int s, c;
        if (ch[i].addr < 0 || (ch[i].vis & 0x0FFFFFFFu) == 0u || unaligned(ch[i].addr)) {
          continue; /* leaves, invisible children and oriented-box nodes stay */
        }
        if (mergeable(ch[i], &s, &c)) {
          continue;
        }
        if (!error.empty()) {
          return false;
        }
        if (area(ch[i]) > ba) {
          ba = area(ch[i]);
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
    return error.empty();
  }

  bool emit(size_t idx, const Ref *ch, int n, std::vector<std::pair<size_t, Ref>> *pending)
  {
    const int W = width;
    std::vector<uint32_t> w(words(), 0u);
    float *f = reinterpret_cast<float *>(w.data());
    for (int s = 0; s < W; s++) {
      /* empty slot: inverted box, never hit (meta 0 also rejects it) */
      f[0 * W + s] = FLT_MAX;
      f[1 * W + s] = -FLT_MAX;
      f[2 * W + s] = FLT_MAX;
      f[3 * W + s] = -FLT_MAX;
      f[4 * W + s] = FLT_MAX;
      f[5 * W + s] = -FLT_MAX;
    }
    int s = 0;
    for (int i = 0; i < n; i++) {
      const uint32_t vis = ch[i].vis & 0x0FFFFFFFu;
      if (vis == 0u) {
        continue; /* invisible to every ray kind */
      }
      for (int a = 0; a < 3; a++) {
        f[(2 * a) * W + s] = ch[i].lo[a];
        f[(2 * a + 1) * W + s] = ch[i].hi[a];
      }
      int start, count;
      if (mergeable(ch[i], &start, &count)) {
        if (start >= (1 << 27)) {
          error = "primitive index beyond the 2^27 leaf-code range";
          return false;
        }
        w[6 * W + s] = ~(((uint32_t)start << 4) | (uint32_t)count);
        w[7 * W + s] = vis | ((uint32_t)count << 28);
      }
      else if (!error.empty()) {
        return false;
      }
      else {
        const size_t child = alloc_node(ch[i].addr);
        w[6 * W + s] = (uint32_t)child | (unaligned(ch[i].addr) ? OBB_CODE : 0u);
        w[7 * W + s] = vis;
        pending->push_back(std::make_pair(child, ch[i]));
      }
      s++;
    }
    memcpy(&out[idx * words()], w.data(), words() * 4);
    return true;
  }

  /* Node slots an OBB node takes (112 B: one slot at every W). */
  size_t obb_slots() const
  {
    return 1;
  }

  /* The unaligned BVH2 node at r.addr copied as an OBB node at idx: words 0..3
   * the stored visibility of both children (PATH_RAY_NODE_UNALIGNED included)
   * and their wide codes, words 4..27 the two children's transforms as stored
   * (bvh_unaligned_node_intersect's operands).  Not widened: a child's
   * oriented box need not lie inside its parent's, so the reference's test of
   * every unaligned node on a path is kept (a ribbon hit outside an
   * ancestor's box is culled there; skipping that test found such hits --
   * measured on the JNK crop: 9 film values off at 1024 spp). */
  bool emit_obb(size_t idx, const Ref &r, std::vector<std::pair<size_t, Ref>> *pending)
  {
    if ((size_t)r.addr + 7 > n_nodes2) {
      error = "unaligned node past __bvh_nodes";
      return false;
    }
    if (idx >= OBB_CODE) {
      error = "wide node index beyond the OBB code range";
      return false;
    }
    const float *n = nodes2 + 4 * (size_t)r.addr;
    uint32_t w0[4];
    memcpy(w0, n, 16);
    std::vector<uint32_t> w(words(), 0u);
    w[0] = w0[0];
    w[1] = w0[1];
    for (int k = 0; k < 2; k++) {
      const int a = (int)w0[2 + k];
      if (a < 0) {
        int start, count;
        if (!leaf_range(a, &start, &count)) {
          return false;
        }
        if (start >= (1 << 27)) {
          error = "primitive index beyond the 2^27 leaf-code range";
          return false;
        }
        w[2 + k] = ~(((uint32_t)start << 4) | (uint32_t)count);
      }
      else {
        const size_t child = alloc_node(a);
        w[2 + k] = (uint32_t)child | (unaligned(a) ? OBB_CODE : 0u);
        Ref c;
        c.addr = a;
        c.vis = w0[k];
        for (int x = 0; x < 3; x++) {
          c.lo[x] = -FLT_MAX;
          c.hi[x] = FLT_MAX;
        }
        pending->push_back(std::make_pair(child, c));
      }
    }
    memcpy(&w[4], n + 4, 24 * 4);
    memcpy(&out[idx * words()], w.data(), words() * 4);
    n_obb++;
    return true;
  }

  /* a fresh node for BVH2 inner node a: one slot, or obb_slots() for an
   * unaligned one */
  size_t alloc_node(int a)
  {
    const size_t child = out.size() / words();
    out.resize(out.size() + (unaligned(a) ? obb_slots() : 1) * words(), 0u);
    return child;
  }

  /* one pending node: an OBB node for an unaligned BVH2 node, else a wide one */
  bool process(size_t idx, const Ref &r, std::vector<Ref> &ch, std::vector<std::pair<size_t, Ref>> *next)
  {
    if (unaligned(r.addr)) {
      return emit_obb(idx, r, next);
    }
    int n = 0;
    return open(r, ch.data(), &n) && emit(idx, ch.data(), n, next);
  }

  std::vector<int> instances; /* objects referenced by instance leaves (may repeat) */

  /* Collapse the BVH2 subtree at `root` into wide nodes starting at a fresh
   * node index, breadth first; returns that index or -1 on error. */
  long collapse(int root)
  {
    const size_t base = out.size() / words();
    out.resize(out.size() + words(), 0u);
    std::vector<std::pair<size_t, Ref>> pending, next;
    std::vector<Ref> ch(width);
    int n = 0;
    if (root < 0) {
      /* single-leaf BVH: one wide node holding the leaf with an unbounded box */
      Ref r;
      r.addr = root;
      r.vis = 0x0FFFFFFFu;
      for (int a = 0; a < 3; a++) {
        r.lo[a] = -FLT_MAX;
        r.hi[a] = FLT_MAX;
      }
      max_depth = std::max(max_depth, 1);
      return emit(base, &r, 1, &pending) ? (long)base : -1;
    }
    Ref r;
    r.addr = root;
    r.vis = 0xFFFFFFFFu;
    if (unaligned(root)) {
      /* an oriented-box root: a wide root with that node as its only child */
      for (int a = 0; a < 3; a++) {
        r.lo[a] = -FLT_MAX;
        r.hi[a] = FLT_MAX;
      }
      r.vis = 0x0FFFFFFFu;
      if (!emit(base, &r, 1, &pending)) {
        return -1;
      }
    }
    else if (!open(r, ch.data(), &n) || !emit(base, ch.data(), n, &pending)) {
      return -1;
    }
    int depth = 1;
    while (!pending.empty()) {
      next.clear();
      for (auto &p : pending) {
        if (!process(p.first, p.second, ch, &next)) {
          return -1;
        }
      }
      pending.swap(next);
      depth++;
    }
    max_depth = std::max(max_depth, depth);
    return (long)base;
  }

  /* root: BVH2 root address (KernelBVH.root).  The top level becomes wide
   * node 0; each instanced object's BVH (root __object_node[object]) is
   * collapsed once per distinct root and recorded in object_root. */
  bool run(int root)
  {
    if (width != 4 && width != 8) {
      error = "width must be 4 or 8";
      return false;
    }
    out.clear();
    n_obb = 0;
    sub_start.assign(n_nodes2 / 4 + 1, -1);
    sub_count.assign(n_nodes2 / 4 + 1, -2);
    instances.clear();
    object_root.assign(n_objects, -1);
    max_depth = 0;
    if (collapse(root) != 0) {
      return false;
    }
    const int top_depth = max_depth;
    int deepest = top_depth;
    std::vector<std::pair<int, long>> done; /* BVH2 root -> wide root */
    for (size_t i = 0; i < instances.size(); i++) {
      const int ob = instances[i];
      if (object_root[ob] >= 0) {
        continue;
      }
      const int r2 = (int)object_node[ob];
      long wr = -1;
      for (auto &d : done) {
        if (d.first == r2) {
          wr = d.second;
        }
      }
      if (wr < 0) {
        max_depth = 0;
        wr = collapse(r2);
        if (wr < 0) {
          return false;
        }
        deepest = std::max(deepest, top_depth + max_depth);
        done.push_back(std::make_pair(r2, wr));
      }
      object_root[ob] = (int)wr;
    }
    max_depth = deepest;
    return true;
  }
};


}  // namespace cybvhw

#endif
