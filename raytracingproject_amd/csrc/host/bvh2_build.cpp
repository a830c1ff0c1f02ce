/*
 * bvh2_build.cpp — host-side BVH2 builder + packer producing the Cycles
 * PackedBVH arrays (stand-in for the unchanged Cycles host builder).
 *
 * The HIP device consumes exactly what the reference host uploads for
 * BVH_LAYOUT_BVH2: this file restates the *layout contract* of
 *   bvh/bvh2.cpp:40-61   pack_leaf         (float4: prim lo, prim hi, visibility, prim type)
 *   bvh/bvh2.cpp:86-116  pack_aligned_node (4 x float4: vis0, vis1, child0, child1 /
 *                                           min/max x, y, z of both children)
 *   bvh/bvh2.cpp:165-236 pack_nodes        (DFS order, leaves in their own array,
 *                                           child index ~i for leaves, root 0 or -1)
 *   bvh/bvh.cpp:279-321  pack_primitives   (prim_tri_index = 3*i, prim_tri_verts)
 *   bvh/bvh2.cpp:133-163 pack_unaligned_node (7 x float4: vis0|UNALIGNED, vis1|UNALIGNED,
 *                                           child0, child1 / child 0's node space /
 *                                           child 1's node space, bvh_unaligned.cpp
 *                                           compute_node_transform)
 * with a binned-SAH builder of its own (the reference's BVHBuild,
 * bvh/bvh_build.cpp:370+, is out of scope — SURVEY.md §2 row 25).  Any valid
 * BVH gives the same closest hits; parity is checked against the reference
 * kernel traversing these same arrays.
 *
 * Hair: curve segments are primitives of kind 2 with explicit boxes; leaves
 * hold one primitive kind (BVHBuild::create_leaf_node); with unaligned nodes
 * on (BVHParams.use_unaligned_nodes, set for scenes with curves) a subtree of
 * curve segments only is bounded in an oriented space along its segments'
 * mean direction, and its parent is packed as an unaligned node.
 *
 * C ABI (host only, no HIP): hcb_build / hcb_build_boxes, hcb_pack, hcb_free.
 */
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct BBox {
  float mn[3], mx[3];
  void reset()
  {
    mn[0] = mn[1] = mn[2] = FLT_MAX;
    mx[0] = mx[1] = mx[2] = -FLT_MAX;
  }
  void grow(const float *p)
  {
    for (int a = 0; a < 3; a++) {
      mn[a] = std::min(mn[a], p[a]);
      mx[a] = std::max(mx[a], p[a]);
    }
  }
  void grow(const BBox &b)
  {
    for (int a = 0; a < 3; a++) {
      mn[a] = std::min(mn[a], b.mn[a]);
      mx[a] = std::max(mx[a], b.mx[a]);
    }
  }
  float area() const
  {
    if (mn[0] > mx[0]) return 0.0f;
    float d0 = mx[0] - mn[0], d1 = mx[1] - mn[1], d2 = mx[2] - mn[2];
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
  }
};

struct Node {
  BBox box;
  int child[2] = {-1, -1};
  int lo = 0, hi = 0; /* prim range for leaves */
  uint32_t visibility = 0;
  bool leaf = false;
  bool unaligned = false; /* curve-only subtree bounded in `space` */
  double space[12];       /* node transform (3 rows of 4), unit box in this space */
};

struct Builder {
  const uint32_t *vis;
  const int32_t *kind = nullptr; /* per primitive: 0 triangle, 1 object instance, 2 curve segment */
  const uint32_t *ptype = nullptr; /* per primitive: packed prim type written into leaves (curves) */
  const float *curve_cp = nullptr; /* per primitive: 4 Bezier control points + radius (16 floats) */
  bool use_unaligned = false;
  int max_leaf;

  /* Leaves hold one primitive kind; an instance is always alone in its leaf
   * (BVHBuild::create_leaf_node keeps object references in leaves of their own,
   * bvh/bvh_build.cpp:777-830, and BVH2::pack_leaf encodes them, bvh2.cpp:40-61). */
  bool leaf_ok(int lo, int hi) const
  {
    if (!kind) return true;
    int inst = 0, curve = 0;
    for (int i = lo; i < hi; i++) {
      inst += kind[order[i]] == 1;
      curve += kind[order[i]] == 2;
    }
    if (inst) return inst == 1 && hi - lo == 1;
    return curve == 0 || curve == hi - lo;
  }

  bool all_curves(int lo, int hi) const
  {
    if (!kind || !curve_cp) return false;
    for (int i = lo; i < hi; i++) {
      if (kind[order[i]] != 2) return false;
    }
    return hi > lo;
  }

  /* Oriented bounds of a curve-only range (BVHUnaligned::compute_aligned_space
   * and compute_node_transform, bvh/bvh_unaligned.cpp:36-165, with a space of
   * our own: z along the mean segment direction).  Writes the node transform
   * that maps the box to the unit cube. */
  void unaligned_space(int lo, int hi, double *out) const
  {
    double ax[3] = {0.0, 0.0, 0.0};
    for (int i = lo; i < hi; i++) {
      const float *c = curve_cp + 16 * (size_t)order[i];
      double d[3] = {(double)c[12] - c[0], (double)c[13] - c[1], (double)c[14] - c[2]};
      const double dot = d[0] * ax[0] + d[1] * ax[1] + d[2] * ax[2];
      const double sgn = dot < 0.0 ? -1.0 : 1.0;
      for (int a = 0; a < 3; a++) ax[a] += sgn * d[a];
    }
    double len = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    double z[3] = {0.0, 0.0, 1.0};
    if (len > 1e-30) {
      for (int a = 0; a < 3; a++) z[a] = ax[a] / len;
    }
    double t[3] = {1.0, 0.0, 0.0};
    if (std::fabs(z[0]) > 0.9) {
      t[0] = 0.0;
      t[1] = 1.0;
    }
    double x[3] = {t[1] * z[2] - t[2] * z[1], t[2] * z[0] - t[0] * z[2], t[0] * z[1] - t[1] * z[0]};
    len = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    for (int a = 0; a < 3; a++) x[a] /= len;
    double y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
    const double *rows[3] = {x, y, z};
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    for (int i = lo; i < hi; i++) {
      const float *c = curve_cp + 16 * (size_t)order[i];
      const double r = std::max(std::max(c[3], c[7]), std::max(c[11], c[15]));
      for (int k = 0; k < 4; k++) {
        for (int a = 0; a < 3; a++) {
          const double v = rows[a][0] * c[4 * k] + rows[a][1] * c[4 * k + 1] + rows[a][2] * c[4 * k + 2];
          mn[a] = std::min(mn[a], v - r);
          mx[a] = std::max(mx[a], v + r);
        }
      }
    }
    for (int a = 0; a < 3; a++) {
      /* conservative: the kernel transforms in float */
      const double pad = 1e-5 * (mx[a] - mn[a]) + 1e-6 * std::max(std::fabs(mn[a]), std::fabs(mx[a])) + 1e-12;
      mn[a] -= pad;
      mx[a] += pad;
      const double inv = 1.0 / std::max(1e-18, mx[a] - mn[a]);
      out[4 * a + 0] = rows[a][0] * inv;
      out[4 * a + 1] = rows[a][1] * inv;
      out[4 * a + 2] = rows[a][2] * inv;
      out[4 * a + 3] = -mn[a] * inv;
    }
  }
  std::vector<BBox> pbox;
  std::vector<float> cent; /* 3 per prim */
  std::vector<int> order;
  std::vector<Node> nodes;

  int build(int lo, int hi, int depth)
  {
    Node node;
    node.box.reset();
    BBox cbox;
    cbox.reset();
    uint32_t visibility = 0;
    for (int i = lo; i < hi; i++) {
      node.box.grow(pbox[order[i]]);
      cbox.grow(&cent[3 * order[i]]);
      visibility |= vis[order[i]];
    }
    node.visibility = visibility;
    if (use_unaligned && all_curves(lo, hi)) {
      node.unaligned = true;
      unaligned_space(lo, hi, node.space);
    }
    const int n = hi - lo;
    int idx = (int)nodes.size();
    nodes.push_back(node);
    if (n <= 1 || (depth > 60 && leaf_ok(lo, hi))) {
      nodes[idx].leaf = true;
      nodes[idx].lo = lo;
      nodes[idx].hi = hi;
      return idx;
    }
    /* binned SAH over the 3 axes */
    const int NB = 32;
    float best_cost = FLT_MAX;
    int best_axis = -1, best_split = -1;
    for (int a = 0; a < 3; a++) {
      float ext = cbox.mx[a] - cbox.mn[a];
      if (!(ext > 0.0f)) continue;
      BBox bb[NB];
      int cnt[NB];
      for (int b = 0; b < NB; b++) {
        bb[b].reset();
        cnt[b] = 0;
      }
      float scale = NB / ext;
      for (int i = lo; i < hi; i++) {
        int p = order[i];
        int b = std::min(NB - 1, (int)((cent[3 * p + a] - cbox.mn[a]) * scale));
        bb[b].grow(pbox[p]);
        cnt[b]++;
      }
      float rarea[NB];
      int rcnt[NB];
      BBox acc;
      acc.reset();
      int c = 0;
      for (int b = NB - 1; b > 0; b--) {
        acc.grow(bb[b]);
        c += cnt[b];
        rarea[b] = acc.area();
        rcnt[b] = c;
      }
      acc.reset();
      c = 0;
      for (int b = 0; b < NB - 1; b++) {
        acc.grow(bb[b]);
        c += cnt[b];
        if (c == 0 || rcnt[b + 1] == 0) continue;
        float cost = acc.area() * c + rarea[b + 1] * rcnt[b + 1];
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = a;
          best_split = b;
        }
      }
    }
    float parea = node.box.area();
    float leaf_cost = (float)n;
    float split_cost = 1.0f + (parea > 0.0f ? best_cost / parea : FLT_MAX);
    int mid;
    if (best_axis < 0) {
      if (n <= max_leaf && leaf_ok(lo, hi)) {
        nodes[idx].leaf = true;
        nodes[idx].lo = lo;
        nodes[idx].hi = hi;
        return idx;
      }
      mid = lo + n / 2; /* coincident centroids: split by count */
    }
    else {
      if (n <= max_leaf && leaf_cost <= split_cost && leaf_ok(lo, hi)) {
        nodes[idx].leaf = true;
        nodes[idx].lo = lo;
        nodes[idx].hi = hi;
        return idx;
      }
      float ext = cbox.mx[best_axis] - cbox.mn[best_axis];
      float scale = NB / ext;
      auto it = std::partition(order.begin() + lo, order.begin() + hi, [&](int p) {
        int b = std::min(NB - 1, (int)((cent[3 * p + best_axis] - cbox.mn[best_axis]) * scale));
        return b <= best_split;
      });
      mid = (int)(it - order.begin());
      if (mid == lo || mid == hi) mid = lo + n / 2;
    }
    int c0 = build(lo, mid, depth + 1);
    int c1 = build(mid, hi, depth + 1);
    nodes[idx].child[0] = c0;
    nodes[idx].child[1] = c1;
    return idx;
  }
};

inline float bits_f(uint32_t u)
{
  float f;
  memcpy(&f, &u, 4);
  return f;
}
inline float bits_i(int32_t i)
{
  float f;
  memcpy(&f, &i, 4);
  return f;
}

}  // namespace

extern "C" {

/*
 * Build + pack.  Inputs: n triangles, verts (n x 9 floats, world space),
 * vis (n, per-triangle object visibility_for_tracing), max_leaf_size.
 * Outputs (caller-allocated):
 *   order       n ints      : BVH slot -> input triangle
 *   nodes_out   4*n_inner float4 (size queried with nodes_out == NULL)
 *   leaves_out  n_leaf float4
 *   counts[0] = n_inner*4 (float4 count), counts[1] = n_leaf, counts[2] = root index
 * Call once with nodes_out == NULL to get counts (the build is cached in ctx).
 */
struct hcb_ctx {
  Builder b;
  int root = 0;
  int n_inner = 0, n_leaf = 0;
  int64_t node_rows = 0; /* float4 rows: 4 per aligned, 7 per unaligned inner node */
};

/* bvh2.cpp pack_inner: a node is packed unaligned when either child is. */
static bool packs_unaligned(const Builder &b, const Node &nd)
{
  return !nd.leaf && (b.nodes[nd.child[0]].unaligned || b.nodes[nd.child[1]].unaligned);
}

static void *build_common(hcb_ctx *ctx, int n, int64_t *counts)
{
  Builder &b = ctx->b;
  b.cent.resize(3 * (size_t)n);
  b.order.resize(n);
  for (int i = 0; i < n; i++) {
    for (int a = 0; a < 3; a++) {
      b.cent[3 * i + a] = 0.5f * (b.pbox[i].mn[a] + b.pbox[i].mx[a]);
    }
    b.order[i] = i;
  }
  b.nodes.reserve(2 * (size_t)n + 1);
  if (n > 0) {
    ctx->root = b.build(0, n, 0);
  }
  for (const Node &nd : b.nodes) {
    if (nd.leaf) ctx->n_leaf++;
    else {
      ctx->n_inner++;
      ctx->node_rows += packs_unaligned(b, nd) ? 7 : 4;
    }
  }
  counts[0] = ctx->node_rows;
  counts[1] = ctx->n_leaf;
  counts[2] = b.nodes.empty() ? 0 : (b.nodes[ctx->root].leaf ? -1 : 0);
  return ctx;
}

void *hcb_build(int n, const float *verts, const uint32_t *vis, int max_leaf_size, int64_t *counts)
{
  hcb_ctx *ctx = new hcb_ctx();
  Builder &b = ctx->b;
  b.vis = vis;
  b.max_leaf = max_leaf_size > 0 ? max_leaf_size : 8;
  b.pbox.resize(n);
  for (int i = 0; i < n; i++) {
    b.pbox[i].reset();
    for (int k = 0; k < 3; k++) {
      b.pbox[i].grow(verts + 9 * (size_t)i + 3 * k);
    }
  }
  return build_common(ctx, n, counts);
}

void *hcb_build_prims(int n, const float *boxes, const uint32_t *vis, const int32_t *kind, const uint32_t *ptype,
                      const float *curve_cp, int use_unaligned, int max_leaf_size, int64_t *counts);

/* Same over explicit primitive boxes (n x 6: min xyz, max xyz) with a kind per
 * primitive (0 triangle, 1 object instance): the top-level BVH of a scene with
 * instanced geometry (BVHBuild::add_reference_object, bvh/bvh_build.cpp:283). */
void *hcb_build_boxes(
    int n, const float *boxes, const uint32_t *vis, const int32_t *kind, int max_leaf_size, int64_t *counts)
{
  return hcb_build_prims(n, boxes, vis, kind, nullptr, nullptr, 0, max_leaf_size, counts);
}

/* Same with curve segments (kind 2): ptype = packed primitive type per
 * primitive (written into leaf.w), curve_cp = 16 floats per primitive (the
 * segment's 4 Bezier control points, each xyz + radius; used for unaligned
 * nodes when use_unaligned). */
void *hcb_build_prims(int n, const float *boxes, const uint32_t *vis, const int32_t *kind, const uint32_t *ptype,
                      const float *curve_cp, int use_unaligned, int max_leaf_size, int64_t *counts)
{
  hcb_ctx *ctx = new hcb_ctx();
  Builder &b = ctx->b;
  b.vis = vis;
  b.kind = kind;
  b.ptype = ptype;
  b.curve_cp = curve_cp;
  b.use_unaligned = use_unaligned != 0 && curve_cp != nullptr;
  b.max_leaf = max_leaf_size > 0 ? max_leaf_size : 8;
  b.pbox.resize(n);
  for (int i = 0; i < n; i++) {
    b.pbox[i].reset();
    b.pbox[i].grow(boxes + 6 * (size_t)i);
    b.pbox[i].grow(boxes + 6 * (size_t)i + 3);
  }
  return build_common(ctx, n, counts);
}

/* Leaf prim type: PRIMITIVE_TRIANGLE, or the packed type given per primitive. */
int hcb_pack(void *h, float *nodes_out, float *leaves_out, int32_t *order_out)
{
  hcb_ctx *ctx = (hcb_ctx *)h;
  Builder &b = ctx->b;
  if (b.nodes.empty()) return 0;
  const uint32_t PATH_RAY_NODE_UNALIGNED = 1u << 13;
  const uint32_t PRIMITIVE_TRIANGLE = 1u;
  struct Entry {
    int node;
    int idx;
  };
  std::vector<Entry> stack;
  int next_node = 0, next_leaf = 0;
  auto node_rows = [&](int node) { return packs_unaligned(b, b.nodes[node]) ? 7 : 4; };
  const Node &root = b.nodes[ctx->root];
  if (root.leaf) {
    stack.push_back({ctx->root, next_leaf++});
  }
  else {
    stack.push_back({ctx->root, next_node});
    next_node += node_rows(ctx->root);
  }
  auto encode = [&](int node, int idx) { return b.nodes[node].leaf ? ~idx : idx; };
  while (!stack.empty()) {
    Entry e = stack.back();
    stack.pop_back();
    const Node &nd = b.nodes[e.node];
    if (nd.leaf) {
      float *d = leaves_out + 4 * (size_t)e.idx;
      if (b.kind && b.kind[b.order[nd.lo]] == 1) {
        /* object instance leaf: ~slot, 0, visibility, prim_type 0 */
        d[0] = bits_i(~nd.lo);
        d[1] = bits_i(0);
        d[2] = bits_f(nd.visibility);
        d[3] = bits_f(0u);
      }
      else {
        d[0] = bits_i(nd.lo);
        d[1] = bits_i(nd.hi);
        d[2] = bits_f(nd.visibility);
        /* pack_leaf: the type of the leaf's first primitive */
        d[3] = bits_f(b.ptype ? b.ptype[b.order[nd.lo]] : PRIMITIVE_TRIANGLE);
      }
    }
    else {
      int idx[2];
      for (int i = 0; i < 2; i++) {
        if (b.nodes[nd.child[i]].leaf) {
          idx[i] = next_leaf++;
        }
        else {
          idx[i] = next_node;
          next_node += node_rows(nd.child[i]);
        }
      }
      stack.push_back({nd.child[0], idx[0]});
      stack.push_back({nd.child[1], idx[1]});
      const Node &c0 = b.nodes[nd.child[0]];
      const Node &c1 = b.nodes[nd.child[1]];
      float *d = nodes_out + 4 * (size_t)e.idx;
      if (packs_unaligned(b, nd)) {
        d[0] = bits_f(c0.visibility | PATH_RAY_NODE_UNALIGNED);
        d[1] = bits_f(c1.visibility | PATH_RAY_NODE_UNALIGNED);
        d[2] = bits_i(encode(nd.child[0], idx[0]));
        d[3] = bits_i(encode(nd.child[1], idx[1]));
        for (int k = 0; k < 2; k++) {
          const Node &c = k == 0 ? c0 : c1;
          double sp[12];
          if (c.unaligned) {
            memcpy(sp, c.space, sizeof(sp));
          }
          else {
            /* an aligned child of an unaligned node: identity space (BVHNode::
             * get_aligned_space), the node transform of its box */
            for (int a = 0; a < 3; a++) {
              const double pad = 1e-6 * std::max(std::fabs((double)c.box.mn[a]), std::fabs((double)c.box.mx[a]));
              const double lo = (double)c.box.mn[a] - pad, hi = (double)c.box.mx[a] + pad;
              const double inv = 1.0 / std::max(1e-18, hi - lo);
              for (int j = 0; j < 3; j++) sp[4 * a + j] = (a == j) ? inv : 0.0;
              sp[4 * a + 3] = -lo * inv;
            }
          }
          for (int j = 0; j < 12; j++) d[4 + 12 * k + j] = (float)sp[j];
        }
      }
      else {
        d[0] = bits_f(c0.visibility & ~PATH_RAY_NODE_UNALIGNED);
        d[1] = bits_f(c1.visibility & ~PATH_RAY_NODE_UNALIGNED);
        d[2] = bits_i(encode(nd.child[0], idx[0]));
        d[3] = bits_i(encode(nd.child[1], idx[1]));
        d[4] = c0.box.mn[0];
        d[5] = c1.box.mn[0];
        d[6] = c0.box.mx[0];
        d[7] = c1.box.mx[0];
        d[8] = c0.box.mn[1];
        d[9] = c1.box.mn[1];
        d[10] = c0.box.mx[1];
        d[11] = c1.box.mx[1];
        d[12] = c0.box.mn[2];
        d[13] = c1.box.mn[2];
        d[14] = c0.box.mx[2];
        d[15] = c1.box.mx[2];
      }
    }
  }
  memcpy(order_out, b.order.data(), sizeof(int32_t) * b.order.size());
  return 0;
}

void hcb_free(void *h)
{
  delete (hcb_ctx *)h;
}

}  // extern "C"
