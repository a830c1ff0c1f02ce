/*
 * tools/host_emu.cpp — debugging aid: the HIP device's per-path code
 * (raytracingproject_amd/csrc/kernel/cy_integrator.h) compiled for the HOST and
 * driven one path at a time, sample-major like the reference CPU device.
 *
 * Built with -DCY_HOST_LIBM_SINCOS it calls the same libm sinf/cosf as the
 * reference kernel, so any difference against oracle/_ref isolates a logic
 * difference of the restatement from GPU arithmetic.  Not part of the product.
 */
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <vector>

/* the device's largest shading variant (csrc/device/k_shade.h CY_DEVICE_MAX_CLOSURE) */
#define CY_MAX_CLOSURE 64
#define CY_INTEGRATOR_EXT 1 /* every extra of the integrator (the _ext shading variants) */
#include "../raytracingproject_amd/csrc/kernel/cy_integrator.h"
#include "../raytracingproject_amd/csrc/kernel/cy_bvhw.h"
#include "../raytracingproject_amd/csrc/host/cy_bvhw_collapse.h"

/* Widen a packed BVH2 like the device library does (hipcycles.hip ensure_bvhw).
 * Returns the number of uint32 written (32 per node), or -1 with the reason
 * copied to err_out. */
/* curve shapes of the scene (1 ribbons, 2 thick, 3 both; hipcycles.hip
 * curve_shapes): ribbon-only scenes widen their hair BVH2 too */
static int g_curve_shapes = 0;
extern "C" void emu_set_curve_shapes(int shapes)
{
  g_curve_shapes = shapes;
}

extern "C" long emu_bvhw_build(int width,
                               int merge_prims,
                               const float *nodes2,
                               long n_nodes2,
                               const float *leaves2,
                               long n_leaves2,
                               int root,
                               const uint32_t *prim_object,
                               long n_prims,
                               const uint32_t *object_node,
                               long n_objects,
                               uint32_t *out,
                               long out_cap,
                               int *object_root,
                               int *depth,
                               char *err_out,
                               int err_len)
{
  cybvhw::Collapser col;
  col.width = width;
  col.merge_prims = merge_prims;
  col.allow_curves = g_curve_shapes != 0;
  col.nodes2 = nodes2;
  col.n_nodes2 = (size_t)n_nodes2;
  col.leaves2 = leaves2;
  col.n_leaves2 = (size_t)n_leaves2;
  col.prim_object = prim_object;
  col.n_prims = (size_t)n_prims;
  col.object_node = object_node;
  col.n_objects = (size_t)n_objects;
  if (!col.run(root)) {
    snprintf(err_out, err_len, "%s", col.error.c_str());
    return -1;
  }
  if ((long)col.out.size() > out_cap) {
    snprintf(err_out, err_len, "output capacity %ld < %zu", out_cap, col.out.size());
    return -1;
  }
  memcpy(out, col.out.data(), col.out.size() * 4);
  memcpy(object_root, col.object_root.data(), col.object_root.size() * 4);
  *depth = col.max_depth;
  return (long)col.out.size();
}

static int g_width = 2;
static int g_instancing = 0; /* emu_set_instancing */

static const int *g_object_root = nullptr;

extern "C" void emu_set_object_root(const int *roots)
{
  g_object_root = roots;
}

static void emu_bind(CyGlobals *kg, const void *data, int n_arrays, const char **names, const void **ptrs,
                     const void *bvhw)
{
  memset(kg, 0, sizeof(*kg));
  kg->data = (const hc_KernelData *)data;
  for (int i = 0; i < n_arrays; i++) {
#define CY_BIND(type, name) \
  if (strcmp(names[i], #name) == 0) \
    kg->name = (const type *)ptrs[i];
    CY_GLOBAL_ARRAYS(CY_BIND)
#undef CY_BIND
  }
  kg->bvhw_nodes = bvhw;
  kg->bvhw_object_root = g_object_root;
  /* generic: the instance paths are always enabled on the host, except that
   * a wide layout over a scene without instances takes the device's
   * non-instanced paths (hipcycles.hip build_globals) */
  kg->have_instancing = (bvhw && !g_instancing) ? 0 : 1;
  kg->tri_index_identity = 0;
  kg->have_curves = kg->data->bvh.have_curves ? 1 : 0;
  if (kg->have_curves && g_curve_shapes != 1) {
    kg->bvhw_nodes = nullptr; /* thick curves keep the BVH2 (hipcycles.hip wide_layout) */
  }
  kg->bvhw_width = kg->bvhw_nodes ? g_width : 0;
}

extern "C" void emu_set_width(int w)
{
  g_width = w;
}

/* instanced scene: the device's wide kernels then traverse the top level in
 * the reference's order and the instances wide (hipcycles.hip scene_traverse) */
extern "C" void emu_set_instancing(int on)
{
  g_instancing = on;
}

template<bool any_hit>
static bool emu_traverse_impl(const CyGlobals *kg, const CyRay *ray, uint vis, CyIsect *isect, uint *err,
                              uint *nn, uint *nl, uint *nt)
{
  if (kg->bvhw_nodes && kg->have_curves) {
    /* ribbon scene on the wide BVH; near-ties and twice-crossed ribbons are
     * re-traced in the reference's order (hipcycles.hip k_intersect_closest) */
    bool tie = false, hit;
    if (g_instancing) {
      hit = g_width == 8 ?
                bvh2_intersect<any_hit, true, 8, CY_LDS_STACK, CY_BLOCK, 1>(kg, ray, vis, isect, err, nn, nl, nt,
                                                                           nullptr, nullptr, &tie) :
                bvh2_intersect<any_hit, true, 4, CY_LDS_STACK, CY_BLOCK, 1>(kg, ray, vis, isect, err, nn, nl, nt,
                                                                           nullptr, nullptr, &tie);
    }
    else {
      hit = g_width == 8 ? bvhw_intersect<8, any_hit, 1>(kg, ray, vis, isect, err, nn, nl, nt, nullptr, &tie) :
                           bvhw_intersect<4, any_hit, 1>(kg, ray, vis, isect, err, nn, nl, nt, nullptr, &tie);
    }
    if (!tie) {
      return hit;
    }
    CyGlobals k2 = *kg;
    k2.bvhw_nodes = nullptr;
    return bvh2_intersect<any_hit, true, 2, CY_LDS_STACK, CY_BLOCK, 3>(&k2, ray, vis, isect, err, nullptr, nullptr,
                                                                        nullptr, nullptr);
  }
  if (kg->bvhw_nodes) {
    bool tie = false, hit;
    if (g_instancing) {
      hit = g_width == 8 ? bvh2_intersect<any_hit, true, 8>(kg, ray, vis, isect, err, nn, nl, nt, nullptr, nullptr, &tie) :
                           bvh2_intersect<any_hit, true, 4>(kg, ray, vis, isect, err, nn, nl, nt, nullptr, nullptr, &tie);
    }
    else {
      hit = g_width == 8 ? bvhw_intersect<8, any_hit>(kg, ray, vis, isect, err, nn, nl, nt, nullptr, &tie) :
                           bvhw_intersect<4, any_hit>(kg, ray, vis, isect, err, nn, nl, nt, nullptr, &tie);
    }
    if (!tie) {
      return hit;
    }
    /* near-tie: re-trace in the reference's order, as shade_path does */
    CyGlobals k2 = *kg;
    k2.bvhw_nodes = nullptr;
#ifdef CY_EMU_SHORT_RETRACE
    /* debugging aid: the re-trace from a t shortened to twice the tie window */
    CyRay rt = *ray;
    rt.t = fminf(ray->t, isect->t * (1.0f + 2.0f * CY_TIE_EPS));
    return bvh2_intersect<any_hit>(&k2, &rt, vis, isect, err, nullptr, nullptr, nullptr, nullptr);
#else
    return bvh2_intersect<any_hit>(&k2, ray, vis, isect, err, nullptr, nullptr, nullptr, nullptr);
#endif
  }
  if (kg->have_curves) {
    return bvh2_intersect<any_hit, true, 2, CY_LDS_STACK, CY_BLOCK, 3>(kg, ray, vis, isect, err, nn, nl, nt,
                                                                         nullptr);
  }
  return bvh2_intersect<any_hit>(kg, ray, vis, isect, err, nn, nl, nt, nullptr);
}

/* Debug aid: with emu_set_check(1) every closest-hit query of a wide-BVH
 * render is repeated with the BVH2 in the reference's order and the first
 * mismatches (ray, both hits) are kept for emu_get_mismatches. */
static int g_check = 0;
static std::vector<float> g_mismatch;
extern "C" void emu_set_check(int on)
{
  g_check = on;
  g_mismatch.clear();
}
extern "C" int emu_get_mismatches(float *out, int max_n)
{
  const int n = std::min<int>(max_n, (int)(g_mismatch.size() / 16));
  memcpy(out, g_mismatch.data(), (size_t)n * 16 * 4);
  return (int)(g_mismatch.size() / 16);
}

template<bool any_hit>
static bool emu_traverse(const CyGlobals *kg, const CyRay *ray, uint vis, CyIsect *isect, uint *err,
                         uint *nn, uint *nl, uint *nt)
{
  const bool hit = emu_traverse_impl<any_hit>(kg, ray, vis, isect, err, nn, nl, nt);
  if (g_check && !any_hit && kg->bvhw_nodes) {
    CyGlobals k2 = *kg;
    k2.bvhw_nodes = nullptr;
    CyIsect i2;
    const bool h2 = kg->have_curves ?
                        bvh2_intersect<false, true, 2, CY_LDS_STACK, CY_BLOCK, 3>(&k2, ray, vis, &i2, err, nullptr,
                                                                                   nullptr, nullptr, nullptr) :
                        bvh2_intersect<false>(&k2, ray, vis, &i2, err, nullptr, nullptr, nullptr, nullptr);
    if (h2 != hit || (hit && (i2.prim != isect->prim || as_uint(i2.t) != as_uint(isect->t)))) {
      const float rec[16] = {ray->P.x, ray->D.x, ray->P.y, ray->D.y, ray->P.z, ray->D.z, ray->t, as_float(vis),
                             (float)isect->prim, isect->t, (float)i2.prim, i2.t, (float)isect->object,
                             (float)i2.object, isect->u, i2.u};
      g_mismatch.insert(g_mismatch.end(), rec, rec + 16);
    }
  }
  return hit;
}

/* scene_intersect on host: rays n x 8 (P, D, t, visibility bits) like
 * k_test_intersect; counters[3] = inner nodes, leaves, triangle tests. */
extern "C" int emu_intersect(const void *data,
                             int n_arrays,
                             const char **names,
                             const void **ptrs,
                             const void *bvhw,
                             const float *rays,
                             int n,
                             int any_hit,
                             float *out_f,
                             int *out_i,
                             unsigned long long *counters)
{
  CyGlobals kg;
  emu_bind(&kg, data, n_arrays, names, ptrs, bvhw);
  uint err = 0;
  for (int i = 0; i < n; i++) {
    const float *r = rays + 8 * i;
    CyRay ray;
    ray.P = mk3(r[0], r[1], r[2]);
    ray.D = mk3(r[3], r[4], r[5]);
    ray.t = r[6];
    const uint visibility = as_uint(r[7]);
    CyIsect isect;
    isect.t = ray.t;
    isect.u = isect.v = 0.0f;
    isect.prim = PRIM_NONE;
    isect.object = OBJECT_NONE;
    isect.type = 0;
    bool hit = false;
    uint nn = 0, nl = 0, nt = 0;
    if (scene_intersect_valid(&ray)) {
      if (any_hit || (visibility & PATH_RAY_SHADOW_OPAQUE)) {
        hit = emu_traverse<true>(&kg, &ray, visibility & PATH_RAY_SHADOW_OPAQUE, &isect, &err, &nn, &nl, &nt);
      }
      else {
        hit = emu_traverse<false>(&kg, &ray, visibility, &isect, &err, &nn, &nl, &nt);
      }
    }
    counters[0] += nn;
    counters[1] += nl;
    counters[2] += nt;
    out_f[3 * i + 0] = isect.t;
    out_f[3 * i + 1] = isect.u;
    out_f[3 * i + 2] = isect.v;
    out_i[4 * i + 0] = hit ? 1 : 0;
    out_i[4 * i + 1] = isect.prim;
    out_i[4 * i + 2] = isect.object;
    out_i[4 * i + 3] = isect.type;
  }
  return (int)err;
}

extern "C" int emu_render(const void *data,
                          int n_arrays,
                          const char **names,
                          const void **ptrs,
                          const void *bvhw,
                          float *buffer,
                          int tx,
                          int ty,
                          int tw,
                          int th,
                          int start_sample,
                          int num_samples,
                          int offset,
                          int stride,
                          int pass_stride)
{
  const hc_KernelData *kd = (const hc_KernelData *)data;
  if (kd->integrator.max_closures > CY_MAX_CLOSURE && !kd->integrator.use_volumes) {
    return -1; /* the device refuses these scenes too (hipcy_load_kernels) */
  }
  CyGlobals kg;
  emu_bind(&kg, data, n_arrays, names, ptrs, bvhw);
  hc_float4 rec[12];
  int isect_type = 0;
  int isect_object = OBJECT_NONE;
  hc_uint4 s0, s1;
  uint item_slot = 0;
  CyPathBuffers b;
  memset(&b, 0, sizeof(b)); /* buffers a feature does not use stay null */
  hc_float4 srec_hits[CY_SHADOW_REC_HITS];
  uint srec_n = CY_SREC_NONE;
  b.ray_P = &rec[0];
  b.ray_D = &rec[1];
  b.isect = &rec[2];
  b.isect_type = &isect_type;
  b.isect_object = &isect_object;
  b.state0 = &s0;
  b.state1 = &s1;
  b.state2 = &rec[3];
  b.throughput = &rec[4];
  b.L = &rec[5];
  b.shadow_P = &rec[6];
  b.shadow_D = &rec[7];
  b.shadow_L = &rec[8];
  b.shadow_T = &rec[9];
  b.item = &item_slot;
  hc_uint4 vol_stack[CY_VOLUME_STACK / 2];
  hc_uint4 vol_rec[2];
  b.vol_stack = vol_stack;
  b.vol_rec = vol_rec;
  hc_float4 sss_rec[CY_SSS_RECS * CY_SSS_REC_F4];
  uint sss_count = 0;
  b.sss_rec = sss_rec;
  b.sss_count = &sss_count;
  hc_uint4 sss_vol[(CY_SSS_RECS + 1) * (CY_VOLUME_STACK / 2)];
  b.sss_vol = sss_vol;
  hc_float4 catcher[CY_CATCHER_F4];
  b.catcher = catcher; /* every scene: a path without a catcher leaves it unused */
  hc_float4 br_rec[CY_BR_RECS * CY_BR_REC_F4];
  uint br_count[2] = {0u, 0u};
  static CyVolumeStep dec_steps[CY_DECOUPLED_STEPS]; /* slot 0's decoupled segment */
  b.dec_steps = dec_steps;
  hc_float4 lp[CY_LP_F4];
  if (((const hc_KernelData *)data)->film.use_light_pass) {
    b.lp = lp;
  }
  if (((const hc_KernelData *)data)->integrator.branched) {
    b.br_rec = br_rec;
    b.br_count = br_count;
  }
  hc_float4 ray_diff[CY_RAY_DIFF_F4];
  hc_float4 shadow_dP[2];
  b.ray_diff = ray_diff;
  b.shadow_dP = shadow_dP;
  /* generic: the differentials are always carried on the host (they change
   * nothing unless a shader reads them) */
  kg.use_ray_diff = getenv("EMU_NO_RAY_DIFF") ? 0 : 1; /* debugging switch */
  const bool vol = ((const hc_KernelData *)data)->integrator.use_volumes != 0;
  uint err = 0;
  CyTile tile;
  tile.x = tx;
  tile.y = ty;
  tile.w = tw;
  tile.h = th;
  tile.npix = (uint)(tw * th);
  tile.n_tiles = 1;
  tile.descs = nullptr;
  tile.aux_offset = 0;
  tile.sample_count_offset = 0;
  tile.write_aux = 0;
  tile.y_step = 1;
  tile.start_sample = start_sample;
  tile.end_sample = start_sample + num_samples;
  tile.offset = offset;
  tile.stride = stride;
  tile.buffer = buffer;
  tile.pass_stride = pass_stride;
  tile.n_items = (uint)(tw * th * num_samples);
  tile.work_next = nullptr;
  std::vector<hc_float4> records(tile.n_items);
  tile.samples_out = records.data();
  /* one slot, items in order: the device runs the same per-item code with
   * many slots in flight; the result per item does not depend on the slot.
   * Each item starts as in the device's camera launch (cam_item set for its
   * first closest and shade stages). */
  for (uint item = 0; item < tile.n_items; item++) {
    uint cam_item = item;
    bool active = true;
    while (active) {
      /* k_intersect_closest */
      CyRay ray;
      uint visibility;
      const bool has_ray = closest_load(&kg, &b, &tile, 0, cam_item, &ray, &visibility);
      CyIsect isect;
      bool hit = false;
      if (has_ray && scene_intersect_valid(&ray)) {
        hit = emu_traverse<false>(&kg, &ray, visibility, &isect, &err, nullptr, nullptr, nullptr);
      }
      closest_store<true>(&b, 0, has_ray, hit, &isect);
      /* k_shade */
      bool shadow = false, finished = false;
      CyClosure closure[CY_MAX_CLOSURE];
      float svm[CY_SVM_STACK];
      CyShadeMem mem;
      mem.closure = closure;
      mem.svm_stack = svm;
      mem.svm_stride = 1;
      mem.svm_fast = CY_SVM_STACK;
      mem.svm_spill = nullptr;
      bool cont = vol ? shade_path<true>(&kg, &b, &tile, 0, cam_item, mem, &shadow, &finished, &err) :
                        shade_path<false>(&kg, &b, &tile, 0, cam_item, mem, &shadow, &finished, &err);
      cam_item = CY_NO_ITEM;
      if (shadow && kg.data->integrator.transparent_shadows) {
        if (!kg.have_instancing) {
          /* k_shadow_record: the traversal stage's record of the shadow ray */
          b.shadow_hits = srec_hits;
          b.shadow_nrec = &srec_n;
          const int hair = kg.have_curves ? g_curve_shapes : 0;
          srec_n = hair == 0 ? shadow_record<0>(&kg, &b, 0, &err) : hair == 1 ? shadow_record<1>(&kg, &b, 0, &err) :
                   hair == 2 ? shadow_record<2>(&kg, &b, 0, &err) : shadow_record<3>(&kg, &b, 0, &err);
        }
        /* k_intersect_shadow_transparent */
        if (vol) {
          shadow_finish_transparent<true>(&kg, &b, &tile, 0, mem, &err);
        }
        else {
          shadow_finish_transparent<false>(&kg, &b, &tile, 0, mem, &err);
        }
      }
      else if (shadow) {
        /* k_intersect_shadow */
        CyRay sr;
        shadow_load(&b, 0, &sr);
        bool blocked = false;
        if (scene_intersect_valid(&sr)) {
          CyIsect si;
          blocked = emu_traverse<true>(&kg, &sr, PATH_RAY_SHADOW_OPAQUE, &si, &err, nullptr, nullptr, nullptr);
        }
        shadow_finish(&b, &tile, 0, blocked);
      }
      active = cont;
    }
  }
  for (int p = 0; p < tw * th; p++) {
    accumulate_pixel(&tile, p);
  }
  return (int)err;
}

/* SHADER task, SHADER_EVAL_BACKGROUND (cy_integrator.h background_evaluate):
 * out[i] (float4) += world colour for input i, num_samples times. */
extern "C" int emu_background(const void *data, int n_arrays, const char **names, const void **ptrs,
                              const unsigned *input, int n, int num_samples, float *out)
{
  CyGlobals kg;
  emu_bind(&kg, data, n_arrays, names, ptrs, nullptr);
  uint err = 0;
  CyClosure closure[1];
  float svm[CY_SVM_STACK];
  CyShadeMem mem;
  mem.closure = closure;
  mem.svm_stack = svm;
  mem.svm_stride = 1;
  mem.svm_fast = CY_SVM_STACK;
  mem.svm_spill = nullptr;
  for (int s = 0; s < num_samples; s++) {
    for (int i = 0; i < n; i++) {
      const cfloat3 c = background_evaluate(&kg, input[4 * i], input[4 * i + 1], mem, &err);
      out[4 * i] += c.x;
      out[4 * i + 1] += c.y;
      out[4 * i + 2] += c.z;
    }
  }
  return (int)err;
}

/* Debug aid: one curve primitive's ribbon test against a ray (P, D, bound):
 * out = (hit, t, u, v) of the reference's form, then (steps hit, first t, min t)
 * of the scanning form. */
extern "C" void emu_ribbon_test(const void *data, int n_arrays, const char **names, const void **ptrs, int prim,
                                const float *ray, float tfar, float *out)
{
  CyGlobals kg;
  emu_bind(&kg, data, n_arrays, names, ptrs, nullptr);
  const cfloat3 P = mk3(ray[0], ray[1], ray[2]);
  const cfloat3 dir = bvh_clamp_direction(mk3(ray[3], ray[4], ray[5]));
  const uint type = kg.__prim_type[prim];
  cy_c4 curve[4];
  curve_segment_keys(&kg, (int)kg.__prim_index[prim], (int)CY_PRIMITIVE_UNPACK_SEGMENT(type), curve);
  cy_c4 c2[4] = {curve[0], curve[1], curve[2], curve[3]};
  float t, u, v, tmin;
  const int hit = ribbon_intersect_steps<false>(P, dir, kg.data->bvh.curve_subdivisions, curve, tfar, &t, &u, &v, &tmin);
  out[0] = (float)hit;
  out[1] = hit ? t : -1.0f;
  out[2] = hit ? u : -1.0f;
  out[3] = hit ? v : -1.0f;
  float t2 = -1.0f, u2, v2, tmin2 = -1.0f;
  const int steps = ribbon_intersect_steps<true>(P, dir, kg.data->bvh.curve_subdivisions, c2, CY_FLT_MAX, &t2, &u2, &v2, &tmin2);
  out[4] = (float)steps;
  out[5] = t2;
  out[6] = tmin2;
}
