/*
 * oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Compiles the reference Cycles CPU kernel *where it lies* under /root/reference
 * (blender/intern/cycles/kernel/kernels/cpu/kernel.cpp, textually included below
 * so that the kernel's inline device functions are reachable) and exposes a small
 * extern "C" surface used as the parity checker and as the CPU baseline:
 *
 *   cref_*  entry points -> reference functions
 *     kernel_const_copy / kernel_global_memory_copy   kernels/cpu/kernel.cpp:67-92
 *     kernel_path_trace (via kernel_cpu_path_trace)     kernel_path.h:643-695,
 *                                                       kernels/cpu/kernel_cpu_impl.h:83-97
 *     scene_intersect                                   kernel/bvh/bvh.h:154-237
 *     kernel_path_trace_setup (camera ray)              kernel_path_common.h:21-46
 *     path_rng_1D                                       kernel_random.h:52-90
 *     ray_offset                                        kernel/bvh/bvh.h:541-586
 *   The tile loop in cref_render mirrors CPUDevice::path_trace
 *   (device/device_cpu.cpp:906-921: sample-outer, pixel-inner) with rows split
 *   over threads; each pixel's samples are still accumulated in sample order.
 *
 * Built by oracle/Makefile into oracle/_ref/libcycles_ref.so (git-ignored).
 * Nothing in this file is shipped; the reference sources are not copied.
 */
#include "kernel/kernels/cpu/kernel.cpp"

#include "hipcycles_kernel_types.h"
#include "render/sobol.h"

#include <cstddef>
#include <cstring>
#include <thread>
#include <vector>

using namespace ccl;

/* Kernel the render entry drives: the generic x86-64 kernel (the parity
 * oracle), or, in the CPU-baseline build (oracle/Makefile ref-avx2), the AVX2
 * kernel stock Blender selects on such hosts (device/device_cpu.cpp:76-134). */
#ifndef CREF_PATH_TRACE
#  define CREF_PATH_TRACE kernel_cpu_path_trace
#  define CREF_ARCH "cpu (generic x86-64, no FMA)"
#endif

namespace {

struct RefContext {
  KernelGlobals kg;
};

KernelGlobals make_globals()
{
  KernelGlobals kg;
  memset((void *)&kg, 0, sizeof(kg));
  return kg;
}

/* Same per-thread initialisation as CPUDevice::thread_kernel_globals_init
 * (device/device_cpu.cpp:1424-1439). */
KernelGlobals thread_globals(const KernelGlobals &base)
{
  KernelGlobals kg = base;
  kg.transparent_shadow_intersections = NULL;
  kg.decoupled_volume_steps[0] = NULL;
  kg.decoupled_volume_steps[1] = NULL;
  kg.decoupled_volume_steps_index = 0;
  kg.coverage_asset = kg.coverage_object = kg.coverage_material = NULL;
  return kg;
}

void thread_globals_free(KernelGlobals &kg)
{
  if (kg.transparent_shadow_intersections) {
    free(kg.transparent_shadow_intersections);
  }
  for (int i = 0; i < 2; i++) {
    if (kg.decoupled_volume_steps[i]) {
      free(kg.decoupled_volume_steps[i]);
    }
  }
}

}  // namespace

extern "C" {

const char *cref_arch(void)
{
  return CREF_ARCH;
}

void *cref_create(void)
{
  RefContext *ctx = new RefContext();
  ctx->kg = make_globals();
  return ctx;
}

void cref_destroy(void *h)
{
  delete (RefContext *)h;
}

int cref_const_copy(void *h, const char *name, const void *host, size_t size)
{
  RefContext *ctx = (RefContext *)h;
  if (strcmp(name, "__data") != 0 || size != sizeof(KernelData)) {
    return -1;
  }
  kernel_const_copy(&ctx->kg, name, (void *)host, size);
  return 0;
}

/* size = number of elements, as CPUDevice::global_alloc passes mem.data_size. */
int cref_global_copy(void *h, const char *name, void *mem, size_t size)
{
  RefContext *ctx = (RefContext *)h;
  kernel_global_memory_copy(&ctx->kg, name, mem, size);
  return 0;
}

/* Render samples [start_sample, start_sample+num_samples) of the tile into
 * buffer (pass_stride floats per pixel), like CPUDevice::path_trace. */
void cref_render(void *h,
                 float *buffer,
                 int start_sample,
                 int num_samples,
                 int tx,
                 int ty,
                 int tw,
                 int th,
                 int offset,
                 int stride,
                 int nthreads)
{
  RefContext *ctx = (RefContext *)h;
  if (nthreads < 1) {
    nthreads = 1;
  }
  auto worker = [&](int t) {
    KernelGlobals kg = thread_globals(ctx->kg);
    for (int sample = start_sample; sample < start_sample + num_samples; sample++) {
      for (int y = ty + t; y < ty + th; y += nthreads) {
        for (int x = tx; x < tx + tw; x++) {
          CREF_PATH_TRACE(&kg, buffer, sample, x, y, offset, stride);
        }
      }
    }
    thread_globals_free(kg);
  };
  if (nthreads == 1) {
    worker(0);
    return;
  }
  std::vector<std::thread> threads;
  for (int t = 0; t < nthreads; t++) {
    threads.emplace_back(worker, t);
  }
  for (auto &th : threads) {
    th.join();
  }
}

/* Adaptive sampling render of one tile, single-threaded, as CPUDevice::render
 * does it (device_cpu.cpp:886-950) with KernelIntegrator.adaptive_stop_per_sample
 * = 0 (the GPU setting): after every sample the tile's pixels are path traced,
 * at need_filter samples (device_task.cpp:184-192) adaptive_sampling_filter
 * (device_cpu.cpp:832-864: stopping per pixel, then filter_x per row and
 * filter_y per column), and at the end adaptive_sampling_post
 * (device_cpu.cpp:866-885).  The reference functions are called as they lie
 * in kernel_adaptive_sampling.h. */
void cref_render_adaptive(void *h,
                          float *buffer,
                          int start_sample,
                          int num_samples,
                          int tx,
                          int ty,
                          int tw,
                          int th,
                          int offset,
                          int stride)
{
  RefContext *ctx = (RefContext *)h;
  KernelGlobals kgt = thread_globals(ctx->kg);
  KernelGlobals *kg = &kgt;
  const int end_sample = start_sample + num_samples;
  const int min_samples = kernel_data.integrator.adaptive_min_samples;
  const int step = kernel_data.integrator.adaptive_step;
  const int ps = kernel_data.film.pass_stride;
  int tile_sample = start_sample;
  for (int sample = start_sample; sample < end_sample; sample++) {
    for (int y = ty; y < ty + th; y++) {
      for (int x = tx; x < tx + tw; x++) {
        CREF_PATH_TRACE(kg, buffer, sample, x, y, offset, stride);
      }
    }
    tile_sample = sample + 1;
    if (sample > min_samples && (sample & (step - 1)) == (step - 1)) {
      WorkTile wtile;
      wtile.x = tx;
      wtile.y = ty;
      wtile.w = tw;
      wtile.h = th;
      wtile.offset = offset;
      wtile.stride = stride;
      wtile.buffer = buffer;
      if (!kernel_data.integrator.adaptive_stop_per_sample) {
        for (int y = ty; y < ty + th; y++) {
          for (int x = tx; x < tx + tw; x++) {
            kernel_do_adaptive_stopping(kg, buffer + (offset + x + y * stride) * ps, sample);
          }
        }
      }
      bool any = false;
      for (int y = ty; y < ty + th; y++) {
        any |= kernel_do_adaptive_filter_x(kg, y, &wtile);
      }
      for (int x = tx; x < tx + tw; x++) {
        any |= kernel_do_adaptive_filter_y(kg, x, &wtile);
      }
      if (!any) {
        tile_sample = end_sample;
        break;
      }
    }
  }
  for (int y = ty; y < ty + th; y++) {
    for (int x = tx; x < tx + tw; x++) {
      float *b = buffer + (offset + x + y * stride) * ps;
      const int sc = kernel_data.film.pass_sample_count;
      if (b[sc] < 0.0f) {
        b[sc] = -b[sc];
        const float mul = tile_sample / max((float)start_sample + 1.0f, b[sc]);
        if (mul != 1.0f) {
          kernel_adaptive_post_adjust(kg, b, mul);
        }
      }
      else {
        kernel_adaptive_post_adjust(kg, b, tile_sample / (tile_sample - 1.0f));
      }
    }
  }
  thread_globals_free(kgt);
}

/* rays: n x 8 floats (P.xyz, D.xyz, t, visibility-as-uint-bits).
 * out_f: n x 3 (t, u, v); out_i: n x 4 (hit, prim, object, type). */
void cref_intersect(void *h, int n, const float *rays, float *out_f, int *out_i)
{
  RefContext *ctx = (RefContext *)h;
  KernelGlobals kg = thread_globals(ctx->kg);
  for (int i = 0; i < n; i++) {
    const float *r = rays + 8 * i;
    Ray ray;
    memset((void *)&ray, 0, sizeof(ray));
    ray.P = make_float3(r[0], r[1], r[2]);
    ray.D = make_float3(r[3], r[4], r[5]);
    ray.t = r[6];
    ray.time = 0.5f;
    uint visibility;
    memcpy(&visibility, &r[7], 4);
    Intersection isect;
    memset((void *)&isect, 0, sizeof(isect));
    bool hit = scene_intersect(&kg, &ray, visibility, &isect);
    out_f[3 * i + 0] = isect.t;
    out_f[3 * i + 1] = isect.u;
    out_f[3 * i + 2] = isect.v;
    out_i[4 * i + 0] = hit ? 1 : 0;
    out_i[4 * i + 1] = isect.prim;
    out_i[4 * i + 2] = isect.object;
    out_i[4 * i + 3] = isect.type;
  }
  thread_globals_free(kg);
}

/* xys: n x 3 ints (x, y, sample). out: n x 8 floats (P.xyz, D.xyz, t, rng_hash bits). */
void cref_camera_rays(void *h, int n, const int *xys, float *out)
{
  RefContext *ctx = (RefContext *)h;
  KernelGlobals kg = thread_globals(ctx->kg);
  for (int i = 0; i < n; i++) {
    uint rng_hash = 0;
    Ray ray;
    memset((void *)&ray, 0, sizeof(ray));
    kernel_path_trace_setup(&kg, xys[3 * i + 2], xys[3 * i + 0], xys[3 * i + 1], &rng_hash, &ray);
    float *o = out + 8 * i;
    o[0] = ray.P.x;
    o[1] = ray.P.y;
    o[2] = ray.P.z;
    o[3] = ray.D.x;
    o[4] = ray.D.y;
    o[5] = ray.D.z;
    o[6] = ray.t;
    memcpy(&o[7], &rng_hash, 4);
  }
  thread_globals_free(kg);
}

/* q: n x 4 uint (rng_hash, sample, num_samples, dimension) -> out n floats. */
void cref_rng_1d(void *h, int n, const uint32_t *q, float *out)
{
  RefContext *ctx = (RefContext *)h;
  KernelGlobals kg = thread_globals(ctx->kg);
  for (int i = 0; i < n; i++) {
    out[i] = path_rng_1D(&kg, q[4 * i + 0], (int)q[4 * i + 1], (int)q[4 * i + 2], (int)q[4 * i + 3]);
  }
  thread_globals_free(kg);
}

/* Sobol direction vectors exactly as the host integrator builds
 * __sample_pattern_lut (render/integrator.cpp:235-243, render/sobol.cpp). */
void cref_sobol_directions(uint32_t *out, int dimensions)
{
  sobol_generate_direction_vectors((uint(*)[SOBOL_BITS])out, dimensions);
}

uint32_t cref_hash_uint2(uint32_t x, uint32_t y)
{
  return hash_uint2(x, y);
}

/* P, Ng: n x 3 floats -> out n x 3. */
void cref_ray_offset(int n, const float *P, const float *Ng, float *out)
{
  for (int i = 0; i < n; i++) {
    float3 r = ray_offset(make_float3(P[3 * i], P[3 * i + 1], P[3 * i + 2]),
                          make_float3(Ng[3 * i], Ng[3 * i + 1], Ng[3 * i + 2]));
    out[3 * i + 0] = r.x;
    out[3 * i + 1] = r.y;
    out[3 * i + 2] = r.z;
  }
}

/* Layout of the reference structs, for the ABI checker. Returns -1 if unknown. */
long cref_sizeof(const char *name)
{
#define HC_SZ(T) \
  if (strcmp(name, #T) == 0) \
    return (long)sizeof(T);
  HC_SZ(KernelData)
  HC_SZ(KernelCamera)
  HC_SZ(KernelFilm)
  HC_SZ(KernelBackground)
  HC_SZ(KernelIntegrator)
  HC_SZ(KernelBVH)
  HC_SZ(KernelTables)
  HC_SZ(KernelBake)
  HC_SZ(KernelObject)
  HC_SZ(KernelLight)
  HC_SZ(KernelLightDistribution)
  HC_SZ(KernelShader)
  HC_SZ(KernelParticle)
  HC_SZ(WorkTile)
#undef HC_SZ
  return -1;
}

long cref_offsetof(const char *sname, const char *fname)
{
#define HC_OFF(S) \
  if (strcmp(sname, #S) == 0) { \
    HC_FIELDS_##S(HC_OFF_FIELD_##S) \
  }
#define HC_FIELDS_KernelCamera HC_KERNEL_CAMERA_FIELDS
#define HC_FIELDS_KernelFilm HC_KERNEL_FILM_FIELDS
#define HC_FIELDS_KernelBackground HC_KERNEL_BACKGROUND_FIELDS
#define HC_FIELDS_KernelIntegrator HC_KERNEL_INTEGRATOR_FIELDS
#define HC_FIELDS_KernelBVH HC_KERNEL_BVH_FIELDS
#define HC_FIELDS_KernelTables HC_KERNEL_TABLES_FIELDS
#define HC_FIELDS_KernelBake HC_KERNEL_BAKE_FIELDS
#define HC_FIELDS_KernelObject HC_KERNEL_OBJECT_FIELDS
#define HC_FIELDS_KernelShader HC_KERNEL_SHADER_FIELDS
#define HC_FIELDS_KernelParticle HC_KERNEL_PARTICLE_FIELDS
#define HC_OFF_FIELD_KernelCamera(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelCamera, f);
#define HC_OFF_FIELD_KernelFilm(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelFilm, f);
#define HC_OFF_FIELD_KernelBackground(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelBackground, f);
#define HC_OFF_FIELD_KernelIntegrator(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelIntegrator, f);
#define HC_OFF_FIELD_KernelBVH(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelBVH, f);
#define HC_OFF_FIELD_KernelTables(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelTables, f);
#define HC_OFF_FIELD_KernelBake(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelBake, f);
#define HC_OFF_FIELD_KernelObject(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelObject, f);
#define HC_OFF_FIELD_KernelShader(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelShader, f);
#define HC_OFF_FIELD_KernelParticle(t, f, c) \
  if (strcmp(fname, #f) == 0) \
    return (long)offsetof(KernelParticle, f);
  HC_OFF(KernelCamera)
  HC_OFF(KernelFilm)
  HC_OFF(KernelBackground)
  HC_OFF(KernelIntegrator)
  HC_OFF(KernelBVH)
  HC_OFF(KernelTables)
  HC_OFF(KernelBake)
  HC_OFF(KernelObject)
  HC_OFF(KernelShader)
  HC_OFF(KernelParticle)
  /* Structs with unions: check the named members explicitly. */
  if (strcmp(sname, "KernelLight") == 0) {
    if (strcmp(fname, "type") == 0) return (long)offsetof(KernelLight, type);
    if (strcmp(fname, "co") == 0) return (long)offsetof(KernelLight, co);
    if (strcmp(fname, "shader_id") == 0) return (long)offsetof(KernelLight, shader_id);
    if (strcmp(fname, "samples") == 0) return (long)offsetof(KernelLight, samples);
    if (strcmp(fname, "max_bounces") == 0) return (long)offsetof(KernelLight, max_bounces);
    if (strcmp(fname, "random") == 0) return (long)offsetof(KernelLight, random);
    if (strcmp(fname, "strength") == 0) return (long)offsetof(KernelLight, strength);
    if (strcmp(fname, "pad1") == 0) return (long)offsetof(KernelLight, pad1);
    if (strcmp(fname, "tfm") == 0) return (long)offsetof(KernelLight, tfm);
    if (strcmp(fname, "itfm") == 0) return (long)offsetof(KernelLight, itfm);
    if (strcmp(fname, "uni") == 0) return (long)offsetof(KernelLight, spot);
  }
  if (strcmp(sname, "KernelLightDistribution") == 0) {
    if (strcmp(fname, "totarea") == 0) return (long)offsetof(KernelLightDistribution, totarea);
    if (strcmp(fname, "prim") == 0) return (long)offsetof(KernelLightDistribution, prim);
    if (strcmp(fname, "shader_flag") == 0)
      return (long)offsetof(KernelLightDistribution, mesh_light.shader_flag);
    if (strcmp(fname, "object_id") == 0)
      return (long)offsetof(KernelLightDistribution, mesh_light.object_id);
  }
  return -1;
}

/* FILM_CONVERT task on the CPU device (device/device_cpu.cpp film_convert ->
 * kernel_cpu_convert_to_byte / _half_float, kernels/cpu/kernel_cpu_impl.h:103-132):
 * every pixel of (x, y, w, h) at index offset + x + y*stride of a full-frame rgba. */
void cref_film_convert(void *h, void *rgba, float *buffer, float sample_scale, int x, int y, int w,
                       int hgt, int offset, int stride, int half)
{
  RefContext *ctx = (RefContext *)h;
  KernelGlobals kg = thread_globals(ctx->kg);
  for (int py = y; py < y + hgt; py++) {
    for (int px = x; px < x + w; px++) {
      if (half) {
        kernel_cpu_convert_to_half_float(&kg, (uchar4 *)rgba, buffer, sample_scale, px, py, offset, stride);
      }
      else {
        kernel_cpu_convert_to_byte(&kg, (uchar4 *)rgba, buffer, sample_scale, px, py, offset, stride);
      }
    }
  }
  thread_globals_free(kg);
}

/* SHADER task on the CPU device (device/device_cpu.cpp shader -> kernel_cpu_shader,
 * kernels/cpu/kernel_cpu_impl.h:152-170 -> kernel_background_evaluate,
 * kernel_bake.h:474-510): output[i] += world colour for i in [x, x + w), per sample. */
void cref_shader_eval(void *h, const void *input, void *output, int type, int x, int w, int num_samples)
{
  RefContext *ctx = (RefContext *)h;
  KernelGlobals kg = thread_globals(ctx->kg);
  for (int sample = 0; sample < num_samples; sample++) {
    for (int i = x; i < x + w; i++) {
      kernel_cpu_shader(&kg, (uint4 *)input, (float4 *)output, type, 0, i, 0, sample);
    }
  }
  thread_globals_free(kg);
}

}  // extern "C"
