/*
 * cy_integrator.h — the wavefront form of kernel_path_trace (kernel_path.h:509-695).
 *
 * The reference runs one camera sample per thread from camera ray to
 * kernel_write_result.  The HIP device keeps a fixed pool of path *slots*
 * resident in HBM and advances all of them one bounce per iteration through
 * three kernels: intersect_closest (bvh), shade (everything between two
 * traversals), intersect_shadow (occlusion of the light sample + deferred light
 * accumulation).  Work items are the tile's (pixel, sample) pairs, numbered
 * sample-major (item = (sample - start) * w*h + pixel); a slot whose path ends
 * takes the next unclaimed item, so the pool stays full until the items run out
 * and the number of iterations is set by the total path length, not by the
 * slowest pixel.  Each finished sample leaves its (L, alpha) record at its item
 * index; k_accumulate then adds every pixel's records to the render buffer in
 * sample order, so the buffer is bit-identical to the CPU kernel's sample-major
 * loop (device_cpu.cpp:906-921) with no float atomics.
 *
 * Radiance accumulation order per path is preserved: the deferred light
 * contribution of bounce k is added after shade(k) and before shade(k+1), exactly
 * where path_radiance_accum_light runs in kernel_branched_path_surface_connect_light.
 */
#ifndef CY_INTEGRATOR_H
#define CY_INTEGRATOR_H

#include "cy_path.h"
#include "cy_subsurface.h"
#include "cy_volume.h"
#include "cy_svm_raytrace.h"

/* Per-slot state, SoA of 16-byte records so every access is one dwordx4. */
typedef struct CyPathBuffers {
  hc_float4 *ray_P;      /* P.xyz, ray t */
  hc_float4 *ray_D;      /* D.xyz, visibility (bits) */
  hc_float4 *isect;      /* t, u, v, prim (bits); prim PRIM_NONE = miss, CY_PRIM_NO_RAY = no camera ray */
  int *isect_type;       /* primitive type of a hit (written only by scenes with curves) */
  int *isect_object;     /* instance object of the hit (written only by instanced scenes) */
  hc_uint4 *state0;      /* flag, rng_hash, rng_offset, sample */
  hc_uint4 *state1;      /* bounce, diffuse_bounce, glossy_bounce, transmission_bounce */
  hc_float4 *state2;     /* transparent_bounce (bits), min_ray_pdf, ray_pdf, ray_t */
  hc_float4 *throughput; /* throughput.xyz, L.transparent */
  hc_float4 *L;          /* L.emission.xyz, (unused) */
  hc_float4 *shadow_P;   /* shadow ray P.xyz, t */
  hc_float4 *shadow_D;   /* shadow ray D.xyz, (unused) */
  hc_float4 *shadow_L;   /* pending light contribution xyz, w: 1 = finish path after; with
                          * transparent shadows the light's BSDF-weighted eval instead */
  hc_float4 *shadow_T;   /* transparent shadows: path throughput xyz, w: bounces (8 bits each:
                          * bounce, transparent, diffuse, glossy); shadow_D.w: transmission bounce */
  uint *item;            /* work item of the path in the slot */
  /* volume scenes (KernelIntegrator.use_volumes): the path's volume stack,
   * CY_VOLUME_STACK / 2 records per slot of two (object, shader) entries, and
   * two records per slot: [0] object, shader, pending stack update flags
   * (CY_VOP_*), volume_bounce; [1] volume_bounds_bounce, the rng_offset the
   * pending shadow ray sees */
  hc_uint4 *vol_stack;
  hc_uint4 *vol_rec;
  /* scenes with disk BSSRDFs: the path's SubsurfaceIndirectRays stack
   * (kernel_types.h:1241-1249) beyond the ray the path continues with,
   * CY_SSS_RECS records of CY_SSS_REC_F4 float4 per slot, and its depth */
  hc_float4 *sss_rec;
  uint *sss_count;
  /* ... in scenes with volumes too: each record's volume stack
   * (CY_VOLUME_STACK / 2 records), and one more per slot for the stack the
   * pending shadow ray of a path that handed its slot to a record sees */
  hc_uint4 *sss_vol;
  /* scenes whose shaders read ray differentials (CyGlobals.use_ray_diff): the
   * path ray's dP / dD, CY_RAY_DIFF_F4 float4 per slot (written when the ray
   * is made; a camera launch's first shade recomputes them), and the shading
   * point's dP the pending transparent shadow ray carries, 2 float4 per slot */
  hc_float4 *ray_diff;
  hc_float4 *shadow_dP;
  /* transparent shadows in non-instanced scenes: the record-all traversal of
   * each pending shadow ray, done by the traversal stage (hipcycles.hip
   * k_shadow_record) before the shading stage evaluates the occluders --
   * per slot CY_SHADOW_REC_HITS hits (t, u, v, prim bits) sorted by distance
   * and their count, or CY_SREC_BLOCKED / CY_SREC_NONE (traverse here) */
  hc_float4 *shadow_hits;
  uint *shadow_nrec;
  /* scenes with shadow catcher objects: the path's shadow-catcher record of
   * PathRadiance (kernel_types.h:540-556), CY_CATCHER_F4 float4 per slot */
  hc_float4 *catcher;
  /* branched path tracing (KernelIntegrator.branched): the paths a camera hit
   * spawned that wait for the slot, CY_BR_RECS records of CY_BR_REC_F4 float4
   * per slot, and per slot the next record to start and the end (first in,
   * first out; cy_branched.h) */
  hc_float4 *br_rec;
  uint *br_count;
  /* light passes (KernelFilm.use_light_pass): the path's PathRadiance
   * components, CY_LP_F4 float4 per slot (CyLightPass) */
  hc_float4 *lp;
  /* decoupled volume ray marching (KernelIntegrator.volume_decoupled): the
   * slot's segment steps, CY_DECOUPLED_STEPS CyVolumeStep of at most
   * CY_DECOUPLED_STEP_BYTES each per slot (the device bounds the slots in
   * flight of such scenes so the 64 KB per slot fit) */
  void *dec_steps;
} CyPathBuffers;

/* The shadow-catcher part of PathRadiance (kernel_accumulate.h:203-233,
 * 526-620): the light a path behind a catcher would have received, shadowed
 * and unshadowed, the background seen through the catcher and the catcher's
 * throughput. */
typedef struct CyCatcher {
  cfloat3 path_total, path_total_shaded, background;
  float throughput, transparency;
  int has;
  int film_transparent; /* KernelBackground.transparent (not stored) */
} CyCatcher;
#define CY_CATCHER_F4 3
/* the kernels with the integrator extras -- shadow catchers, branched path
 * tracing, light passes (the _ext shading variants, which hipcy_load_kernels
 * picks for such scenes; kept out of the _tex variants, whose private memory
 * they would double) */
#ifndef CY_INTEGRATOR_EXT
#  define CY_INTEGRATOR_EXT 0
#endif
#define CY_CATCHER (CY_CLOSURE_EXT && CY_SVM_TEX && CY_INTEGRATOR_EXT)
/* the volume extras -- decoupled ray marching, a camera inside a volume
 * object, subsurface scattering in volume scenes (their stacks per exit ray):
 * the _vext shading variants (hipcy_load_kernels picks them); the _vol
 * variants keep the distance-sampled volume path alone */
#ifndef CY_VOLUME_EXT
#  define CY_VOLUME_EXT 1
#endif


#define CY_SHADOW_REC_HITS 4
#define CY_SREC_BLOCKED 0x100u
#define CY_SREC_NONE 0x200u

#define CY_SSS_RECS (BSSRDF_MAX_HITS - 1)
#define CY_BR_RECS 16
#define CY_BR_REC_F4 10 /* a path record (CY_SSS_REC_F4) and its branch factor */
#define CY_SSS_REC_F4 9 /* state (3), ray (2), throughput, ray differentials (3) */
#define CY_RAY_DIFF_F4 3

/* Pending volume stack update of a slot (cy_volume.h volume_stack_enter_exit
 * of the surface in vol_rec[0].xy): the reference updates the stack when the
 * path bounces through the surface, after the surface's light sample was
 * traced with the old stack; the wavefront traces that shadow ray in the next
 * stage, so the update is recorded and applied by the next shade. */
#define CY_VOP_PATH 1u       /* apply to the path's stack at its next shade */
#define CY_VOP_SHADOW 2u     /* apply to the shadow ray's copy (kernel_shadow.h:22-45) */
#define CY_VOP_BACKFACING 4u /* the surface was hit from behind (SD_BACKFACING) */
#define CY_VOP_OWN_STACK 8u  /* the shadow ray's stack is the slot's sss_vol[CY_SSS_RECS] */
#define CY_VOP_INIT_CAMERA 16u /* a new path's camera ray sets up the stack (camera inside a volume) */

/* One RenderTile of a multi-tile pass (hipcy_path_trace_tiles), or of a lane's
 * tile stream (hipcy_render_feed). */
typedef struct CyTileDesc {
  int x, y, w, h;
  int offset, stride;
  float *buffer;
  uint px_begin;    /* first pixel of the tile in the pass's (tile streams: its group's) pixel numbering */
  int start_sample; /* tile streams: the tile's first sample */
  uint item_begin;  /* tile streams: first work item of the tile's group in the lane's item numbering */
  int num_samples;  /* tile streams: samples of the tile */
  /* tile streams: a group of tiles with one sample range shares its items,
   * numbered sample-major over the group's pixels (group_npix per sample,
   * this tile's at px_begin ..), so the rays in flight at one time spread over
   * every tile of the group as a whole-frame pass's do; group_first is the
   * descriptor index of the group's first tile.  A tile alone (or one sample
   * range of a tile too large for the record ring) is a group of one. */
  uint group_npix;
  uint group_first;
} CyTileDesc;

typedef struct CyTile {
  int x, y, w, h;
  int y_step; /* rows of the tile are image rows y, y+y_step, ... (1 = contiguous) */
  int start_sample, end_sample; /* the sample range of this pass */
  int offset, stride;
  float *buffer;
  int pass_stride;
  uint n_items;           /* w * h * (end_sample - start_sample) */
  uint item_base;         /* first item of a camera launch: slot s holds item item_base + (s - slot_base) */
  uint *work_next;        /* next unclaimed item (atomic) */
  hc_float4 *samples_out; /* per item: L.xyz, alpha; alpha NaN = no camera ray */
  uint npix;              /* pixels of the pass (w * h for one tile) */
  int n_tiles;            /* > 1: the pass covers descs[0 .. n_tiles-1], pixels numbered tile by tile */
  const CyTileDesc *descs;
  /* adaptive sampling: KernelFilm pass_adaptive_aux_buffer / pass_sample_count
   * offsets (0 = pass absent) and pass_adaptive_aux_buffer && adaptive_threshold > 0 */
  int aux_offset;
  int sample_count_offset;
  int write_aux;
  /* Tile streams (hipcy_render_feed): work items are numbered tile by tile,
   * each tile's samples sample-major inside it (descs[k].item_begin), and
   * only tiles desc_lo .. n_tiles-1 can still hand out items; records live in
   * a ring indexed by item & ring_mask (all ones for ordinary passes). */
  int stream = 0;
  uint desc_lo = 0;
  uint ring_mask = 0xFFFFFFFFu;
} CyTile;

typedef struct CyStats {
  unsigned long long nodes, leaves, tris, rays;
  unsigned long long lane_iters, wave_iters; /* loop iterations: per lane summed, per wave max summed */
} CyStats; /* [0] closest-hit traversal, [1] shadow traversal */

CY_FN hc_float4 mkf4(float x, float y, float z, float w)
{
  hc_float4 r;
  r.x = x;
  r.y = y;
  r.z = z;
  r.w = w;
  return r;
}

/* Path-slot records are touched once per iteration and the whole pool is far
 * larger than the L2 and the 256 MB Infinity Cache: read and write them with
 * non-temporal hints so they stream past the caches and leave the scene
 * (BVH, triangles, shaders) resident for the random accesses. */
#if defined(__HIPCC__)
typedef float cy_v4f __attribute__((ext_vector_type(4)));
typedef unsigned int cy_v4u __attribute__((ext_vector_type(4)));
CY_FN hc_float4 cy_ld(const hc_float4 *p)
{
  const cy_v4f v = __builtin_nontemporal_load((const cy_v4f *)p);
  return mkf4(v.x, v.y, v.z, v.w);
}
CY_FN hc_uint4 cy_ld(const hc_uint4 *p)
{
  const cy_v4u v = __builtin_nontemporal_load((const cy_v4u *)p);
  hc_uint4 r;
  r.x = v.x;
  r.y = v.y;
  r.z = v.z;
  r.w = v.w;
  return r;
}
CY_FN int cy_ld(const int *p)
{
  return __builtin_nontemporal_load(p);
}
CY_FN uint cy_ld(const uint *p)
{
  return __builtin_nontemporal_load(p);
}
CY_FN void cy_st(hc_float4 *p, hc_float4 v)
{
  cy_v4f x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, (cy_v4f *)p);
}
CY_FN void cy_st(hc_uint4 *p, hc_uint4 v)
{
  cy_v4u x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, (cy_v4u *)p);
}
CY_FN void cy_st(int *p, int v)
{
  __builtin_nontemporal_store(v, p);
}
CY_FN void cy_st(uint *p, uint v)
{
  __builtin_nontemporal_store(v, p);
}
#else
template<typename T> static inline T cy_ld(const T *p)
{
  return *p;
}
template<typename T> static inline void cy_st(T *p, T v)
{
  *p = v;
}
#endif

CY_FN void load_state(const CyPathBuffers *b, int slot, CyPathState *s, const CyGlobals *kg)
{
  hc_uint4 s0 = cy_ld(&b->state0[slot]);
  hc_uint4 s1 = cy_ld(&b->state1[slot]);
  hc_float4 s2 = cy_ld(&b->state2[slot]);
  s->flag = (int)s0.x;
  s->rng_hash = s0.y;
  s->rng_offset = (int)s0.z;
  s->sample = (int)s0.w;
  s->num_samples = KD->integrator.aa_samples;
  s->bounce = (int)s1.x;
  s->diffuse_bounce = (int)s1.y;
  s->glossy_bounce = (int)s1.z;
  s->transmission_bounce = (int)s1.w;
  s->transparent_bounce = as_int(s2.x);
  s->min_ray_pdf = s2.y;
  s->ray_pdf = s2.z;
  s->ray_t = s2.w;
}

CY_FN void store_state(const CyPathBuffers *b, int slot, const CyPathState *s)
{
  hc_uint4 s0, s1;
  s0.x = (uint)s->flag;
  s0.y = s->rng_hash;
  s0.z = (uint)s->rng_offset;
  s0.w = (uint)s->sample;
  s1.x = (uint)s->bounce;
  s1.y = (uint)s->diffuse_bounce;
  s1.z = (uint)s->glossy_bounce;
  s1.w = (uint)s->transmission_bounce;
  cy_st(&b->state0[slot], s0);
  cy_st(&b->state1[slot], s1);
  cy_st(&b->state2[slot], mkf4(int_as_float(s->transparent_bounce), s->min_ray_pdf, s->ray_pdf, s->ray_t));
}

#if CY_CLOSURE_EXT
/* A ray's differentials dP, dD in three float4. */
CY_FN void diff_store(hc_float4 *dst, const CyDiff3 &dP, const CyDiff3 &dD)
{
  cy_st(&dst[0], mkf4(dP.dx.x, dP.dx.y, dP.dx.z, dP.dy.x));
  cy_st(&dst[1], mkf4(dP.dy.y, dP.dy.z, dD.dx.x, dD.dx.y));
  cy_st(&dst[2], mkf4(dD.dx.z, dD.dy.x, dD.dy.y, dD.dy.z));
}

CY_FN void diff_load(const hc_float4 *src, CyDiff3 *dP, CyDiff3 *dD)
{
  const hc_float4 a = cy_ld(&src[0]);
  const hc_float4 c = cy_ld(&src[1]);
  const hc_float4 e = cy_ld(&src[2]);
  dP->dx = mk3(a.x, a.y, a.z);
  dP->dy = mk3(a.w, c.x, c.y);
  dD->dx = mk3(c.z, c.w, e.x);
  dD->dy = mk3(e.y, e.z, e.w);
}

/* A subsurface indirect ray of the slot (state, ray, throughput; with ray
 * differentials their dP, dD). */
CY_FN void path_rec_store(hc_float4 *dst, const CyPathState *s, const CyRay *ray, cfloat3 throughput,
                          const CyDiff3 *dP, const CyDiff3 *dD)
{
  cy_st(&dst[0], mkf4(int_as_float(s->flag), as_float(s->rng_hash), int_as_float(s->rng_offset),
                      int_as_float(s->sample)));
  cy_st(&dst[1], mkf4(int_as_float(s->bounce), int_as_float(s->diffuse_bounce), int_as_float(s->glossy_bounce),
                      int_as_float(s->transmission_bounce)));
  cy_st(&dst[2], mkf4(int_as_float(s->transparent_bounce), s->min_ray_pdf, s->ray_pdf, s->ray_t));
  cy_st(&dst[3], mkf4(ray->P.x, ray->P.y, ray->P.z, ray->t));
  cy_st(&dst[4], mkf4(ray->D.x, ray->D.y, ray->D.z, int_as_float(s->volume_bounce)));
  cy_st(&dst[5], mkf4(throughput.x, throughput.y, throughput.z, int_as_float(s->volume_bounds_bounce)));
  if (dP) {
    diff_store(&dst[6], *dP, *dD);
  }
}

CY_FN void sss_rec_store(const CyPathBuffers *b, int slot, int r, const CyPathState *s, const CyRay *ray,
                         cfloat3 throughput, const CyDiff3 *dP = nullptr, const CyDiff3 *dD = nullptr)
{
  path_rec_store(b->sss_rec + ((size_t)slot * CY_SSS_RECS + (size_t)r) * CY_SSS_REC_F4, s, ray, throughput, dP, dD);
}

CY_FN void path_rec_load(const hc_float4 *src, const CyGlobals *kg, CyPathState *s, CyRay *ray, cfloat3 *throughput,
                         CyDiff3 *dP, CyDiff3 *dD)
{
  const hc_float4 r0 = cy_ld(&src[0]);
  const hc_float4 r1 = cy_ld(&src[1]);
  const hc_float4 r2 = cy_ld(&src[2]);
  const hc_float4 r3 = cy_ld(&src[3]);
  const hc_float4 r4 = cy_ld(&src[4]);
  const hc_float4 r5 = cy_ld(&src[5]);
  s->flag = as_int(r0.x);
  s->rng_hash = as_uint(r0.y);
  s->rng_offset = as_int(r0.z);
  s->sample = as_int(r0.w);
  s->num_samples = KD->integrator.aa_samples;
  s->bounce = as_int(r1.x);
  s->diffuse_bounce = as_int(r1.y);
  s->glossy_bounce = as_int(r1.z);
  s->transmission_bounce = as_int(r1.w);
  s->transparent_bounce = as_int(r2.x);
  s->min_ray_pdf = r2.y;
  s->ray_pdf = r2.z;
  s->ray_t = r2.w;
  s->volume_bounce = as_int(r4.w);
  s->volume_bounds_bounce = as_int(r5.w);
  ray->P = mk3(r3.x, r3.y, r3.z);
  ray->t = r3.w;
  ray->D = mk3(r4.x, r4.y, r4.z);
  *throughput = mk3(r5.x, r5.y, r5.z);
  if (dP) {
    diff_load(&src[6], dP, dD);
  }
}

CY_FN void sss_rec_load(const CyPathBuffers *b, int slot, int r, const CyGlobals *kg, CyPathState *s, CyRay *ray,
                        cfloat3 *throughput, CyDiff3 *dP = nullptr, CyDiff3 *dD = nullptr)
{
  path_rec_load(b->sss_rec + ((size_t)slot * CY_SSS_RECS + (size_t)r) * CY_SSS_REC_F4, kg, s, ray, throughput, dP,
                dD);
}

/* branch record r of the slot (the branch factor in its last float4) */
CY_FN hc_float4 *br_rec_at(const CyPathBuffers *b, int slot, int r)
{
  return b->br_rec + ((size_t)slot * CY_BR_RECS + (size_t)r) * CY_BR_REC_F4;
}

/* The slot's volume stack and pending update records (CyPathBuffers.vol_*);
 * a volume stack kept at src / dst (CY_VOLUME_STACK / 2 records). */
CY_FN void vol_stack_read(const hc_uint4 *src, CyVolumeStack *st)
{
  for (int k = 0; k < CY_VOLUME_STACK / 2; k++) {
    const hc_uint4 r = cy_ld(&src[k]);
    st->e[2 * k].object = (int)r.x;
    st->e[2 * k].shader = (int)r.y;
    st->e[2 * k + 1].object = (int)r.z;
    st->e[2 * k + 1].shader = (int)r.w;
    if ((int)r.y == SHADER_NONE || (int)r.w == SHADER_NONE) {
      break;
    }
  }
}

CY_FN void vol_stack_write(hc_uint4 *dst, const CyVolumeStack *st)
{
  for (int k = 0; k < CY_VOLUME_STACK / 2; k++) {
    hc_uint4 r;
    r.x = (uint)st->e[2 * k].object;
    r.y = (uint)st->e[2 * k].shader;
    r.z = (uint)st->e[2 * k + 1].object;
    r.w = (uint)st->e[2 * k + 1].shader;
    cy_st(&dst[k], r);
    if ((int)r.y == SHADER_NONE || (int)r.w == SHADER_NONE) {
      break;
    }
  }
}

CY_FN void vol_stack_load(const CyPathBuffers *b, int slot, CyVolumeStack *st)
{
  vol_stack_read(b->vol_stack + (size_t)slot * (CY_VOLUME_STACK / 2), st);
}

CY_FN void vol_stack_store(const CyPathBuffers *b, int slot, const CyVolumeStack *st)
{
  vol_stack_write(b->vol_stack + (size_t)slot * (CY_VOLUME_STACK / 2), st);
}

/* record r's volume stack (r == CY_SSS_RECS: the pending shadow ray's) */
CY_FN hc_uint4 *sss_vol_at(const CyPathBuffers *b, int slot, int r)
{
  return b->sss_vol + ((size_t)slot * (CY_SSS_RECS + 1) + (size_t)r) * (CY_VOLUME_STACK / 2);
}

CY_FN void vol_rec_store(const CyPathBuffers *b, int slot, uint object, uint shader, uint flags,
                         const CyPathState *state, int shadow_rng_offset)
{
  hc_uint4 r0, r1;
  r0.x = object;
  r0.y = shader;
  r0.z = flags;
  r0.w = (uint)state->volume_bounce;
  r1.x = (uint)state->volume_bounds_bounce;
  r1.y = (uint)shadow_rng_offset;
  r1.z = 0u;
  r1.w = 0u;
  cy_st(&b->vol_rec[2 * (size_t)slot], r0);
  cy_st(&b->vol_rec[2 * (size_t)slot + 1], r1);
}

/* A new path in the slot: the stack of a camera ray (kernel_path_state.h:62-68) */
CY_FN void vol_slot_init(const CyGlobals *kg, const CyPathBuffers *b, int slot)
{
  CyVolumeStack st;
  volume_stack_init(kg, &st);
  vol_stack_store(b, slot, &st);
  CyPathState s;
  s.volume_bounce = 0;
  s.volume_bounds_bounce = 0;
  vol_rec_store(b, slot, 0u, 0u, KD->cam.is_inside_volume ? CY_VOP_INIT_CAMERA : 0u, &s, 0);
}

#endif

/* kernel_path_state.h:19-71 (the volume stack: vol_slot_init / shade_path). */
CY_FN void path_state_init(const CyGlobals *kg, CyPathState *s, uint rng_hash, int sample)
{
  s->flag = PATH_RAY_CAMERA | PATH_RAY_MIS_SKIP | PATH_RAY_TRANSPARENT_BACKGROUND;
  s->rng_hash = rng_hash;
  s->rng_offset = PRNG_BASE_NUM;
  s->sample = sample;
  s->num_samples = KD->integrator.aa_samples;
  s->bounce = 0;
  s->diffuse_bounce = 0;
  s->glossy_bounce = 0;
  s->transmission_bounce = 0;
  s->transparent_bounce = 0;
  s->min_ray_pdf = CY_FLT_MAX;
  s->ray_pdf = 0.0f;
  s->ray_t = 0.0f;
  s->volume_bounce = 0;
  s->volume_bounds_bounce = 0;
}

/* kernel_path_state.h:72-178 */
template<bool VOL = false> CY_FN void path_state_next(const CyGlobals *kg, CyPathState *s, int label)
{
  if (label & LABEL_TRANSPARENT) {
    s->flag |= PATH_RAY_TRANSPARENT;
    s->transparent_bounce++;
    if (s->transparent_bounce >= KD->integrator.transparent_max_bounce) {
      s->flag |= PATH_RAY_TERMINATE_IMMEDIATE;
    }
    if (!KD->integrator.transparent_shadows) {
      s->flag |= PATH_RAY_MIS_SKIP;
    }
    s->rng_offset += PRNG_BOUNCE_NUM;
    return;
  }
  s->bounce++;
  if (s->bounce >= KD->integrator.max_bounce) {
    s->flag |= PATH_RAY_TERMINATE_AFTER_TRANSPARENT;
  }
  s->flag &= ~(PATH_RAY_ALL_VISIBILITY | PATH_RAY_MIS_SKIP);
  if (VOL && (label & LABEL_VOLUME_SCATTER)) {
    s->flag |= PATH_RAY_VOLUME_SCATTER;
    s->flag &= ~PATH_RAY_TRANSPARENT_BACKGROUND;
    s->volume_bounce++;
    if (s->volume_bounce >= KD->integrator.max_volume_bounce) {
      s->flag |= PATH_RAY_TERMINATE_AFTER_TRANSPARENT;
    }
    s->rng_offset += PRNG_BOUNCE_NUM;
    return;
  }
  if (label & LABEL_REFLECT) {
    s->flag |= PATH_RAY_REFLECT;
    s->flag &= ~PATH_RAY_TRANSPARENT_BACKGROUND;
    if (label & LABEL_DIFFUSE) {
      s->diffuse_bounce++;
      if (s->diffuse_bounce >= KD->integrator.max_diffuse_bounce) {
        s->flag |= PATH_RAY_TERMINATE_AFTER_TRANSPARENT;
      }
    }
    else {
      s->glossy_bounce++;
      if (s->glossy_bounce >= KD->integrator.max_glossy_bounce) {
        s->flag |= PATH_RAY_TERMINATE_AFTER_TRANSPARENT;
      }
    }
  }
  else {
    s->flag |= PATH_RAY_TRANSMIT;
    if (!(label & LABEL_TRANSMIT_TRANSPARENT)) {
      s->flag &= ~PATH_RAY_TRANSPARENT_BACKGROUND;
    }
    s->transmission_bounce++;
    if (s->transmission_bounce >= KD->integrator.max_transmission_bounce) {
      s->flag |= PATH_RAY_TERMINATE_AFTER_TRANSPARENT;
    }
  }
  if (label & LABEL_DIFFUSE) {
    s->flag |= PATH_RAY_DIFFUSE | PATH_RAY_DIFFUSE_ANCESTOR;
  }
  else if (label & LABEL_GLOSSY) {
    s->flag |= PATH_RAY_GLOSSY;
  }
  else {
    s->flag |= PATH_RAY_GLOSSY | PATH_RAY_SINGULAR | PATH_RAY_MIS_SKIP;
  }
  s->rng_offset += PRNG_BOUNCE_NUM;
}

/* kernel_path_state.h:197-206 */
CY_FN uint path_state_ray_visibility(const CyPathState *s)
{
  uint flag = (uint)s->flag & PATH_RAY_ALL_VISIBILITY;
  if (flag & PATH_RAY_TRANSMIT) {
    flag &= ~(PATH_RAY_DIFFUSE | PATH_RAY_GLOSSY);
  }
  if (s->flag & PATH_RAY_VOLUME_SCATTER) {
    flag |= PATH_RAY_DIFFUSE;
  }
  return flag;
}

/* kernel_path_state.h:208-244 */
CY_FN float path_state_continuation_probability(const CyGlobals *kg,
                                                const CyPathState *s,
                                                cfloat3 throughput,
                                                float branch_factor = 1.0f)
{
  if (s->flag & PATH_RAY_TERMINATE_IMMEDIATE) {
    return 0.0f;
  }
  else if (s->flag & PATH_RAY_TRANSPARENT) {
    if (s->transparent_bounce <= KD->integrator.transparent_min_bounce) {
      return 1.0f;
    }
    else if ((s->flag & PATH_RAY_SHADOW_CATCHER) && s->transparent_bounce <= 8) {
      return 1.0f; /* kernel_path_state.h:218-222: no RR behind a shadow catcher */
    }
  }
  else {
    if (s->bounce <= KD->integrator.min_bounce) {
      return 1.0f;
    }
    else if ((s->flag & PATH_RAY_SHADOW_CATCHER) && s->bounce <= 3) {
      return 1.0f; /* kernel_path_state.h:230-234 */
    }
  }
  /* branch_factor is 1.0 outside branched path tracing */
  return cmin(sqrtf(max3f(fabs3(throughput)) * branch_factor), 1.0f);
}

CY_FN bool path_state_ao_bounce(const CyGlobals *kg, const CyPathState *s)
{
  if (s->bounce <= KD->integrator.ao_bounces) {
    return false;
  }
  int bounce = s->bounce - s->transmission_bounce - (s->glossy_bounce > 0);
  return (bounce > KD->integrator.ao_bounces);
}

/* kernel_accumulate.h:276-284 */
CY_FN cfloat3 path_radiance_clamp(const CyGlobals *kg, cfloat3 L, int bounce)
{
  float limit = (bounce > 0) ? KD->integrator.sample_clamp_indirect :
                               KD->integrator.sample_clamp_direct;
  float sum = reduce_add3(fabs3(L));
  if (sum > limit) {
    L = mul3f(L, limit / sum);
  }
  return L;
}

/* PathRadiance with light passes (kernel_types.h:523-578): the components a
 * path adds to (emission stays the radiance L itself) and PathRadianceState,
 * the first bounce's BSDF weights per component */
typedef struct CyLightPass {
  cfloat3 background, direct_emission, indirect;
  cfloat3 direct_diffuse, direct_glossy, direct_transmission, direct_volume;
  cfloat3 color_diffuse, color_glossy, color_transmission;
  cfloat3 state_diffuse, state_glossy, state_transmission, state_volume, state_direct;
  cfloat3 shadow;
  float mist;
} CyLightPass;
#define CY_LP_F4 16

CY_FN void lightpass_init(CyLightPass *p)
{
  const cfloat3 z = mk3(0.0f, 0.0f, 0.0f);
  p->background = p->direct_emission = p->indirect = z;
  p->direct_diffuse = p->direct_glossy = p->direct_transmission = p->direct_volume = z;
  p->color_diffuse = p->color_glossy = p->color_transmission = z;
  p->state_diffuse = p->state_glossy = p->state_transmission = p->state_volume = p->state_direct = z;
  p->shadow = z;
  p->mist = 0.0f;
}

CY_FN void lightpass_load(const CyPathBuffers *b, int slot, CyLightPass *p)
{
  const hc_float4 *src = b->lp + (size_t)slot * CY_LP_F4;
  cfloat3 *f[15] = {&p->background, &p->direct_emission, &p->indirect, &p->direct_diffuse, &p->direct_glossy,
                    &p->direct_transmission, &p->direct_volume, &p->color_diffuse, &p->color_glossy,
                    &p->color_transmission, &p->state_diffuse, &p->state_glossy, &p->state_transmission,
                    &p->state_volume, &p->state_direct};
  for (int k = 0; k < 15; k++) {
    const hc_float4 r = cy_ld(&src[k]);
    *f[k] = mk3(r.x, r.y, r.z);
  }
  const hc_float4 r = cy_ld(&src[15]);
  p->shadow = mk3(r.x, r.y, r.z);
  p->mist = r.w;
}

CY_FN void lightpass_store(const CyPathBuffers *b, int slot, const CyLightPass *p)
{
  hc_float4 *dst = b->lp + (size_t)slot * CY_LP_F4;
  const cfloat3 *f[15] = {&p->background, &p->direct_emission, &p->indirect, &p->direct_diffuse, &p->direct_glossy,
                          &p->direct_transmission, &p->direct_volume, &p->color_diffuse, &p->color_glossy,
                          &p->color_transmission, &p->state_diffuse, &p->state_glossy, &p->state_transmission,
                          &p->state_volume, &p->state_direct};
  for (int k = 0; k < 15; k++) {
    cy_st(&dst[k], mkf4(f[k]->x, f[k]->y, f[k]->z, 0.0f));
  }
  cy_st(&dst[15], mkf4(p->shadow.x, p->shadow.y, p->shadow.z, p->mist));
}

/* path_radiance_accum_emission with light passes (kernel_accumulate.h:320-330) */
CY_FN void lightpass_accum_emission(CyLightPass *p, cfloat3 *L, int bounce, cfloat3 contribution)
{
  if (bounce == 0) {
    *L = add3(*L, contribution);
  }
  else if (bounce == 1) {
    p->direct_emission = add3(p->direct_emission, contribution);
  }
  else {
    p->indirect = add3(p->indirect, contribution);
  }
}

/* the slot's catcher record (CyPathBuffers.catcher) */
CY_FN void catcher_init(const CyGlobals *kg, CyCatcher *c)
{
  c->film_transparent = KD->background.transparent;
  c->path_total = c->path_total_shaded = c->background = mk3(0.0f, 0.0f, 0.0f);
  c->throughput = 0.0f;
  c->transparency = 1.0f;
  c->has = 0;
}

CY_FN void catcher_load(const CyGlobals *kg, const CyPathBuffers *b, int slot, CyCatcher *c)
{
  c->film_transparent = KD->background.transparent;
  const hc_float4 *src = b->catcher + (size_t)slot * CY_CATCHER_F4;
  const hc_float4 r0 = cy_ld(&src[0]);
  const hc_float4 r1 = cy_ld(&src[1]);
  const hc_float4 r2 = cy_ld(&src[2]);
  c->path_total = mk3(r0.x, r0.y, r0.z);
  c->throughput = r0.w;
  c->path_total_shaded = mk3(r1.x, r1.y, r1.z);
  c->transparency = r1.w;
  c->background = mk3(r2.x, r2.y, r2.z);
  c->has = as_int(r2.w);
}

CY_FN void catcher_store(const CyPathBuffers *b, int slot, const CyCatcher *c)
{
  hc_float4 *dst = b->catcher + (size_t)slot * CY_CATCHER_F4;
  cy_st(&dst[0], mkf4(c->path_total.x, c->path_total.y, c->path_total.z, c->throughput));
  cy_st(&dst[1], mkf4(c->path_total_shaded.x, c->path_total_shaded.y, c->path_total_shaded.z, c->transparency));
  cy_st(&dst[2], mkf4(c->background.x, c->background.y, c->background.z, int_as_float(c->has)));
}

/* Record the finished sample: kernel_passes.h:338-433 with only the combined
 * pass (kernel_accumulate.h:622-688, use_light_pass == 0, no shadow catcher);
 * the buffer addition itself happens in accumulate_pixel. */
CY_FN void write_sample(const CyTile *tile, uint item, cfloat3 L_emission, float L_transparent,
                        const CyCatcher *catcher = nullptr)
{
  cfloat3 L_sum = L_emission;
  float sum = fabsf(L_sum.x) + fabsf(L_sum.y) + fabsf(L_sum.z);
  if (!isfinite_safe(sum)) {
    L_sum = mk3(0.0f, 0.0f, 0.0f);
  }
  float alpha = 1.0f - L_transparent;
  if (catcher && catcher->has) {
    /* path_radiance_sum_shadowcatcher (kernel_accumulate.h:590-620) */
    const float path_total = average3(catcher->path_total);
    float shadow;
    if (!isfinite_safe(path_total)) {
      shadow = 0.0f;
    }
    else if (path_total == 0.0f) {
      shadow = catcher->transparency;
    }
    else {
      shadow = average3(catcher->path_total_shaded) / path_total;
    }
    if (catcher->film_transparent) {
      alpha -= catcher->throughput * shadow;
    }
    else {
      L_sum = add3(L_sum, mul3f(catcher->background, shadow));
    }
  }
  cy_st(&tile->samples_out[item & tile->ring_mask], mkf4(L_sum.x, L_sum.y, L_sum.z, alpha));
}

#define CY_NO_ITEM 0xFFFFFFFFu
#define CY_PRIM_NO_RAY (-2)

/* Tile of pixel p in a multi-tile pass (binary search of the tiles' first pixels). */
CY_FN int tile_of_pixel(const CyTile *tile, uint p)
{
  int lo = 0, hi = tile->n_tiles - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tile->descs[mid].px_begin <= p) {
      lo = mid;
    }
    else {
      hi = mid - 1;
    }
  }
  return lo;
}

/* Image position of pixel p of the pass. */
CY_FN void pass_pixel(const CyTile *tile, uint p, int *x, int *y)
{
  if (tile->n_tiles > 1) {
    const CyTileDesc &d = tile->descs[tile_of_pixel(tile, p)];
    const int local = (int)(p - d.px_begin);
    *x = d.x + local % d.w;
    *y = d.y + local / d.w;
  }
  else {
    *x = tile->x + (int)p % tile->w;
    *y = tile->y + ((int)p / tile->w) * tile->y_step;
  }
}

/* Group of a tile stream's work item: the last descriptor whose group starts
 * at or before it (binary search over the tiles that can still hand out
 * items; the tiles of one group share item_begin, so this is the group's last
 * tile). */
CY_FN int tile_of_item(const CyTile *tile, uint item)
{
  int lo = (int)tile->desc_lo, hi = tile->n_tiles - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tile->descs[mid].item_begin <= item) {
      lo = mid;
    }
    else {
      hi = mid - 1;
    }
  }
  return lo;
}

/* Pixel and sample of a work item (items are numbered sample-major; in a tile
 * stream, sample-major over each group's pixels). */
CY_FN void item_pixel(const CyTile *tile, uint item, int *x, int *y, int *sample)
{
  if (tile->stream) {
    int k = tile_of_item(tile, item);
    const CyTileDesc &g = tile->descs[k];
    const uint local = item - g.item_begin;
    const uint q = local % g.group_npix;
    *sample = g.start_sample + (int)(local / g.group_npix);
    /* the group's tile holding pixel q: the last with px_begin <= q */
    int lo = (int)g.group_first;
    while (lo < k) {
      const int mid = (lo + k + 1) >> 1;
      if (tile->descs[mid].px_begin <= q) {
        lo = mid;
      }
      else {
        k = mid - 1;
      }
    }
    const CyTileDesc &d = tile->descs[lo];
    const uint p = q - d.px_begin;
    *x = d.x + (int)(p % (uint)d.w);
    *y = d.y + (int)(p / (uint)d.w);
    return;
  }
  const uint p = item % tile->npix;
  *sample = tile->start_sample + (int)(item / tile->npix);
  pass_pixel(tile, p, x, y);
}

/* Render-buffer pixel of pass pixel p (the tile's rows stored contiguously). */
CY_FN float *pixel_buffer(const CyTile *tile, uint p)
{
  if (tile->n_tiles > 1) {
    const CyTileDesc &d = tile->descs[tile_of_pixel(tile, p)];
    const int local = (int)(p - d.px_begin);
    return d.buffer + (size_t)(d.offset + d.x + local % d.w + (d.y + local / d.w) * d.stride) * tile->pass_stride;
  }
  const int x = tile->x + (int)(p % (uint)tile->w);
  const int ybuf = tile->y + (int)(p / (uint)tile->w);
  return tile->buffer + (size_t)(tile->offset + x + ybuf * tile->stride) * tile->pass_stride;
}

/* Render-buffer pixel of work item `item` (its RenderTile's buffer at the
 * tile's offset / stride): where the camera path's AOV outputs are added. */
CY_FN float *item_buffer(const CyTile *tile, uint item);

/* path_radiance_clamp_and_sum with light passes (kernel_accumulate.h:622-676)
 * and kernel_write_light_passes (kernel_passes.h:292-337): the combined value
 * summed from the components (returned), the light passes added to the pixel */
CY_FN cfloat3 lightpass_finish(const CyGlobals *kg, float *buffer, cfloat3 emission, CyLightPass *p)
{
  /* path_radiance_sum_indirect (kernel_accumulate.h:536-556) */
  const cfloat3 dE = safe_divide_color(p->direct_emission, p->state_direct);
  p->direct_diffuse = add3(p->direct_diffuse, mul3(p->state_diffuse, dE));
  p->direct_glossy = add3(p->direct_glossy, mul3(p->state_glossy, dE));
  p->direct_transmission = add3(p->direct_transmission, mul3(p->state_transmission, dE));
  p->direct_volume = add3(p->direct_volume, mul3(p->state_volume, dE));
  const cfloat3 ind = safe_divide_color(p->indirect, p->state_direct);
  const cfloat3 z = mk3(0.0f, 0.0f, 0.0f);
  cfloat3 indirect_diffuse = add3(z, mul3(p->state_diffuse, ind));
  cfloat3 indirect_glossy = add3(z, mul3(p->state_glossy, ind));
  cfloat3 indirect_transmission = add3(z, mul3(p->state_transmission, ind));
  cfloat3 indirect_volume = add3(z, mul3(p->state_volume, ind));
  cfloat3 L_direct = add3(add3(add3(add3(p->direct_diffuse, p->direct_glossy), p->direct_transmission),
                               p->direct_volume),
                          emission);
  const cfloat3 L_indirect = add3(add3(add3(indirect_diffuse, indirect_glossy), indirect_transmission),
                                  indirect_volume);
  if (!KD->background.transparent) {
    L_direct = add3(L_direct, p->background);
  }
  cfloat3 L_sum = add3(L_direct, L_indirect);
  const float sum = fabsf(L_sum.x) + fabsf(L_sum.y) + fabsf(L_sum.z);
  if (!isfinite_safe(sum)) {
    L_sum = z;
    p->direct_diffuse = p->direct_glossy = p->direct_transmission = p->direct_volume = z;
    indirect_diffuse = indirect_glossy = indirect_transmission = indirect_volume = z;
    emission = z;
  }
  const int flag = KD->film.light_pass_flag;
  auto add = [&](int bit, int offset, cfloat3 v) {
    if (flag & (1 << bit)) {
      cy_pass_add(buffer + offset + 0, v.x);
      cy_pass_add(buffer + offset + 1, v.y);
      cy_pass_add(buffer + offset + 2, v.z);
    }
  };
  /* PASSMASK(type) = 1 << (type % 32), PassType MIST 32 .. VOLUME_INDIRECT 51 */
  add(7, KD->film.pass_diffuse_indirect, indirect_diffuse);
  add(10, KD->film.pass_glossy_indirect, indirect_glossy);
  add(13, KD->film.pass_transmission_indirect, indirect_transmission);
  add(19, KD->film.pass_volume_indirect, indirect_volume);
  add(6, KD->film.pass_diffuse_direct, p->direct_diffuse);
  add(9, KD->film.pass_glossy_direct, p->direct_glossy);
  add(12, KD->film.pass_transmission_direct, p->direct_transmission);
  add(18, KD->film.pass_volume_direct, p->direct_volume);
  add(1, KD->film.pass_emission, emission);
  add(2, KD->film.pass_background, p->background);
  add(8, KD->film.pass_diffuse_color, p->color_diffuse);
  add(11, KD->film.pass_glossy_color, p->color_glossy);
  add(14, KD->film.pass_transmission_color, p->color_transmission);
  if (flag & (1 << 4)) {
    float *q = buffer + KD->film.pass_shadow;
    cy_pass_add(q + 0, p->shadow.x);
    cy_pass_add(q + 1, p->shadow.y);
    cy_pass_add(q + 2, p->shadow.z);
    cy_pass_add(q + 3, KD->film.pass_shadow_scale);
  }
  if (flag & (1 << 0)) {
    cy_pass_add(buffer + KD->film.pass_mist, 1.0f - p->mist);
  }
  return L_sum;
}

CY_FN float *item_buffer(const CyTile *tile, uint item)
{
  if (tile->stream) {
    int k = tile_of_item(tile, item);
    const CyTileDesc &g = tile->descs[k];
    const uint q = (item - g.item_begin) % g.group_npix;
    int lo = (int)g.group_first;
    while (lo < k) {
      const int mid = (lo + k + 1) >> 1;
      if (tile->descs[mid].px_begin <= q) {
        lo = mid;
      }
      else {
        k = mid - 1;
      }
    }
    const CyTileDesc &d = tile->descs[lo];
    const uint p = q - d.px_begin;
    const int x = d.x + (int)(p % (uint)d.w), y = d.y + (int)(p / (uint)d.w);
    return d.buffer + (size_t)(d.offset + x + y * d.stride) * tile->pass_stride;
  }
  return pixel_buffer(tile, item % tile->npix);
}

/* kernel_path_trace_setup (kernel_path_common.h:21-46) for a work item.  With
 * adaptive sampling a pixel whose aux buffer marks it converged takes no
 * sample (kernel_path.h:654-659): reported as no camera ray (t = 0). */
CY_FN void item_camera_ray(const CyGlobals *kg, const CyTile *tile, uint item, uint *rng_hash, int *sample, CyRay *ray)
{
  int x, y;
  item_pixel(tile, item, &x, &y, sample);
  if (tile->aux_offset != 0 && pixel_buffer(tile, item % tile->npix)[tile->aux_offset + 3] > 0.0f) {
    *rng_hash = 0;
    ray->t = 0.0f;
    return;
  }
  camera_sample_ray(kg, x, y, *sample, rng_hash, ray);
}

#if CY_CLOSURE_EXT
/* The differentials of the slot's ray: a camera launch's first shade
 * recomputes the camera ray's (camera_sample_ray), later ones read the slot's
 * record. */
CY_FN void ray_diff_load(const CyGlobals *kg, const CyPathBuffers *b, const CyTile *tile, int slot, uint cam_item,
                         CyDiff3 *dP, CyDiff3 *dD)
{
  if (cam_item != CY_NO_ITEM) {
    int x, y, sample;
    uint rng_hash;
    CyRay ray;
    item_pixel(tile, cam_item, &x, &y, &sample);
    camera_sample_ray(kg, x, y, sample, &rng_hash, &ray, dP, dD);
  }
  else {
    diff_load(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, dP, dD);
  }
}
#endif

CY_FN void write_no_sample(const CyTile *tile, uint item)
{
  cy_st(&tile->samples_out[item & tile->ring_mask], mkf4(0.0f, 0.0f, 0.0f, __builtin_nanf("")));
}

/* Start work item `item` in the slot (refills after the camera launch).
 * Returns false when the sample has no camera ray (t == 0: no write,
 * kernel_path.h:660-662); the caller then claims another item. */
CY_FN bool slot_start(const CyGlobals *kg, const CyPathBuffers *b, const CyTile *tile, int slot, uint item)
{
  uint rng_hash;
  int sample;
  CyRay ray;
#if CY_CLOSURE_EXT
  if (kg->use_ray_diff) {
    CyDiff3 dP, dD;
    ray_diff_load(kg, b, tile, slot, item, &dP, &dD);
    diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, dP, dD);
  }
#endif
  item_camera_ray(kg, tile, item, &rng_hash, &sample, &ray);
  if (ray.t == 0.0f) {
    write_no_sample(tile, item);
    return false;
  }
  CyPathState s;
  path_state_init(kg, &s, rng_hash, sample);
  store_state(b, slot, &s);
#if CY_CLOSURE_EXT
  if (KD->integrator.use_volumes) {
    vol_slot_init(kg, b, slot);
  }
#endif
  cy_st(&b->item[slot], item);
  cy_st(&b->ray_P[slot], mkf4(ray.P.x, ray.P.y, ray.P.z, ray.t));
  cy_st(&b->ray_D[slot], mkf4(ray.D.x, ray.D.y, ray.D.z, as_float(path_state_ray_visibility(&s))));
  cy_st(&b->throughput[slot], mkf4(1.0f, 1.0f, 1.0f, 0.0f));
  cy_st(&b->L[slot], mkf4(0.0f, 0.0f, 0.0f, 1.0f)); /* w: the branch factor */
  if (b->br_rec) {
    cy_st(&b->br_count[2 * (size_t)slot], 0u); /* no waiting branched paths */
    cy_st(&b->br_count[2 * (size_t)slot + 1], 0u);
  }
  if (b->catcher) {
    CyCatcher c;
    catcher_init(kg, &c);
    catcher_store(b, slot, &c);
  }
#if CY_CLOSURE_EXT
  if (b->lp) {
    CyLightPass p;
    lightpass_init(&p);
    lightpass_store(b, slot, &p);
  }
#endif
  return true;
}

/* Finish the path in a slot: record its sample; the slot then needs new work. */
CY_FN void slot_finish(const CyPathBuffers *b, const CyTile *tile, int slot, uint item, cfloat3 L_emission,
                       float L_transparent, const CyCatcher *catcher = nullptr)
{
  write_sample(tile, item != CY_NO_ITEM ? item : cy_ld(&b->item[slot]), L_emission, L_transparent, catcher);
}

/* ---------------------------------------------------------------------------
 * Stage 1 (closest hit), around the traversal.  A camera launch (cam_item !=
 * CY_NO_ITEM) generates the work item's camera ray itself, so the first
 * traversal of a path reads no slot state at all and nothing is written for it
 * before its first shade.  Returns false when there is no ray to trace. */
CY_FN bool closest_load(const CyGlobals *kg, const CyPathBuffers *b, const CyTile *tile, int slot, uint cam_item,
                        CyRay *ray, uint *visibility)
{
  if (cam_item != CY_NO_ITEM) {
    uint rng_hash;
    int sample;
    item_camera_ray(kg, tile, cam_item, &rng_hash, &sample, ray);
    CyPathState s;
    path_state_init(kg, &s, rng_hash, sample);
    *visibility = path_state_ray_visibility(&s);
    return ray->t != 0.0f;
  }
  const hc_float4 rp = cy_ld(&b->ray_P[slot]);
  const hc_float4 rd = cy_ld(&b->ray_D[slot]);
  ray->P = mk3(rp.x, rp.y, rp.z);
  ray->t = rp.w;
  ray->D = mk3(rd.x, rd.y, rd.z);
  *visibility = as_uint(rd.w);
  return true;
}

template<bool INST>
CY_FN void closest_store(const CyPathBuffers *b, int slot, bool has_ray, bool hit, const CyIsect *isect)
{
  if (hit) {
    cy_st(&b->isect[slot], mkf4(isect->t, isect->u, isect->v, int_as_float(isect->prim)));
    if (INST) {
      cy_st(&b->isect_object[slot], isect->object);
    }
  }
  else {
    cy_st(&b->isect[slot], mkf4(0.0f, 0.0f, 0.0f, int_as_float(has_ray ? PRIM_NONE : CY_PRIM_NO_RAY)));
  }
}

/* Stage 3 (shadow), around the any-hit traversal: the shadow ray of the slot. */
CY_FN void shadow_load(const CyPathBuffers *b, int slot, CyRay *ray)
{
  const hc_float4 sp = cy_ld(&b->shadow_P[slot]);
  const hc_float4 sdr = cy_ld(&b->shadow_D[slot]);
  ray->P = mk3(sp.x, sp.y, sp.z);
  ray->t = sp.w;
  ray->D = mk3(sdr.x, sdr.y, sdr.z);
}

/* Deferred light add (path_radiance_accum_light) once occlusion is known;
 * returns true when the path ended with this light sample and its sample was
 * recorded. */
CY_FN bool shadow_finish(const CyPathBuffers *b, const CyTile *tile, int slot, bool blocked)
{
  const hc_float4 sl = cy_ld(&b->shadow_L[slot]);
  hc_float4 L4 = cy_ld(&b->L[slot]);
  if (!blocked) {
    L4.x = L4.x + sl.x;
    L4.y = L4.y + sl.y;
    L4.z = L4.z + sl.z;
  }
  if (sl.w != 0.0f) {
    /* (a path behind a shadow catcher traces its light samples itself: it
     * never ends here) */
    slot_finish(b, tile, slot, CY_NO_ITEM, mk3(L4.x, L4.y, L4.z), cy_ld(&b->throughput[slot]).w);
    return true;
  }
  cy_st(&b->L[slot], L4);
  return false;
}

/* kernel_shadow.h:386-462 shadow_blocked with transparent shadows, record-all
 * (the CPU kernel's __SHADOW_RECORD_ALL__ branch, kernel_shadow.h:130-230):
 * the occluders' shaders are evaluated in distance order, each from the ray
 * moved to the previous one, and their transparency attenuates *shadow.
 * Returns true when the light is blocked. */
#ifndef CY_SHADOW_MAX_HITS
#  define CY_SHADOW_MAX_HITS 64 /* kernel_shadow.h:127 SHADOW_STACK_MAX_HITS */
#endif
template<bool VOL = false>
CY_FN bool shadow_blocked_transparent(const CyGlobals *kg, CyRay ray, const CyPathState *state, CyShadeMem mem,
                                      cfloat3 *shadow, uint *err, void *volume_stack = nullptr,
                                      const CyDiff3 *ray_dP = nullptr, uint rec = CY_SREC_NONE,
                                      const hc_float4 *rec_hits = nullptr, uint visibility = PATH_RAY_SHADOW)
{
#if CY_CLOSURE_EXT
  /* volume scenes: the shadow ray's copy of the path's volume stack, crossed
   * at every transparent surface (kernel_shadow.h:49-85), and the volumes'
   * attenuation of each segment between surfaces */
  CyVolumeStack *vstack = (CyVolumeStack *)volume_stack;
#endif
  *shadow = mk3(1.0f, 1.0f, 1.0f);
  if (ray.t == 0.0f) {
    return false;
  }
  const int transparent_max_bounce = KD->integrator.transparent_max_bounce;
  if (state->transparent_bounce >= transparent_max_bounce) {
    return true;
  }
  const uint max_hits = (uint)(transparent_max_bounce - state->transparent_bounce - 1);
  CyIsect hits[CY_SHADOW_MAX_HITS];
  uint num_hits = 0;
  bool blocked;
  bool wide = kg->bvhw_nodes != nullptr && !kg->have_instancing;
  if (rec == CY_SREC_BLOCKED) {
    return true; /* the traversal stage's record-all met an occluder (blocked: no volume work) */
  }
  if (rec <= CY_SHADOW_REC_HITS) {
    /* the traversal stage's hits: sorted, distinct distances */
    for (uint k = 0; k < rec; k++) {
      const hc_float4 h = cy_ld(&rec_hits[k]);
      hits[k].t = h.x;
      hits[k].u = h.y;
      hits[k].v = h.z;
      hits[k].prim = as_int(h.w);
      hits[k].object = OBJECT_NONE;
      hits[k].type = kg->have_curves ? (int)kg->__prim_type[hits[k].prim] : PRIMITIVE_TRIANGLE;
    }
    num_hits = rec;
    blocked = false;
    wide = false;
  }
  else if (wide) {
    /* the wide layout's record-all (same hits, another recording order) */
    blocked = kg->have_curves ? bvhw_shadow_all<1>(kg, &ray, hits, visibility, max_hits, &num_hits, err) :
                                bvhw_shadow_all<0>(kg, &ray, hits, visibility, max_hits, &num_hits, err);
  }
  else {
    blocked = kg->have_curves ?
                  bvh2_shadow_all<true, 3>(kg, &ray, hits, visibility, max_hits, &num_hits, err) :
                  bvh2_shadow_all<true>(kg, &ray, hits, visibility, max_hits, &num_hits, err);
  }
  if (blocked || num_hits == 0) {
#if CY_CLOSURE_EXT
    if (VOL && !blocked && vstack->e[0].shader != SHADER_NONE) {
      CySD vsd;
      volume_shadow(kg, &vsd, state, vstack, &ray, shadow, mem, err);
    }
#endif
    return blocked;
  }
  /* sort_intersections (bvh/bvh.h:606-626): stable, by distance */
  for (int pass = 0; pass < 2; pass++) {
    for (uint i = 1; i < num_hits; i++) {
      const CyIsect h = hits[i];
      int j = (int)i - 1;
      while (j >= 0 && hits[j].t > h.t) {
        hits[j + 1] = hits[j];
        j--;
      }
      hits[j + 1] = h;
    }
    bool shared = false;
    for (uint i = 1; wide && i < num_hits; i++) {
      shared |= hits[i].t == hits[i - 1].t;
    }
    if (!shared) {
      break;
    }
    /* two hits at one distance: the first one recorded is shaded and the
     * other skipped, so the reference's recording order decides -- the BVH2
     * query gives it (the set of hits, and so blocked, stays the same) */
    wide = false;
    num_hits = 0;
    blocked = kg->have_curves ?
                  bvh2_shadow_all<true, 3>(kg, &ray, hits, visibility, max_hits, &num_hits, err) :
                  bvh2_shadow_all<true>(kg, &ray, hits, visibility, max_hits, &num_hits, err);
    if (blocked) {
      /* the two queries record the same set of hits, so this does not happen;
       * should it, the reference's own query decides, as in the first exit */
      return true;
    }
  }
  cfloat3 throughput = mk3(1.0f, 1.0f, 1.0f);
  const cfloat3 Pend = add3(ray.P, mul3f(ray.D, ray.t));
  float last_t = 0.0f;
  for (uint k = 0; k < num_hits; k++) {
    CyIsect isect = hits[k];
    const float new_t = isect.t;
    isect.t -= last_t;
    if (last_t == new_t) {
      continue;
    }
    last_t = new_t;
    /* shadow_handle_transparent_isect (kernel_shadow.h:49-85) */
#if CY_CLOSURE_EXT
    if (VOL && vstack->e[0].shader != SHADER_NONE) {
      CyRay segment_ray = ray;
      segment_ray.t = isect.t;
      CySD vsd;
      volume_shadow(kg, &vsd, state, vstack, &segment_ray, &throughput, mem, err);
    }
#endif
    CySD sd;
    sd.closure = mem.closure;
    sd.svm_stack = mem.svm_stack;
    sd.svm_stride = mem.svm_stride;
    sd.svm_fast = mem.svm_fast;
    sd.svm_spill = mem.svm_spill;
#if CY_CLOSURE_EXT
    /* the shadow ray carries the shading point's dP and no dD
     * (kernel_emission.h:193-194) */
    CyDiff3 zero_dD;
    zero_dD.dx = zero_dD.dy = mk3(0.0f, 0.0f, 0.0f);
    shader_setup_from_ray(kg, &sd, &isect, &ray, ray_dP, &zero_dD);
#else
    shader_setup_from_ray(kg, &sd, &isect, &ray);
#endif
    if (!VOL || !(sd.flag & SD_HAS_ONLY_VOLUME)) {
      CyPathState st = *state;
      st.bounce += 1; /* path_state_modify_bounce */
      shader_eval_surface(kg, &sd, &st, PATH_RAY_SHADOW, err);
      throughput = mul3(throughput, shader_bsdf_transparency(&sd));
    }
    if (is_zero3(throughput)) {
      return true;
    }
#if CY_CLOSURE_EXT
    if (VOL) {
      volume_stack_enter_exit(sd.flag, sd.object, sd.shader, vstack);
    }
#endif
    ray.P = sd.P;
    if (ray.t != CY_FLT_MAX) {
      ray.D = normalize_len3(sub3(Pend, ray.P), &ray.t);
    }
  }
#if CY_CLOSURE_EXT
  if (VOL && vstack->e[0].shader != SHADER_NONE) {
    /* the last segment, towards the light */
    CySD vsd;
    volume_shadow(kg, &vsd, state, vstack, &ray, &throughput, mem, err);
  }
#endif
  *shadow = throughput;
  return is_zero3(throughput);
}

#if CY_CLOSURE_EXT
/* shadow_blocked_transparent<true> for the light samples the shading stage
 * traces itself (subsurface exit points, decoupled volume segments): one
 * out-of-line copy instead of one inlined per call site. */
CY_NOINLINE bool shadow_blocked_volume_inline(const CyGlobals *kg, const CyRay *ray, const CyPathState *state,
                                              CyShadeMem mem, cfloat3 *shadow, uint *err, CyVolumeStack *stack,
                                              const CyDiff3 *ray_dP)
{
  return shadow_blocked_transparent<true>(kg, *ray, state, mem, shadow, err, stack, ray_dP);
}
#endif

/* The traversal half of a pending transparent shadow ray (hipcycles.hip
 * k_shadow_record; non-instanced scenes): the record-all query, its hits
 * sorted and stored in the slot's record when they fit and their distances
 * are distinct.  Returns the record word (hit count, CY_SREC_BLOCKED or
 * CY_SREC_NONE); shadow_finish_transparent takes it from there. */
template<int HAIR>
CY_FN uint shadow_record(const CyGlobals *kg, const CyPathBuffers *b, int slot, uint *err)
{
  CyRay ray;
  shadow_load(b, slot, &ray);
  const uint transparent_bounce = (as_uint(cy_ld(&b->shadow_T[slot]).w) >> 8) & 0xFFu;
  const int transparent_max_bounce = KD->integrator.transparent_max_bounce;
  if (ray.t == 0.0f || (int)transparent_bounce >= transparent_max_bounce) {
    return CY_SREC_NONE; /* shadow_blocked_transparent ends these before traversing */
  }
  const uint max_hits = (uint)(transparent_max_bounce - (int)transparent_bounce - 1);
  CyIsect hits[CY_SHADOW_MAX_HITS];
  uint n = 0;
  bool blocked;
  if constexpr (HAIR <= 1) {
    blocked = kg->bvhw_nodes ? bvhw_shadow_all<HAIR>(kg, &ray, hits, PATH_RAY_SHADOW, max_hits, &n, err) :
                               bvh2_shadow_all<false, HAIR>(kg, &ray, hits, PATH_RAY_SHADOW, max_hits, &n, err);
  }
  else {
    blocked = bvh2_shadow_all<false, HAIR>(kg, &ray, hits, PATH_RAY_SHADOW, max_hits, &n, err);
  }
  if (blocked) {
    return CY_SREC_BLOCKED;
  }
  if (n > CY_SHADOW_REC_HITS) {
    return CY_SREC_NONE;
  }
  /* sort_intersections (bvh/bvh.h:606-626): stable, by distance */
  for (uint k = 1; k < n; k++) {
    const CyIsect h = hits[k];
    int j = (int)k - 1;
    while (j >= 0 && hits[j].t > h.t) {
      hits[j + 1] = hits[j];
      j--;
    }
    hits[j + 1] = h;
  }
  for (uint k = 1; k < n; k++) {
    if (hits[k].t == hits[k - 1].t) {
      return CY_SREC_NONE; /* the recording order decides: the shading kernel traverses in the BVH2's */
    }
  }
  hc_float4 *out = b->shadow_hits + (size_t)slot * CY_SHADOW_REC_HITS;
  for (uint k = 0; k < n; k++) {
    cy_st(&out[k], mkf4(hits[k].t, hits[k].u, hits[k].v, int_as_float(hits[k].prim)));
  }
  return n;
}

/* The transparent-shadow counterpart of shadow_finish: occlusion and
 * attenuation of the pending light sample, then its contribution
 * (path_radiance_accum_light: throughput * shadow, times the eval, clamped). */
template<bool VOL = false>
CY_FN bool shadow_finish_transparent(const CyGlobals *kg, const CyPathBuffers *b, const CyTile *tile, int slot,
                                     CyShadeMem mem, uint *err)
{
  CyRay ray;
  shadow_load(b, slot, &ray);
  const hc_float4 sl = cy_ld(&b->shadow_L[slot]);
  const hc_float4 st4 = cy_ld(&b->shadow_T[slot]);
  const uint packed = as_uint(st4.w);
  CyPathState state;
  load_state(b, slot, &state, kg);
  state.bounce = (int)(packed & 0xFF);
  state.transparent_bounce = (int)((packed >> 8) & 0xFF);
  state.diffuse_bounce = (int)((packed >> 16) & 0xFF);
  state.glossy_bounce = (int)(packed >> 24);
  state.transmission_bounce = as_int(cy_ld(&b->shadow_D[slot]).w);
  const uint rec = b->shadow_nrec ? cy_ld(&b->shadow_nrec[slot]) : CY_SREC_NONE;
  const hc_float4 *rec_hits = b->shadow_hits ? b->shadow_hits + (size_t)slot * CY_SHADOW_REC_HITS : nullptr;
  cfloat3 shadow;
  bool blocked;
#if CY_CLOSURE_EXT
  CyDiff3 sdP;
  const CyDiff3 *sdP_ptr = nullptr;
  if (kg->use_ray_diff) {
    const hc_float4 a = cy_ld(&b->shadow_dP[2 * (size_t)slot]);
    const hc_float4 c = cy_ld(&b->shadow_dP[2 * (size_t)slot + 1]);
    sdP.dx = mk3(a.x, a.y, a.z);
    sdP.dy = mk3(a.w, c.x, c.y);
    sdP_ptr = &sdP;
  }
  if (VOL) {
    /* the stack the light sample saw, crossing the surface when the ray
     * leaves through it, and the rng offset of the sample's bounce */
    CyVolumeStack vstack;
    vol_stack_load(b, slot, &vstack);
    const hc_uint4 r0 = cy_ld(&b->vol_rec[2 * (size_t)slot]);
    const hc_uint4 r1 = cy_ld(&b->vol_rec[2 * (size_t)slot + 1]);
    if (r0.z & CY_VOP_OWN_STACK) {
      vol_stack_read(sss_vol_at(b, slot, CY_SSS_RECS), &vstack);
    }
    if (r0.z & CY_VOP_SHADOW) {
      volume_stack_enter_exit(SD_HAS_VOLUME | ((r0.z & CY_VOP_BACKFACING) ? SD_BACKFACING : 0), (int)r0.x,
                              (int)r0.y, &vstack);
    }
    state.rng_offset = (int)r1.y;
    blocked = shadow_blocked_transparent<true>(kg, ray, &state, mem, &shadow, err, &vstack, sdP_ptr, rec, rec_hits);
  }
  else
  {
    blocked = shadow_blocked_transparent<false>(kg, ray, &state, mem, &shadow, err, nullptr, sdP_ptr, rec,
                                                rec_hits);
  }
#else
  blocked = shadow_blocked_transparent<false>(kg, ray, &state, mem, &shadow, err, nullptr, nullptr, rec, rec_hits);
#endif
  hc_float4 L4 = cy_ld(&b->L[slot]);
  if (!blocked) {
    const cfloat3 shaded_throughput = mul3(mul3f(mk3(st4.x, st4.y, st4.z), 1.0f), shadow);
    cfloat3 contribution = mul3(shaded_throughput, mk3(sl.x, sl.y, sl.z));
    contribution = path_radiance_clamp(kg, contribution, state.bounce);
    L4.x = L4.x + contribution.x;
    L4.y = L4.y + contribution.y;
    L4.z = L4.z + contribution.z;
  }
  if (sl.w != 0.0f) {
    CyCatcher catcher;
    if (b->catcher) {
      catcher_load(kg, b, slot, &catcher);
    }
    slot_finish(b, tile, slot, CY_NO_ITEM, mk3(L4.x, L4.y, L4.z), cy_ld(&b->throughput[slot]).w,
                b->catcher ? &catcher : nullptr);
    return true;
  }
  cy_st(&b->L[slot], L4);
  return false;
}

/* Add pixel p's sample records to the render buffer in sample order
 * (kernel_write_pass_float4, kernel_write_passes.h:49-65, once per sample).
 * With adaptive sampling every recorded sample also does what the rest of
 * kernel_write_result does (kernel_passes.h:394-432): samples with
 * sample_is_even (kernel_random.h:294-318; for Sobol `sample & 1`) add twice
 * their radiance to the aux buffer, and the sample count pass is made
 * negative and decremented.  The tile's rows are stored contiguously. */
CY_FN void accumulate_pixel(const CyTile *tile, int p)
{
  const int npix = (int)tile->npix;
  float *buf = pixel_buffer(tile, (uint)p);
  float b0 = buf[0], b1 = buf[1], b2 = buf[2], b3 = buf[3];
  const int n = tile->end_sample - tile->start_sample;
  if (tile->aux_offset == 0 && tile->sample_count_offset == 0) {
    for (int k = 0; k < n; k++) {
      const hc_float4 r = cy_ld(&tile->samples_out[(size_t)k * npix + p]);
      if (r.w == r.w) {
        b0 += r.x;
        b1 += r.y;
        b2 += r.z;
        b3 += r.w;
      }
    }
  }
  else {
    float *aux = buf + tile->aux_offset;
    float a0 = aux[0], a1 = aux[1], a2 = aux[2], a3 = aux[3];
    float sc = tile->sample_count_offset ? buf[tile->sample_count_offset] : 0.0f;
    for (int k = 0; k < n; k++) {
      const hc_float4 r = cy_ld(&tile->samples_out[(size_t)k * npix + p]);
      if (r.w == r.w) {
        b0 += r.x;
        b1 += r.y;
        b2 += r.z;
        b3 += r.w;
        if (tile->write_aux && ((tile->start_sample + k) & 1)) {
          a0 += r.x * 2.0f;
          a1 += r.y * 2.0f;
          a2 += r.z * 2.0f;
          a3 += 0.0f;
        }
        if (tile->sample_count_offset) {
          if (sc > 0.0f) {
            sc *= -1.0f;
          }
          sc += -1.0f;
        }
      }
    }
    if (tile->aux_offset) {
      aux[0] = a0;
      aux[1] = a1;
      aux[2] = a2;
      aux[3] = a3;
    }
    if (tile->sample_count_offset) {
      buf[tile->sample_count_offset] = sc;
    }
  }
  buf[0] = b0;
  buf[1] = b1;
  buf[2] = b2;
  buf[3] = b3;
}

/* accumulate_pixel for pixel p of tile d of a tile stream: the tile's records
 * of sample k sit at item d.item_begin + k * group_npix + px_begin + p of the
 * lane's ring. */
CY_FN void accumulate_stream_pixel(const CyTileDesc &d, const hc_float4 *ring, uint ring_mask, int pass_stride,
                                   int p)
{
  float *buf = d.buffer + (size_t)(d.offset + d.x + p % d.w + (d.y + p / d.w) * d.stride) * pass_stride;
  float b0 = buf[0], b1 = buf[1], b2 = buf[2], b3 = buf[3];
  const uint npix = d.group_npix;
  const uint first = d.item_begin + d.px_begin + (uint)p;
  /* the records of 8 samples are requested before they are added (in
   * sample order): a tile has few pixels, so each thread needs several
   * loads in flight */
  constexpr int U = 8;
  int k = 0;
  for (; k + U <= d.num_samples; k += U) {
    hc_float4 r[U];
#pragma unroll
    for (int j = 0; j < U; j++) {
      r[j] = cy_ld(&ring[(first + (uint)(k + j) * npix) & ring_mask]);
    }
#pragma unroll
    for (int j = 0; j < U; j++) {
      if (r[j].w == r[j].w) {
        b0 += r[j].x;
        b1 += r[j].y;
        b2 += r[j].z;
        b3 += r[j].w;
      }
    }
  }
  for (; k < d.num_samples; k++) {
    const hc_float4 r = cy_ld(&ring[(first + (uint)k * npix) & ring_mask]);
    if (r.w == r.w) {
      b0 += r.x;
      b1 += r.y;
      b2 += r.z;
      b3 += r.w;
    }
  }
  buf[0] = b0;
  buf[1] = b1;
  buf[2] = b2;
  buf[3] = b3;
}

/* shader_setup_from_background (kernel_shader.h:397-439): P = D, N = Ng = I = -D */
CY_FN void shader_setup_from_background(const CyGlobals *kg, CySD *sd, cfloat3 D, CyShadeMem mem,
                                        const CyDiff3 *ray_dD = nullptr)
{
  sd->closure = mem.closure;
  sd->svm_stack = mem.svm_stack;
  sd->svm_stride = mem.svm_stride;
  sd->svm_fast = mem.svm_fast;
  sd->svm_spill = mem.svm_spill;
  sd->P = D;
  sd->N = neg3(D);
  sd->Ng = neg3(D);
  sd->I = neg3(D);
  sd->shader = KD->background.surface_shader;
  sd->flag = kg->__shaders[sd->shader & SHADER_MASK].flags;
  sd->object_flag = 0;
  sd->ray_length = 0.0f;
  sd->object = OBJECT_NONE;
  sd->prim = PRIM_NONE;
  sd->type = 0; /* PRIMITIVE_NONE */
#if CY_CLOSURE_EXT
  sd->dPdu = mk3(0.0f, 0.0f, 0.0f);
  sd->dPdv = mk3(0.0f, 0.0f, 0.0f);
  /* dP = the ray's dD, dI = -dD (kernel_shader.h:426-432) */
  sd_zero_differentials(sd);
  if (ray_dD) {
    sd->dP = *ray_dD;
    sd->dI.dx = neg3(ray_dD->dx);
    sd->dI.dy = neg3(ray_dD->dy);
  }
#endif
  sd->u = 0.0f;
  sd->v = 0.0f;
  sd->svm_closure_weight = mk3(0.0f, 0.0f, 0.0f);
  sd->closure_emission_background = mk3(0.0f, 0.0f, 0.0f);
  sd->closure_transparent_extinction = mk3(0.0f, 0.0f, 0.0f);
}

/* shader_background_eval (kernel_shader.h:996-1004) */
CY_FN cfloat3 shader_background_eval(const CySD *sd)
{
  return (sd->flag & SD_EMISSION) ? sd->closure_emission_background : mk3(0.0f, 0.0f, 0.0f);
}

/* indirect_background's non-constant branch (kernel_emission.h:309-321): the
 * world shader evaluated along the ray with the bounce raised for the
 * light-path node (path_state_modify_bounce); also direct_emissive_eval's
 * background-light branch (kernel_emission.h:40-51, path flag EMISSION only). */
CY_FN cfloat3 background_eval_svm(const hc_KernelData *data,
                                        const hc_uint4 *svm_nodes,
                                        const hc_KernelShader *shaders,
                                        const hc_KernelObject *objects,
                                        const hc_TextureInfo *texture_info,
                                        cfloat3 D,
                                        CyShadeMem mem,
                                        CyPathState state,
                                        int path_flag,
                                        uint *err,
                                        const CyDiff3 *ray_dD = nullptr)
{
  CyGlobals kgv;
  kgv.data = data;
  kgv.__svm_nodes = svm_nodes;
  kgv.__shaders = shaders;
  kgv.__objects = objects;
  kgv.__texture_info = texture_info;
  const CyGlobals *kg = &kgv;
  CySD esd;
  shader_setup_from_background(kg, &esd, D, mem, ray_dD);
  state.bounce += 1;
  shader_eval_surface(kg, &esd, &state, path_flag, err);
  return shader_background_eval(&esd);
}

#if CY_SVM_TEX
/* direct_emissive_eval's non-constant branch for a mesh-light or lamp sample
 * (kernel_emission.h:54-88): shader_setup_from_sample (kernel_shader.h:244-360;
 * world space, no differentials; a lamp's transform is the identity the host
 * packs) and the emitter's SVM program with PATH_RAY_EMISSION, which stores no
 * closures (shader_eval_surface: max_closures 0), so the shading point's
 * closure array in `mem` is left intact; then shader_emissive_eval
 * (kernel_shader.h, emissive_simple_eval).  The caller flips ls.Ng to the
 * emitter's backfacing-corrected normal (ls->Ng = emission_sd->Ng), which is
 * the same flip the constant branch makes.  Inlined by default.  This
 * out-of-line form (CY_EMISSIVE_OOL) is bit-exact on the GPU;
 * the r03 form that produced non-finite films wrote ls->Ng through a pointer
 * into the caller's private frame. */
#ifdef CY_EMISSIVE_OOL /* diagnostic build (build.py --variant ... -DCY_EMISSIVE_OOL): the out-of-line form */
CY_NOINLINE
#else
CY_FN
#endif
cfloat3 emissive_eval_svm(const CyGlobals *kg, cfloat3 P, cfloat3 Ng, cfloat3 I, int shader, int object,
                                      int prim, int lamp, float u, float v, float t, CyShadeMem mem, CyPathState state,
                                      uint *err)
{
  CySD esd;
  esd.closure = mem.closure;
  esd.svm_stack = mem.svm_stack;
  esd.svm_stride = mem.svm_stride;
  esd.svm_fast = mem.svm_fast;
  esd.svm_spill = mem.svm_spill;
  esd.P = P;
  esd.N = Ng;
  esd.Ng = Ng;
  esd.I = I;
  esd.shader = shader;
  esd.type = (prim != PRIM_NONE) ? PRIMITIVE_TRIANGLE : ((lamp != LAMP_NONE) ? (1 << 6) /* PRIMITIVE_LAMP */ : 0);
  esd.lamp = lamp;
  esd.object = object;
  esd.prim = prim;
  esd.u = u;
  esd.v = v;
  esd.ray_length = t;
  esd.flag = kg->__shaders[(uint)esd.shader & SHADER_MASK].flags;
  esd.object_flag = (esd.object != OBJECT_NONE) ? (int)kg->__object_flag[esd.object] : 0;
  if ((esd.type & PRIMITIVE_TRIANGLE) && ((uint)esd.shader & SHADER_SMOOTH_NORMAL)) {
    esd.N = triangle_smooth_normal(kg, Ng, esd.prim, esd.u, esd.v);
    if (!(esd.object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
      esd.N = object_normal_transform(kg, esd.object, esd.N);
    }
  }
#if CY_CLOSURE_EXT
  esd.dPdu = mk3(0.0f, 0.0f, 0.0f);
  esd.dPdv = mk3(0.0f, 0.0f, 0.0f);
  if (esd.type & PRIMITIVE_TRIANGLE) {
    triangle_dPdudv(kg, esd.prim, &esd.dPdu, &esd.dPdv);
    if (!(esd.object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
      esd.dPdu = transform_direction(object_tfm(kg, esd.object), esd.dPdu);
      esd.dPdv = transform_direction(object_tfm(kg, esd.object), esd.dPdv);
    }
  }
#endif
  if (esd.prim != PRIM_NONE && dot3(esd.Ng, esd.I) < 0.0f) {
    esd.flag |= SD_BACKFACING;
    esd.Ng = neg3(esd.Ng);
    esd.N = neg3(esd.N);
#if CY_CLOSURE_EXT
    esd.dPdu = neg3(esd.dPdu);
    esd.dPdv = neg3(esd.dPdv);
#endif
  }
#if CY_CLOSURE_EXT
  sd_zero_differentials(&esd); /* shader_setup_from_sample: no ray differentials */
#endif
  esd.closure_emission_background = mk3(0.0f, 0.0f, 0.0f);
  esd.closure_transparent_extinction = mk3(0.0f, 0.0f, 0.0f);
  esd.svm_closure_weight = mk3(0.0f, 0.0f, 0.0f);
  state.bounce += 1; /* path_state_modify_bounce(state, true) */
  shader_eval_surface(kg, &esd, &state, PATH_RAY_EMISSION, err);
  if (!(esd.flag & SD_EMISSION)) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  const float res = (fabsf(dot3(esd.Ng, esd.I)) > 0.0f) ? 1.0f : 0.0f;
  return mul3(mk3(res, res, res), esd.closure_emission_background);
}
#endif

#if CY_CLOSURE_EXT
/* light_sample (kernel_light.h:628-661) with a chosen lamp: lamp < 0 picks a
 * light from the distribution as light_sample does. */
CY_FN bool light_sample_lamp(const CyGlobals *kg, int lamp, float randu, float randv, cfloat3 P, int bounce,
                             CyLightSample *ls, uint *err)
{
  if (lamp < 0) {
    return light_sample(kg, randu, randv, P, bounce, ls, err);
  }
  if ((float)bounce > kg->__lights[lamp].max_bounces) {
    return false;
  }
  return lamp_light_sample(kg, lamp, randu, randv, P, ls, err);
}
#endif

/* Direct light at a shading point, one light sample (kernel_path_surface.h:23-140
 * kernel_branched_path_surface_connect_light with one sample, or
 * kernel_path_volume_connect_light, kernel_path_volume.h:21-61, when PHASE: a
 * volume scatter point lit through its phase closures): light_sample +
 * direct_emission (kernel_emission.h:101-205).  An occluded-or-not light
 * sample is left in the slot's shadow records and *shadow set; *shadow_D is
 * the shadow ray's direction then. */
template<bool PHASE, bool INLINE = false>
CY_FN void connect_light(const CyGlobals *kg, const CyPathBuffers *b, int slot, const CySD *sd,
                         const CyPathState *state, cfloat3 throughput, cfloat3 *L, bool *shadow, cfloat3 *shadow_D,
                         CyShadeMem mem, uint *err, const void *inline_vstack = nullptr)
{
  float light_u, light_v;
  path_state_rng_2D(kg, state, PRNG_LIGHT_U, &light_u, &light_v);
  float terminate = (KD->integrator.light_inv_rr_threshold > 0.0f) ?
                        path_state_rng_1D(kg, state, PRNG_LIGHT_TERMINATE) :
                        0.0f;
  CyLightSample ls;
  CY_DBG3(state, "light uv", mk3(light_u, light_v, terminate));
  if (light_sample(kg, light_u, light_v, sd->P, state->bounce, &ls, err) && ls.pdf != 0.0f) {
    CY_DBG3(state, "ls.P", ls.P);
    CY_DBG3(state, "ls.D", ls.D);
    CY_DBG3(state, "ls.Ng", ls.Ng);
    CY_DBG3(state, "ls.t pdf fac", mk3(ls.t, ls.pdf, ls.eval_fac));
    cfloat3 light_eval = mk3(0.0f, 0.0f, 0.0f);
    cfloat3 I = neg3(ls.D);
    if (shader_constant_emission_eval(kg, ls.shader, &light_eval)) {
      if ((ls.prim != PRIM_NONE) && dot3(ls.Ng, I) < 0.0f) {
        ls.Ng = neg3(ls.Ng);
      }
    }
#if CY_SVM_TEX
    else if (ls.type == LIGHT_BACKGROUND) {
      /* direct_emissive_eval (kernel_emission.h:37-86): the world
       * shader toward the sampled direction */
      light_eval = background_eval_svm(kg->data, kg->__svm_nodes, kg->__shaders, kg->__objects, kg->__texture_info, ls.D, mem,
                                       *state, PATH_RAY_EMISSION, err);
    }
    else {
      /* a mesh light or lamp whose emission depends on its shader's nodes */
      light_eval = emissive_eval_svm(kg, ls.P, ls.Ng, I, ls.shader, ls.object, ls.prim, ls.lamp, ls.u, ls.v, ls.t, mem,
                                     *state, err);
      if ((ls.prim != PRIM_NONE) && dot3(ls.Ng, I) < 0.0f) {
        ls.Ng = neg3(ls.Ng);
      }
    }
#else
    else {
      cy_set_error(err, CY_ERR_FEATURE, 7); /* non-constant emitter: a _tex variant scans it */
    }
#endif
    light_eval = mul3f(light_eval, ls.eval_fac);
    if (ls.lamp != LAMP_NONE) {
      light_eval = mul3(light_eval, klight_vec(kg->__lights[ls.lamp].strength));
    }
    if (!is_zero3(light_eval)) {
      cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
      float bpdf;
#if CY_CLOSURE_EXT
      if (PHASE) {
        /* direct_emission at a volume point (kernel_emission.h:127-138): the
         * phase functions, the MIS weight on the light's eval */
        eval = shader_volume_phase_eval(sd, ls.D, &bpdf);
        if ((uint)ls.shader & SHADER_USE_MIS) {
          light_eval = mul3f(light_eval, power_heuristic(ls.pdf, bpdf));
        }
      }
      else
#endif
#if CY_CLOSURE_EXT && CY_SVM_TEX
      if (KD->integrator.branched) {
        /* shader_bsdf_eval of branched path tracing (kernel_shader.h:626-628) */
        cfloat3 no_mis;
        shader_bsdf_eval_branched(sd, ls.D, ls.pdf, ((uint)ls.shader & SHADER_USE_MIS) != 0, &eval, &no_mis);
      }
      else
#endif
      {
        /* shader_bsdf_eval (kernel_shader.h:606-636) */
        shader_bsdf_multi_eval(sd, ls.D, &bpdf, -1, &eval, 0.0f, 0.0f);
        if ((uint)ls.shader & SHADER_USE_MIS) {
          float weight = power_heuristic(ls.pdf, bpdf);
          eval = mul3f(eval, weight);
        }
      }
      CY_DBG3(state, "light_eval", light_eval);
      CY_DBG3(state, "bsdf eval(light)", eval);
      CY_DBG1(state, "bsdf pdf(light)", bpdf);
      eval = mul3(eval, div3f(light_eval, ls.pdf));
      if (((uint)ls.shader & SHADER_EXCLUDE_ANY) &&
          ((uint)ls.shader & SHADER_EXCLUDE_DIFFUSE)) {
        eval = mk3(0.0f, 0.0f, 0.0f);
      }
      bool has_emission = !is_zero3(eval);
      if (has_emission && KD->integrator.light_inv_rr_threshold > 0.0f) {
        float lprob = max3f(fabs3(eval)) * KD->integrator.light_inv_rr_threshold;
        if (lprob < 1.0f) {
          if (terminate >= lprob) {
            has_emission = false;
          }
          else {
            eval = mul3f(eval, 1.0f / lprob);
          }
        }
      }
      if (has_emission) {
        /* path_radiance_accum_light, contribution precomputed */
        cfloat3 shaded_throughput = mul3(mul3f(throughput, 1.0f), mk3(1.0f, 1.0f, 1.0f));
        cfloat3 contribution = mul3(shaded_throughput, eval);
        contribution = path_radiance_clamp(kg, contribution, state->bounce);
        if ((uint)ls.shader & SHADER_CAST_SHADOW) {
          bool transmit = (dot3(sd->Ng, ls.D) < 0.0f);
          cfloat3 sP = ray_offset(sd->P, transmit ? neg3(sd->Ng) : sd->Ng);
          cfloat3 sD;
          float st;
          if (ls.t == CY_FLT_MAX) {
            /* distant light */
            sD = ls.D;
            st = ls.t;
          }
          else {
            sD = normalize_len3(sub3(ray_offset(ls.P, ls.Ng), sP), &st);
          }
          *shadow_D = sD;
#if CY_CLOSURE_EXT
          if (INLINE) {
            /* a subsurface exit point: the light sample is occluded here and
             * now (one of up to BSSRDF_MAX_HITS per shade); *shadow reports
             * that the transparent-shadow evaluation reused sd's closure
             * memory */
            CyRay sray;
            sray.P = sP;
            sray.D = sD;
            sray.t = st;
            if (KD->integrator.transparent_shadows) {
              cfloat3 attenuation;
              bool blocked;
              if (inline_vstack) {
                /* volume scenes: the path's stack as the shadow ray sees it
                 * (shadow_blocked_volume_path_state, kernel_shadow.h:23-45) */
                CyVolumeStack sstack = *(const CyVolumeStack *)inline_vstack;
                if (dot3(sd->Ng, sD) < 0.0f) {
                  volume_stack_enter_exit(sd->flag, sd->object, sd->shader, &sstack);
                }
                blocked = shadow_blocked_volume_inline(kg, &sray, state, mem, &attenuation, err, &sstack,
                                                       kg->use_ray_diff ? &sd->dP : nullptr);
              }
              else {
                blocked = shadow_blocked_transparent<false>(kg, sray, state, mem, &attenuation, err, nullptr,
                                                            kg->use_ray_diff ? &sd->dP : nullptr);
              }
              *shadow = true;
              if (!blocked) {
                const cfloat3 shaded = mul3(mul3f(throughput, 1.0f), attenuation);
                *L = add3(*L, path_radiance_clamp(kg, mul3(shaded, eval), state->bounce));
              }
            }
            else {
              bool blocked = false;
#ifdef CY_EXP_SSS_NO_SHADOW /* profiling experiment only: exit points never occluded */
              if (false) {
#else
              if (scene_intersect_valid(&sray)) {
#endif
                CyIsect si;
                blocked = kg->have_curves ?
                              bvh2_intersect<true, true, 2, CY_LDS_STACK, CY_BLOCK, 3>(
                                  kg, &sray, PATH_RAY_SHADOW_OPAQUE, &si, err, nullptr, nullptr, nullptr) :
                              bvh2_intersect<true>(kg, &sray, PATH_RAY_SHADOW_OPAQUE, &si, err, nullptr, nullptr,
                                                   nullptr);
              }
              if (!blocked) {
                *L = add3(*L, contribution);
              }
            }
            return;
          }
#endif
          cy_st(&b->shadow_P[slot], mkf4(sP.x, sP.y, sP.z, st));
          if (KD->integrator.transparent_shadows) {
            /* the shadow's attenuation multiplies the throughput before
             * the eval (path_radiance_accum_light): keep both, and the
             * bounces the occluders' shaders see (kernel_shadow.h:60-75) */
            cy_st(&b->shadow_D[slot], mkf4(sD.x, sD.y, sD.z, int_as_float(state->transmission_bounce)));
            cy_st(&b->shadow_L[slot], mkf4(eval.x, eval.y, eval.z, 0.0f));
            const uint packed = (uint)state->bounce | ((uint)state->transparent_bounce << 8) |
                                ((uint)state->diffuse_bounce << 16) | ((uint)state->glossy_bounce << 24);
            cy_st(&b->shadow_T[slot], mkf4(throughput.x, throughput.y, throughput.z, as_float(packed)));
#if CY_CLOSURE_EXT
            if (kg->use_ray_diff) {
              cy_st(&b->shadow_dP[2 * (size_t)slot], mkf4(sd->dP.dx.x, sd->dP.dx.y, sd->dP.dx.z, sd->dP.dy.x));
              cy_st(&b->shadow_dP[2 * (size_t)slot + 1], mkf4(sd->dP.dy.y, sd->dP.dy.z, 0.0f, 0.0f));
            }
#endif
          }
          else {
            cy_st(&b->shadow_D[slot], mkf4(sD.x, sD.y, sD.z, 0.0f));
            cy_st(&b->shadow_L[slot], mkf4(contribution.x, contribution.y, contribution.z, 0.0f));
          }
          *shadow = (st != 0.0f);
          if (!*shadow) {
            *L = add3(*L, contribution);
          }
        }
        else {
          *L = add3(*L, contribution);
        }
      }
    }
  }
}

#include "cy_branched.h"

#if CY_CLOSURE_EXT && CY_SVM_TEX

/* direct_emission (kernel_emission.h:101-205) at a volume scatter point (sd->prim
 * == PRIM_NONE: the phase functions, MIS on the light's eval): *eval is the
 * light's contribution per unit throughput; *light_ray the shadow ray (t = 0:
 * the light casts no shadow).  False: no contribution. */
CY_FN bool volume_direct_emission(const CyGlobals *kg, const CySD *sd, CyLightSample *ls, const CyPathState *state,
                                  float rand_terminate, cfloat3 *eval, CyRay *light_ray, CyShadeMem mem, uint *err)
{
  if (ls->pdf == 0.0f) {
    return false;
  }
  cfloat3 light_eval = mk3(0.0f, 0.0f, 0.0f);
  const cfloat3 I = neg3(ls->D);
  /* direct_emissive_eval (kernel_emission.h:20-99) */
  if (shader_constant_emission_eval(kg, ls->shader, &light_eval)) {
    if ((ls->prim != PRIM_NONE) && dot3(ls->Ng, I) < 0.0f) {
      ls->Ng = neg3(ls->Ng);
    }
  }
  else if (ls->type == LIGHT_BACKGROUND) {
    light_eval = background_eval_svm(kg->data, kg->__svm_nodes, kg->__shaders, kg->__objects, kg->__texture_info,
                                     ls->D, mem, *state, PATH_RAY_EMISSION, err);
  }
  else {
    light_eval = emissive_eval_svm(kg, ls->P, ls->Ng, I, ls->shader, ls->object, ls->prim, ls->lamp, ls->u, ls->v,
                                   ls->t, mem, *state, err);
    if ((ls->prim != PRIM_NONE) && dot3(ls->Ng, I) < 0.0f) {
      ls->Ng = neg3(ls->Ng);
    }
  }
  light_eval = mul3f(light_eval, ls->eval_fac);
  if (ls->lamp != LAMP_NONE) {
    light_eval = mul3(light_eval, klight_vec(kg->__lights[ls->lamp].strength));
  }
  if (is_zero3(light_eval)) {
    return false;
  }
  float bpdf;
  cfloat3 e = shader_volume_phase_eval(sd, ls->D, &bpdf);
  if ((uint)ls->shader & SHADER_USE_MIS) {
    light_eval = mul3f(light_eval, power_heuristic(ls->pdf, bpdf));
  }
  e = mul3(e, div3f(light_eval, ls->pdf));
  if (((uint)ls->shader & SHADER_EXCLUDE_ANY) && ((uint)ls->shader & SHADER_EXCLUDE_DIFFUSE)) {
    e = mk3(0.0f, 0.0f, 0.0f);
  }
  if (is_zero3(e)) {
    return false;
  }
  if (KD->integrator.light_inv_rr_threshold > 0.0f) {
    const float probability = max3f(fabs3(e)) * KD->integrator.light_inv_rr_threshold;
    if (probability < 1.0f) {
      if (rand_terminate >= probability) {
        return false;
      }
      e = mul3f(e, 1.0f / probability);
    }
  }
  if ((uint)ls->shader & SHADER_CAST_SHADOW) {
    const bool transmit = (dot3(sd->Ng, ls->D) < 0.0f);
    light_ray->P = ray_offset(sd->P, transmit ? neg3(sd->Ng) : sd->Ng);
    if (ls->t == CY_FLT_MAX) {
      light_ray->D = ls->D;
      light_ray->t = ls->t;
    }
    else {
      light_ray->D = normalize_len3(sub3(ray_offset(ls->P, ls->Ng), light_ray->P), &light_ray->t);
    }
  }
  else {
    light_ray->t = 0.0f;
  }
  *eval = e;
  return true;
}

/* kernel_branched_path_volume_connect_light (kernel_path_volume.h:131-257):
 * direct light at points of the recorded segment, one light sample per lamp
 * (or all lamps' samples and the mesh lights' with sample_all_lights), each
 * at its own scatter distance (decoupled scatter toward the light sample,
 * equiangular / MIS by the volumes' sampling method), occluded inline
 * through transparent surfaces and volumes (the shadow ray's own copy of the
 * volume stack, shadow_blocked_volume_path_state), added to *L in the
 * reference's order.  The closure memory is shared with the shadow's surface
 * evaluations: decoupled_scatter evaluates the segment's closures again
 * before each light's phase evaluation. */
CY_FN void volume_connect_all_lights(const CyGlobals *kg, CySD *sd, cfloat3 throughput, const CyPathState *state,
                                     cfloat3 *L, bool sample_all_lights, const CyRay *ray,
                                     const CyVolumeSegment *segment, const CyVolumeStack *stack, CyShadeMem mem,
                                     uint *err)
{
  /* One LightSample for the whole loop: a light_sample that fails early (a
   * triangle light facing away: pdf 0 before P and t are set) leaves the
   * previous sample's P and t in place, and the equiangular sampling below
   * then aims at that point.  In the reference the sample is a loop-local
   * left uninitialised, which the CPU build keeps in one stack slot across
   * the iterations: the same stale values (found on volume_mis_decoupled,
   * one path whose mesh-light sample failed after a lamp sample). */
  CyLightSample ls;
  ls.P = mk3(0.0f, 0.0f, 0.0f);
  ls.t = CY_FLT_MAX;
  int num_lights = 1;
  if (sample_all_lights) {
    num_lights = KD->integrator.num_all_lights;
    if (KD->integrator.pdf_triangles != 0.0f) {
      num_lights += 1;
    }
  }
  for (int i = 0; i < num_lights; ++i) {
    int num_samples = 1;
    int num_all_lights = 1;
    uint lamp_rng_hash = state->rng_hash;
    bool double_pdf = false;
    bool is_mesh_light = false;
    bool is_lamp = false;
    if (sample_all_lights) {
      is_lamp = i < KD->integrator.num_all_lights;
      if (is_lamp) {
        if ((float)state->bounce > kg->__lights[i].max_bounces) {
          continue;
        }
        num_samples = kg->__lights[i].samples;
        num_all_lights = KD->integrator.num_all_lights;
        lamp_rng_hash = cmj_hash(state->rng_hash, (uint)i);
        double_pdf = KD->integrator.pdf_triangles != 0.0f;
      }
      else {
        num_samples = KD->integrator.mesh_light_samples;
        double_pdf = KD->integrator.num_all_lights != 0;
        is_mesh_light = true;
      }
    }
    const float num_samples_inv = 1.0f / (float)(num_samples * num_all_lights);
    for (int j = 0; j < num_samples; j++) {
      CyRay light_ray;
      light_ray.t = 0.0f;
      bool has_emission = false;
      cfloat3 tp = throughput;
      cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
      if (KD->integrator.use_direct_light) {
        float light_u, light_v;
        path_branched_rng_2D(kg, lamp_rng_hash, state, j, num_samples, PRNG_LIGHT_U, &light_u, &light_v);
        if (is_mesh_light && double_pdf) {
          light_u = 0.5f * light_u;
        }
        const int lamp = is_lamp ? i : -1;
        const bool ls_ok = light_sample_lamp(kg, lamp, light_u, light_v, ray->P, state->bounce, &ls, err);
        CY_DBGF(state, "ls_ok %d pdf %08x lamp %d\n", (int)ls_ok, __builtin_bit_cast(unsigned, ls.pdf), ls.lamp);
        const float rphase = path_rng_1D(kg, state->rng_hash, state->sample * num_samples + j,
                                         state->rng_offset + PRNG_PHASE_CHANNEL);
        const float rscatter = path_rng_1D(kg, state->rng_hash, state->sample * num_samples + j,
                                           state->rng_offset + PRNG_SCATTER_DISTANCE);
        const cfloat3 light_P = ls.P;
        CY_DBGF(state, "light %d sample %d\n", i, j);
        CY_DBG3(state, "light uv rphase", mk3(light_u, light_v, rphase));
        CY_DBG3(state, "ls.P", ls.P);
        CY_DBG1(state, "ls.t", ls.t);
        const int result = volume_decoupled_scatter(kg, state, ray, sd, stack, &tp, rphase, rscatter, segment,
                                                    (ls.t != CY_FLT_MAX) ? &light_P : nullptr, false, err);
        if (result == VOLUME_PATH_SCATTERED) {
          if (light_sample_lamp(kg, lamp, light_u, light_v, sd->P, state->bounce, &ls, err)) {
            if (double_pdf) {
              ls.pdf *= 2.0f;
            }
            const float terminate = (KD->integrator.light_inv_rr_threshold > 0.0f) ?
                                        path_rng_1D(kg, state->rng_hash, state->sample * num_samples + j,
                                                    state->rng_offset + PRNG_LIGHT_TERMINATE) :
                                        0.0f;
            has_emission = volume_direct_emission(kg, sd, &ls, state, terminate, &eval, &light_ray, mem, err);
          }
        }
      }
      /* shadow_blocked: the path's volume stack as the shadow ray sees it
       * (shadow_blocked_volume_path_state, kernel_shadow.h:23-45) */
      bool blocked = false;
      cfloat3 shadow = mk3(1.0f, 1.0f, 1.0f);
      if (light_ray.t != 0.0f) {
        CyVolumeStack sstack = *stack;
        if (dot3(sd->Ng, light_ray.D) < 0.0f) {
          volume_stack_enter_exit(sd->flag, sd->object, sd->shader, &sstack);
        }
        blocked = shadow_blocked_volume_inline(kg, &light_ray, state, mem, &shadow, err, &sstack,
                                               kg->use_ray_diff ? &sd->dP : nullptr);
      }
      CY_DBGF(state, "has_emission %d blocked %d\n", (int)has_emission, (int)blocked);
      CY_DBG3(state, "eval", eval);
      CY_DBG3(state, "shadow", shadow);
      CY_DBG3(state, "tp", tp);
      if (has_emission && !blocked) {
        /* path_radiance_accum_light (kernel_accumulate.h:402-459) */
        const cfloat3 shaded_throughput = mul3(mul3f(tp, num_samples_inv), shadow);
        *L = add3(*L, path_radiance_clamp(kg, mul3(shaded_throughput, eval), state->bounce));
      }
    }
  }
}

/* kernel_path_volume (kernel_path.h:186-215), decoupled branch: the segment
 * recorded once, its emission, direct light over all lights, then the
 * indirect scatter decision.  Returns VOLUME_PATH_SCATTERED (vsd at the
 * scatter point, throughput weighted) or VOLUME_PATH_ATTENUATED (throughput
 * times the segment's transmittance). */
CY_NOINLINE int volume_decoupled_path(const CyGlobals *kg, CySD *vsd, CyPathState *state,
                                      const CyVolumeStack *stack, const CyRay *volume_ray, cfloat3 *L,
                                      cfloat3 *throughput, float step_size, int sampling_method, CyShadeMem mem,
                                      CyVolumeStep *steps, uint *err)
{
  CyVolumeSegment segment;
  shader_setup_from_volume(vsd, volume_ray, mem);
  volume_decoupled_record(kg, state, volume_ray, vsd, stack, &segment, step_size, steps, err);
  segment.sampling_method = sampling_method;
  if (segment.closure_flag & SD_EMISSION) {
    volume_accum_emission(kg, state, L, *throughput, segment.accum_emission);
  }
  int result = VOLUME_PATH_ATTENUATED;
  if (segment.closure_flag & SD_SCATTER) {
    const bool all = KD->integrator.sample_all_lights_indirect != 0;
    volume_connect_all_lights(kg, vsd, *throughput, state, L, all, volume_ray, &segment, stack, mem, err);
    const float rphase = path_state_rng_1D(kg, state, PRNG_PHASE_CHANNEL);
    const float rscatter = path_state_rng_1D(kg, state, PRNG_SCATTER_DISTANCE);
    result = volume_decoupled_scatter(kg, state, volume_ray, vsd, stack, throughput, rphase, rscatter, &segment,
                                      nullptr, true, err);
  }
  if (result != VOLUME_PATH_SCATTERED) {
    *throughput = mul3(*throughput, segment.accum_transmittance);
    return VOLUME_PATH_ATTENUATED;
  }
  return VOLUME_PATH_SCATTERED;
}
#endif

#if CY_CLOSURE_EXT
/* connect_light<false, true> for a subsurface exit point in a volume scene
 * (the light sample traced through the fog with the path's stack): one
 * out-of-line copy for the disk and random-walk exit points of the volume
 * kernels. */
CY_NOINLINE void connect_light_exit_vol(const CyGlobals *kg, const CyPathBuffers *b, int slot, const CySD *sd,
                                        const CyPathState *state, cfloat3 throughput, cfloat3 *L, bool *reused,
                                        CyShadeMem mem, uint *err, const CyVolumeStack *vstack)
{
  cfloat3 shadow_D;
  connect_light<false, true>(kg, b, slot, sd, state, throughput, L, reused, &shadow_D, mem, err, vstack);
}

/* kernel_path_surface_bounce (kernel_path_surface.h:270-358) for the diffuse
 * closure at a subsurface exit point; with vstack (volume scenes) the ray's
 * stack enters / leaves the surface's volume on a transmission bounce
 * (kernel_path_surface.h:325-329). */
CY_FN bool subsurface_exit_bounce(const CyGlobals *kg, const CySD *sd, cfloat3 *throughput, CyPathState *state,
                                  CyRay *ray, uint *err, CyDiff3 *domega_in = nullptr, CyVolumeStack *vstack = nullptr)
{
  if (!(sd->flag & SD_BSDF)) {
    return false;
  }
  float bsdf_u, bsdf_v;
  path_state_rng_2D(kg, state, PRNG_BSDF_U, &bsdf_u, &bsdf_v);
  cfloat3 bsdf_eval_v = mk3(0.0f, 0.0f, 0.0f);
  cfloat3 omega_in = mk3(0.0f, 0.0f, 0.0f);
  float bsdf_pdf = 0.0f;
  const int label = shader_bsdf_sample(kg, sd, bsdf_u, bsdf_v, &bsdf_eval_v, &omega_in, &bsdf_pdf, err, domega_in);
  if (bsdf_pdf == 0.0f || is_zero3(bsdf_eval_v)) {
    return false;
  }
  const float inverse_pdf = 1.0f / bsdf_pdf;
  *throughput = mul3(*throughput, mul3f(bsdf_eval_v, inverse_pdf));
  if (!(label & LABEL_TRANSPARENT)) {
    state->ray_pdf = bsdf_pdf;
    state->ray_t = 0.0f;
    state->min_ray_pdf = fminf(bsdf_pdf, state->min_ray_pdf);
  }
  path_state_next(kg, state, label);
  ray->P = ray_offset(sd->P, (label & LABEL_TRANSMIT) ? neg3(sd->Ng) : sd->Ng);
  ray->D = normalize3(omega_in);
  if (state->bounce == 0) {
    ray->t -= sd->ray_length;
  }
  else {
    ray->t = CY_FLT_MAX;
  }
  if (vstack && (label & LABEL_TRANSMIT)) {
    volume_stack_enter_exit(sd->flag, sd->object, sd->shader, vstack);
  }
  return true;
}

/* kernel_path_subsurface_scatter (kernel_path_subsurface.h:26-110) for a disk
 * BSSRDF: up to BSSRDF_MAX_HITS exit points, each lit with the path's state and
 * throughput (its shadow ray traced here), each bouncing into an indirect ray
 * with rng_offset + PRNG_BOUNCE_NUM.  The reference ends the path there and
 * then traces the indirect rays last to first, ray k with rng_offset +
 * k * PRNG_BOUNCE_NUM (kernel_path_subsurface_setup_indirect): the last one
 * replaces the path's state, ray and throughput here, the others wait in the
 * slot's SSS records until the path before them ends (shade_path).  Returns
 * the number of indirect rays. */
template<bool VOL = false>
CY_FN int subsurface_disk_paths(const CyGlobals *kg, const CyPathBuffers *b, int slot, uint cam_item, CySD *sd,
                                const CyClosure *sc, float bssrdf_u, float bssrdf_v, CyPathState *state,
                                CyRay *ray, cfloat3 *throughput, cfloat3 *L, CyShadeMem mem, uint *err,
                                CyVolumeStack *vstack = nullptr, CySD *stack_sd = nullptr)
{
  if (!b->sss_rec || (cam_item == CY_NO_ITEM && cy_ld(&b->sss_count[slot]) != 0u)) {
    cy_set_error(err, CY_ERR_FEATURE, 12); /* no indirect-ray records, or a second scatter on one path */
    return 0;
  }
  const int bssrdf_type = sc->type;
  const float bssrdf_rough = bssrdf_roughness(sc);
  uint lcg_state = lcg_init(state->rng_hash + (uint)state->rng_offset + (uint)state->sample * 0x68bc21ebu);
  CyLocalHits li;
  CyRay ss_ray;
#ifdef CY_EXP_SSS_OFF /* profiling experiment only: no exit points */
  const int num_hits = 0;
  (void)lcg_state;
#else
  const int num_hits = subsurface_scatter_disk(kg, &li, sd, sc, &lcg_state, bssrdf_u, bssrdf_v, &ss_ray, err);
#endif
  int pushed = 0;
  CyPathState top_state;
  CyRay top_ray;
  cfloat3 top_tp = mk3(0.0f, 0.0f, 0.0f);
  /* with ray differentials each indirect ray carries the entry point's dP
   * (shader_setup_from_subsurface keeps sd->dP, dI) and its sampled dD */
  const bool diff = kg->use_ray_diff != 0;
  CyDiff3 top_dD, hit_dD;
  /* volume scenes: each indirect ray's own stack, from the path's, crossed by
   * the ray from the path's previous point to the exit point when the object
   * intersects a volume (kernel_path_subsurface.h:56-57, 92-99) */
  const bool update_stack = vstack && (sd->object_flag & SD_OBJECT_INTERSECTS_VOLUME);
  CyVolumeStack top_stack, hit_stack;
  for (int hit = 0; hit < num_hits; hit++) {
    /* subsurface_scatter_multi_setup (kernel_subsurface.h:284-313) */
    shader_setup_from_subsurface(kg, sd, &li.hits[hit], &ss_ray);
    cfloat3 weight = li.weight[hit];
    cfloat3 N = sd->N;
    subsurface_color_bump_blur(kg, sd, state, &weight, &N, err);
    subsurface_scatter_setup_diffuse_bsdf(kg, sd, bssrdf_type, bssrdf_rough, weight, N);
    if (KD->integrator.use_direct_light && (sd->flag & SD_BSDF_HAS_EVAL)) {
      bool reused = false;
      cfloat3 shadow_D;
      if (VOL) {
        connect_light_exit_vol(kg, b, slot, sd, state, *throughput, L, &reused, mem, err, vstack);
      }
      else {
        connect_light<false, true>(kg, b, slot, sd, state, *throughput, L, &reused, &shadow_D, mem, err);
      }
      if (reused) {
        shader_setup_from_subsurface(kg, sd, &li.hits[hit], &ss_ray);
        subsurface_scatter_setup_diffuse_bsdf(kg, sd, bssrdf_type, bssrdf_rough, weight, N);
      }
    }
    CyPathState hit_state = *state;
    CyRay hit_ray = *ray;
    cfloat3 hit_tp = *throughput;
    hit_state.rng_offset += PRNG_BOUNCE_NUM;
    if (vstack) {
      hit_stack = *vstack;
    }
    if (subsurface_exit_bounce(kg, sd, &hit_tp, &hit_state, &hit_ray, err, diff ? &hit_dD : nullptr,
                               vstack ? &hit_stack : nullptr)) {
      hit_state.ray_t = 0.0f;
      if (update_stack) {
        CyRay volume_ray = *ray;
        volume_ray.D = normalize_len3(sub3(hit_ray.P, volume_ray.P), &volume_ray.t);
        volume_stack_update_for_subsurface(kg, stack_sd, &volume_ray, &hit_stack, err);
      }
      if (pushed > 0) {
        top_state.rng_offset += (pushed - 1) * PRNG_BOUNCE_NUM;
        sss_rec_store(b, slot, pushed - 1, &top_state, &top_ray, top_tp, diff ? &sd->dP : nullptr, &top_dD);
        if (vstack) {
          vol_stack_write(sss_vol_at(b, slot, pushed - 1), &top_stack);
        }
      }
      top_state = hit_state;
      top_ray = hit_ray;
      top_tp = hit_tp;
      top_dD = hit_dD;
      if (vstack) {
        top_stack = hit_stack;
      }
      pushed++;
    }
  }
  if (pushed > 0) {
    top_state.rng_offset += (pushed - 1) * PRNG_BOUNCE_NUM;
    *state = top_state;
    *ray = top_ray;
    *throughput = top_tp;
    if (vstack) {
      *vstack = top_stack;
    }
    if (diff) {
      diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, sd->dP, top_dD);
    }
    if (pushed > 1) {
      cy_st(&b->sss_count[slot], (uint)(pushed - 1));
    }
  }
  return pushed;
}
#endif

/* ---------------------------------------------------------------------------
 * Stage 2: shade one path at one bounce.  Returns true when the slot must be
 * enqueued for the next closest-hit traversal.  *shadow is set when a shadow ray
 * was emitted (the slot then goes to the shadow queue; if the path ends at this
 * bounce the shadow stage finishes it).  *finished is set when the path ended
 * here and its sample was recorded.
 */
#if CY_CLOSURE_EXT
/* kernel_path_volume_bounce: a new direction from the phase closures */
CY_FN bool volume_bounce(const CyGlobals *kg, const CySD *sd, cfloat3 *throughput, CyPathState *state, CyRay *ray)
{
  float phase_u, phase_v;
  path_state_rng_2D(kg, state, PRNG_BSDF_U, &phase_u, &phase_v);
  cfloat3 phase_eval = mk3(0.0f, 0.0f, 0.0f);
  cfloat3 omega_in = mk3(0.0f, 0.0f, 0.0f);
  float phase_pdf = 0.0f;
  const int label = shader_volume_phase_sample(sd, phase_u, phase_v, &phase_eval, &omega_in, &phase_pdf);
  if (phase_pdf == 0.0f || is_zero3(phase_eval)) {
    return false;
  }
  /* path_radiance_bsdf_bounce */
  const float inverse_pdf = 1.0f / phase_pdf;
  *throughput = mul3(*throughput, mul3f(phase_eval, inverse_pdf));
  state->ray_pdf = phase_pdf;
  state->ray_t = 0.0f;
  state->min_ray_pdf = fminf(phase_pdf, state->min_ray_pdf);
  path_state_next<true>(kg, state, label);
  const float probability = path_state_continuation_probability(kg, state, *throughput);
  if (probability == 0.0f) {
    return false;
  }
  else if (probability != 1.0f) {
    const float terminate = path_state_rng_1D(kg, state, PRNG_TERMINATE - PRNG_BOUNCE_NUM);
    if (terminate >= probability) {
      return false;
    }
    *throughput = div3f(*throughput, probability);
  }
  ray->P = sd->P;
  ray->D = omega_in;
  ray->t = CY_FLT_MAX;
  return true;
}
#endif

#if CY_CLOSURE_EXT
/* PassType bits of KernelFilm.pass_flag (kernel_types.h:353-364) */
#define CY_PASS_DEPTH (1 << 2)
#define CY_PASS_NORMAL (1 << 3)
#define CY_PASS_UV (1 << 4)
#define CY_PASS_OBJECT_ID (1 << 5)
#define CY_PASS_MATERIAL_ID (1 << 6)
#define CY_DATA_PASSES (CY_PASS_DEPTH | CY_PASS_NORMAL | CY_PASS_UV | CY_PASS_OBJECT_ID | CY_PASS_MATERIAL_ID)
#define ATTR_STD_UV_ID 3u /* AttributeStandard ATTR_STD_UV */

/* kernel_write_data_passes (kernel_passes.h:173-225), the writes at the
 * camera path's first opaque-enough hit: depth, object and material index on
 * the pixel's sample 0, the average BSDF normal and the UV map every sample
 * (kernel_write_pass_float: added; atomically on the device, as the
 * reference's GPU devices do). */
CY_FN void write_data_passes(const CyGlobals *kg, float *buffer, const CySD *sd, const CyPathState *state)
{
  const int flag = KD->film.pass_flag;
  if (state->sample == 0) {
    if (flag & CY_PASS_DEPTH) {
      /* camera_z_depth (kernel_camera.h:449-460) */
      float depth;
      if (KD->cam.type != 2 /* CAMERA_PANORAMA */) {
        depth = transform_point((const struct cy_tfm *)&KD->cam.worldtocamera, sd->P).z;
      }
      else {
        const hc_Transform &c = KD->cam.cameratoworld;
        depth = len3(sub3(sd->P, mk3(c.x.w, c.y.w, c.z.w)));
      }
      cy_pass_add(buffer + KD->film.pass_depth, depth);
    }
    if (flag & CY_PASS_OBJECT_ID) {
      /* object_pass_id (geom_object.h:237-243) */
      cy_pass_add(buffer + KD->film.pass_object_id,
                  (sd->object == OBJECT_NONE) ? 0.0f : kg->__objects[sd->object].pass_id);
    }
    if (flag & CY_PASS_MATERIAL_ID) {
      /* shader_pass_id (geom_object.h:345-348) */
      cy_pass_add(buffer + KD->film.pass_material_id,
                  (float)kg->__shaders[(uint)sd->shader & SHADER_MASK].pass_id);
    }
  }
  if (flag & CY_PASS_NORMAL) {
    /* shader_bsdf_average_normal (kernel_shader.h:913-924) */
    cfloat3 N = mk3(0.0f, 0.0f, 0.0f);
    for (int i = 0; i < sd->num_closure; i++) {
      const CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_BSDF_OR_BSSRDF(sc->type)) {
        N = add3(N, mul3f(sc->N, fabsf(average3(sc->weight))));
      }
    }
    N = is_zero3(N) ? sd->N : normalize3(N);
    float *p = buffer + KD->film.pass_normal;
    cy_pass_add(p + 0, N.x);
    cy_pass_add(p + 1, N.y);
    cy_pass_add(p + 2, N.z);
  }
  if (flag & CY_PASS_UV) {
    /* primitive_uv (geom_primitive.h:259-268) */
    cfloat3 uv = mk3(0.0f, 0.0f, 0.0f);
    const CyAttr desc = find_attribute(kg, sd->object, sd->prim, ATTR_STD_UV_ID);
    if (desc.offset != (int)ATTR_STD_NOT_FOUND) {
      float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (sd->type & PRIMITIVE_ALL_TRIANGLE) {
        triangle_attribute(kg, desc, sd->prim, sd->u, sd->v, 2, f);
      }
      else if (sd->type & PRIMITIVE_ALL_CURVE) {
        curve_attribute(kg, desc, sd->prim, sd->type, sd->u, 2, f);
      }
      uv = mk3(f[0], f[1], 1.0f);
    }
    float *p = buffer + KD->film.pass_uv;
    cy_pass_add(p + 0, uv.x);
    cy_pass_add(p + 1, uv.y);
    cy_pass_add(p + 2, uv.z);
  }
}
#endif

#if CY_CLOSURE_EXT && CY_SVM_TEX
/* kernel_branched_path_integrate's work at a camera hit (kernel_path_branched.h:
 * 470-500) after the shader is applied: the direct light of all lights (or one),
 * then per BSDF closure its diffuse / glossy / transmission samples' indirect
 * paths (kernel_branched_path_surface_indirect_light, :201-280), and the camera
 * ray carried on through the surface's transparency.  The first of these paths
 * replaces the slot's (true returned, *state .. *branch_factor set), the others
 * wait in the slot's branch records in the reference's order. */
CY_FN bool branched_camera_hit(const CyGlobals *kg, const CyPathBuffers *b, int slot, const CySD *sd,
                               CyPathState *state, cfloat3 *throughput, CyRay *ray, cfloat3 *L, float *branch_factor,
                               CyCatcher *catcher, CyShadeMem mem, uint *err)
{
  const bool all = KD->integrator.sample_all_lights_direct || (state->flag & PATH_RAY_SHADOW_CATCHER);
  connect_light_branched(kg, sd, state, *throughput, 1.0f, all, L, catcher, mem, err);
  const bool diff = kg->use_ray_diff != 0;
  bool have_first = false;
  CyPathState first_state;
  CyRay first_ray;
  cfloat3 first_tp = mk3(0.0f, 0.0f, 0.0f);
  float first_bf = 1.0f;
  CyDiff3 first_dP, first_dD, dD;
  int n = 0;
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    /* transparency is not handled here, but in the camera loop */
    if (!CLOSURE_IS_BSDF(sc->type) || sc->type == CLOSURE_BSDF_TRANSPARENT_ID) {
      continue;
    }
    int num_samples;
    if (CLOSURE_IS_BSDF_DIFFUSE(sc->type)) {
      num_samples = KD->integrator.diffuse_samples;
    }
    else if (sc->type == CLOSURE_BSDF_BSSRDF_ID || sc->type == CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID) {
      num_samples = 1;
    }
    else if ((sc->type >= CLOSURE_BSDF_REFLECTION_ID && sc->type <= CLOSURE_BSDF_HAIR_REFLECTION_ID) ||
             sc->type == CLOSURE_BSDF_HAIR_PRINCIPLED_ID) {
      num_samples = KD->integrator.glossy_samples;
    }
    else {
      num_samples = KD->integrator.transmission_samples;
    }
    const float num_samples_inv = 1.0f / (float)num_samples;
    for (int j = 0; j < num_samples; j++) {
      CyPathState ps = *state;
      cfloat3 tp = *throughput;
      CyRay bray;
      float bf = *branch_factor;
      ps.rng_hash = cmj_hash(state->rng_hash, (uint)i);
      if (!branched_surface_bounce(kg, sd, sc, j, num_samples, &tp, &ps, &bray, &bf, diff ? &dD : nullptr, err)) {
        continue;
      }
      ps.rng_hash = state->rng_hash;
      tp = mul3f(tp, num_samples_inv);
      if (!have_first) {
        have_first = true;
        first_state = ps;
        first_ray = bray;
        first_tp = tp;
        first_bf = bf;
        first_dP = sd->dP;
        first_dD = dD;
      }
      else if (n >= CY_BR_RECS) {
        cy_set_error(err, CY_ERR_FEATURE, 15); /* more branched samples than the slot's records */
      }
      else {
        hc_float4 *rec = br_rec_at(b, slot, n++);
        path_rec_store(rec, &ps, &bray, tp, diff ? &sd->dP : nullptr, &dD);
        cy_st(&rec[CY_BR_REC_F4 - 1], mkf4(bf, 0.0f, 0.0f, 0.0f));
      }
    }
  }
  /* continue in case of transparency (kernel_path_branched.h:487-516) */
  const cfloat3 tpc = mul3(*throughput, shader_bsdf_transparency(sd));
  if (!is_zero3(tpc)) {
    CyPathState cs = *state;
    path_state_next(kg, &cs, LABEL_TRANSPARENT);
    CyRay cr;
    cr.P = ray_offset(sd->P, neg3(sd->Ng));
    cr.D = ray->D;
    cr.t = ray->t - sd->ray_length;
    CyDiff3 cdD;
    cdD.dx = neg3(sd->dI.dx);
    cdD.dy = neg3(sd->dI.dy);
    if (!have_first) {
      have_first = true;
      first_state = cs;
      first_ray = cr;
      first_tp = tpc;
      first_bf = *branch_factor;
      first_dP = sd->dP;
      first_dD = cdD;
    }
    else if (n >= CY_BR_RECS) {
      cy_set_error(err, CY_ERR_FEATURE, 15);
    }
    else {
      hc_float4 *rec = br_rec_at(b, slot, n++);
      path_rec_store(rec, &cs, &cr, tpc, diff ? &sd->dP : nullptr, &cdD);
      cy_st(&rec[CY_BR_REC_F4 - 1], mkf4(*branch_factor, 0.0f, 0.0f, 0.0f));
    }
  }
  cy_st(&b->br_count[2 * (size_t)slot], 0u);
  cy_st(&b->br_count[2 * (size_t)slot + 1], (uint)n);
  if (!have_first) {
    return false;
  }
  *state = first_state;
  *ray = first_ray;
  *throughput = first_tp;
  *branch_factor = first_bf;
  if (diff) {
    diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, first_dP, first_dD);
  }
  return true;
}
#endif

/* indirect_background (kernel_emission.h:288-345): the world seen along the
 * ray (its light-path exclusions, the world shader evaluated with the bounce
 * raised, the background MIS weight). */
CY_FN cfloat3 indirect_background(const CyGlobals *kg, const CyPathBuffers *b, const CyTile *tile, int slot,
                                  uint cam_item, const CyPathState *state, const CyRay *ray, CyShadeMem mem,
                                  uint *err)
{
  uint shader = (uint)KD->background.surface_shader;
  bool excluded = false;
  if (shader & SHADER_EXCLUDE_ANY) {
    if (((shader & SHADER_EXCLUDE_DIFFUSE) && (state->flag & PATH_RAY_DIFFUSE)) ||
        ((shader & SHADER_EXCLUDE_GLOSSY) &&
         ((state->flag & (PATH_RAY_GLOSSY | PATH_RAY_REFLECT)) ==
          (PATH_RAY_GLOSSY | PATH_RAY_REFLECT))) ||
        ((shader & SHADER_EXCLUDE_TRANSMIT) && (state->flag & PATH_RAY_TRANSMIT)) ||
        ((shader & SHADER_EXCLUDE_CAMERA) && (state->flag & PATH_RAY_CAMERA)) ||
        ((shader & SHADER_EXCLUDE_SCATTER) && (state->flag & PATH_RAY_VOLUME_SCATTER))) {
      excluded = true;
    }
  }
  cfloat3 L_background = mk3(0.0f, 0.0f, 0.0f);
  if (!excluded) {
    if (!shader_constant_emission_eval(kg, (int)shader, &L_background)) {
      /* world shader evaluated along the ray, bounce raised for the
       * light-path node (path_state_modify_bounce) */
#if CY_SVM_TEX
#if CY_CLOSURE_EXT
      CyDiff3 rdP, rdD;
      if (kg->use_ray_diff) {
        ray_diff_load(kg, b, tile, slot, cam_item, &rdP, &rdD);
      }
      L_background = background_eval_svm(kg->data, kg->__svm_nodes, kg->__shaders, kg->__objects, kg->__texture_info, ray->D,
                                         mem, *state, state->flag | PATH_RAY_EMISSION, err,
                                         kg->use_ray_diff ? &rdD : nullptr);
#else
      L_background = background_eval_svm(kg->data, kg->__svm_nodes, kg->__shaders, kg->__objects, kg->__texture_info, ray->D,
                                         mem, *state, state->flag | PATH_RAY_EMISSION, err);
#endif
#else
      cy_set_error(err, CY_ERR_FEATURE, 3); /* node world in the kernel without texture nodes */
#endif
    }
    /* background MIS weight (kernel_emission.h:325-335) */
    if (!(state->flag & PATH_RAY_MIS_SKIP) && KD->background.use_mis) {
      const float pdf = background_light_pdf(kg, ray->D);
      const float mis_weight = power_heuristic(state->ray_pdf, pdf);
      L_background = mul3f(L_background, mis_weight);
    }
  }
  return L_background;
}

template<bool VOL = false>
CY_FN bool shade_path(const CyGlobals *kg,
                      const CyPathBuffers *b,
                      const CyTile *tile,
                      int slot,
                      uint cam_item,
                      CyShadeMem mem,
                      bool *shadow,
                      bool *finished,
                      uint *err)
{
  *shadow = false;
  *finished = false;
  hc_float4 is4 = cy_ld(&b->isect[slot]);
  CyPathState state;
  CyRay ray;
  cfloat3 throughput, L;
  float L_transparent;
  float branch_factor = 1.0f; /* PathState.branch_factor (path_state_branch) */
  uint rng_hash = 0, ray_visibility = 0;
  int sample = 0;
  if (cam_item != CY_NO_ITEM) {
    /* first bounce of a camera launch: the path starts here (the closest
     * stage traced the same camera ray) */
    if (as_int(is4.w) == CY_PRIM_NO_RAY) {
      write_no_sample(tile, cam_item);
      *finished = true;
      return false;
    }
    item_camera_ray(kg, tile, cam_item, &rng_hash, &sample, &ray);
  }
  else {
    const hc_float4 rp = cy_ld(&b->ray_P[slot]);
    const hc_float4 rd = cy_ld(&b->ray_D[slot]);
    ray.P = mk3(rp.x, rp.y, rp.z);
    ray.t = rp.w;
    ray.D = mk3(rd.x, rd.y, rd.z);
    ray_visibility = as_uint(rd.w);
  }

  int hit_object = OBJECT_NONE;
  if (as_int(is4.w) >= 0 && (as_int(is4.w) & CY_PRIM_TIE)) {
    /* near-tie of the wide traversal (hipcycles.hip k_intersect_closest):
     * re-trace with the bound BVH2 in the reference's visiting order, before
     * the path state is loaded (little is live here).  The re-trace starts
     * from the ray's own t, as the reference does: a t shortened to the tie
     * window would be rescaled by every instance push / pop on the way
     * (bvh_instance_push leaves FLT_MAX unscaled, any other t is multiplied
     * and divided again), so the t each candidate is tested against would
     * drift from the reference's by a rounding -- enough to flip exactly the
     * near-equal comparisons a tie is about (measured: 364 pixels of the BBS
     * stand-in's instanced frame). */
    if (cam_item != CY_NO_ITEM) {
      CyPathState cs;
      cs.flag = PATH_RAY_CAMERA | PATH_RAY_MIS_SKIP | PATH_RAY_TRANSPARENT_BACKGROUND; /* path_state_init */
      ray_visibility = path_state_ray_visibility(&cs);
    }
    CyRay rt = ray;
    CyIsect ti;
    if (bvh2_intersect<false>(kg, &rt, ray_visibility, &ti, err, nullptr, nullptr, nullptr)) {
      is4 = mkf4(ti.t, ti.u, ti.v, int_as_float(ti.prim));
      hit_object = ti.object;
    }
    else {
      is4.w = int_as_float(PRIM_NONE); /* unreachable: the wide traversal's hit lies inside the window */
    }
  }
  else if (kg->have_instancing && as_int(is4.w) >= 0) {
    hit_object = cy_ld(&b->isect_object[slot]);
  }

  if (cam_item != CY_NO_ITEM) {
    path_state_init(kg, &state, rng_hash, sample);
    throughput = mk3(1.0f, 1.0f, 1.0f);
    L_transparent = 0.0f;
    L = mk3(0.0f, 0.0f, 0.0f);
  }
  else {
    load_state(b, slot, &state, kg);
    const hc_float4 tp4 = cy_ld(&b->throughput[slot]);
    throughput = mk3(tp4.x, tp4.y, tp4.z);
    L_transparent = tp4.w;
    const hc_float4 L4 = cy_ld(&b->L[slot]);
    L = mk3(L4.x, L4.y, L4.z);
#if CY_CATCHER
    if (KD->integrator.branched) {
      branch_factor = L4.w; /* an indirect path of branched path tracing */
    }
#endif
  }
#if CY_CATCHER
  CyCatcher catcher;
  if (b->catcher) {
    if (cam_item != CY_NO_ITEM) {
      catcher_init(kg, &catcher);
    }
    else {
      catcher_load(kg, b, slot, &catcher);
    }
  }
  /* light passes: the path's PathRadiance components */
  CyLightPass lp;
  if (b->lp) {
    if (cam_item != CY_NO_ITEM) {
      lightpass_init(&lp);
    }
    else {
      lightpass_load(b, slot, &lp);
    }
  }
#endif
#ifdef CY_DBG_X
  {
    int dx, dy, ds;
    item_pixel(tile, cam_item != CY_NO_ITEM ? cam_item : cy_ld(&b->item[slot]), &dx, &dy, &ds);
    state.dbg = dx == CY_DBG_X && dy == CY_DBG_Y && ds == CY_DBG_S;
  }
  CY_DBGF(&state, "bounce %d flag %08x\n", state.bounce, state.flag);
  CY_DBG3(&state, "ray.P", ray.P);
  CY_DBG3(&state, "ray.D", ray.D);
  CY_DBG1(&state, "ray.t", ray.t);
  CY_DBG3(&state, "isect", mk3(is4.x, is4.y, is4.z));
  CY_DBGF(&state, "prim %d\n", as_int(is4.w));
  CY_DBG3(&state, "throughput", throughput);
  CY_DBG3(&state, "L", L);
#endif

#if CY_CLOSURE_EXT
  /* the path's volume stack, with the update its last surface left pending */
  CyVolumeStack vstack;
  uint vop_object = 0u, vop_shader = 0u, vop_flags = 0u; /* this bounce's pending update */
  int shadow_rng_offset = 0;
  if (VOL) {
    if (cam_item != CY_NO_ITEM) {
      if (CY_VOLUME_EXT && KD->cam.is_inside_volume) {
        CySD stack_sd;
        volume_stack_init_camera(kg, &stack_sd, &ray, (uint)state.flag, &vstack, err);
      }
      else {
        volume_stack_init(kg, &vstack);
      }
    }
    else {
      vol_stack_load(b, slot, &vstack);
      const hc_uint4 r0 = cy_ld(&b->vol_rec[2 * (size_t)slot]);
      const hc_uint4 r1 = cy_ld(&b->vol_rec[2 * (size_t)slot + 1]);
      state.volume_bounce = (int)r0.w;
      state.volume_bounds_bounce = (int)r1.x;
      if (CY_VOLUME_EXT && (r0.z & CY_VOP_INIT_CAMERA)) {
        /* path_state_init's kernel_volume_stack_init (kernel_path_state.h:62-68) */
        CySD stack_sd;
        volume_stack_init_camera(kg, &stack_sd, &ray, (uint)state.flag, &vstack, err);
      }
      if (r0.z & CY_VOP_PATH) {
        volume_stack_enter_exit(SD_HAS_VOLUME | ((r0.z & CY_VOP_BACKFACING) ? SD_BACKFACING : 0), (int)r0.x,
                                (int)r0.y, &vstack);
      }
    }
  }
#endif

  const bool hit = as_int(is4.w) != PRIM_NONE;
  /* isect->type: the primitive's packed type (a curve's carries its segment) */
  const int type = hit ? (kg->have_curves ? (int)kg->__prim_type[as_int(is4.w)] : PRIMITIVE_TRIANGLE) : 0;

  /* kernel_path_lamp_emission (kernel_path.h:86-113): lamps hit by the ray
   * segment since the last non-transparent bounce, MIS-weighted
   * (indirect_lamp_emission, kernel_emission.h:235-286) */
  if (KD->integrator.use_lamp_mis && !(state.flag & PATH_RAY_CAMERA)) {
    const float isect_t = hit ? is4.x : ray.t;
    const cfloat3 light_P = sub3(ray.P, mul3f(ray.D, state.ray_t));
    state.ray_t += isect_t;
    for (int lamp = 0; lamp < KD->integrator.num_all_lights; lamp++) {
      CyLightSample ls;
      if (!lamp_light_eval(kg, lamp, light_P, ray.D, state.ray_t, &ls)) {
        continue;
      }
      const uint lsh = (uint)ls.shader;
      if (lsh & SHADER_EXCLUDE_ANY) {
        if (((lsh & SHADER_EXCLUDE_DIFFUSE) && (state.flag & PATH_RAY_DIFFUSE)) ||
            ((lsh & SHADER_EXCLUDE_GLOSSY) &&
             ((state.flag & (PATH_RAY_GLOSSY | PATH_RAY_REFLECT)) == (PATH_RAY_GLOSSY | PATH_RAY_REFLECT))) ||
            ((lsh & SHADER_EXCLUDE_TRANSMIT) && (state.flag & PATH_RAY_TRANSMIT)) ||
            ((lsh & SHADER_EXCLUDE_SCATTER) && (state.flag & PATH_RAY_VOLUME_SCATTER))) {
          continue;
        }
      }
      /* direct_emissive_eval (kernel_emission.h:20-99) */
      cfloat3 lamp_L = mk3(0.0f, 0.0f, 0.0f);
      if (!shader_constant_emission_eval(kg, ls.shader, &lamp_L)) {
#if CY_SVM_TEX
        lamp_L = emissive_eval_svm(kg, ls.P, ls.Ng, neg3(ray.D), ls.shader, ls.object, ls.prim, ls.lamp, ls.u, ls.v,
                                   ls.t, mem, state, err);
#else
        cy_set_error(err, CY_ERR_FEATURE, 7); /* non-constant emitter: a _tex variant scans it */
#endif
      }
      lamp_L = mul3f(lamp_L, ls.eval_fac);
      lamp_L = mul3(lamp_L, klight_vec(kg->__lights[lamp].strength));
#if CY_CLOSURE_EXT
      if (VOL && vstack.e[0].shader != SHADER_NONE) {
        /* shadow attenuation by the volumes along the segment (kernel_emission.h:264-272) */
        CyRay volume_ray;
        volume_ray.P = light_P;
        volume_ray.D = ray.D;
        volume_ray.t = ls.t;
        cfloat3 volume_tp = mk3(1.0f, 1.0f, 1.0f);
        CySD esd;
        volume_shadow(kg, &esd, &state, &vstack, &volume_ray, &volume_tp, mem, err);
        lamp_L = mul3(lamp_L, volume_tp);
      }
#endif
      if (!(state.flag & PATH_RAY_MIS_SKIP)) {
        lamp_L = mul3f(lamp_L, power_heuristic(state.ray_pdf, ls.pdf));
      }
      /* path_radiance_accum_emission (kernel_accumulate.h:304-335; nothing
       * behind a shadow catcher) */
      cfloat3 contribution = mul3(throughput, lamp_L);
      contribution = path_radiance_clamp(kg, contribution, state.bounce - 1);
#if CY_CATCHER
      if (b->lp) {
        lightpass_accum_emission(&lp, &L, state.bounce, contribution);
      }
      else if (!(state.flag & PATH_RAY_SHADOW_CATCHER))
#endif
      {
        L = add3(L, contribution);
      }
    }
  }

  bool cont = false; /* path continues with a new ray */
  cfloat3 shadow_D = mk3(0.0f, 0.0f, 0.0f);
  bool vol_scattered = false;
  int sss_disk_rays = -1; /* >= 0: a disk BSSRDF scattered at this bounce */

#if CY_CLOSURE_EXT
  if (VOL) {
    /* kernel_path_volume (kernel_path.h:149-247), distance sampling */
    if (!hit) {
      volume_stack_clean(kg, &vstack);
    }
    if (vstack.e[0].shader != SHADER_NONE) {
      CyRay volume_ray = ray;
      volume_ray.t = hit ? is4.x : CY_FLT_MAX;
      const float step_size = volume_stack_step_size(kg, &vstack);
      CySD vsd;
      /* kernel_path.h:180-215: the CPU device's decoupled ray marching (direct
       * light from all lights inline, cy_volume_decoupled.h), or distance
       * sampling with one deferred light sample */
      const int sampling_method = volume_stack_sampling_method(kg, &vstack);
      const bool decoupled = CY_VOLUME_EXT && volume_use_decoupled(kg, (state.flag & PATH_RAY_CAMERA) != 0,
                                                                   sampling_method);
      const int result = decoupled ? volume_decoupled_path(kg, &vsd, &state, &vstack, &volume_ray, &L, &throughput,
                                                           step_size, sampling_method, mem,
                                                           (CyVolumeStep *)b->dec_steps +
                                                               (size_t)slot * CY_DECOUPLED_STEPS,
                                                           err) :
                                     volume_integrate(kg, &state, &vsd, &vstack, &volume_ray, &L, &throughput,
                                                      step_size, mem, err);
      if (result == VOLUME_PATH_SCATTERED) {
        vol_scattered = true;
        if (!decoupled) {
          connect_light<true>(kg, b, slot, &vsd, &state, throughput, &L, shadow, &shadow_D, mem, err);
        }
        shadow_rng_offset = state.rng_offset;
        if (volume_bounce(kg, &vsd, &throughput, &state, &ray)) {
          cont = true;
          if (kg->use_ray_diff) {
            /* kernel_path_volume.h:123-124: dP = the volume point's dP (the
             * segment ray's dD, shader_setup_from_volume), dD = the phase
             * sample's (zero, volume.h:146-147) */
            CyDiff3 rdP, rdD;
            ray_diff_load(kg, b, tile, slot, cam_item, &rdP, &rdD);
            CyDiff3 zero;
            zero.dx = zero.dy = mk3(0.0f, 0.0f, 0.0f);
            diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, rdD, zero);
          }
        }
      }
    }
  }
#endif

  if (vol_scattered) {
    /* the segment scattered: no surface or background at its end */
  }
  else if (!hit) {
    /* kernel_path_background (kernel_path.h:115-144) */
    bool skip = false;
    if (KD->background.transparent && (state.flag & PATH_RAY_TRANSPARENT_BACKGROUND)) {
      L_transparent += average3(throughput);
      if (!(KD->film.light_pass_flag & (1 << 2))) { /* PASSMASK(BACKGROUND) */
        skip = true;
      }
    }
    if (!skip) {
      if (path_state_ao_bounce(kg, &state)) {
        throughput = mul3f(throughput, KD->background.ao_bounces_factor);
      }
      const cfloat3 L_background = indirect_background(kg, b, tile, slot, cam_item, &state, &ray, mem, err);
      /* path_radiance_accum_background (kernel_accumulate.h:478-520) */
      bool catcher_path = false;
#if CY_CATCHER
      if (b->catcher && (state.flag & PATH_RAY_STORE_SHADOW_INFO)) {
        catcher.path_total = add3(catcher.path_total, mul3(throughput, L_background));
        catcher.path_total_shaded = add3(catcher.path_total_shaded,
                                         mul3f(mul3(throughput, L_background), catcher.transparency));
        catcher_path = (state.flag & PATH_RAY_SHADOW_CATCHER) != 0;
      }
#endif
      if (!catcher_path) {
        cfloat3 contribution = mul3(throughput, L_background);
        contribution = path_radiance_clamp(kg, contribution, state.bounce - 1);
#if CY_CATCHER
        if (b->lp) {
          /* path_radiance_accum_background with light passes (kernel_accumulate.h:500-510) */
          if (state.flag & PATH_RAY_TRANSPARENT_BACKGROUND) {
            lp.background = add3(lp.background, contribution);
          }
          else if (state.bounce == 1) {
            lp.direct_emission = add3(lp.direct_emission, contribution);
          }
          else {
            lp.indirect = add3(lp.indirect, contribution);
          }
        }
        else
#endif
        {
          L = add3(L, contribution);
        }
      }
    }
  }
  else if (!path_state_ao_bounce(kg, &state)) {
    CyIsect isect;
    isect.t = is4.x;
    isect.u = is4.y;
    isect.v = is4.z;
    isect.prim = as_int(is4.w);
    isect.object = hit_object;
    isect.type = type;

    CySD sd;
    sd.closure = mem.closure;
    sd.svm_stack = mem.svm_stack;
    sd.svm_stride = mem.svm_stride;
    sd.svm_fast = mem.svm_fast;
    sd.svm_spill = mem.svm_spill;
#if CY_CLOSURE_EXT
    CyDiff3 rdP, rdD;
    if (kg->use_ray_diff) {
      ray_diff_load(kg, b, tile, slot, cam_item, &rdP, &rdD);
    }
    shader_setup_from_ray(kg, &sd, &isect, &ray, kg->use_ray_diff ? &rdP : nullptr, &rdD);
#else
    shader_setup_from_ray(kg, &sd, &isect, &ray);
#endif
#ifdef CY_DBG_X
    sd.dbg = state.dbg;
#endif
    CY_DBG3(&state, "sd.P", sd.P);
    CY_DBG3(&state, "sd.N", sd.N);
    CY_DBG3(&state, "sd.Ng", sd.Ng);
    CY_DBG3(&state, "sd.I", sd.I);
    CY_DBG3(&state, "sd.uv", mk3(sd.u, sd.v, sd.ray_length));
#if CY_CLOSURE_EXT
    CY_DBG3(&state, "sd.dP.dx", sd.dP.dx);
    CY_DBG3(&state, "sd.dP.dy", sd.dP.dy);
    CY_DBG3(&state, "sd.dI.dx", sd.dI.dx);
    CY_DBG3(&state, "sd.dI.dy", sd.dI.dy);
    CY_DBG3(&state, "sd.du", mk3(sd.du.dx, sd.du.dy, sd.dv.dx));
    CY_DBG1(&state, "sd.dv.dy", sd.dv.dy);
#endif
#if CY_CLOSURE_EXT
    if (VOL && (sd.flag & SD_HAS_ONLY_VOLUME)) {
      /* volume bounding surface: pass through without a bounce
       * (kernel_path_surface.h:332-352, path_state_volume_next) */
      state.volume_bounds_bounce++;
      if (state.volume_bounds_bounce <= VOLUME_BOUNDS_MAX) {
        if (state.volume_bounds_bounce > 1) {
          state.rng_offset += PRNG_BOUNCE_NUM;
        }
        if (state.bounce == 0) {
          ray.t -= sd.ray_length;
        }
        else {
          ray.t = CY_FLT_MAX;
        }
        ray.P = ray_offset(sd.P, neg3(sd.Ng));
        if (kg->use_ray_diff) {
          /* kernel_path_surface.h:346: dP transferred, dD kept */
          diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, sd.dP, rdD);
        }
        vop_object = (uint)sd.object;
        vop_shader = (uint)sd.shader;
        vop_flags = CY_VOP_PATH | ((sd.flag & SD_BACKFACING) ? CY_VOP_BACKFACING : 0u);
        cont = true;
      }
    }
    else
#endif
    {
#ifdef CY_EXP_FIXED_SVM /* profiling experiment only: one diffuse closure, no SVM */
    sd.num_closure = 1;
    sd.num_closure_left = 0;
    sd.closure[0].type = CLOSURE_BSDF_DIFFUSE_ID;
    sd.closure[0].weight = mk3(0.8f, 0.8f, 0.8f);
    sd.closure[0].sample_weight = 0.8f;
    sd.closure[0].N = sd.N;
    sd.flag |= SD_BSDF | SD_BSDF_HAS_EVAL;
#else
    {
      /* the camera path's pixel for the AOV outputs (svm_aov.h), when the
       * film has AOV passes */
      float *aov_buffer = nullptr;
      if ((KD->film.pass_aov_color_num > 0 || KD->film.pass_aov_value_num > 0) && (state.flag & PATH_RAY_CAMERA)) {
        aov_buffer = item_buffer(tile, cam_item != CY_NO_ITEM ? cam_item : cy_ld(&b->item[slot]));
      }
      shader_eval_surface(kg, &sd, &state, state.flag, err, aov_buffer);
    }
#endif
#if CY_CATCHER
    /* kernel_branched_path_integrate: the camera segment of branched path
     * tracing merges identical closures instead (kernel_path_branched.h:440) */
    const bool branched_cam = KD->integrator.branched && (state.flag & PATH_RAY_CAMERA);
    if (branched_cam) {
      shader_merge_closures(&sd);
    }
    else
#else
    const bool branched_cam = false;
#endif
    {
      shader_prepare_closures(&sd, &state);
    }
#ifdef CY_DBG_X
    CY_DBGF(&state, "closures %d flag %08x\n", sd.num_closure, sd.flag);
    CY_DBG3(&state, "sd.N'", sd.N);
    for (int i = 0; i < sd.num_closure; i++) {
      CY_DBGF(&state, "closure %d type %d sw %08x\n", i, sd.closure[i].type,
              __builtin_bit_cast(unsigned, sd.closure[i].sample_weight));
      CY_DBG3(&state, "  weight", sd.closure[i].weight);
      CY_DBG3(&state, "  N", sd.closure[i].N);
      CY_DBG3(&state, "  a", mk3(sd.closure[i].alpha_x, sd.closure[i].alpha_y, sd.closure[i].ior));
    }
#endif

    /* kernel_path_shader_apply (kernel_path.h:254-321) */
    bool terminated = false;
#if CY_CATCHER
    if (sd.object_flag & SD_OBJECT_SHADOW_CATCHER) {
      if (state.flag & PATH_RAY_TRANSPARENT_BACKGROUND) {
        /* a camera (or transparent) ray reaches the catcher: the path goes on
         * behind it, recording the light it would have received
         * (path_radiance_accum_shadowcatcher, kernel_accumulate.h:529-537) */
        state.flag |= PATH_RAY_SHADOW_CATCHER | PATH_RAY_STORE_SHADOW_INFO;
        cfloat3 bg = mk3(0.0f, 0.0f, 0.0f);
        if (!KD->background.transparent) {
          bg = indirect_background(kg, b, tile, slot, cam_item, &state, &ray, mem, err);
        }
        catcher.throughput += average3(throughput);
        catcher.background = add3(catcher.background, mul3(throughput, bg));
        catcher.has = 1;
      }
    }
    else if (state.flag & PATH_RAY_SHADOW_CATCHER) {
      /* only update transparency after the catcher bounce */
      catcher.transparency *= average3(shader_bsdf_transparency(&sd));
    }
#else
    if (sd.object_flag & SD_OBJECT_SHADOW_CATCHER) {
      cy_set_error(err, CY_ERR_FEATURE, 5); /* the _ext kernels render shadow catchers */
    }
#endif
    if (((sd.flag & SD_HOLDOUT) || (sd.object_flag & SD_OBJECT_HOLDOUT_MASK)) &&
        (state.flag & PATH_RAY_TRANSPARENT_BACKGROUND)) {
      /* holdout (kernel_path.h:285-296): the holdout weight makes the pixel
       * transparent; a full holdout ends the path */
      const cfloat3 holdout_weight = shader_holdout_apply(&sd);
      if (KD->background.transparent) {
        L_transparent += average3(mul3(holdout_weight, throughput));
      }
      if (holdout_weight.x == 1.0f && holdout_weight.y == 1.0f && holdout_weight.z == 1.0f) {
        terminated = true;
      }
    }
    if (!terminated) {
    if ((state.flag & PATH_RAY_CAMERA) && !(state.flag & PATH_RAY_SINGLE_PASS_DONE)) {
      /* kernel_write_data_passes (kernel_passes.h:173-225): no data passes,
       * only the single-pass flag, set at the first hit that is not
       * transparent enough to show what is behind it (the AOV outputs of
       * later hits are skipped) */
      bool single_pass = true;
      if (!(!(sd.flag & SD_TRANSPARENT) || KD->film.pass_alpha_threshold == 0.0f)) {
        /* shader_bsdf_alpha (kernel_shader.h:860-868) */
        const cfloat3 tr = shader_bsdf_transparency(&sd);
        cfloat3 alpha = mk3(1.0f - tr.x, 1.0f - tr.y, 1.0f - tr.z);
        alpha = mk3(cmax(alpha.x, 0.0f), cmax(alpha.y, 0.0f), cmax(alpha.z, 0.0f));
        alpha = mk3(cmin(alpha.x, 1.0f), cmin(alpha.y, 1.0f), cmin(alpha.z, 1.0f));
        single_pass = average3(alpha) >= KD->film.pass_alpha_threshold;
      }
      if (single_pass) {
#if CY_CLOSURE_EXT
        if (KD->film.pass_flag & CY_DATA_PASSES) {
          write_data_passes(kg, item_buffer(tile, cam_item != CY_NO_ITEM ? cam_item : cy_ld(&b->item[slot])), &sd,
                            &state);
        }
#endif
        state.flag |= PATH_RAY_SINGLE_PASS_DONE;
      }
    }
#if CY_CATCHER
    if (b->lp && (state.flag & PATH_RAY_CAMERA)) {
      /* kernel_passes.h:251-281: colour passes and mist at camera hits */
      const int lflag = KD->film.light_pass_flag;
      cfloat3 cd = mk3(0.0f, 0.0f, 0.0f), cg = cd, ct = cd;
      for (int i = 0; i < sd.num_closure; i++) {
        const CyClosure *sc = &sd.closure[i];
        if (CLOSURE_IS_BSDF_DIFFUSE(sc->type) || CLOSURE_IS_BSSRDF(sc->type) || CLOSURE_IS_BSDF_BSSRDF(sc->type)) {
          cd = add3(cd, sc->weight);
        }
        if (CLOSURE_IS_BSDF_GLOSSY(sc->type)) {
          cg = add3(cg, sc->weight);
        }
        if (CLOSURE_IS_BSDF_TRANSMISSION(sc->type)) {
          ct = add3(ct, sc->weight);
        }
      }
      if (lflag & ((1 << 6) | (1 << 7) | (1 << 8))) {
        lp.color_diffuse = add3(lp.color_diffuse, mul3(cd, throughput));
      }
      if (lflag & ((1 << 9) | (1 << 10) | (1 << 11))) {
        lp.color_glossy = add3(lp.color_glossy, mul3(cg, throughput));
      }
      if (lflag & ((1 << 12) | (1 << 13) | (1 << 14))) {
        lp.color_transmission = add3(lp.color_transmission, mul3(ct, throughput));
      }
      if (lflag & 1) {
        /* camera_distance (kernel_camera.h:472-482) */
        const hc_Transform &c = KD->cam.cameratoworld;
        const cfloat3 camP = mk3(c.x.w, c.y.w, c.z.w);
        float depth;
        if (KD->cam.type == 1 /* CAMERA_ORTHOGRAPHIC */) {
          const cfloat3 camD = mk3(c.x.z, c.y.z, c.z.z);
          depth = fabsf(dot3(sub3(sd.P, camP), camD));
        }
        else {
          depth = len3(sub3(sd.P, camP));
        }
        float mist = saturate((depth - KD->film.mist_start) * KD->film.mist_inv_depth);
        const float falloff = KD->film.mist_falloff;
        if (falloff == 1.0f) {
        }
        else if (falloff == 2.0f) {
          mist = mist * mist;
        }
        else if (falloff == 0.5f) {
          mist = sqrtf(mist);
        }
        else {
          mist = cy_powf(mist, falloff);
        }
        const cfloat3 tr = shader_bsdf_transparency(&sd);
        cfloat3 alpha = mk3(1.0f - tr.x, 1.0f - tr.y, 1.0f - tr.z);
        alpha = mk3(cmax(alpha.x, 0.0f), cmax(alpha.y, 0.0f), cmax(alpha.z, 0.0f));
        alpha = mk3(cmin(alpha.x, 1.0f), cmin(alpha.y, 1.0f), cmin(alpha.z, 1.0f));
        lp.mist += (1.0f - mist) * average3(mul3(throughput, alpha));
      }
    }
#endif
    if (KD->integrator.filter_glossy != CY_FLT_MAX) {
      float blur_pdf = KD->integrator.filter_glossy * state.min_ray_pdf;
      if (blur_pdf < 1.0f) {
        float blur_roughness = sqrtf(1.0f - blur_pdf) * 0.5f;
        for (int i = 0; i < sd.num_closure; i++) {
          CyClosure *sc = &sd.closure[i];
          /* bsdf.h:706-735 bsdf_blur: GGX (all variants), multiscatter GGX,
           * Beckmann and Ashikhmin-Shirley raise their roughness alike */
          if (sc->type == CLOSURE_BSDF_MICROFACET_GGX_ID || sc->type == CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_BECKMANN_ID ||
              sc->type == CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID ||
              sc->type == CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID) {
            sc->alpha_x = fmaxf(blur_roughness, sc->alpha_x);
            sc->alpha_y = fmaxf(blur_roughness, sc->alpha_y);
          }
#if CY_CLOSURE_EXT
          else if (sc->type == CLOSURE_BSDF_HAIR_PRINCIPLED_ID) {
            bsdf_principled_hair_blur(&sd, sc, blur_roughness);
          }
#endif
        }
      }
    }
    if (sd.flag & SD_EMISSION) {
      /* indirect_primitive_emission (kernel_emission.h:209-233) */
      float res = (fabsf(dot3(sd.Ng, sd.I)) > 0.0f) ? 1.0f : 0.0f;
      cfloat3 emission = mul3(mk3(res, res, res), sd.closure_emission_background);
      if (!(state.flag & PATH_RAY_MIS_SKIP) && (sd.flag & SD_USE_MIS) &&
          (sd.type & PRIMITIVE_ALL_TRIANGLE)) {
        float pdf = triangle_light_pdf(kg, &sd, sd.ray_length);
        float mis_weight = power_heuristic(state.ray_pdf, pdf);
        emission = mul3f(emission, mis_weight);
      }
      /* path_radiance_accum_emission (kernel_accumulate.h:304-335) */
      cfloat3 contribution = mul3(throughput, emission);
      contribution = path_radiance_clamp(kg, contribution, state.bounce - 1);
#if CY_CATCHER
      if (b->lp) {
        lightpass_accum_emission(&lp, &L, state.bounce, contribution);
      }
      else if (!(state.flag & PATH_RAY_SHADOW_CATCHER))
#endif
      {
        L = add3(L, contribution);
      }
    }

    /* Russian roulette (kernel_path.h:587-599; on the camera segment of
     * branched path tracing only behind transparency, kernel_path_branched.h:
     * 449-466) */
    const float probability = (branched_cam && !(state.flag & PATH_RAY_TRANSPARENT)) ?
                                  1.0f :
                                  path_state_continuation_probability(kg, &state, throughput, branch_factor);
    if (probability == 0.0f) {
      terminated = true;
    }
    else if (probability != 1.0f) {
      float terminate = path_state_rng_1D(kg, &state, PRNG_TERMINATE);
      if (terminate >= probability) {
        terminated = true;
      }
      else {
        throughput = div3f(throughput, probability);
      }
    }
    } /* !holdout end */

    /* kernel_path_subsurface_scatter (kernel_path_subsurface.h:26-110): a
     * picked BSSRDF moves the shading point to where the random walk leaves
     * the object, with a diffuse closure carrying the walk's weight; light is
     * connected there with the path's state, the bounce uses rng_offset +
     * PRNG_BOUNCE_NUM (the indirect ray's state), and a walk that never leaves
     * ends the path */
    bool sss_bounce = false;
#if CY_CLOSURE_EXT
    bool sss_update = false; /* random walk: the exit ray's volume stack is updated */
    CyIsect ss_hit;
    cfloat3 ss_weight, ss_N;
    CyRay ss_ray;
    int ss_type = 0;
    float ss_rough = 0.0f;
    const cfloat3 in_P = ray.P;
#endif
    if (!terminated) {
      if (KD->integrator.use_ambient_occlusion) {
        cy_set_error(err, CY_ERR_FEATURE, 6);
      }
#if CY_CLOSURE_EXT
      if (sd.flag & SD_BSSRDF) {
        float bssrdf_u, bssrdf_v;
        path_state_rng_2D(kg, &state, PRNG_BSDF_U, &bssrdf_u, &bssrdf_v);
        const CyClosure *sc = shader_bssrdf_pick(&sd, &throughput, &bssrdf_u);
        if (sc) {
          const int bssrdf_type = sc->type;
          const float bssrdf_rough = bssrdf_roughness(sc);
          if (CLOSURE_IS_DISK_BSSRDF(bssrdf_type)) {
            /* the exit points' light and bounces replace the path's own */
            if constexpr (VOL && CY_VOLUME_EXT) {
              CySD stack_sd;
              sss_disk_rays = subsurface_disk_paths<true>(kg, b, slot, cam_item, &sd, sc, bssrdf_u, bssrdf_v,
                                                          &state, &ray, &throughput, &L, mem, err, &vstack,
                                                          &stack_sd);
            }
            else {
              sss_disk_rays = subsurface_disk_paths(kg, b, slot, cam_item, &sd, sc, bssrdf_u, bssrdf_v, &state,
                                                    &ray, &throughput, &L, mem, err);
            }
            terminated = true;
          }
          else if (subsurface_random_walk(kg, &sd, &state, sc, bssrdf_u, bssrdf_v, &ss_hit, &ss_weight, &ss_ray,
                                          err)) {
            /* subsurface_scatter_multi_setup (kernel_subsurface.h:284-313) */
            shader_setup_from_subsurface(kg, &sd, &ss_hit, &ss_ray);
            ss_N = sd.N;
            subsurface_color_bump_blur(kg, &sd, &state, &ss_weight, &ss_N, err);
            subsurface_scatter_setup_diffuse_bsdf(kg, &sd, bssrdf_type, bssrdf_rough, ss_weight, ss_N);
            sss_bounce = true;
            if (VOL && CY_VOLUME_EXT && (sd.object_flag & SD_OBJECT_INTERSECTS_VOLUME)) {
              /* the exit ray's stack is updated after its bounce, so the exit
               * point's light sample is traced here with the path's stack */
              sss_update = true;
              ss_type = bssrdf_type;
              ss_rough = bssrdf_rough;
            }
          }
          else {
            terminated = true;
          }
        }
      }
#else
      if (sd.flag & SD_BSSRDF) {
        cy_set_error(err, CY_ERR_FEATURE, 6);
      }
#endif
    }
#if CY_CATCHER
    if (!terminated && branched_cam) {
      cont = branched_camera_hit(kg, b, slot, &sd, &state, &throughput, &ray, &L, &branch_factor, &catcher, mem,
                                 err);
      terminated = true;
    }
#endif
    if (!terminated) {
      /* Direct light: kernel_branched_path_surface_connect_light with one sample
       * (kernel_path_surface.h:23-140), light_sample + direct_emission
       * (kernel_emission.h:101-205). */
#ifdef CY_EXP_NO_LIGHT /* profiling experiment only: skip next-event estimation */
      if (false) {
#else
      if (KD->integrator.use_direct_light && (sd.flag & SD_BSDF_HAS_EVAL)) {
#endif
#if CY_CLOSURE_EXT
        if (VOL && CY_VOLUME_EXT && sss_update) {
          bool reused = false;
          connect_light_exit_vol(kg, b, slot, &sd, &state, throughput, &L, &reused, mem, err, &vstack);
          if (reused) {
            shader_setup_from_subsurface(kg, &sd, &ss_hit, &ss_ray);
            subsurface_scatter_setup_diffuse_bsdf(kg, &sd, ss_type, ss_rough, ss_weight, ss_N);
          }
        }
        else
#endif
#if CY_CATCHER
        if (b->lp) {
          /* light passes: the light sample traced here, added per component */
          connect_light_branched(kg, &sd, &state, throughput, 1.0f, (state.flag & PATH_RAY_SHADOW_CATCHER) != 0, &L,
                                 &catcher, mem, err, &lp);
        }
        else if ((state.flag & PATH_RAY_SHADOW_CATCHER) ||
                 (KD->integrator.branched && KD->integrator.sample_all_lights_indirect)) {
          /* kernel_path_indirect (kernel_path.h:470-476) / a path behind a
           * shadow catcher: all lights */
          connect_light_branched(kg, &sd, &state, throughput, 1.0f, true, &L, &catcher, mem, err);
        }
        else
#endif
        {
          connect_light<false>(kg, b, slot, &sd, &state, throughput, &L, shadow, &shadow_D, mem, err);
        }
      }
#if CY_CLOSURE_EXT
      if (VOL && *shadow) {
        /* the shadow ray leaves through the surface: its copy of the stack
         * crosses it (shadow_blocked_volume_path_state) */
        shadow_rng_offset = state.rng_offset;
        if ((sd.flag & SD_HAS_VOLUME) && dot3(sd.Ng, shadow_D) < 0.0f) {
          vop_object = (uint)sd.object;
          vop_shader = (uint)sd.shader;
          vop_flags |= CY_VOP_SHADOW | ((sd.flag & SD_BACKFACING) ? CY_VOP_BACKFACING : 0u);
        }
      }
#endif

      /* kernel_path_surface_bounce (kernel_path_surface.h:270-358) */
      if (sss_bounce) {
        state.rng_offset += PRNG_BOUNCE_NUM; /* hit_state of the subsurface indirect ray */
      }
      if (sd.flag & SD_BSDF) {
        float bsdf_u, bsdf_v;
        path_state_rng_2D(kg, &state, PRNG_BSDF_U, &bsdf_u, &bsdf_v);
        cfloat3 bsdf_eval_v = mk3(0.0f, 0.0f, 0.0f);
        cfloat3 omega_in = mk3(0.0f, 0.0f, 0.0f);
        float bsdf_pdf = 0.0f;
#if CY_CLOSURE_EXT
        CyDiff3 domega;
        CyBsdfEvalLP ev_lp;
        int label;
        if (CY_CATCHER && b->lp) {
          label = shader_bsdf_sample_lp(kg, &sd, bsdf_u, bsdf_v, &ev_lp, &omega_in, &bsdf_pdf, err,
                                        kg->use_ray_diff ? &domega : nullptr);
          /* bsdf_eval_is_zero over every component (the transparent one too) */
          bsdf_eval_v = bsdf_eval_lp_is_zero(&ev_lp) ? mk3(0.0f, 0.0f, 0.0f) : mk3(1.0f, 1.0f, 1.0f);
        }
        else {
          label = shader_bsdf_sample(kg, &sd, bsdf_u, bsdf_v, &bsdf_eval_v, &omega_in, &bsdf_pdf, err,
                                     kg->use_ray_diff ? &domega : nullptr);
        }
#else
        int label = shader_bsdf_sample(kg, &sd, bsdf_u, bsdf_v, &bsdf_eval_v, &omega_in, &bsdf_pdf, err);
#endif
        CY_DBGF(&state, "bsdf label %d\n", label);
        CY_DBG3(&state, "bsdf eval", bsdf_eval_v);
        CY_DBG3(&state, "omega_in", omega_in);
        CY_DBG1(&state, "bsdf pdf", bsdf_pdf);
        if (!(bsdf_pdf == 0.0f || is_zero3(bsdf_eval_v))) {
          float inverse_pdf = 1.0f / bsdf_pdf;
#if CY_CATCHER
          if (b->lp) {
            /* path_radiance_bsdf_bounce with light passes (kernel_accumulate.h:247-265) */
            if (state.bounce == 0 && !(label & LABEL_TRANSPARENT)) {
              const cfloat3 value = mul3f(throughput, inverse_pdf);
              lp.state_diffuse = mul3(ev_lp.diffuse, value);
              lp.state_glossy = mul3(ev_lp.glossy, value);
              lp.state_transmission = mul3(ev_lp.transmission, value);
              lp.state_volume = mul3(ev_lp.volume, value);
              throughput = add3(add3(add3(lp.state_diffuse, lp.state_glossy), lp.state_transmission),
                                lp.state_volume);
              lp.state_direct = throughput;
            }
            else {
              const cfloat3 sum = mul3f(add3(bsdf_eval_lp_sum(&ev_lp), ev_lp.transparent), inverse_pdf);
              throughput = mul3(throughput, sum);
            }
          }
          else
#endif
          {
            throughput = mul3(throughput, mul3f(bsdf_eval_v, inverse_pdf));
          }
          if (!(label & LABEL_TRANSPARENT)) {
            state.ray_pdf = bsdf_pdf;
            state.ray_t = 0.0f;
            state.min_ray_pdf = fminf(bsdf_pdf, state.min_ray_pdf);
          }
          path_state_next(kg, &state, label);
          ray.P = ray_offset(sd.P, (label & LABEL_TRANSMIT) ? neg3(sd.Ng) : sd.Ng);
          ray.D = normalize3(omega_in);
          if (state.bounce == 0) {
            ray.t -= sd.ray_length;
          }
          else {
            ray.t = CY_FLT_MAX;
          }
          cont = true;
#if CY_CLOSURE_EXT
          if (kg->use_ray_diff) {
            /* kernel_path_surface.h:321-322 */
            diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, sd.dP, domega);
          }
          if (VOL && (label & LABEL_TRANSMIT) && (sd.flag & SD_HAS_VOLUME)) {
            /* enter/exit the surface's volume (kernel_path_surface.h:325-329) */
            vop_object = (uint)sd.object;
            vop_shader = (uint)sd.shader;
            vop_flags |= CY_VOP_PATH | ((sd.flag & SD_BACKFACING) ? CY_VOP_BACKFACING : 0u);
          }
          if (VOL && CY_VOLUME_EXT && sss_update) {
            /* kernel_path_subsurface.h:92-99: the surface's own update, then
             * the volume surfaces from the path's previous point to the exit
             * point (no shadow is pending: it was traced above) */
            if (vop_flags & CY_VOP_PATH) {
              volume_stack_enter_exit(sd.flag, sd.object, sd.shader, &vstack);
              vop_flags &= ~(CY_VOP_PATH | CY_VOP_BACKFACING);
            }
            CyRay volume_ray;
            volume_ray.P = in_P;
            volume_ray.D = normalize_len3(sub3(ray.P, in_P), &volume_ray.t);
            CySD stack_sd;
            volume_stack_update_for_subsurface(kg, &stack_sd, &volume_ray, &vstack, err);
          }
#endif
        }
      }
    }
    }
  }

#if CY_CLOSURE_EXT
  if (sss_disk_rays > 0) {
    cont = true; /* the last indirect ray of the exit points */
  }
  else if (!cont && b->sss_rec) {
    /* the path ended: the next subsurface indirect ray of the slot
     * (kernel_path_subsurface_setup_indirect), if any */
    const int pending = (sss_disk_rays == 0 || cam_item != CY_NO_ITEM) ? 0 : (int)cy_ld(&b->sss_count[slot]);
    if (pending > 0) {
      if (VOL && CY_VOLUME_EXT) {
        /* the record's own stack; a shadow ray still pending keeps the ended
         * path's (and its own crossing of the surface) */
        if (*shadow) {
          vol_stack_write(sss_vol_at(b, slot, CY_SSS_RECS), &vstack);
          vop_flags |= CY_VOP_OWN_STACK;
        }
        vop_flags &= ~CY_VOP_PATH;
        vol_stack_read(sss_vol_at(b, slot, pending - 1), &vstack);
      }
      if (kg->use_ray_diff) {
        CyDiff3 pdP, pdD;
        sss_rec_load(b, slot, pending - 1, kg, &state, &ray, &throughput, &pdP, &pdD);
        diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, pdP, pdD);
      }
      else {
        sss_rec_load(b, slot, pending - 1, kg, &state, &ray, &throughput);
      }
      cy_st(&b->sss_count[slot], (uint)(pending - 1));
      cont = true;
    }
  }
#if CY_CATCHER
  if (!cont && b->br_rec && cam_item == CY_NO_ITEM) {
    /* the path ended: the next path its camera hit spawned, if any */
    const uint next = cy_ld(&b->br_count[2 * (size_t)slot]);
    const uint end = cy_ld(&b->br_count[2 * (size_t)slot + 1]);
    if (next < end) {
      const hc_float4 *rec = br_rec_at(b, slot, (int)next);
      if (kg->use_ray_diff) {
        CyDiff3 pdP, pdD;
        path_rec_load(rec, kg, &state, &ray, &throughput, &pdP, &pdD);
        diff_store(b->ray_diff + (size_t)slot * CY_RAY_DIFF_F4, pdP, pdD);
      }
      else {
        path_rec_load(rec, kg, &state, &ray, &throughput, nullptr, nullptr);
      }
      branch_factor = cy_ld(&rec[CY_BR_REC_F4 - 1]).x;
      cy_st(&b->br_count[2 * (size_t)slot], next + 1);
      cont = true;
    }
  }
#endif
  if (VOL && (cont || *shadow)) {
    vol_stack_store(b, slot, &vstack);
    vol_rec_store(b, slot, vop_object, vop_shader, vop_flags, &state, shadow_rng_offset);
  }
#endif

#if CY_CATCHER
  if (b->catcher && (cont || *shadow)) {
    catcher_store(b, slot, &catcher);
  }
  if (b->lp && (cont || *shadow)) {
    lightpass_store(b, slot, &lp);
  }
#endif
  if (cont) {
    store_state(b, slot, &state);
    if (cam_item != CY_NO_ITEM) {
      cy_st(&b->item[slot], cam_item);
    }
    cy_st(&b->ray_P[slot], mkf4(ray.P.x, ray.P.y, ray.P.z, ray.t));
    cy_st(&b->ray_D[slot], mkf4(ray.D.x, ray.D.y, ray.D.z, as_float(path_state_ray_visibility(&state))));
    cy_st(&b->throughput[slot], mkf4(throughput.x, throughput.y, throughput.z, L_transparent));
    cy_st(&b->L[slot], mkf4(L.x, L.y, L.z, branch_factor));
    return true;
  }
  if (*shadow) {
    /* the path ends after its pending light contribution: the shadow stage
     * adds it, writes the sample and regenerates the slot */
    if (cam_item != CY_NO_ITEM) {
      cy_st(&b->item[slot], cam_item);
    }
    cy_st(&b->throughput[slot], mkf4(throughput.x, throughput.y, throughput.z, L_transparent));
    cy_st(&b->L[slot], mkf4(L.x, L.y, L.z, branch_factor));
    hc_float4 sl = cy_ld(&b->shadow_L[slot]);
    sl.w = 1.0f;
    cy_st(&b->shadow_L[slot], sl);
    return false;
  }
#if CY_CATCHER
  if (b->catcher) {
    CY_DBG3(&state, "catcher total", catcher.path_total);
    CY_DBG3(&state, "catcher shaded", catcher.path_total_shaded);
    CY_DBG3(&state, "catcher background", catcher.background);
    CY_DBG3(&state, "catcher tp transp has", mk3(catcher.throughput, catcher.transparency, (float)catcher.has));
  }
  if (b->lp) {
    /* light passes: the combined value summed from the components */
    const uint fitem = cam_item != CY_NO_ITEM ? cam_item : cy_ld(&b->item[slot]);
    L = lightpass_finish(kg, item_buffer(tile, fitem), L, &lp);
  }
  slot_finish(b, tile, slot, cam_item, L, L_transparent, b->catcher ? &catcher : nullptr);
#else
  slot_finish(b, tile, slot, cam_item, L, L_transparent);
#endif
  *finished = true;
  return false;
}

/* ---------------------------------------------------------------------------
 * SHADER task, SHADER_EVAL_BACKGROUND: the world shader seen along one
 * equirectangular direction (kernel_bake.h:474-510 kernel_background_evaluate;
 * LightManager feeds (u, v) = ((x + 0.5) / w, (y + 0.5) / h) as float bits,
 * light.cpp:38-60, and builds the background importance map from the result).
 */

/* kernel_projection.h:67-83: equirectangular_range_to_direction with the
 * default range (-2pi, pi, -pi, pi) */
CY_FN cfloat3 equirectangular_to_direction(float u, float v)
{
  const float m_2pi = 6.2831853071795864f;
  const float phi = -m_2pi * u + CY_PI_F;
  const float theta = -CY_PI_F * v + CY_PI_F;
  const float sin_theta = cy_sinf(theta);
  return mk3(sin_theta * cy_cosf(phi), sin_theta * cy_sinf(phi), cy_cosf(theta));
}

CY_FN cfloat3 background_evaluate(const CyGlobals *kg, uint in_u, uint in_v, CyShadeMem mem, uint *err)
{
  const cfloat3 D = equirectangular_to_direction(as_float(in_u), as_float(in_v));
  CySD sd;
  shader_setup_from_background(kg, &sd, D, mem);
  /* path_flag 0 | PATH_RAY_EMISSION: no BSDF closures are kept */
  shader_eval_surface(kg, &sd, nullptr, PATH_RAY_EMISSION, err);
  return shader_background_eval(&sd);
}

#endif /* CY_INTEGRATOR_H */
