/*
 * cy_oracle.h — TEST INFRASTRUCTURE ONLY: plain-C restatement of the primitive
 * operations of the Cycles path-tracing hot path, used as an independent CPU
 * checker of the HIP device on the GPU box (where the reference tree is absent).
 * Pinned against the reference CPU kernel (oracle/_ref) and the committed golden
 * vectors in tests/golden/ (tests/test_oracle.py).
 */
#ifndef CY_ORACLE_H
#define CY_ORACLE_H

#include <stdint.h>

uint32_t cyo_hash_uint2(uint32_t kx, uint32_t ky);
uint32_t cyo_cmj_hash_simple(uint32_t i, uint32_t p);
/* lut: 32 * dims uints; returns path_rng_1D(rng_hash, sample, dimension) */
float cyo_path_rng_1d(const uint32_t *lut, uint32_t rng_hash, int sample, int dimension);
void cyo_ray_offset(const float P[3], const float Ng[3], float out[3]);
int cyo_ray_triangle_intersect(const float P[3], const float D[3], float ray_t,
                               const float a[3], const float b[3], const float c[3],
                               float *u, float *v, float *t);
/* Brute-force closest hit over n_prims triangles of prim_tri_verts (3 float4 per
 * prim, in BVH slot order) with per-prim visibility: independent of any BVH.
 * rays: n x 8 floats (P, D, t, visibility bits); out_f n x 3, out_i n x 4. */
void cyo_intersect_brute(const float *prim_tri_verts, const uint32_t *prim_visibility, int n_prims,
                         const float *rays, int n, int any_hit, float *out_f, int32_t *out_i);
/* Same with instancing: top-level slots [0, n_top) hold world-space triangles
 * (prim_type 1) and object instances (prim_type 0, object prim_object[slot]);
 * an instance's triangles are slots [obj_first, +obj_count) in object space,
 * tested with the reference's push/pop of the ray and t (obj_itfm: 12 floats
 * per object).  out_i[2] is the instance object or -1. */
void cyo_intersect_brute_instanced(const float *prim_tri_verts, const uint32_t *prim_tri_index,
                                   const uint32_t *prim_type, const uint32_t *prim_object,
                                   const uint32_t *prim_visibility, int n_top, const float *obj_itfm,
                                   const int32_t *obj_first, const int32_t *obj_count, const float *rays,
                                   int n, int any_hit, float *out_f, int32_t *out_i);

/* Film convert of the combined display pass (kernel/kernel_film.h:19-141,
 * util/util_color.h:77-83, util/util_half.h:80-118 SSE2 branch): pixels
 * (x, y, w, h) of buffer (pass_stride floats per pixel) at index
 * offset + x + y*stride into rgba (4 bytes, or 4 half bit patterns, per pixel).
 * film: pass_stride, display_pass_stride, display_pass_components,
 * display_divide_pass_stride, use_display_exposure, use_display_pass_alpha. */
void cyo_film_convert(const int32_t film[6], float exposure, const float *buffer, void *rgba, float sample_scale,
                      int x, int y, int w, int h, int offset, int stride, int half);


/* Background importance map CDFs (render/light.cpp:530-565 background_cdf and
 * 676-716 marginal CDF): pixels res_y x res_x float4 (rgb used), marg
 * (res_y + 1) float pairs, cond res_y x (res_x + 1) float pairs. */
void cyo_background_cdf(const float *pixels, int res_x, int res_y, float *marg, float *cond);

#endif
