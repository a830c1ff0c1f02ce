/*
 * cy_oracle.c — TEST INFRASTRUCTURE ONLY (see cy_oracle.h).  Never linked into
 * the product.  Each function restates the reference at the cited lines:
 *   cyo_hash_uint2          util/util_hash.h:28-93
 *   cyo_cmj_hash_simple     kernel/kernel_jitter.h:122-129
 *   cyo_path_rng_1d         kernel/kernel_random.h:40-90 (Sobol branch)
 *   cyo_ray_offset          kernel/bvh/bvh.h:541-586
 *   cyo_ray_triangle_intersect util/util_math_intersect.h:88-195 (scalar branch)
 *   cyo_intersect_brute     closest hit = minimum t over all visible triangles,
 *                           later primitive wins ties (geom_triangle_intersect.h:25-72
 *                           accepts t <= current); any-hit = first hit.
 * Compiled with -ffp-contract=off like the reference generic CPU kernel.
 */
#include "cy_oracle.h"

#include <math.h>
#include <string.h>

static float u2f(uint32_t u)
{
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static uint32_t f2u(float f)
{
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

#define ROT(x, k) (((x) << (k)) | ((x) >> (32 - (k))))

uint32_t cyo_hash_uint2(uint32_t kx, uint32_t ky)
{
  uint32_t a, b, c;
  a = b = c = 0xdeadbeef + (2 << 2) + 13;
  b += ky;
  a += kx;
  c ^= b; c -= ROT(b, 14);
  a ^= c; a -= ROT(c, 11);
  b ^= a; b -= ROT(a, 25);
  c ^= b; c -= ROT(b, 16);
  a ^= c; a -= ROT(c, 4);
  b ^= a; b -= ROT(a, 14);
  c ^= b; c -= ROT(b, 24);
  return c;
}

uint32_t cyo_cmj_hash_simple(uint32_t i, uint32_t p)
{
  i = (i ^ 61) ^ p;
  i += i << 3;
  i ^= i >> 4;
  i *= 0x27d4eb2d;
  return i;
}

float cyo_path_rng_1d(const uint32_t *lut, uint32_t rng_hash, int sample, int dimension)
{
  uint32_t result = 0;
  uint32_t i = (uint32_t)sample + 64u; /* SOBOL_SKIP */
  int j = 0;
  while (i) {
    int x = __builtin_ffs((int)i);
    j += x;
    result ^= lut[32 * dimension + j - 1];
    i >>= x;
  }
  float r = (float)result * (1.0f / (float)0xFFFFFFFF);
  uint32_t tmp_rng = cyo_cmj_hash_simple((uint32_t)dimension, rng_hash);
  float shift = (float)tmp_rng * (1.0f / (float)0xFFFFFFFF);
  return r + shift - floorf(r + shift);
}

static float offset1(float p, float n)
{
  if (fabsf(p) < 1.0f) {
    return p + n * 1e-5f;
  }
  uint32_t ip = f2u(p);
  ip += ((ip ^ f2u(n)) >> 31) ? (uint32_t)-32 : 32u;
  return u2f(ip);
}

void cyo_ray_offset(const float P[3], const float Ng[3], float out[3])
{
  for (int k = 0; k < 3; k++) {
    out[k] = offset1(P[k], Ng[k]);
  }
}

static void sub(const float *a, const float *b, float *r)
{
  r[0] = a[0] - b[0];
  r[1] = a[1] - b[1];
  r[2] = a[2] - b[2];
}
static void add(const float *a, const float *b, float *r)
{
  r[0] = a[0] + b[0];
  r[1] = a[1] + b[1];
  r[2] = a[2] + b[2];
}
static void cross(const float *a, const float *b, float *r)
{
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
static float dot(const float *a, const float *b)
{
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static float fmin_c(float a, float b)
{
  return (a < b) ? a : b;
}
static float fmax_c(float a, float b)
{
  return (a > b) ? a : b;
}

int cyo_ray_triangle_intersect(const float P[3], const float D[3], float ray_t,
                               const float a[3], const float b[3], const float c[3],
                               float *u, float *v, float *t)
{
  float v0[3], v1[3], v2[3], e0[3], e1[3], e2[3], s[3], cr[3];
  sub(c, P, v0);
  sub(a, P, v1);
  sub(b, P, v2);
  sub(v2, v0, e0);
  sub(v0, v1, e1);
  sub(v1, v2, e2);
  add(v2, v0, s);
  cross(s, e0, cr);
  const float U = dot(cr, D);
  add(v0, v1, s);
  cross(s, e1, cr);
  const float V = dot(cr, D);
  add(v1, v2, s);
  cross(s, e2, cr);
  const float W = dot(cr, D);
  const float minUVW = fmin_c(U, fmin_c(V, W));
  const float maxUVW = fmax_c(U, fmax_c(V, W));
  if (minUVW < 0.0f && maxUVW > 0.0f) {
    return 0;
  }
  float Ng1[3], Ng[3];
  cross(e1, e0, Ng1);
  add(Ng1, Ng1, Ng);
  const float den = dot(Ng, D);
  if (den == 0.0f) {
    return 0;
  }
  const float T = dot(v0, Ng);
  const uint32_t sign_den = f2u(den) & 0x80000000u;
  const float sign_T = u2f(f2u(T) ^ sign_den);
  if ((sign_T < 0.0f) || (sign_T > ray_t * u2f(f2u(den) ^ sign_den))) {
    return 0;
  }
  const float inv_den = 1.0f / den;
  *u = U * inv_den;
  *v = V * inv_den;
  *t = T * inv_den;
  return 1;
}

void cyo_intersect_brute(const float *prim_tri_verts, const uint32_t *prim_visibility, int n_prims,
                         const float *rays, int n, int any_hit, float *out_f, int32_t *out_i)
{
  const float ooeps = 8.271806E-25f;
  for (int r = 0; r < n; r++) {
    const float *ray = rays + 8 * r;
    float P[3] = {ray[0], ray[1], ray[2]};
    float D[3];
    for (int k = 0; k < 3; k++) {
      float d = ray[3 + k];
      D[k] = (fabsf(d) > ooeps) ? d : copysignf(ooeps, d);
    }
    const uint32_t vis = f2u(ray[7]) & (any_hit ? ((1u << 7) | (1u << 8)) : 0xFFFFFFFFu);
    float best_t = ray[6], bu = 0.0f, bv = 0.0f;
    int best = -1;
    for (int p = 0; p < n_prims; p++) {
      const float *tv = prim_tri_verts + 12 * (size_t)p;
      float u, v, t;
      if (cyo_ray_triangle_intersect(P, D, best_t, tv, tv + 4, tv + 8, &u, &v, &t)) {
        if (prim_visibility[p] & vis) {
          best = p;
          best_t = t;
          bu = u;
          bv = v;
          if (any_hit) {
            break;
          }
        }
      }
    }
    out_f[3 * r + 0] = best_t;
    out_f[3 * r + 1] = bu;
    out_f[3 * r + 2] = bv;
    out_i[4 * r + 0] = best >= 0;
    out_i[4 * r + 1] = best;
    out_i[4 * r + 2] = -1;
    out_i[4 * r + 3] = best >= 0 ? 1 : 0;
  }
}

/* transform_point / transform_direction (util_transform.h, scalar branch) */
static void xform(const float *m, const float *a, int point, float *r)
{
  for (int k = 0; k < 3; k++) {
    const float *row = m + 4 * k;
    r[k] = a[0] * row[0] + a[1] * row[1] + a[2] * row[2];
    if (point) {
      r[k] = r[k] + row[3];
    }
  }
}

static void clamp_dir(const float *d, float *r)
{
  const float ooeps = 8.271806E-25f;
  for (int k = 0; k < 3; k++) {
    r[k] = (fabsf(d[k]) > ooeps) ? d[k] : copysignf(ooeps, d[k]);
  }
}

void cyo_intersect_brute_instanced(const float *prim_tri_verts, const uint32_t *prim_tri_index,
                                   const uint32_t *prim_type, const uint32_t *prim_object,
                                   const uint32_t *prim_visibility, int n_top, const float *obj_itfm,
                                   const int32_t *obj_first, const int32_t *obj_count, const float *rays,
                                   int n, int any_hit, float *out_f, int32_t *out_i)
{
  for (int r = 0; r < n; r++) {
    const float *ray = rays + 8 * r;
    const float P[3] = {ray[0], ray[1], ray[2]};
    float D[3];
    clamp_dir(ray + 3, D);
    const uint32_t vis = f2u(ray[7]) & (any_hit ? ((1u << 7) | (1u << 8)) : 0xFFFFFFFFu);
    float best_t = ray[6], bu = 0.0f, bv = 0.0f;
    int best = -1, best_obj = -1, done = 0;
    for (int p = 0; p < n_top && !done; p++) {
      float u, v, t;
      if (prim_type[p] == 1u) {
        const float *tv = prim_tri_verts + 4 * (size_t)prim_tri_index[p];
        if (cyo_ray_triangle_intersect(P, D, best_t, tv, tv + 4, tv + 8, &u, &v, &t) &&
            (prim_visibility[p] & vis)) {
          best = p;
          best_obj = -1;
          best_t = t;
          bu = u;
          bv = v;
          done = any_hit;
        }
        continue;
      }
      /* instance: bvh_instance_push / pop (geom/geom_object.h:425-470) */
      const int ob = (int)prim_object[p];
      const float *itfm = obj_itfm + 12 * (size_t)ob;
      float Po[3], Dt[3], Do[3];
      xform(itfm, P, 1, Po);
      xform(itfm, ray + 3, 0, Dt);
      const float len = sqrtf(dot(Dt, Dt));
      const float inv = 1.0f / len;
      const float Dn[3] = {Dt[0] * inv, Dt[1] * inv, Dt[2] * inv};
      clamp_dir(Dn, Do);
      float t_obj = (best_t != 3.402823466e+38f) ? best_t * len : best_t;
      for (int q = obj_first[ob]; q < obj_first[ob] + obj_count[ob]; q++) {
        const float *tv = prim_tri_verts + 4 * (size_t)prim_tri_index[q];
        if (cyo_ray_triangle_intersect(Po, Do, t_obj, tv, tv + 4, tv + 8, &u, &v, &t) &&
            (prim_visibility[q] & vis)) {
          best = q;
          best_obj = ob;
          t_obj = t;
          bu = u;
          bv = v;
          if (any_hit) {
            done = 1;
            break;
          }
        }
      }
      if (t_obj != 3.402823466e+38f) {
        xform(itfm, ray + 3, 0, Dt);
        t_obj /= sqrtf(dot(Dt, Dt));
      }
      best_t = t_obj;
    }
    out_f[3 * r + 0] = best_t;
    out_f[3 * r + 1] = bu;
    out_f[3 * r + 2] = bv;
    out_i[4 * r + 0] = best >= 0;
    out_i[4 * r + 1] = best;
    out_i[4 * r + 2] = best_obj;
    out_i[4 * r + 3] = best >= 0 ? 1 : 0;
  }
}


/* ---- film convert (kernel_film.h) ---------------------------------------- */

static float f_min(float a, float b) { return (a < b) ? a : b; }
static float f_max(float a, float b) { return (a > b) ? a : b; }
static float f_saturate(float a) { return f_min(f_max(a, 0.0f), 1.0f); }

/* util_color.h:77-83; powf is libm's, as in the reference */
static float srgb(float c)
{
  if (c < 0.0031308f) {
    return (c < 0.0f) ? 0.0f : c * 12.92f;
  }
  return 1.055f * powf(c, 1.0f / 2.4f) - 0.055f;
}

/* util_half.h:80-118 (SSE2 branch of float4_store_half): truncating conversion */
static uint16_t to_half(float v, float scale)
{
  float f = v * scale;
  f = (f > 0.0f) ? ((f < 65504.0f) ? f : 65504.0f) : 0.0f;
  int32_t x;
  memcpy(&x, &f, 4);
  const int32_t absolute = x & 0x7FFFFFFF;
  const int32_t Z = (int32_t)((uint32_t)absolute + 0xC8000000u);
  const int32_t result = (absolute < 0x38800000) ? 0 : Z;
  return (uint16_t)((result >> 13) & 0x7FFF);
}

void cyo_film_convert(const int32_t film[6], float exposure, const float *buffer, void *rgba, float sample_scale,
                      int x, int y, int w, int h, int offset, int stride, int half)
{
  const int pass_stride = film[0], dstride = film[1], dcomp = film[2], ddiv = film[3];
  const int use_exposure = film[4], use_alpha = film[5];
  const int use_scale = (ddiv == -1);
  for (int py = y; py < y + h; py++) {
    for (int px = x; px < x + w; px++) {
      const int index = offset + px + py * stride;
      float r[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      /* film_get_pass_result (kernel_film.h:19-63) */
      const float *in = buffer + dstride + (long)index * pass_stride;
      if (dcomp == 4) {
        const float alpha = use_scale ? (use_alpha ? in[3] : 1.0f / sample_scale) : 1.0f;
        r[0] = in[0];
        r[1] = in[1];
        r[2] = in[2];
        r[3] = alpha;
        if (ddiv != -1) {
          const float *dv = buffer + ddiv + (long)index * pass_stride;
          float q[3];
          for (int c = 0; c < 3; c++) {
            q[c] = (dv[c] != 0.0f) ? r[c] / dv[c] : 0.0f;
          }
          if (dv[0] == 0.0f) {
            if (dv[1] == 0.0f) { q[0] = q[2]; q[1] = q[2]; }
            else if (dv[2] == 0.0f) { q[0] = q[1]; q[2] = q[1]; }
            else q[0] = 0.5f * (q[1] + q[2]);
          }
          else if (dv[1] == 0.0f) {
            if (dv[2] == 0.0f) { q[1] = q[0]; q[2] = q[0]; }
            else q[1] = 0.5f * (q[0] + q[2]);
          }
          else if (dv[2] == 0.0f) {
            q[2] = 0.5f * (q[0] + q[1]);
          }
          r[0] = q[0];
          r[1] = q[1];
          r[2] = q[2];
        }
        if (use_exposure) {
          r[0] *= exposure;
          r[1] *= exposure;
          r[2] *= exposure;
          r[3] *= 1.0f;
        }
      }
      else if (dcomp == 1) {
        r[0] = r[1] = r[2] = in[0];
        r[3] = 1.0f / sample_scale;
      }
      const float scale = use_scale ? sample_scale : 1.0f;
      if (half) {
        uint16_t *o = (uint16_t *)rgba + (long)index * 4;
        for (int c = 0; c < 4; c++) {
          o[c] = to_half(r[c], scale);
        }
      }
      else {
        /* film_map + film_float_to_byte (kernel_film.h:65-92) */
        const float m[4] = {srgb(r[0] * scale), srgb(r[1] * scale), srgb(r[2] * scale), f_saturate(r[3] * scale)};
        uint8_t *o = (uint8_t *)rgba + (long)index * 4;
        for (int c = 0; c < 4; c++) {
          o[c] = (uint8_t)(f_saturate(m[c]) * 255.0f);
        }
      }
    }
  }
}

/* render/light.cpp:530-565 background_cdf: per row, the luminance-times-sine
 * function and its running sum (each step adds the previous value / res_x),
 * normalised by the row total which the entry past the end keeps. */
static void cyo_cdf_row(const float *pixels, int i, int res_x, int res_y, float *cond)
{
  const int w = res_x + 1;
  float *c = cond + 2 * (long)i * w;
  const float s = sinf(3.14159265358979323846f * ((float)i + 0.5f) / (float)res_y);
  for (int j = 0; j < res_x; j++) {
    const float *p = pixels + 4 * ((long)i * res_x + j);
    float lum = p[0] + p[1];
    lum = lum + p[2];
    lum = lum * (1.0f / 3.0f);
    c[2 * j] = lum * s;
    if (j == 0) {
      c[1] = 0.0f;
    }
    else {
      const float step = c[2 * j - 2] / (float)res_x;
      c[2 * j + 1] = c[2 * j - 1] + step;
    }
  }
  const float last_step = c[2 * res_x - 2] / (float)res_x;
  const float total = c[2 * res_x - 1] + last_step;
  const float inv = 1.0f / total;
  c[2 * res_x] = total;
  if (total > 0.0f) {
    for (int j = 1; j < res_x; j++) {
      c[2 * j + 1] = c[2 * j + 1] * inv;
    }
  }
  c[2 * res_x + 1] = 1.0f;
}

/* render/light.cpp:676-716 marginal CDF over the row totals */
void cyo_background_cdf(const float *pixels, int res_x, int res_y, float *marg, float *cond)
{
  for (int i = 0; i < res_y; i++) {
    cyo_cdf_row(pixels, i, res_x, res_y, cond);
  }
  const int w = res_x + 1;
  for (int i = 0; i < res_y; i++) {
    marg[2 * i] = cond[2 * ((long)i * w + res_x)];
    marg[2 * i + 1] = (i == 0) ? 0.0f : marg[2 * i - 1] + marg[2 * i - 2] / (float)res_y;
  }
  const float total = marg[2 * res_y - 1] + marg[2 * res_y - 2] / (float)res_y;
  marg[2 * res_y] = total;
  if (total > 0.0f) {
    for (int i = 1; i < res_y; i++) {
      marg[2 * i + 1] = marg[2 * i + 1] / total;
    }
  }
  marg[2 * res_y + 1] = 1.0f;
}
