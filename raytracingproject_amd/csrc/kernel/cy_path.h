/*
 * cy_path.h — device functions of the Cycles path-tracing hot path for gfx950.
 *
 * A restatement (not a translation) of the reference megakernel's per-sample
 * logic, regrouped into the three wavefront stages the HIP device runs
 * (intersect_closest -> shade -> intersect_shadow).  The per-sample arithmetic is
 * kept operation-for-operation identical to the reference scalar code so that the
 * render buffer matches the reference CPU kernel; each function cites the
 * reference it follows.
 */
#ifndef CY_PATH_H
#define CY_PATH_H

#include "cy_globals.h"
#include "cy_types.h"

#define KD (kg->data)

CY_FN cfloat3 f4to3(hc_float4 a)
{
  return mk3(a.x, a.y, a.z);
}

CY_FN void cy_set_error(uint *err, uint code, uint detail)
{
#if defined(__HIP_DEVICE_COMPILE__)
  if (err) {
    atomicCAS(err, 0u, (code << 24) | (detail & 0xFFFFFFu));
  }
#else
  (void)err;
  (void)code;
  (void)detail;
#endif
}

/* ---------------------------------------------------------------------------
 * Random numbers: kernel_random.h:40-153 (Sobol + Cranley-Patterson rotation).
 */
/* kernel_random.h sobol_dimension: XOR of the direction numbers of the set
 * bits of index + SOBOL_SKIP.  The reference walks the set bits with a
 * dependent loop; here each group of 8 bits reads its 8 contiguous direction
 * numbers at once (two 16-B loads, one memory latency) and masks them.  XOR is
 * order-independent, so the result is identical. */
CY_FN uint sobol_dimension(const CyGlobals *kg, int index, int dimension)
{
  uint result = 0;
  const uint i = (uint)index + SOBOL_SKIP;
  const uint *dirs = kg->__sample_pattern_lut + 32 * dimension;
  for (int base = 0; base < 32 && (i >> base) != 0u; base += 8) {
    uint v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      v[k] = dirs[base + k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      result ^= ((i >> (base + k)) & 1u) ? v[k] : 0u;
    }
  }
  return result;
}

CY_FN float path_rng_1D(const CyGlobals *kg, uint rng_hash, int sample, int dimension)
{
  uint result = sobol_dimension(kg, sample, dimension);
  float r = (float)result * (1.0f / (float)0xFFFFFFFF);
  uint tmp_rng = cmj_hash_simple((uint)dimension, rng_hash);
  float shift = (float)tmp_rng * (1.0f / (float)0xFFFFFFFF);
  return r + shift - floorf(r + shift);
}

CY_FN void path_rng_2D(
    const CyGlobals *kg, uint rng_hash, int sample, int dimension, float *fx, float *fy)
{
  *fx = path_rng_1D(kg, rng_hash, sample, dimension);
  *fy = path_rng_1D(kg, rng_hash, sample, dimension + 1);
}

CY_FN float path_state_rng_1D(const CyGlobals *kg, const CyPathState *s, int dimension)
{
  return path_rng_1D(kg, s->rng_hash, s->sample, s->rng_offset + dimension);
}

CY_FN void path_state_rng_2D(
    const CyGlobals *kg, const CyPathState *s, int dimension, float *fx, float *fy)
{
  path_rng_2D(kg, s->rng_hash, s->sample, s->rng_offset + dimension, fx, fy);
}

/* kernel_globals.h:213-227 */
CY_FN float lookup_table_read(const CyGlobals *kg, float x, int offset, int size)
{
  x = saturate(x) * (size - 1);
  int index = imin((int)x, size - 1);
  int nindex = imin(index + 1, size - 1);
  float t = x - index;
  float data0 = kg->__lookup_table[index + offset];
  if (t == 0.0f) {
    return data0;
  }
  float data1 = kg->__lookup_table[nindex + offset];
  return (1.0f - t) * data0 + t * data1;
}

/* ---------------------------------------------------------------------------
 * Camera: kernel_path_common.h:21-46 (kernel_path_trace_setup) and
 * kernel_camera.h:19-369: perspective, orthographic and panorama cameras
 * (equirectangular, fisheye equidistant / equisolid, mirror ball,
 * kernel_projection.h), depth of field with disk or polygonal apertures and
 * anamorphic ratio, near/far clipping.  Motion blur and stereo are rejected at
 * load_kernels.
 */
#define CY_M_PI_2_F 1.57079632679489661923f
#define CY_M_PI_4_F 0.785398163397448309616f

/* kernel_montecarlo.h:150-169 */
CY_FN void concentric_sample_disk(float u1, float u2, float *x, float *y)
{
  float phi, r;
  const float a = 2.0f * u1 - 1.0f;
  const float b = 2.0f * u2 - 1.0f;
  if (a == 0.0f && b == 0.0f) {
    *x = 0.0f;
    *y = 0.0f;
    return;
  }
  else if (a * a > b * b) {
    r = a;
    phi = CY_M_PI_4_F * (b / a);
  }
  else {
    r = b;
    phi = CY_M_PI_2_F - CY_M_PI_4_F * (a / b);
  }
  *x = r * cy_cosf(phi);
  *y = r * cy_sinf(phi);
}

/* kernel_montecarlo.h:172-194 */
CY_FN void regular_polygon_sample(float corners, float rotation, float u, float v, float *x, float *y)
{
  const float corner = floorf(u * corners);
  u = u * corners - corner;
  u = sqrtf(u);
  v = v * u;
  u = 1.0f - u;
  const float angle = CY_PI_F / corners;
  const float px = (u + v) * cy_cosf(angle);
  const float py = (u - v) * cy_sinf(angle);
  rotation += corner * 2.0f * angle;
  const float cr = cy_cosf(rotation);
  const float sr = cy_sinf(rotation);
  *x = cr * px - sr * py;
  *y = sr * px + cr * py;
}

/* kernel_camera.h:21-40 camera_sample_aperture, scaled by aperturesize */
CY_FN void camera_sample_aperture(const CyGlobals *kg, float u, float v, float *x, float *y)
{
  const float blades = KD->cam.blades;
  if (blades == 0.0f) {
    concentric_sample_disk(u, v, x, y);
  }
  else {
    regular_polygon_sample(blades, KD->cam.bladesrotation, u, v, x, y);
  }
  *x *= KD->cam.inv_aperture_ratio;
  const float size = KD->cam.aperturesize;
  *x = *x * size;
  *y = *y * size;
}

/* kernel_projection.h:64-71 equirectangular_range_to_direction */
CY_FN cfloat3 equirectangular_range_to_direction(float u, float v, hc_float4 range)
{
  const float phi = range.x * u + range.y;
  const float theta = range.z * v + range.w;
  const float sin_theta = cy_sinf(theta);
  return mk3(sin_theta * cy_cosf(phi), sin_theta * cy_sinf(phi), cy_cosf(theta));
}

/* kernel_projection.h:94-111 fisheye_to_direction */
CY_FN cfloat3 fisheye_to_direction(float u, float v, float fov)
{
  u = (u - 0.5f) * 2.0f;
  v = (v - 0.5f) * 2.0f;
  const float r = sqrtf(u * u + v * v);
  if (r > 1.0f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float phi = safe_acosf((r != 0.0f) ? u / r : 0.0f);
  const float theta = r * fov * 0.5f;
  if (v < 0.0f) {
    phi = -phi;
  }
  return mk3(cy_cosf(theta), -cy_cosf(phi) * cy_sinf(theta), cy_sinf(phi) * cy_sinf(theta));
}

/* kernel_projection.h:126-145 fisheye_equisolid_to_direction */
CY_FN cfloat3 fisheye_equisolid_to_direction(float u, float v, float lens, float fov, float width, float height)
{
  u = (u - 0.5f) * width;
  v = (v - 0.5f) * height;
  const float rmax = 2.0f * lens * cy_sinf(fov * 0.25f);
  const float r = sqrtf(u * u + v * v);
  if (r > rmax) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float phi = safe_acosf((r != 0.0f) ? u / r : 0.0f);
  const float theta = 2.0f * cy_asinf(r / (2.0f * lens));
  if (v < 0.0f) {
    phi = -phi;
  }
  return mk3(cy_cosf(theta), -cy_cosf(phi) * cy_sinf(theta), cy_sinf(phi) * cy_sinf(theta));
}

/* kernel_projection.h:149-166 mirrorball_to_direction */
CY_FN cfloat3 mirrorball_to_direction(float u, float v)
{
  cfloat3 dir;
  dir.x = 2.0f * u - 1.0f;
  dir.z = 2.0f * v - 1.0f;
  if (dir.x * dir.x + dir.z * dir.z > 1.0f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  dir.y = -sqrtf(fmaxf(1.0f - dir.x * dir.x - dir.z * dir.z, 0.0f));
  const cfloat3 I = mk3(0.0f, -1.0f, 0.0f);
  return sub3(mul3f(dir, 2.0f * dot3(dir, I)), I);
}

/* kernel_projection.h:184-199 panorama_to_direction */
CY_FN cfloat3 panorama_to_direction(const CyGlobals *kg, float u, float v)
{
  switch (KD->cam.panorama_type) {
    case 0: /* PANORAMA_EQUIRECTANGULAR */
      return equirectangular_range_to_direction(u, v, KD->cam.equirectangular_range);
    case 3: /* PANORAMA_MIRRORBALL */
      return mirrorball_to_direction(u, v);
    case 1: /* PANORAMA_FISHEYE_EQUIDISTANT */
      return fisheye_to_direction(u, v, KD->cam.fisheye_fov);
    case 2: /* PANORAMA_FISHEYE_EQUISOLID */
    default:
      return fisheye_equisolid_to_direction(u, v, KD->cam.fisheye_lens, KD->cam.fisheye_fov, KD->cam.sensorwidth,
                                            KD->cam.sensorheight);
  }
}

CY_FN void camera_sample_ray(const CyGlobals *kg, int x, int y, int sample, uint *rng_hash_out, CyRay *ray,
                             CyDiff3 *dP = nullptr, CyDiff3 *dD = nullptr)
{
  /* path_rng_init (kernel_random.h:129-153) */
  uint rng_hash = hash_uint2((uint)x, (uint)y);
  rng_hash ^= (uint)KD->integrator.seed;
  float filter_u, filter_v;
  if (sample == 0) {
    filter_u = 0.5f;
    filter_v = 0.5f;
  }
  else {
    path_rng_2D(kg, rng_hash, sample, PRNG_FILTER_U, &filter_u, &filter_v);
  }
  *rng_hash_out = rng_hash;
  float lens_u = 0.0f, lens_v = 0.0f;
  const bool dof = KD->cam.aperturesize > 0.0f;
  if (dof) {
    path_rng_2D(kg, rng_hash, sample, PRNG_LENS_U, &lens_u, &lens_v);
  }

  /* camera_sample (kernel_camera.h:296-356): pixel filter */
  const int filter_table_offset = KD->film.filter_table_offset;
  const float raster_x = x + lookup_table_read(kg, filter_u, filter_table_offset, FILTER_TABLE_SIZE);
  const float raster_y = y + lookup_table_read(kg, filter_v, filter_table_offset, FILTER_TABLE_SIZE);

  const struct cy_ptfm *rastertocamera = (const struct cy_ptfm *)&KD->cam.rastertocamera;
  const struct cy_tfm *cameratoworld = (const struct cy_tfm *)&KD->cam.cameratoworld;
  const cfloat3 Pcamera = transform_perspective(rastertocamera, mk3(raster_x, raster_y, 0.0f));
  const int type = KD->cam.type;
  if (type == 0) {
    /* camera_sample_perspective (kernel_camera.h:42-171) */
    cfloat3 P = mk3(0.0f, 0.0f, 0.0f);
    cfloat3 D = Pcamera;
    if (dof) {
      float lx, ly;
      camera_sample_aperture(kg, lens_u, lens_v, &lx, &ly);
      const float ft = KD->cam.focaldistance / D.z;
      const cfloat3 Pfocus = mul3f(D, ft);
      P = mk3(lx, ly, 0.0f);
      D = normalize3(sub3(Pfocus, P));
    }
    P = transform_point(cameratoworld, P);
    D = normalize3(transform_direction(cameratoworld, D));
    ray->P = P;
    ray->D = D;
    if (dP) {
      /* kernel_camera.h:114-120 */
      const cfloat3 Dcenter = transform_direction(cameratoworld, Pcamera);
      const cfloat3 cdx = mk3(KD->cam.dx.x, KD->cam.dx.y, KD->cam.dx.z);
      const cfloat3 cdy = mk3(KD->cam.dy.x, KD->cam.dy.y, KD->cam.dy.z);
      dP->dx = mk3(0.0f, 0.0f, 0.0f);
      dP->dy = mk3(0.0f, 0.0f, 0.0f);
      dD->dx = sub3(normalize3(add3(Dcenter, cdx)), normalize3(Dcenter));
      dD->dy = sub3(normalize3(add3(Dcenter, cdy)), normalize3(Dcenter));
    }
    /* camera clipping (__CAMERA_CLIPPING__) */
    const float z_inv = 1.0f / normalize3(Pcamera).z;
    const float nearclip = KD->cam.nearclip * z_inv;
    ray->P = add3(ray->P, mul3f(ray->D, nearclip));
    if (dP) {
      dP->dx = add3(dP->dx, mul3f(dD->dx, nearclip));
      dP->dy = add3(dP->dy, mul3f(dD->dy, nearclip));
    }
    ray->t = KD->cam.cliplength * z_inv;
  }
  else if (type == 1) {
    /* camera_sample_orthographic (kernel_camera.h:174-233) */
    cfloat3 P;
    cfloat3 D = mk3(0.0f, 0.0f, 1.0f);
    if (dof) {
      float lx, ly;
      camera_sample_aperture(kg, lens_u, lens_v, &lx, &ly);
      const cfloat3 Pfocus = mul3f(D, KD->cam.focaldistance);
      const cfloat3 lensuvw = mk3(lx, ly, 0.0f);
      P = add3(Pcamera, lensuvw);
      D = normalize3(sub3(Pfocus, lensuvw));
    }
    else {
      P = Pcamera;
    }
    ray->P = transform_point(cameratoworld, P);
    ray->D = normalize3(transform_direction(cameratoworld, D));
    if (dP) {
      /* kernel_camera.h:221-227 */
      dP->dx = mk3(KD->cam.dx.x, KD->cam.dx.y, KD->cam.dx.z);
      dP->dy = mk3(KD->cam.dy.x, KD->cam.dy.y, KD->cam.dy.z);
      dD->dx = mk3(0.0f, 0.0f, 0.0f);
      dD->dy = mk3(0.0f, 0.0f, 0.0f);
    }
    ray->t = KD->cam.cliplength;
  }
  else {
    /* camera_sample_panorama (kernel_camera.h:237-291) */
    cfloat3 P = mk3(0.0f, 0.0f, 0.0f);
    cfloat3 D = panorama_to_direction(kg, Pcamera.x, Pcamera.y);
    if (D.x == 0.0f && D.y == 0.0f && D.z == 0.0f) {
      /* outside the lens: no camera ray */
      ray->P = P;
      ray->D = D;
      ray->t = 0.0f;
      return;
    }
    if (dof) {
      float lx, ly;
      camera_sample_aperture(kg, lens_u, lens_v, &lx, &ly);
      const cfloat3 Dfocus = normalize3(D);
      const cfloat3 Pfocus = mul3f(Dfocus, KD->cam.focaldistance);
      const cfloat3 U = normalize3(sub3(mk3(1.0f, 0.0f, 0.0f), mul3f(Dfocus, Dfocus.x)));
      const cfloat3 V = normalize3(cross3(Dfocus, U));
      P = add3(mul3f(U, lx), mul3f(V, ly));
      D = normalize3(sub3(Pfocus, P));
    }
    P = transform_point(cameratoworld, P);
    D = normalize3(transform_direction(cameratoworld, D));
    ray->P = P;
    ray->D = D;
    if (dP) {
      /* kernel_camera.h:305-339: the centre and the two neighbouring pixels'
       * rays (without depth of field) */
      const cfloat3 Pcenter = transform_point(cameratoworld, Pcamera);
      const cfloat3 Dcenter =
          normalize3(transform_direction(cameratoworld, panorama_to_direction(kg, Pcamera.x, Pcamera.y)));
      const cfloat3 Px0 = transform_perspective(rastertocamera, mk3(raster_x + 1.0f, raster_y, 0.0f));
      const cfloat3 Dx = normalize3(transform_direction(cameratoworld, panorama_to_direction(kg, Px0.x, Px0.y)));
      const cfloat3 Px = transform_point(cameratoworld, Px0);
      dP->dx = sub3(Px, Pcenter);
      dD->dx = sub3(Dx, Dcenter);
      const cfloat3 Py0 = transform_perspective(rastertocamera, mk3(raster_x, raster_y + 1.0f, 0.0f));
      const cfloat3 Dy = normalize3(transform_direction(cameratoworld, panorama_to_direction(kg, Py0.x, Py0.y)));
      const cfloat3 Py = transform_point(cameratoworld, Py0);
      dP->dy = sub3(Py, Pcenter);
      dD->dy = sub3(Dy, Dcenter);
    }
    const float nearclip = KD->cam.nearclip;
    ray->P = add3(ray->P, mul3f(ray->D, nearclip));
    if (dP) {
      dP->dx = add3(dP->dx, mul3f(dD->dx, nearclip));
      dP->dy = add3(dP->dy, mul3f(dD->dy, nearclip));
    }
    ray->t = KD->cam.cliplength;
  }
}

/* ---------------------------------------------------------------------------
 * BVH2 traversal over the packed Cycles layout (bvh/bvh_traversal.h:34-227,
 * bvh_nodes.h:31-77, geom_triangle_intersect.h:25-72, util_math_intersect.h:88-195).
 * Two-level: instance leaves enter an object's own BVH in object space.
 */
CY_FN cfloat3 bvh_clamp_direction(cfloat3 dir)
{
  const float ooeps = 8.271806E-25f;
  return mk3((fabsf(dir.x) > ooeps) ? dir.x : copysignf(ooeps, dir.x),
             (fabsf(dir.y) > ooeps) ? dir.y : copysignf(ooeps, dir.y),
             (fabsf(dir.z) > ooeps) ? dir.z : copysignf(ooeps, dir.z));
}

/* ray_triangle_intersect against the bound ray_t, also reporting whether the
 * hit passes the same test against a second bound t_exact (cy_bvhw.h: hits
 * are collected against a widened bound and judged at the exact one). */
CY_FN bool ray_triangle_intersect2(cfloat3 P,
                                   cfloat3 dir,
                                   float ray_t,
                                   float t_exact,
                                   cfloat3 tri_a,
                                   cfloat3 tri_b,
                                   cfloat3 tri_c,
                                   float *isect_u,
                                   float *isect_v,
                                   float *isect_t,
                                   bool *exact_ok)
{
  const cfloat3 v0 = sub3(tri_c, P);
  const cfloat3 v1 = sub3(tri_a, P);
  const cfloat3 v2 = sub3(tri_b, P);
  const cfloat3 e0 = sub3(v2, v0);
  const cfloat3 e1 = sub3(v0, v1);
  const cfloat3 e2 = sub3(v1, v2);
  const float U = dot3(cross3(add3(v2, v0), e0), dir);
  const float V = dot3(cross3(add3(v0, v1), e1), dir);
  const float W = dot3(cross3(add3(v1, v2), e2), dir);
  const float minUVW = cmin(U, cmin(V, W));
  const float maxUVW = cmax(U, cmax(V, W));
  if (minUVW < 0.0f && maxUVW > 0.0f) {
    return false;
  }
  const cfloat3 Ng1 = cross3(e1, e0);
  const cfloat3 Ng = add3(Ng1, Ng1);
  const float den = dot3(Ng, dir);
  if (den == 0.0f) {
    return false;
  }
  const float T = dot3(v0, Ng);
  const int sign_den = (as_int(den) & 0x80000000);
  const float sign_T = xor_signmask(T, sign_den);
  const float abs_den = xor_signmask(den, sign_den);
  if ((sign_T < 0.0f) || (sign_T > ray_t * abs_den)) {
    return false;
  }
  *exact_ok = !(sign_T > t_exact * abs_den);
  const float inv_den = 1.0f / den;
  *isect_u = U * inv_den;
  *isect_v = V * inv_den;
  *isect_t = T * inv_den;
  return true;
}

/* util/util_math_intersect.h:88-195 (ray_triangle_intersect, the
 * non-SSE/watertight-style path the generic x86 kernel compiles). */
CY_FN bool ray_triangle_intersect(cfloat3 P,
                                  cfloat3 dir,
                                  float ray_t,
                                  cfloat3 tri_a,
                                  cfloat3 tri_b,
                                  cfloat3 tri_c,
                                  float *isect_u,
                                  float *isect_v,
                                  float *isect_t)
{
  bool exact_ok;
  return ray_triangle_intersect2(P, dir, ray_t, ray_t, tri_a, tri_b, tri_c, isect_u, isect_v, isect_t, &exact_ok);
}

CY_FN bool scene_intersect_valid(const CyRay *ray)
{
  return isfinite_safe(ray->P.x) && isfinite_safe(ray->D.x) && len_squared3(ray->D) != 0.0f;
}

/* Closest hit (any_hit == false) or opaque-shadow any hit (any_hit == true).
 * Returns true on hit; counters (when non-null) gather traversal statistics for
 * the algorithmic-bytes roofline (inner nodes, leaves, triangle tests). */
/* Traversal stack (bvh_types.h:30-33: 192 entries).  On the device the first
 * CY_LDS_STACK entries live in LDS, one column per thread (entry i of thread t
 * at lds_base[i * CY_BLOCK + t]: 64 consecutive lanes hit 64 consecutive dwords,
 * conflict-free); deeper entries spill to a private array that is only touched
 * by rays descending more than CY_LDS_STACK levels below their stack bottom. */
/* The stack is a pair of locals of bvh2_intersect (an LDS column pointer and
 * the private spill array), never an object whose address is taken, so the
 * compiler keeps the pointer in a register and uses ds_* for the LDS part. */

/* Object transforms (geom/geom_object.h:37-48): static objects only. */
CY_FN const struct cy_tfm *object_tfm(const CyGlobals *kg, int object)
{
  return (const struct cy_tfm *)&kg->__objects[object].tfm;
}
CY_FN const struct cy_tfm *object_itfm(const CyGlobals *kg, int object)
{
  return (const struct cy_tfm *)&kg->__objects[object].itfm;
}

/* bvh_instance_push / bvh_instance_pop (geom/geom_object.h:425-470): the ray
 * enters an instance in object space, its t scaled by the direction length. */
CY_FN float bvh_instance_push(
    const CyGlobals *kg, int object, const CyRay *ray, cfloat3 *P, cfloat3 *dir, cfloat3 *idir, float t)
{
  const struct cy_tfm *tfm = object_itfm(kg, object);
  *P = transform_point(tfm, ray->P);
  float len;
  *dir = bvh_clamp_direction(normalize_len3(transform_direction(tfm, ray->D), &len));
  *idir = rcp3(*dir);
  if (t != CY_FLT_MAX) {
    t *= len;
  }
  return t;
}

CY_FN float bvh_instance_pop(
    const CyGlobals *kg, int object, const CyRay *ray, cfloat3 *P, cfloat3 *dir, cfloat3 *idir, float t)
{
  if (t != CY_FLT_MAX) {
    t /= len3(transform_direction(object_itfm(kg, object), ray->D));
  }
  *P = ray->P;
  *dir = bvh_clamp_direction(ray->D);
  *idir = rcp3(*dir);
  return t;
}

#include "cy_curve.h"

/* One BVH2 inner node (bvh_nodes.h): the aligned two-child slab test
 * (bvh_aligned_node_intersect :31-77) or, in scenes with curves, the
 * oriented-box test of a node whose first word carries PATH_RAY_NODE_UNALIGNED
 * (bvh_unaligned_node_intersect :79-135: each child's box is the unit cube in
 * the affine space stored for it, 7 float4 per node).  Returns the traverse
 * mask; dist = entry distances. */
CY_FN bool bvh_obb_intersect(hc_float4 sx, hc_float4 sy, hc_float4 sz, cfloat3 P, cfloat3 dir, float t, float *dist)
{
  struct cy_tfm space;
  space.x.x = sx.x, space.x.y = sx.y, space.x.z = sx.z, space.x.w = sx.w;
  space.y.x = sy.x, space.y.y = sy.y, space.y.z = sy.z, space.y.w = sy.w;
  space.z.x = sz.x, space.z.y = sz.y, space.z.z = sz.z, space.z.w = sz.w;
  const cfloat3 aligned_dir = transform_direction(&space, dir);
  const cfloat3 aligned_P = transform_point(&space, P);
  const cfloat3 nrdir = neg3(rcp3(aligned_dir));
  const cfloat3 lower_xyz = mul3(aligned_P, nrdir);
  const cfloat3 upper_xyz = sub3(lower_xyz, nrdir);
  const float near_x = cmin(lower_xyz.x, upper_xyz.x);
  const float near_y = cmin(lower_xyz.y, upper_xyz.y);
  const float near_z = cmin(lower_xyz.z, upper_xyz.z);
  const float far_x = cmax(lower_xyz.x, upper_xyz.x);
  const float far_y = cmax(lower_xyz.y, upper_xyz.y);
  const float far_z = cmax(lower_xyz.z, upper_xyz.z);
  const float tnear = max4(0.0f, near_x, near_y, near_z);
  const float tfar = min4(t, far_x, far_y, far_z);
  *dist = tnear;
  return tnear <= tfar;
}

CY_FN bool bvh_unaligned_node_intersect_child(const hc_float4 *nodes, int node_addr, int child, cfloat3 P,
                                              cfloat3 dir, float t, float *dist)
{
  const int child_addr = node_addr + child * 3;
  return bvh_obb_intersect(nodes[child_addr + 1], nodes[child_addr + 2], nodes[child_addr + 3], P, dir, t, dist);
}

template<int HAIR>
CY_FN int bvh2_node_intersect(const hc_float4 *nodes, int node_addr, hc_float4 cnodes, cfloat3 P, cfloat3 dir,
                              cfloat3 idir, float t, uint visibility, float *c0min_o, float *c1min_o)
{
  if (HAIR != 0 && (as_uint(cnodes.x) & PATH_RAY_NODE_UNALIGNED)) {
    int mask = 0;
    if (bvh_unaligned_node_intersect_child(nodes, node_addr, 0, P, dir, t, c0min_o)) {
      if (as_uint(cnodes.x) & visibility) {
        mask |= 1;
      }
    }
    if (bvh_unaligned_node_intersect_child(nodes, node_addr, 1, P, dir, t, c1min_o)) {
      if (as_uint(cnodes.y) & visibility) {
        mask |= 2;
      }
    }
    return mask;
  }
  const hc_float4 node0 = nodes[node_addr + 1];
  const hc_float4 node1 = nodes[node_addr + 2];
  const hc_float4 node2 = nodes[node_addr + 3];
  float c0lox = (node0.x - P.x) * idir.x;
  float c0hix = (node0.z - P.x) * idir.x;
  float c0loy = (node1.x - P.y) * idir.y;
  float c0hiy = (node1.z - P.y) * idir.y;
  float c0loz = (node2.x - P.z) * idir.z;
  float c0hiz = (node2.z - P.z) * idir.z;
  float c0min = max4(0.0f, cmin(c0lox, c0hix), cmin(c0loy, c0hiy), cmin(c0loz, c0hiz));
  float c0max = min4(t, cmax(c0lox, c0hix), cmax(c0loy, c0hiy), cmax(c0loz, c0hiz));
  float c1lox = (node0.y - P.x) * idir.x;
  float c1hix = (node0.w - P.x) * idir.x;
  float c1loy = (node1.y - P.y) * idir.y;
  float c1hiy = (node1.w - P.y) * idir.y;
  float c1loz = (node2.y - P.z) * idir.z;
  float c1hiz = (node2.w - P.z) * idir.z;
  float c1min = max4(0.0f, cmin(c1lox, c1hix), cmin(c1loy, c1hiy), cmin(c1loz, c1hiz));
  float c1max = min4(t, cmax(c1lox, c1hix), cmax(c1loy, c1hiy), cmax(c1loz, c1hiz));
  *c0min_o = c0min;
  *c1min_o = c1min;
  return (((c0max >= c0min) && (as_uint(cnodes.x) & visibility)) ? 1 : 0) |
         (((c1max >= c1min) && (as_uint(cnodes.y) & visibility)) ? 2 : 0);
}

/* Resumable traversal (iteration budget, hipcy_set_traversal_budget): the
 * position of a traversal that ran out of iterations -- the next stack code to
 * process, the LDS ring's top and fill, the near-tie flag -- so that it can
 * continue in a later launch, bit for bit as if it had not stopped.  The ring
 * entries themselves are saved and restored by the caller (hipcycles.hip
 * cont_save / cont_load).  A traversal with entries in the private overflow
 * arrays never suspends. */
struct CyTravCursor {
  int code;
  float code_t; /* entry distance of code's box */
  int top;
  int n_ring;
  bool tie;
  bool suspended;
};

/* Forward declaration: the wide traversal of one instance's BVH (cy_bvhw.h). */
template<int W, bool any_hit, int HAIR = 0>
CY_FN bool bvhw_traverse(const CyGlobals *kg, int root, cfloat3 P, cfloat3 dir, cfloat3 idir, int object,
                         uint visibility, CyIsect *isect, uint *err, uint *cnt_nodes, uint *cnt_leaves,
                         uint *cnt_tris, CY_LDS CyStackEntry *lds_ring, bool *tie_out, int budget = 0,
                         CyTravCursor *cur = nullptr, CY_LDS const hc_float4 *top_nodes = nullptr,
                         int n_top = 0);

/* Closest hit / opaque any hit with the bound BVH2 in the reference's order
 * (bvh/bvh_traversal.h:34-227).  The first LDSN stack entries live in LDS,
 * entry i of this thread at lds_stack[i * LDS_STRIDE] (ints).
 *
 * WI > 2 (instanced scenes with the device's wide BVH): the top level is
 * traversed here, in the reference's order, and each instance entered is
 * traversed with the W-wide BVH of its object (bvhw_traverse from the object's
 * wide root, object space).  The closest hit inside one instance does not
 * depend on the visiting order (near-ties excepted: *tie, see bvhw_traverse), so
 * the sequence of instances entered -- and with it every bvh_instance_push/pop
 * rounding of t -- is the reference's. */
/* HAIR: 0 triangles only, else the curve shapes compiled in (curve_intersect). */
template<bool any_hit, bool INST = true, int WI = 2, int LDSN = CY_LDS_STACK, int LDS_STRIDE = CY_BLOCK,
         int HAIR = 0>
CY_FN bool bvh2_intersect(const CyGlobals *kg,
                          const CyRay *ray,
                          uint visibility,
                          CyIsect *isect,
                          uint *err,
                          uint *cnt_nodes,
                          uint *cnt_leaves,
                          uint *cnt_tris,
                          CY_LDS int *lds_stack = nullptr,
                          CY_LDS CyStackEntry *lds_ring = nullptr,
                          bool *tie = nullptr)
{
  int stack_spill[BVH_STACK_SIZE];
  auto stack_set = [&](int i, int v) {
    if (lds_stack && i < LDSN) {
      lds_stack[i * LDS_STRIDE] = v;
    }
    else {
      stack_spill[i] = v;
    }
  };
  auto stack_get = [&](int i) -> int { return (lds_stack && i < LDSN) ? lds_stack[i * LDS_STRIDE] : stack_spill[i]; };
  stack_set(0, ENTRYPOINT_SENTINEL);
  int stack_ptr = 0;
  int node_addr = KD->bvh.root;
  int object = OBJECT_NONE;
  cfloat3 P = ray->P;
  cfloat3 dir = bvh_clamp_direction(ray->D);
  cfloat3 idir = rcp3(dir);

  isect->t = ray->t;
  isect->u = 0.0f;
  isect->v = 0.0f;
  isect->prim = PRIM_NONE;
  isect->object = OBJECT_NONE;
  isect->type = 0;

  uint n_nodes = 0, n_leaves = 0, n_tris = 0;
  const hc_float4 *nodes = kg->__bvh_nodes;

  do {
    do {
      while (node_addr >= 0 && node_addr != ENTRYPOINT_SENTINEL) {
        n_nodes++;
        const hc_float4 cnodes = nodes[node_addr + 0];
        float c0min, c1min;
        const int traverse_mask = bvh2_node_intersect<HAIR>(nodes, node_addr, cnodes, P, dir, idir, isect->t,
                                                            visibility, &c0min, &c1min);

        node_addr = as_int(cnodes.z);
        int node_addr_child1 = as_int(cnodes.w);

        if (traverse_mask == 3) {
          bool is_closest_child1 = (c1min < c0min);
          if (is_closest_child1) {
            int tmp = node_addr;
            node_addr = node_addr_child1;
            node_addr_child1 = tmp;
          }
          ++stack_ptr;
          if (stack_ptr >= BVH_STACK_SIZE) {
            cy_set_error(err, CY_ERR_BVH_STACK, 0);
            return false;
          }
          stack_set(stack_ptr, node_addr_child1);
        }
        else {
          if (traverse_mask == 2) {
            node_addr = node_addr_child1;
          }
          else if (traverse_mask == 0) {
            node_addr = stack_get(stack_ptr);
            --stack_ptr;
          }
        }
      }

      if (node_addr < 0) {
        n_leaves++;
        const hc_float4 leaf = kg->__bvh_leaf_nodes[-node_addr - 1];
        int prim_addr = as_int(leaf.x);
        if (prim_addr >= 0) {
          const int prim_addr2 = as_int(leaf.y);
          const uint type = as_uint(leaf.w);
          node_addr = stack_get(stack_ptr);
          --stack_ptr;
          if ((type & PRIMITIVE_ALL) == PRIMITIVE_TRIANGLE) {
            for (; prim_addr < prim_addr2; prim_addr++) {
              n_tris++;
              const uint tri_vindex = kg->__prim_tri_index[prim_addr];
              const hc_float4 *tv = kg->__prim_tri_verts + tri_vindex;
              float tt, uu, vv;
              if (ray_triangle_intersect(
                      P, dir, isect->t, f4to3(tv[0]), f4to3(tv[1]), f4to3(tv[2]), &uu, &vv, &tt)) {
                if (kg->__prim_visibility[prim_addr] & visibility) {
                  isect->prim = prim_addr;
                  isect->object = object;
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
          else if (HAIR != 0 && (type & PRIMITIVE_ALL_CURVE)) {
            /* curve segments (bvh_traversal.h:166-184) */
            for (; prim_addr < prim_addr2; prim_addr++) {
              n_tris++;
              const uint curve_type = kg->__prim_type[prim_addr];
              if (curve_intersect<HAIR>(kg, isect, P, dir, visibility, object, prim_addr, curve_type) && any_hit) {
                if (cnt_nodes) {
                  *cnt_nodes += n_nodes;
                  *cnt_leaves += n_leaves;
                  *cnt_tris += n_tris;
                }
                return true;
              }
            }
          }
          else {
            cy_set_error(err, CY_ERR_PRIMITIVE, type);
          }
        }
        else if (!INST) {
          cy_set_error(err, CY_ERR_FEATURE, 1); /* instance leaf in a kernel built without instancing */
          return false;
        }
        else {
          /* instance push (bvh_traversal.h:190-205) */
          object = (int)kg->__prim_object[-prim_addr - 1];
          isect->t = bvh_instance_push(kg, object, ray, &P, &dir, &idir, isect->t);
          if constexpr (WI > 2) {
            /* the instance's own BVH, wide; then the instance pop and the
             * top-level continuation, as the reference does at the sentinel */
            const bool h = bvhw_traverse<WI, any_hit, HAIR>(kg, kg->bvhw_object_root[object], P, dir, idir, object,
                                                       visibility, isect, err, cnt_nodes, cnt_leaves, cnt_tris,
                                                       lds_ring, tie);
            if (any_hit && h) {
              if (cnt_nodes) {
                *cnt_nodes += n_nodes;
                *cnt_leaves += n_leaves;
                *cnt_tris += n_tris;
              }
              return true;
            }
            isect->t = bvh_instance_pop(kg, object, ray, &P, &dir, &idir, isect->t);
            object = OBJECT_NONE;
            node_addr = stack_get(stack_ptr);
            --stack_ptr;
            continue;
          }
          ++stack_ptr;
          if (stack_ptr >= BVH_STACK_SIZE) {
            cy_set_error(err, CY_ERR_BVH_STACK, 0);
            return false;
          }
          stack_set(stack_ptr, ENTRYPOINT_SENTINEL);
          node_addr = (int)kg->__object_node[object];
        }
      }
    } while (node_addr != ENTRYPOINT_SENTINEL);

    if (INST && stack_ptr >= 0) {
      /* instance pop (bvh_traversal.h:209-222) */
      isect->t = bvh_instance_pop(kg, object, ray, &P, &dir, &idir, isect->t);
      object = OBJECT_NONE;
      node_addr = stack_get(stack_ptr);
      --stack_ptr;
    }
  } while (node_addr != ENTRYPOINT_SENTINEL);

  if (cnt_nodes) {
    *cnt_nodes += n_nodes;
    *cnt_leaves += n_leaves;
    *cnt_tris += n_tris;
  }
  return (isect->prim != PRIM_NONE);
}

/* Record-all shadow traversal with the bound BVH2 in the reference's order
 * (bvh/bvh_shadow_all.h:40-258): every primitive hit within the ray is recorded
 * (hits holds max_hits + 1 entries) until one whose shader has no transparent
 * shadow, or more than max_hits of them, blocks the light.  Hits inside an
 * instance get their t scaled to world space at the instance pop. */
template<bool INST, int HAIR = 0>
CY_FN bool bvh2_shadow_all(const CyGlobals *kg,
                           const CyRay *ray,
                           CyIsect *hits,
                           uint visibility,
                           uint max_hits,
                           uint *num_hits,
                           uint *err)
{
  int stack[BVH_STACK_SIZE];
  stack[0] = ENTRYPOINT_SENTINEL;
  int stack_ptr = 0;
  int node_addr = KD->bvh.root;
  const float tmax = ray->t;
  cfloat3 P = ray->P;
  cfloat3 dir = bvh_clamp_direction(ray->D);
  cfloat3 idir = rcp3(dir);
  int object = OBJECT_NONE;
  float isect_t = tmax;
  int num_hits_in_instance = 0;
  *num_hits = 0;
  const hc_float4 *nodes = kg->__bvh_nodes;
  do {
    do {
      while (node_addr >= 0 && node_addr != ENTRYPOINT_SENTINEL) {
        const hc_float4 cnodes = nodes[node_addr + 0];
        float c0min, c1min;
        const int traverse_mask = bvh2_node_intersect<HAIR>(nodes, node_addr, cnodes, P, dir, idir, isect_t,
                                                            visibility, &c0min, &c1min);
        node_addr = as_int(cnodes.z);
        int node_addr_child1 = as_int(cnodes.w);
        if (traverse_mask == 3) {
          if (c1min < c0min) {
            const int tmp = node_addr;
            node_addr = node_addr_child1;
            node_addr_child1 = tmp;
          }
          if (++stack_ptr >= BVH_STACK_SIZE) {
            cy_set_error(err, CY_ERR_BVH_STACK, 0);
            return true;
          }
          stack[stack_ptr] = node_addr_child1;
        }
        else if (traverse_mask == 2) {
          node_addr = node_addr_child1;
        }
        else if (traverse_mask == 0) {
          node_addr = stack[stack_ptr];
          --stack_ptr;
        }
      }
      if (node_addr < 0) {
        const hc_float4 leaf = kg->__bvh_leaf_nodes[-node_addr - 1];
        int prim_addr = as_int(leaf.x);
        if (prim_addr >= 0) {
          const int prim_addr2 = as_int(leaf.y);
          const uint type = as_uint(leaf.w);
          node_addr = stack[stack_ptr];
          --stack_ptr;
          const bool curves = HAIR != 0 && (type & PRIMITIVE_ALL_CURVE);
          if ((type & PRIMITIVE_ALL) != PRIMITIVE_TRIANGLE && !curves) {
            cy_set_error(err, CY_ERR_PRIMITIVE, type);
            return true;
          }
          for (; prim_addr < prim_addr2; prim_addr++) {
            CyIsect *h = &hits[*num_hits];
            bool hit;
            int shader;
            if (curves) {
              /* bvh_shadow_all.h:161-169: the record's t bounds the curve test */
              h->t = isect_t;
              hit = curve_intersect<HAIR>(kg, h, P, dir, visibility, object, prim_addr, kg->__prim_type[prim_addr]);
              shader = hit ? as_int(kg->__curves[kg->__prim_index[prim_addr]].z) : 0;
            }
            else {
              const uint tri_vindex = kg->__prim_tri_index[prim_addr];
              const hc_float4 *tv = kg->__prim_tri_verts + tri_vindex;
              float tt, uu, vv;
              hit = ray_triangle_intersect(P, dir, isect_t, f4to3(tv[0]), f4to3(tv[1]), f4to3(tv[2]), &uu, &vv,
                                           &tt) &&
                    (kg->__prim_visibility[prim_addr] & visibility);
              if (hit) {
                h->prim = prim_addr;
                h->object = object;
                h->type = PRIMITIVE_TRIANGLE;
                h->u = uu;
                h->v = vv;
                h->t = tt;
              }
              shader = hit ? (int)kg->__tri_shader[kg->__prim_index[prim_addr]] : 0;
            }
            if (hit) {
              const int flag = kg->__shaders[shader & SHADER_MASK].flags;
              if (!(flag & SD_HAS_TRANSPARENT_SHADOW)) {
                return true;
              }
              if (*num_hits == max_hits) {
                return true;
              }
              (*num_hits)++;
              num_hits_in_instance++;
            }
          }
        }
        else if (!INST) {
          cy_set_error(err, CY_ERR_FEATURE, 1);
          return true;
        }
        else {
          /* instance push */
          object = (int)kg->__prim_object[-prim_addr - 1];
          isect_t = bvh_instance_push(kg, object, ray, &P, &dir, &idir, isect_t);
          num_hits_in_instance = 0;
          if (++stack_ptr >= BVH_STACK_SIZE) {
            cy_set_error(err, CY_ERR_BVH_STACK, 0);
            return true;
          }
          stack[stack_ptr] = ENTRYPOINT_SENTINEL;
          node_addr = (int)kg->__object_node[object];
        }
      }
    } while (node_addr != ENTRYPOINT_SENTINEL);
    if (INST && stack_ptr >= 0) {
      /* instance pop: recorded t back to world space (bvh_instance_pop_factor) */
      if (num_hits_in_instance) {
        const float t_fac = 1.0f / len3(transform_direction(object_itfm(kg, object), ray->D));
        for (int i = 0; i < num_hits_in_instance; i++) {
          hits[*num_hits - 1 - i].t *= t_fac;
        }
        P = ray->P;
        dir = bvh_clamp_direction(ray->D);
        idir = rcp3(dir);
      }
      else {
        bvh_instance_pop(kg, object, ray, &P, &dir, &idir, CY_FLT_MAX);
      }
      isect_t = tmax;
      object = OBJECT_NONE;
      node_addr = stack[stack_ptr];
      --stack_ptr;
    }
  } while (node_addr != ENTRYPOINT_SENTINEL);
  return false;
}

#if CY_CLOSURE_EXT
/* scene_intersect_volume_all (bvh/bvh.h:500-531, bvh/bvh_volume_all.h:38-327)
 * on the BVH2: every triangle of an object with a volume (SD_OBJECT_HAS_VOLUME)
 * the ray crosses within its own t, recorded in traversal order up to max_hits;
 * instances without a volume are not entered, curves are never recorded.  Hits
 * inside an instance get their t scaled to world space at the pop (or when
 * max_hits ends the query inside it).  Returns the number of hits. */
template<bool INST, int HAIR = 0>
CY_FN uint bvh2_volume_all(const CyGlobals *kg, const CyRay *ray, CyIsect *hits, uint max_hits, uint visibility,
                           uint *err)
{
  int stack[BVH_STACK_SIZE];
  stack[0] = ENTRYPOINT_SENTINEL;
  int stack_ptr = 0;
  int node_addr = KD->bvh.root;
  const float tmax = ray->t;
  cfloat3 P = ray->P;
  cfloat3 dir = bvh_clamp_direction(ray->D);
  cfloat3 idir = rcp3(dir);
  int object = OBJECT_NONE;
  float isect_t = tmax;
  uint num_hits_in_instance = 0;
  uint num_hits = 0;
  const hc_float4 *nodes = kg->__bvh_nodes;
  do {
    do {
      while (node_addr >= 0 && node_addr != ENTRYPOINT_SENTINEL) {
        const hc_float4 cnodes = nodes[node_addr + 0];
        float c0min, c1min;
        const int traverse_mask = bvh2_node_intersect<HAIR>(nodes, node_addr, cnodes, P, dir, idir, isect_t,
                                                            visibility, &c0min, &c1min);
        node_addr = as_int(cnodes.z);
        int node_addr_child1 = as_int(cnodes.w);
        if (traverse_mask == 3) {
          if (c1min < c0min) {
            const int tmp = node_addr;
            node_addr = node_addr_child1;
            node_addr_child1 = tmp;
          }
          if (++stack_ptr >= BVH_STACK_SIZE) {
            cy_set_error(err, CY_ERR_BVH_STACK, 0);
            return num_hits;
          }
          stack[stack_ptr] = node_addr_child1;
        }
        else if (traverse_mask == 2) {
          node_addr = node_addr_child1;
        }
        else if (traverse_mask == 0) {
          node_addr = stack[stack_ptr];
          --stack_ptr;
        }
      }
      if (node_addr < 0) {
        const hc_float4 leaf = kg->__bvh_leaf_nodes[-node_addr - 1];
        int prim_addr = as_int(leaf.x);
        if (prim_addr >= 0) {
          const int prim_addr2 = as_int(leaf.y);
          const uint type = as_uint(leaf.w);
          node_addr = stack[stack_ptr];
          --stack_ptr;
          if ((type & PRIMITIVE_ALL) == PRIMITIVE_TRIANGLE) {
            for (; prim_addr < prim_addr2; prim_addr++) {
              const int tri_object = (object == OBJECT_NONE) ? (int)kg->__prim_object[prim_addr] : object;
              if (!(kg->__object_flag[tri_object] & SD_OBJECT_HAS_VOLUME)) {
                continue;
              }
              const uint tri_vindex = kg->__prim_tri_index[prim_addr];
              const hc_float4 *tv = kg->__prim_tri_verts + tri_vindex;
              float tt, uu, vv;
              if (ray_triangle_intersect(P, dir, isect_t, f4to3(tv[0]), f4to3(tv[1]), f4to3(tv[2]), &uu, &vv,
                                         &tt) &&
                  (kg->__prim_visibility[prim_addr] & visibility)) {
                CyIsect *h = &hits[num_hits];
                h->prim = prim_addr;
                h->object = object;
                h->type = PRIMITIVE_TRIANGLE;
                h->u = uu;
                h->v = vv;
                h->t = tt;
                num_hits++;
                num_hits_in_instance++;
                if (num_hits == max_hits) {
                  if (INST && object != OBJECT_NONE) {
                    /* bvh_volume_all.h:180-186 scales by the instance-space direction here */
                    const float t_fac = 1.0f / len3(transform_direction(object_itfm(kg, object), dir));
                    for (uint i = 0; i < num_hits_in_instance; i++) {
                      hits[num_hits - 1 - i].t *= t_fac;
                    }
                  }
                  return num_hits;
                }
              }
            }
          }
          else if (!(HAIR != 0 && (type & PRIMITIVE_ALL_CURVE))) {
            cy_set_error(err, CY_ERR_PRIMITIVE, type);
            return num_hits;
          }
        }
        else if (!INST) {
          cy_set_error(err, CY_ERR_FEATURE, 1);
          return num_hits;
        }
        else {
          object = (int)kg->__prim_object[-prim_addr - 1];
          if (kg->__object_flag[object] & SD_OBJECT_HAS_VOLUME) {
            /* instance push */
            isect_t = bvh_instance_push(kg, object, ray, &P, &dir, &idir, isect_t);
            num_hits_in_instance = 0;
            if (++stack_ptr >= BVH_STACK_SIZE) {
              cy_set_error(err, CY_ERR_BVH_STACK, 0);
              return num_hits;
            }
            stack[stack_ptr] = ENTRYPOINT_SENTINEL;
            node_addr = (int)kg->__object_node[object];
          }
          else {
            object = OBJECT_NONE;
            node_addr = stack[stack_ptr];
            --stack_ptr;
          }
        }
      }
    } while (node_addr != ENTRYPOINT_SENTINEL);
    if (INST && stack_ptr >= 0) {
      /* instance pop */
      if (num_hits_in_instance) {
        const float t_fac = 1.0f / len3(transform_direction(object_itfm(kg, object), ray->D));
        for (uint i = 0; i < num_hits_in_instance; i++) {
          hits[num_hits - 1 - i].t *= t_fac;
        }
        P = ray->P;
        dir = bvh_clamp_direction(ray->D);
        idir = rcp3(dir);
      }
      else {
        bvh_instance_pop(kg, object, ray, &P, &dir, &idir, CY_FLT_MAX);
      }
      isect_t = tmax;
      object = OBJECT_NONE;
      node_addr = stack[stack_ptr];
      --stack_ptr;
    }
  } while (node_addr != ENTRYPOINT_SENTINEL);
  return num_hits;
}
#endif

/* Record-all shadow traversal of the W-wide layout (non-instanced scenes;
 * kg->bvhw_width 4 or 8, oriented-box nodes in ribbon scenes): the query of
 * bvh2_shadow_all above with the same bound (the ray's own t, which no
 * recorded hit shortens), the same slab arithmetic on the same boxes and the
 * same primitive tests, so it records the same set of hits and blocks on the
 * same conditions (an occluder without transparent shadow, or more than
 * max_hits hits) -- only the recording order differs, which the caller's
 * sort by distance removes unless two hits share a distance
 * (shadow_blocked_transparent then repeats the query in the BVH2's order). */
#ifndef CY_SHADOW_WIDE_STACK
#  define CY_SHADOW_WIDE_STACK 96
#endif
template<int HAIR>
CY_FN bool bvhw_shadow_all(const CyGlobals *kg, const CyRay *ray, CyIsect *hits, uint visibility, uint max_hits,
                           uint *num_hits, uint *err)
{
  const int Q = kg->bvhw_width >> 2;
  const hc_float4 *nodes = (const hc_float4 *)kg->bvhw_nodes;
  const float tmax = ray->t;
  const cfloat3 P = ray->P;
  const cfloat3 dir = bvh_clamp_direction(ray->D);
  const cfloat3 idir = rcp3(dir);
  int stack[CY_SHADOW_WIDE_STACK];
  int sp = 0;
  int code = 0;
  *num_hits = 0;
  while (true) {
    if (code >= 0) {
      /* the node's hit children, visited nearest first (an occluder that
       * blocks the light then ends the query early, as in the BVH2's order) */
      const bool obb = HAIR != 0 && (code & (1 << 30));
      const hc_float4 *np = nodes + (size_t)(code & ~(1 << 30)) * (size_t)(8 * Q);
      float tn[8];
      int cc[8];
      int n_hit = 0;
      if (obb) {
        /* oriented-box node (cy_bvhw_collapse.h emit_obb): two children */
        const hc_float4 h = np[0];
        float d;
        if ((as_uint(h.x) & visibility) && bvh_obb_intersect(np[1], np[2], np[3], P, dir, tmax, &d)) {
          tn[n_hit] = d;
          cc[n_hit] = as_int(h.z);
          n_hit++;
        }
        if ((as_uint(h.y) & visibility) && bvh_obb_intersect(np[4], np[5], np[6], P, dir, tmax, &d)) {
          tn[n_hit] = d;
          cc[n_hit] = as_int(h.w);
          n_hit++;
        }
      }
      else {
        for (int q = 0; q < Q; q++) {
          const hc_float4 lx = np[0 * Q + q], hx = np[1 * Q + q];
          const hc_float4 ly = np[2 * Q + q], hy = np[3 * Q + q];
          const hc_float4 lz = np[4 * Q + q], hz = np[5 * Q + q];
          const hc_float4 ch = np[6 * Q + q], mt = np[7 * Q + q];
          const float alx[4] = {lx.x, lx.y, lx.z, lx.w}, ahx[4] = {hx.x, hx.y, hx.z, hx.w};
          const float aly[4] = {ly.x, ly.y, ly.z, ly.w}, ahy[4] = {hy.x, hy.y, hy.z, hy.w};
          const float alz[4] = {lz.x, lz.y, lz.z, lz.w}, ahz[4] = {hz.x, hz.y, hz.z, hz.w};
          const int ach[4] = {as_int(ch.x), as_int(ch.y), as_int(ch.z), as_int(ch.w)};
          const uint amt[4] = {as_uint(mt.x), as_uint(mt.y), as_uint(mt.z), as_uint(mt.w)};
          for (int j = 0; j < 4; j++) {
            const float clox = (alx[j] - P.x) * idir.x;
            const float chix = (ahx[j] - P.x) * idir.x;
            const float cloy = (aly[j] - P.y) * idir.y;
            const float chiy = (ahy[j] - P.y) * idir.y;
            const float cloz = (alz[j] - P.z) * idir.z;
            const float chiz = (ahz[j] - P.z) * idir.z;
            const float cmn = max4(0.0f, cmin(clox, chix), cmin(cloy, chiy), cmin(cloz, chiz));
            const float cmx = min4(tmax, cmax(clox, chix), cmax(cloy, chiy), cmax(cloz, chiz));
            if ((cmx >= cmn) && (amt[j] & 0x0FFFFFFFu & visibility)) {
              tn[n_hit] = cmn;
              cc[n_hit] = ach[j];
              n_hit++;
            }
          }
        }
      }
      if (n_hit > 0) {
        /* insertion sort by entry distance; push far to near */
        for (int a = 1; a < n_hit; a++) {
          const float t0 = tn[a];
          const int c0 = cc[a];
          int b = a - 1;
          while (b >= 0 && tn[b] > t0) {
            tn[b + 1] = tn[b];
            cc[b + 1] = cc[b];
            b--;
          }
          tn[b + 1] = t0;
          cc[b + 1] = c0;
        }
        if (sp + n_hit - 1 > CY_SHADOW_WIDE_STACK) {
          cy_set_error(err, CY_ERR_BVH_STACK, 3);
          return true;
        }
        for (int a = n_hit - 1; a >= 1; a--) {
          stack[sp++] = cc[a];
        }
        code = cc[0];
        continue;
      }
    }
    else {
      const int packed = ~code;
      int prim_addr = packed >> 4;
      const int prim_end = prim_addr + (packed & 15);
      if ((packed & 15) == 0) {
        cy_set_error(err, CY_ERR_FEATURE, 1); /* instanced scenes keep bvh2_shadow_all */
        return true;
      }
      const bool curves = HAIR != 0 && (kg->__prim_type[prim_addr] & PRIMITIVE_ALL_CURVE);
      for (; prim_addr < prim_end; prim_addr++) {
        CyIsect *h = &hits[*num_hits];
        bool hit;
        int shader;
        if (curves) {
          h->t = tmax;
          hit = curve_intersect<HAIR>(kg, h, P, dir, visibility, OBJECT_NONE, prim_addr, kg->__prim_type[prim_addr]);
          shader = hit ? as_int(kg->__curves[kg->__prim_index[prim_addr]].z) : 0;
        }
        else {
          const uint tri_vindex = kg->__prim_tri_index[prim_addr];
          const hc_float4 *tv = kg->__prim_tri_verts + tri_vindex;
          float tt, uu, vv;
          hit = ray_triangle_intersect(P, dir, tmax, f4to3(tv[0]), f4to3(tv[1]), f4to3(tv[2]), &uu, &vv, &tt) &&
                (kg->__prim_visibility[prim_addr] & visibility);
          if (hit) {
            h->prim = prim_addr;
            h->object = OBJECT_NONE;
            h->type = PRIMITIVE_TRIANGLE;
            h->u = uu;
            h->v = vv;
            h->t = tt;
          }
          shader = hit ? (int)kg->__tri_shader[kg->__prim_index[prim_addr]] : 0;
        }
        if (hit) {
          if (!(kg->__shaders[shader & SHADER_MASK].flags & SD_HAS_TRANSPARENT_SHADOW)) {
            return true;
          }
          if (*num_hits == max_hits) {
            return true;
          }
          (*num_hits)++;
        }
      }
    }
    if (sp == 0) {
      break;
    }
    code = stack[--sp];
  }
  return false;
}

/* ---------------------------------------------------------------------------
 * Ray offset (bvh/bvh.h:541-586, __INTERSECTION_REFINE__ branch).
 */
CY_FN cfloat3 ray_offset(cfloat3 P, cfloat3 Ng)
{
  const float epsilon_f = 1e-5f;
  const float epsilon_test = 1.0f;
  const int epsilon_i = 32;
  cfloat3 res;
  if (fabsf(P.x) < epsilon_test) {
    res.x = P.x + Ng.x * epsilon_f;
  }
  else {
    uint ix = as_uint(P.x);
    ix += ((ix ^ as_uint(Ng.x)) >> 31) ? -epsilon_i : epsilon_i;
    res.x = as_float(ix);
  }
  if (fabsf(P.y) < epsilon_test) {
    res.y = P.y + Ng.y * epsilon_f;
  }
  else {
    uint iy = as_uint(P.y);
    iy += ((iy ^ as_uint(Ng.y)) >> 31) ? -epsilon_i : epsilon_i;
    res.y = as_float(iy);
  }
  if (fabsf(P.z) < epsilon_test) {
    res.z = P.z + Ng.z * epsilon_f;
  }
  else {
    uint iz = as_uint(P.z);
    iz += ((iz ^ as_uint(Ng.z)) >> 31) ? -epsilon_i : epsilon_i;
    res.z = as_float(iz);
  }
  return res;
}

/* ---------------------------------------------------------------------------
 * Triangle geometry: geom_triangle.h:26-110, geom_triangle_intersect.h:195-250.
 */
CY_FN void triangle_verts(const CyGlobals *kg, int prim, cfloat3 V[3])
{
  const hc_uint4 tri_vindex = kg->__tri_vindex[prim];
  V[0] = f4to3(kg->__prim_tri_verts[tri_vindex.w + 0]);
  V[1] = f4to3(kg->__prim_tri_verts[tri_vindex.w + 1]);
  V[2] = f4to3(kg->__prim_tri_verts[tri_vindex.w + 2]);
}

#if CY_CLOSURE_EXT
/* triangle_dPdudv (geom_triangle.h): derivatives of P w.r.t. the barycentric u, v */
CY_FN void triangle_dPdudv(const CyGlobals *kg, int prim, cfloat3 *dPdu, cfloat3 *dPdv)
{
  cfloat3 V[3];
  triangle_verts(kg, prim, V);
  *dPdu = sub3(V[0], V[2]);
  *dPdv = sub3(V[1], V[2]);
}
#endif

CY_FN cfloat3 triangle_normal(const CyGlobals *kg, const CySD *sd)
{
  cfloat3 V[3];
  triangle_verts(kg, sd->prim, V);
  if (sd->object_flag & SD_OBJECT_NEGATIVE_SCALE_APPLIED) {
    return normalize3(cross3(sub3(V[2], V[0]), sub3(V[1], V[0])));
  }
  return normalize3(cross3(sub3(V[1], V[0]), sub3(V[2], V[0])));
}

CY_FN cfloat3 triangle_smooth_normal(const CyGlobals *kg, cfloat3 Ng, int prim, float u, float v)
{
  const hc_uint4 tri_vindex = kg->__tri_vindex[prim];
  cfloat3 n0 = f4to3(kg->__tri_vnormal[tri_vindex.x]);
  cfloat3 n1 = f4to3(kg->__tri_vnormal[tri_vindex.y]);
  cfloat3 n2 = f4to3(kg->__tri_vnormal[tri_vindex.z]);
  cfloat3 N = safe_normalize3(add3(add3(mul3f(n2, (1.0f - u - v)), mul3f(n0, u)), mul3f(n1, v)));
  return is_zero3(N) ? Ng : N;
}

CY_FN cfloat3 triangle_refine(const CyGlobals *kg, const CyIsect *isect, const CyRay *ray)
{
  cfloat3 P = ray->P;
  cfloat3 D = ray->D;
  float t = isect->t;
  if (isect->object != OBJECT_NONE) {
    /* instanced geometry: refine in object space */
    if (t == 0.0f) {
      return P;
    }
    const struct cy_tfm *itfm = object_itfm(kg, isect->object);
    P = transform_point(itfm, P);
    D = transform_direction(itfm, mul3f(D, t));
    D = normalize_len3(D, &t);
  }
  P = add3(P, mul3f(D, t));
  const uint tri_vindex = kg->__prim_tri_index[isect->prim];
  const hc_float4 tri_a = kg->__prim_tri_verts[tri_vindex + 0];
  const hc_float4 tri_b = kg->__prim_tri_verts[tri_vindex + 1];
  const hc_float4 tri_c = kg->__prim_tri_verts[tri_vindex + 2];
  cfloat3 edge1 = mk3(tri_a.x - tri_c.x, tri_a.y - tri_c.y, tri_a.z - tri_c.z);
  cfloat3 edge2 = mk3(tri_b.x - tri_c.x, tri_b.y - tri_c.y, tri_b.z - tri_c.z);
  cfloat3 tvec = mk3(P.x - tri_c.x, P.y - tri_c.y, P.z - tri_c.z);
  cfloat3 qvec = cross3(tvec, edge1);
  cfloat3 pvec = cross3(D, edge2);
  float det = dot3(edge1, pvec);
  if (det != 0.0f) {
    float rt = dot3(edge2, qvec) / det;
    P = add3(P, mul3f(D, rt));
  }
  if (isect->object != OBJECT_NONE) {
    P = transform_point(object_tfm(kg, isect->object), P);
  }
  return P;
}

/* object_normal_transform (geom_object.h:168-177, __OBJECT_MOTION__ form:
 * sd->ob_itfm is the static inverse transform) */
CY_FN cfloat3 object_normal_transform(const CyGlobals *kg, int object, cfloat3 N)
{
  return normalize3(transform_direction_transposed(object_itfm(kg, object), N));
}

/* kernel_shader.h:54-153 (static triangles and curves, instanced or not; no
 * differentials: the differentials only feed texture filtering, which this
 * node subset lacks). */
#if CY_CLOSURE_EXT
/* kernel_differential.h: the ray differential transferred to the hit plane,
 * the incoming direction's, and the barycentric u / v differentials */
CY_FN void differential_transfer(CyDiff3 *dP_, const CyDiff3 &dP, cfloat3 D, const CyDiff3 &dD, cfloat3 Ng, float t)
{
  const cfloat3 tmp = div3f(D, dot3(D, Ng));
  const cfloat3 tmpx = add3(dP.dx, mul3f(dD.dx, t));
  const cfloat3 tmpy = add3(dP.dy, mul3f(dD.dy, t));
  dP_->dx = sub3(tmpx, mul3f(tmp, dot3(tmpx, Ng)));
  dP_->dy = sub3(tmpy, mul3f(tmp, dot3(tmpy, Ng)));
}

CY_FN void differential_dudv(CyDiff *du, CyDiff *dv, cfloat3 dPdu, cfloat3 dPdv, CyDiff3 dP, cfloat3 Ng)
{
  const float xn = fabsf(Ng.x);
  const float yn = fabsf(Ng.y);
  const float zn = fabsf(Ng.z);
  if (zn < xn || zn < yn) {
    if (yn < xn || yn < zn) {
      dPdu.x = dPdu.y;
      dPdv.x = dPdv.y;
      dP.dx.x = dP.dx.y;
      dP.dy.x = dP.dy.y;
    }
    dPdu.y = dPdu.z;
    dPdv.y = dPdv.z;
    dP.dx.y = dP.dx.z;
    dP.dy.y = dP.dy.z;
  }
  float det = (dPdu.x * dPdv.y - dPdv.x * dPdu.y);
  if (det != 0.0f) {
    det = 1.0f / det;
  }
  du->dx = (dP.dx.x * dPdv.y - dP.dx.y * dPdv.x) * det;
  dv->dx = (dP.dx.y * dPdu.x - dP.dx.x * dPdu.y) * det;
  du->dy = (dP.dy.x * dPdv.y - dP.dy.y * dPdv.x) * det;
  dv->dy = (dP.dy.y * dPdu.x - dP.dy.x * dPdu.y) * det;
}

CY_FN void sd_zero_differentials(CySD *sd)
{
  sd->dP.dx = sd->dP.dy = sd->dI.dx = sd->dI.dy = mk3(0.0f, 0.0f, 0.0f);
  sd->du.dx = sd->du.dy = sd->dv.dx = sd->dv.dy = 0.0f;
}
#endif

CY_FN void shader_setup_from_ray(const CyGlobals *kg, CySD *sd, const CyIsect *isect, const CyRay *ray,
                                 const CyDiff3 *ray_dP = nullptr, const CyDiff3 *ray_dD = nullptr)
{
  sd->object = (isect->object == OBJECT_NONE) ? (int)kg->__prim_object[isect->prim] : isect->object;
  sd->type = isect->type;
  sd->flag = 0;
  sd->object_flag = (int)kg->__object_flag[sd->object];
  sd->prim = (int)kg->__prim_index[isect->prim];
  sd->ray_length = isect->t;
  sd->u = isect->u;
  sd->v = isect->v;

  if (kg->have_curves && (sd->type & PRIMITIVE_ALL_CURVE)) {
    curve_shader_setup(kg, sd, isect, ray);
  }
  else {
    cfloat3 Ng = triangle_normal(kg, sd);
    sd->shader = (int)kg->__tri_shader[sd->prim];
    sd->P = triangle_refine(kg, isect, ray);
    sd->Ng = Ng;
    sd->N = Ng;
    if ((uint)sd->shader & SHADER_SMOOTH_NORMAL) {
      sd->N = triangle_smooth_normal(kg, Ng, sd->prim, sd->u, sd->v);
    }
#if CY_CLOSURE_EXT
    triangle_dPdudv(kg, sd->prim, &sd->dPdu, &sd->dPdv);
#endif
  }
  sd->I = neg3(ray->D);
  sd->flag |= kg->__shaders[(uint)sd->shader & SHADER_MASK].flags;
  if (isect->object != OBJECT_NONE) {
    /* instance transform */
    sd->N = object_normal_transform(kg, sd->object, sd->N);
    sd->Ng = object_normal_transform(kg, sd->object, sd->Ng);
#if CY_CLOSURE_EXT
    sd->dPdu = transform_direction(object_tfm(kg, sd->object), sd->dPdu);
    sd->dPdv = transform_direction(object_tfm(kg, sd->object), sd->dPdv);
#endif
  }

  bool backfacing = (dot3(sd->Ng, sd->I) < 0.0f);
  if (backfacing) {
    sd->flag |= SD_BACKFACING;
    sd->Ng = neg3(sd->Ng);
    sd->N = neg3(sd->N);
#if CY_CLOSURE_EXT
    sd->dPdu = neg3(sd->dPdu);
    sd->dPdv = neg3(sd->dPdv);
#endif
  }
#if CY_CLOSURE_EXT
  if (ray_dP) {
    /* kernel_shader.h:145-149 */
    differential_transfer(&sd->dP, *ray_dP, ray->D, *ray_dD, sd->Ng, isect->t);
    sd->dI.dx = neg3(ray_dD->dx);
    sd->dI.dy = neg3(ray_dD->dy);
    differential_dudv(&sd->du, &sd->dv, sd->dPdu, sd->dPdv, sd->dP, sd->Ng);
  }
  else {
    sd_zero_differentials(sd);
  }
#endif
}

/* ---------------------------------------------------------------------------
 * Closures (closure/alloc.h, bsdf_diffuse.h, bsdf_microfacet.h GGX,
 * bsdf_reflection.h, bsdf_refraction.h, bsdf_util.h).
 */
CY_FN CyClosure *closure_alloc(CySD *sd, int type, cfloat3 weight)
{
  if (sd->num_closure_left == 0) {
    return 0;
  }
  CyClosure *sc = &sd->closure[sd->num_closure];
  sc->type = type;
  sc->weight = weight;
  sd->num_closure++;
  sd->num_closure_left--;
  return sc;
}

/* closure/bsdf_transparent.h:37-80: transparency accumulates in
 * closure_transparent_extinction and in one transparent closure (allocated
 * even on a terminated path, for its transparency). */
CY_FN void bsdf_transparent_setup(CySD *sd, cfloat3 weight, int path_flag)
{
  const float sample_weight = fabsf(average3(weight));
  if (!(sample_weight >= CLOSURE_WEIGHT_CUTOFF)) {
    return;
  }
  if (sd->flag & SD_TRANSPARENT) {
    sd->closure_transparent_extinction = add3(sd->closure_transparent_extinction, weight);
    for (int i = 0; i < sd->num_closure; i++) {
      CyClosure *sc = &sd->closure[i];
      if (sc->type == CLOSURE_BSDF_TRANSPARENT_ID) {
        sc->weight = add3(sc->weight, weight);
        sc->sample_weight += sample_weight;
        break;
      }
    }
  }
  else {
    sd->flag |= SD_BSDF | SD_TRANSPARENT;
    sd->closure_transparent_extinction = weight;
    if (path_flag & PATH_RAY_TERMINATE) {
      sd->num_closure_left = 1;
    }
    CyClosure *bsdf = closure_alloc(sd, CLOSURE_BSDF_TRANSPARENT_ID, weight);
    if (bsdf) {
      bsdf->sample_weight = sample_weight;
      bsdf->N = sd->N;
    }
    else if (path_flag & PATH_RAY_TERMINATE) {
      sd->num_closure_left = 0;
    }
  }
}

/* kernel_shader.h:736-746 shader_bsdf_transparency (no volumes) */
CY_FN cfloat3 shader_bsdf_transparency(const CySD *sd)
{
  return (sd->flag & SD_TRANSPARENT) ? sd->closure_transparent_extinction : mk3(0.0f, 0.0f, 0.0f);
}

/* kernel_shader.h:1020-1053 shader_holdout_apply.  A holdout object keeps its
 * transparent closure and retypes the rest to NBUILTIN_CLOSURES (sampled and
 * evaluated by nobody); the flag mask is the reference's arithmetic
 * SD_CLOSURE_FLAGS - (SD_TRANSPARENT | SD_BSDF), which clears SD_TRANSPARENT
 * and keeps SD_BSDF_NEEDS_LCG. */
CY_FN cfloat3 shader_holdout_apply(CySD *sd)
{
  cfloat3 weight = mk3(0.0f, 0.0f, 0.0f);
  if (sd->object_flag & SD_OBJECT_HOLDOUT_MASK) {
    if ((sd->flag & SD_TRANSPARENT) && !(sd->flag & SD_HAS_ONLY_VOLUME)) {
      weight = sub3(mk3(1.0f, 1.0f, 1.0f), sd->closure_transparent_extinction);
      for (int i = 0; i < sd->num_closure; i++) {
        CyClosure *sc = &sd->closure[i];
        if (sc->type != CLOSURE_BSDF_TRANSPARENT_ID) {
          sc->type = NBUILTIN_CLOSURES;
        }
      }
      sd->flag &= ~(SD_CLOSURE_FLAGS - (SD_TRANSPARENT | SD_BSDF));
    }
    else {
      weight = mk3(1.0f, 1.0f, 1.0f);
    }
  }
  else {
    for (int i = 0; i < sd->num_closure; i++) {
      const CyClosure *sc = &sd->closure[i];
      if (sc->type == CLOSURE_HOLDOUT_ID) {
        weight = add3(weight, sc->weight);
      }
    }
  }
  return weight;
}

CY_FN CyClosure *bsdf_alloc(CySD *sd, cfloat3 weight)
{
  CyClosure *sc = closure_alloc(sd, CLOSURE_NONE_ID, weight);
  if (sc == 0) {
    return 0;
  }
  float sample_weight = fabsf(average3(weight));
  sc->sample_weight = sample_weight;
  return (sample_weight >= CLOSURE_WEIGHT_CUTOFF) ? sc : 0;
}

#include "cy_closures.h"

/* ---------------------------------------------------------------------------
 * BSSRDF closures (closure/bssrdf.h:330-425).  A BSSRDF keeps its radius in
 * the closure's T.  The random walk keeps its albedo in (alpha_x, alpha_y,
 * ior); the disk profiles (cubic / gaussian / burley / principled) need no
 * albedo after setup and keep the cubic sharpness in alpha_x and the channel
 * count in alpha_y.  `extra` (float bits) holds the roughness of the
 * principled types and the texture blur of the Subsurface Scattering node's
 * (whose roughness is 0, as the principled types' texture blur is). */
#if CY_CLOSURE_EXT
CY_FN bool bssrdf_is_principled(int type)
{
  return type == CLOSURE_BSSRDF_PRINCIPLED_ID || type == CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID;
}
CY_FN cfloat3 bssrdf_radius(const CyClosure *sc)
{
  return sc->T;
}
CY_FN cfloat3 bssrdf_albedo(const CyClosure *sc)
{
  return mk3(sc->alpha_x, sc->alpha_y, sc->ior);
}
CY_FN float bssrdf_roughness(const CyClosure *sc)
{
  return bssrdf_is_principled((int)sc->type) ? int_as_float(sc->extra) : 0.0f;
}
CY_FN float bssrdf_texture_blur(const CyClosure *sc)
{
  return bssrdf_is_principled((int)sc->type) ? 0.0f : int_as_float(sc->extra);
}

/* bssrdf_alloc (bssrdf.h:332-343) */
CY_FN CyClosure *bssrdf_alloc(CySD *sd, cfloat3 weight)
{
  CyClosure *sc = closure_alloc(sd, CLOSURE_NONE_ID, weight);
  if (sc == 0) {
    return 0;
  }
  const float sample_weight = fabsf(average3(weight));
  sc->sample_weight = sample_weight;
  return (sample_weight >= CLOSURE_WEIGHT_CUTOFF) ? sc : 0;
}

/* bssrdf_burley_fitting / _compatible_mfp / _setup (bssrdf.h:196-220) */
CY_FN float bssrdf_burley_fitting(float A)
{
  return 1.9f - A + 3.5f * (A - 0.8f) * (A - 0.8f);
}

/* bssrdf_setup (bssrdf.h:345-423): radii below BSSRDF_MIN_RADIUS move their
 * channel's weight to a diffuse closure; the BSSRDF's sample weight counts its
 * channels; burley-type profiles (and the random walk) remap the radius to the
 * mean free path. */
CY_FN int bssrdf_setup(CySD *sd, CyClosure *bssrdf, int type, cfloat3 radius, cfloat3 albedo, float roughness,
                       float sharpness, float texture_blur)
{
  int flag = 0;
  int bssrdf_channels = 3;
  cfloat3 diffuse_weight = mk3(0.0f, 0.0f, 0.0f);
  if (radius.x < BSSRDF_MIN_RADIUS) {
    diffuse_weight.x = bssrdf->weight.x;
    bssrdf->weight.x = 0.0f;
    radius.x = 0.0f;
    bssrdf_channels--;
  }
  if (radius.y < BSSRDF_MIN_RADIUS) {
    diffuse_weight.y = bssrdf->weight.y;
    bssrdf->weight.y = 0.0f;
    radius.y = 0.0f;
    bssrdf_channels--;
  }
  if (radius.z < BSSRDF_MIN_RADIUS) {
    diffuse_weight.z = bssrdf->weight.z;
    bssrdf->weight.z = 0.0f;
    radius.z = 0.0f;
    bssrdf_channels--;
  }
  const cfloat3 bssrdf_N = bssrdf->N;
  if (bssrdf_channels < 3) {
    /* the type set before the diffuse setup is overwritten by it, as in the
     * reference: these are plain (principled) diffuse closures */
    CyClosure *bsdf = bsdf_alloc(sd, diffuse_weight);
    if (type == CLOSURE_BSSRDF_PRINCIPLED_ID || type == CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID) {
      if (bsdf) {
        bsdf->N = bssrdf_N;
        bsdf->alpha_x = roughness;
        bsdf->type = CLOSURE_BSDF_PRINCIPLED_DIFFUSE_ID;
        flag |= SD_BSDF | SD_BSDF_HAS_EVAL;
      }
    }
    else if (bsdf) {
      bsdf->N = bssrdf_N;
      flag |= bsdf_diffuse_setup(bsdf);
    }
  }
  if (bssrdf_channels > 0) {
    bssrdf->type = type;
    bssrdf->sample_weight = fabsf(average3(bssrdf->weight)) * (float)bssrdf_channels;
    texture_blur = saturate(texture_blur);
    sharpness = saturate(sharpness);
    if (type == CLOSURE_BSSRDF_BURLEY_ID || type == CLOSURE_BSSRDF_PRINCIPLED_ID ||
        type == CLOSURE_BSSRDF_RANDOM_WALK_ID || type == CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID) {
      const cfloat3 l = mul3f(radius, 0.25f * CY_1_PI_F);
      const cfloat3 sfit = mk3(bssrdf_burley_fitting(albedo.x), bssrdf_burley_fitting(albedo.y),
                               bssrdf_burley_fitting(albedo.z));
      radius = div3(l, sfit);
    }
    flag |= SD_BSSRDF;
  }
  else {
    bssrdf->type = type;
    bssrdf->sample_weight = 0.0f;
  }
  bssrdf->T = radius;
  if (type == CLOSURE_BSSRDF_RANDOM_WALK_ID || type == CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID) {
    bssrdf->alpha_x = albedo.x;
    bssrdf->alpha_y = albedo.y;
    bssrdf->ior = albedo.z;
  }
  else {
    bssrdf->alpha_x = sharpness;
    bssrdf->alpha_y = (float)bssrdf_channels;
  }
  bssrdf->extra = as_int(bssrdf_is_principled(type) ? roughness : texture_blur);
  return flag;
}
#endif

/* ---------------------------------------------------------------------------
 * SVM interpreter subset (svm/svm.h:220-549, svm_closure.h, svm_value.h,
 * svm_fresnel.h).  Unknown nodes set CY_ERR_SVM_NODE and stop the shader.
 */
/* SVM stack view: element i < fast at p[i * stride] (an LDS column on the
 * device), deeper elements at spill[i - fast] */
typedef struct CySvmStack {
  float *p;
  int stride;
  int fast;
  float *spill;
} CySvmStack;

CY_FN float svm_load(CySvmStack stack, uint a, uint *err)
{
  if (a >= CY_SVM_STACK) {
    cy_set_error(err, CY_ERR_SVM_STACK, a);
    return 0.0f;
  }
  return ((int)a < stack.fast) ? stack.p[(int)a * stack.stride] : stack.spill[(int)a - stack.fast];
}
CY_FN void svm_store(CySvmStack stack, uint a, float f, uint *err)
{
  if (a >= CY_SVM_STACK) {
    cy_set_error(err, CY_ERR_SVM_STACK, a);
    return;
  }
  if ((int)a < stack.fast) {
    stack.p[(int)a * stack.stride] = f;
  }
  else {
    stack.spill[(int)a - stack.fast] = f;
  }
}
CY_FN cfloat3 svm_load3(CySvmStack stack, uint a, uint *err)
{
  return mk3(svm_load(stack, a, err), svm_load(stack, a + 1, err), svm_load(stack, a + 2, err));
}
CY_FN void svm_store3(CySvmStack stack, uint a, cfloat3 f, uint *err)
{
  svm_store(stack, a, f.x, err);
  svm_store(stack, a + 1, f.y, err);
  svm_store(stack, a + 2, f.z, err);
}

#include "cy_svm_nodes.h"
#include "cy_svm_noise.h"
#include "cy_svm_extra.h"
#include "cy_attribute.h"

/* svm_closure.h:21-56 */
CY_FN void svm_node_glass_setup(CySD *sd, CyClosure *b, int type, float eta, float roughness, bool refract)
{
  if (type == CLOSURE_BSDF_SHARP_GLASS_ID) {
    b->alpha_y = 0.0f;
    b->alpha_x = 0.0f;
    if (refract) {
      b->ior = eta;
      b->type = CLOSURE_BSDF_REFRACTION_ID;
    }
    else {
      b->ior = 0.0f;
      b->type = CLOSURE_BSDF_REFLECTION_ID;
    }
    sd->flag |= SD_BSDF;
  }
#if CY_CLOSURE_EXT
  else if (type == CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID) {
    b->alpha_x = roughness;
    b->alpha_y = roughness;
    b->ior = eta;
    sd->flag |= refract ? bsdf_microfacet_beckmann_refraction_setup(b) : bsdf_microfacet_beckmann_setup(b);
  }
#endif
  else {
    b->alpha_x = roughness;
    b->alpha_y = roughness;
    b->ior = eta;
    sd->flag |= refract ? bsdf_microfacet_ggx_refraction_setup(b) : bsdf_microfacet_ggx_setup(b);
  }
}

#if CY_CLOSURE_EXT
/* svm_closure.h:100-463: the Principled BSDF with the GGX distribution
 * (the multiscatter distribution is rejected at load_kernels).  On the
 * reference CPU kernel __SUBSURFACE__ is defined, so the diffuse lobe is
 * gated by the subsurface mix; subsurface > 0 needs a BSSRDF and sets
 * CY_ERR_CLOSURE.  The tangent input is read only when linked (the
 * reference reads stack slot 255 otherwise). */
CY_FN void svm_node_principled_bsdf(const CyGlobals *kg,
                                    CySD *sd,
                                    CySvmStack stack,
                                    hc_uint4 data_node,
                                    cfloat3 N,
                                    float param1,
                                    float param2,
                                    float mix_weight,
                                    int path_flag,
                                    int *offset,
                                    uint *err)
{
  hc_uint4 data_node2 = kg->__svm_nodes[(*offset)++];
  cfloat3 T = (data_node.y != SVM_STACK_INVALID) ? svm_load3(stack, data_node.y, err) : mk3(0.0f, 0.0f, 0.0f);
  const uint specular_offset = data_node.z & 0xFF, roughness_offset = (data_node.z >> 8) & 0xFF;
  const uint specular_tint_offset = (data_node.z >> 16) & 0xFF, anisotropic_offset = (data_node.z >> 24) & 0xFF;
  const uint sheen_offset = data_node.w & 0xFF, sheen_tint_offset = (data_node.w >> 8) & 0xFF;
  const uint clearcoat_offset = (data_node.w >> 16) & 0xFF, clearcoat_roughness_offset = (data_node.w >> 24) & 0xFF;
  const uint eta_offset = data_node2.x & 0xFF, transmission_offset = (data_node2.x >> 8) & 0xFF;
  const uint anisotropic_rotation_offset = (data_node2.x >> 16) & 0xFF;
  const uint transmission_roughness_offset = (data_node2.x >> 24) & 0xFF;
  float metallic = param1;
  float subsurface = param2;
  float specular = svm_load(stack, specular_offset, err);
  float roughness = svm_load(stack, roughness_offset, err);
  float specular_tint = svm_load(stack, specular_tint_offset, err);
  float anisotropic = svm_load(stack, anisotropic_offset, err);
  float sheen = svm_load(stack, sheen_offset, err);
  float sheen_tint = svm_load(stack, sheen_tint_offset, err);
  float clearcoat = svm_load(stack, clearcoat_offset, err);
  float clearcoat_roughness = svm_load(stack, clearcoat_roughness_offset, err);
  float transmission = svm_load(stack, transmission_offset, err);
  float anisotropic_rotation = svm_load(stack, anisotropic_rotation_offset, err);
  float transmission_roughness = svm_load(stack, transmission_roughness_offset, err);
  float eta = fmaxf(svm_load(stack, eta_offset, err), 1e-5f);
  const uint distribution = data_node2.y;
  if (anisotropic_rotation != 0.0f) {
    T = rotate_around_axis(T, N, anisotropic_rotation * CY_2PI_F);
  }
  float ior = (sd->flag & SD_BACKFACING) ? 1.0f / eta : eta;
  float cosNO = dot3(N, sd->I);
  float fresnel = fresnel_dielectric_cos(cosNO, ior);
  float diffuse_weight = (1.0f - saturate(metallic)) * (1.0f - saturate(transmission));
  float final_transmission = saturate(transmission) * (1.0f - saturate(metallic));
  float specular_weight = (1.0f - final_transmission);

  hc_uint4 data_base_color = kg->__svm_nodes[(*offset)++];
  cfloat3 base_color = (data_base_color.x != SVM_STACK_INVALID) ?
                           svm_load3(stack, data_base_color.x, err) :
                           mk3(as_float(data_base_color.y), as_float(data_base_color.z),
                               as_float(data_base_color.w));
  hc_uint4 data_cn_ssr = kg->__svm_nodes[(*offset)++];
  cfloat3 clearcoat_normal = (data_cn_ssr.x != SVM_STACK_INVALID) ? svm_load3(stack, data_cn_ssr.x, err) : sd->N;
  hc_uint4 data_subsurface_color = kg->__svm_nodes[(*offset)++];
  cfloat3 subsurface_color = (data_subsurface_color.x != SVM_STACK_INVALID) ?
                                 svm_load3(stack, data_subsurface_color.x, err) :
                                 mk3(as_float(data_subsurface_color.y), as_float(data_subsurface_color.z),
                                     as_float(data_subsurface_color.w));
  cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);

  /* diffuse, gated by the subsurface mix (__SUBSURFACE__ branch) */
  cfloat3 mixed_ss_base_color = add3(mul3f(subsurface_color, subsurface), mul3f(base_color, (1.0f - subsurface)));
  if (path_flag & PATH_RAY_DIFFUSE_ANCESTOR) {
    subsurface = 0.0f;
    base_color = mixed_ss_base_color;
  }
  if (fabsf(average3(mixed_ss_base_color)) > CLOSURE_WEIGHT_CUTOFF) {
    if (subsurface <= CLOSURE_WEIGHT_CUTOFF && diffuse_weight > CLOSURE_WEIGHT_CUTOFF) {
      cfloat3 diff_weight = mul3f(mul3(weight, base_color), diffuse_weight);
      CyClosure *b = bsdf_alloc(sd, diff_weight);
      if (b) {
        b->N = N;
        b->alpha_x = roughness;
        b->type = CLOSURE_BSDF_PRINCIPLED_DIFFUSE_ID;
        sd->flag |= SD_BSDF | SD_BSDF_HAS_EVAL;
      }
    }
    else if (subsurface > CLOSURE_WEIGHT_CUTOFF) {
      /* svm_closure.h:220-236 */
      const cfloat3 subsurf_weight = mul3f(mul3(weight, mixed_ss_base_color), diffuse_weight);
      CyClosure *bssrdf = bssrdf_alloc(sd, subsurf_weight);
      if (bssrdf) {
        const int subsurface_method = (int)data_node2.z;
        const cfloat3 subsurface_radius = (data_cn_ssr.y != SVM_STACK_INVALID) ? svm_load3(stack, data_cn_ssr.y, err) :
                                                                                 mk3(1.0f, 1.0f, 1.0f);
        bssrdf->N = N;
        sd->flag |= bssrdf_setup(sd, bssrdf, subsurface_method, mul3f(subsurface_radius, subsurface),
                                 (subsurface_method == CLOSURE_BSSRDF_PRINCIPLED_ID) ? subsurface_color :
                                                                                     mixed_ss_base_color,
                                 roughness, 0.0f, 0.0f);
      }
    }
  }

  /* sheen */
  if (diffuse_weight > CLOSURE_WEIGHT_CUTOFF && sheen > CLOSURE_WEIGHT_CUTOFF) {
    float m_cdlum = dot3(base_color, mk3(KD->film.rgb_to_y.x, KD->film.rgb_to_y.y, KD->film.rgb_to_y.z));
    cfloat3 m_ctint = m_cdlum > 0.0f ? div3f(base_color, m_cdlum) : mk3(1.0f, 1.0f, 1.0f);
    cfloat3 sheen_color = add3(mul3f(mk3(1.0f, 1.0f, 1.0f), (1.0f - sheen_tint)), mul3f(m_ctint, sheen_tint));
    cfloat3 sheen_weight = mul3f(mul3(mul3f(weight, sheen), sheen_color), diffuse_weight);
    CyClosure *b = bsdf_alloc(sd, sheen_weight);
    if (b) {
      b->N = N;
      sd->flag |= bsdf_principled_sheen_setup(sd, b);
    }
  }

  /* specular reflection */
  if (KD->integrator.caustics_reflective || (path_flag & PATH_RAY_DIFFUSE) == 0) {
    if (specular_weight > CLOSURE_WEIGHT_CUTOFF &&
        (specular > CLOSURE_WEIGHT_CUTOFF || metallic > CLOSURE_WEIGHT_CUTOFF)) {
      cfloat3 spec_weight = mul3f(weight, specular_weight);
      CyClosure *b = bsdf_alloc(sd, spec_weight);
      int extra = (b != 0) ? closure_alloc_extra(sd) : -1;
      if (b && extra >= 0) {
        CyClosure *ex = &sd->closure[extra];
        b->N = N;
        b->ior = (2.0f / (1.0f - safe_sqrtf(0.08f * specular))) - 1.0f;
        b->T = T;
        b->extra = extra;
        float aspect = safe_sqrtf(1.0f - anisotropic * 0.9f);
        float r2 = roughness * roughness;
        b->alpha_x = r2 / aspect;
        b->alpha_y = r2 * aspect;
        float m_cdlum = 0.3f * base_color.x + 0.6f * base_color.y + 0.1f * base_color.z;
        cfloat3 m_ctint = m_cdlum > 0.0f ? div3f(base_color, m_cdlum) : mk3(0.0f, 0.0f, 0.0f);
        cfloat3 tmp_col = add3(mul3f(mk3(1.0f, 1.0f, 1.0f), (1.0f - specular_tint)), mul3f(m_ctint, specular_tint));
        ex->N = add3(mul3f(mul3f(tmp_col, specular * 0.08f), (1.0f - metallic)), mul3f(base_color, metallic));
        ex->weight = base_color;
        ex->alpha_x = 0.0f;
        if (distribution == CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID || roughness <= 0.075f) {
          sd->flag |= bsdf_microfacet_ggx_fresnel_setup(b, sd);
        }
        else {
          /* multi-scatter GGX (svm_closure.h:281-283) */
          sd->flag |= bsdf_microfacet_multi_ggx_fresnel_setup(sd, b);
        }
      }
    }
  }

  /* glass */
  if (KD->integrator.caustics_reflective || KD->integrator.caustics_refractive ||
      (path_flag & PATH_RAY_DIFFUSE) == 0) {
    if (final_transmission > CLOSURE_WEIGHT_CUTOFF) {
      cfloat3 glass_weight = mul3f(weight, final_transmission);
      cfloat3 cspec0 = add3(mul3f(base_color, specular_tint), mul3f(mk3(1.0f, 1.0f, 1.0f), (1.0f - specular_tint)));
      if (roughness <= 5e-2f || distribution == CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID) {
        float refl_roughness = roughness;
        if (KD->integrator.caustics_reflective || (path_flag & PATH_RAY_DIFFUSE) == 0) {
          CyClosure *b = bsdf_alloc(sd, mul3f(glass_weight, fresnel));
          int extra = (b != 0) ? closure_alloc_extra(sd) : -1;
          if (b && extra >= 0) {
            CyClosure *ex = &sd->closure[extra];
            b->N = N;
            b->T = mk3(0.0f, 0.0f, 0.0f);
            b->extra = extra;
            b->alpha_x = refl_roughness * refl_roughness;
            b->alpha_y = refl_roughness * refl_roughness;
            b->ior = ior;
            ex->weight = base_color;
            ex->N = cspec0;
            ex->alpha_x = 0.0f;
            sd->flag |= bsdf_microfacet_ggx_fresnel_setup(b, sd);
          }
        }
        if (KD->integrator.caustics_refractive || (path_flag & PATH_RAY_DIFFUSE) == 0) {
          CyClosure *b = bsdf_alloc(sd, mul3f(mul3(base_color, glass_weight), (1.0f - fresnel)));
          if (b) {
            b->N = N;
            b->T = mk3(0.0f, 0.0f, 0.0f);
            b->extra = -1;
            if (distribution == CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID) {
              transmission_roughness = 1.0f - (1.0f - refl_roughness) * (1.0f - transmission_roughness);
            }
            else {
              transmission_roughness = refl_roughness;
            }
            b->alpha_x = transmission_roughness * transmission_roughness;
            b->alpha_y = transmission_roughness * transmission_roughness;
            b->ior = ior;
            sd->flag |= bsdf_microfacet_ggx_refraction_setup(b);
          }
        }
      }
      else {
        /* multi-scatter GGX (svm_closure.h:403-426) */
        CyClosure *b = bsdf_alloc(sd, glass_weight);
        int extra = (b != 0) ? closure_alloc_extra(sd) : -1;
        if (b && extra >= 0) {
          CyClosure *ex = &sd->closure[extra];
          b->N = N;
          b->extra = extra;
          b->T = mk3(0.0f, 0.0f, 0.0f);
          b->alpha_x = roughness * roughness;
          b->alpha_y = roughness * roughness;
          b->ior = ior;
          ex->weight = base_color;
          ex->N = cspec0;
          ex->alpha_x = 0.0f;
          sd->flag |= bsdf_microfacet_multi_ggx_glass_fresnel_setup(sd, b);
        }
      }
    }
  }

  /* clearcoat */
  if (KD->integrator.caustics_reflective || (path_flag & PATH_RAY_DIFFUSE) == 0) {
    if (clearcoat > CLOSURE_WEIGHT_CUTOFF) {
      CyClosure *b = bsdf_alloc(sd, weight);
      int extra = (b != 0) ? closure_alloc_extra(sd) : -1;
      if (b && extra >= 0) {
        CyClosure *ex = &sd->closure[extra];
        b->N = clearcoat_normal;
        b->T = mk3(0.0f, 0.0f, 0.0f);
        b->ior = 1.5f;
        b->extra = extra;
        b->alpha_x = clearcoat_roughness * clearcoat_roughness;
        b->alpha_y = clearcoat_roughness * clearcoat_roughness;
        ex->weight = mk3(0.0f, 0.0f, 0.0f);
        ex->N = mk3(0.04f, 0.04f, 0.04f);
        ex->alpha_x = clearcoat;
        sd->flag |= bsdf_microfacet_ggx_clearcoat_setup(b, sd);
      }
    }
  }
}
#endif

/* svm_closure.h:58-735 svm_node_closure_bsdf (every BSDF the SVM compiler
 * emits except Principled, multiscatter GGX and hair; those set
 * CY_ERR_CLOSURE). */
CY_FN void svm_node_closure_bsdf(const CyGlobals *kg,
                                 CySD *sd,
                                 CySvmStack stack,
                                 hc_uint4 node,
                                 int path_flag,
                                 int *offset,
                                 uint *err)
{
  uint type = node.y & 0xFF, param1_offset = (node.y >> 8) & 0xFF;
  uint param2_offset = (node.y >> 16) & 0xFF, mix_weight_offset = (node.y >> 24) & 0xFF;
  float mix_weight = (mix_weight_offset != SVM_STACK_INVALID) ?
                         svm_load(stack, mix_weight_offset, err) :
                         1.0f;
  hc_uint4 data_node = kg->__svm_nodes[*offset];
  (*offset)++;
  if (mix_weight == 0.0f) {
    if (type == CLOSURE_BSDF_PRINCIPLED_ID) {
      *offset += 4; /* the principled node's extra data */
    }
#if CY_CLOSURE_EXT
    else if (type == CLOSURE_BSDF_HAIR_PRINCIPLED_ID) {
      /* the reference skips none of the principled hair node's three extra
       * data nodes here and runs them as instructions (svm_closure.h:75-85) */
      cy_set_error(err, CY_ERR_FEATURE, 13);
    }
#endif
    return;
  }
  cfloat3 N = (data_node.x != SVM_STACK_INVALID) ? svm_load3(stack, data_node.x, err) : sd->N;
  float param1 = (param1_offset != SVM_STACK_INVALID) ? svm_load(stack, param1_offset, err) :
                                                        as_float(node.z);
  float param2 = (param2_offset != SVM_STACK_INVALID) ? svm_load(stack, param2_offset, err) :
                                                        as_float(node.w);
  switch (type) {
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_PRINCIPLED_ID:
      svm_node_principled_bsdf(kg, sd, stack, data_node, N, param1, param2, mix_weight, path_flag, offset, err);
      break;
#endif
    case CLOSURE_BSDF_DIFFUSE_ID: {
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *b = bsdf_alloc(sd, weight);
      if (b) {
        b->N = N;
        float roughness = param1;
        if (roughness == 0.0f) {
          sd->flag |= bsdf_diffuse_setup(b);
        }
        else {
#if CY_CLOSURE_EXT
          b->alpha_x = roughness;
          sd->flag |= bsdf_oren_nayar_setup(b);
#else
          cy_set_error(err, CY_ERR_CLOSURE, CLOSURE_BSDF_OREN_NAYAR_ID);
#endif
        }
      }
      break;
    }
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_TRANSLUCENT_ID: {
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *b = bsdf_alloc(sd, weight);
      if (b) {
        b->N = N;
        sd->flag |= bsdf_translucent_setup(b);
      }
      break;
    }
#endif
    case CLOSURE_BSDF_TRANSPARENT_ID:
      bsdf_transparent_setup(sd, mul3f(sd->svm_closure_weight, mix_weight), path_flag);
      break;
    case CLOSURE_BSDF_REFLECTION_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_ID:
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_MICROFACET_BECKMANN_ID:
    case CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID:
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
#endif
    {
      if (!KD->integrator.caustics_reflective && (path_flag & PATH_RAY_DIFFUSE)) {
        break;
      }
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *b = bsdf_alloc(sd, weight);
      if (!b) {
        break;
      }
      float roughness = sqr(param1);
      b->N = N;
      b->ior = 0.0f;
      if (data_node.y == SVM_STACK_INVALID) {
#if CY_CLOSURE_EXT
        b->T = mk3(0.0f, 0.0f, 0.0f);
#endif
        b->alpha_x = roughness;
        b->alpha_y = roughness;
      }
      else {
#if !CY_CLOSURE_EXT
        cy_set_error(err, CY_ERR_CLOSURE, 1000 + type); /* anisotropic: extended closure set */
#else
        b->T = svm_load3(stack, data_node.y, err);
        float rotation = svm_load(stack, data_node.z, err);
        if (rotation != 0.0f) {
          b->T = rotate_around_axis(b->T, b->N, rotation * CY_2PI_F);
        }
        float anisotropy = cclamp(param2, -0.99f, 0.99f);
        if (anisotropy < 0.0f) {
          b->alpha_x = roughness / (1.0f + anisotropy);
          b->alpha_y = roughness * (1.0f + anisotropy);
        }
        else {
          b->alpha_x = roughness * (1.0f - anisotropy);
          b->alpha_y = roughness / (1.0f - anisotropy);
        }
#endif
      }
      if (type == CLOSURE_BSDF_REFLECTION_ID) {
        b->type = CLOSURE_BSDF_REFLECTION_ID;
        sd->flag |= SD_BSDF;
      }
#if CY_CLOSURE_EXT
      else if (type == CLOSURE_BSDF_MICROFACET_BECKMANN_ID) {
        sd->flag |= bsdf_microfacet_beckmann_setup(b);
      }
      else if (type == CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID) {
        sd->flag |= bsdf_ashikhmin_shirley_setup(b);
      }
      else if (type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID) {
        /* svm_closure.h:345-356: the color (param4) in a MicrofacetExtra */
        const int extra = closure_alloc_extra(sd);
        if (extra >= 0) {
          CyClosure *ex = &sd->closure[extra];
          b->extra = extra;
          ex->weight = svm_load3(stack, data_node.w, err);
          ex->N = mk3(0.0f, 0.0f, 0.0f);
          ex->alpha_x = 0.0f;
          sd->flag |= bsdf_microfacet_multi_ggx_setup(sd, b);
        }
      }
#endif
      else {
        sd->flag |= bsdf_microfacet_ggx_setup(b);
      }
      break;
    }
    case CLOSURE_BSDF_REFRACTION_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID:
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID:
#endif
    {
      if (!KD->integrator.caustics_refractive && (path_flag & PATH_RAY_DIFFUSE)) {
        break;
      }
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *b = bsdf_alloc(sd, weight);
      if (b) {
        b->N = N;
#if CY_CLOSURE_EXT
        b->T = mk3(0.0f, 0.0f, 0.0f);
#endif
        float eta = fmaxf(param2, 1e-5f);
        eta = (sd->flag & SD_BACKFACING) ? 1.0f / eta : eta;
        if (type == CLOSURE_BSDF_REFRACTION_ID) {
          b->alpha_x = 0.0f;
          b->alpha_y = 0.0f;
          b->ior = eta;
          b->type = CLOSURE_BSDF_REFRACTION_ID;
          sd->flag |= SD_BSDF;
        }
        else {
          float roughness = sqr(param1);
          b->alpha_x = roughness;
          b->alpha_y = roughness;
          b->ior = eta;
#if CY_CLOSURE_EXT
          if (type == CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID) {
            sd->flag |= bsdf_microfacet_beckmann_refraction_setup(b);
          }
          else
#endif
          {
            sd->flag |= bsdf_microfacet_ggx_refraction_setup(b);
          }
        }
      }
      break;
    }
    case CLOSURE_BSDF_SHARP_GLASS_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID:
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID:
#endif
    {
      if (!KD->integrator.caustics_reflective && !KD->integrator.caustics_refractive &&
          (path_flag & PATH_RAY_DIFFUSE)) {
        break;
      }
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      float eta = fmaxf(param2, 1e-5f);
      eta = (sd->flag & SD_BACKFACING) ? 1.0f / eta : eta;
      float cosNO = dot3(N, sd->I);
      float fresnel = fresnel_dielectric_cos(cosNO, eta);
      float roughness = sqr(param1);
      if (KD->integrator.caustics_reflective || (path_flag & PATH_RAY_DIFFUSE) == 0) {
        CyClosure *b = bsdf_alloc(sd, mul3f(weight, fresnel));
        if (b) {
          b->N = N;
#if CY_CLOSURE_EXT
          b->T = mk3(0.0f, 0.0f, 0.0f);
#endif
          svm_node_glass_setup(sd, b, (int)type, eta, roughness, false);
        }
      }
      if (KD->integrator.caustics_refractive || (path_flag & PATH_RAY_DIFFUSE) == 0) {
        CyClosure *b = bsdf_alloc(sd, mul3f(weight, (1.0f - fresnel)));
        if (b) {
          b->N = N;
#if CY_CLOSURE_EXT
          b->T = mk3(0.0f, 0.0f, 0.0f);
#endif
          svm_node_glass_setup(sd, b, (int)type, eta, roughness, true);
        }
      }
      break;
    }
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID: {
      /* svm_closure.h:664-698 (Glass BSDF, Multiscatter GGX) */
      if (!KD->integrator.caustics_reflective && !KD->integrator.caustics_refractive &&
          (path_flag & PATH_RAY_DIFFUSE)) {
        break;
      }
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *b = bsdf_alloc(sd, weight);
      if (!b) {
        break;
      }
      const int extra = closure_alloc_extra(sd);
      if (extra < 0) {
        break;
      }
      CyClosure *ex = &sd->closure[extra];
      b->N = N;
      b->extra = extra;
      b->T = mk3(0.0f, 0.0f, 0.0f);
      float roughness = sqr(param1);
      b->alpha_x = roughness;
      b->alpha_y = roughness;
      float eta = fmaxf(param2, 1e-5f);
      b->ior = (sd->flag & SD_BACKFACING) ? 1.0f / eta : eta;
      ex->weight = svm_load3(stack, data_node.z, err);
      ex->N = mk3(0.0f, 0.0f, 0.0f);
      ex->alpha_x = 0.0f;
      sd->flag |= bsdf_microfacet_multi_ggx_glass_setup(sd, b);
      break;
    }
    case CLOSURE_BSDF_ASHIKHMIN_VELVET_ID: {
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *b = bsdf_alloc(sd, weight);
      if (b) {
        b->N = N;
        b->alpha_x = saturate(param1);
        sd->flag |= bsdf_ashikhmin_velvet_setup(b);
      }
      break;
    }
    case CLOSURE_BSDF_GLOSSY_TOON_ID:
      if (!KD->integrator.caustics_reflective && (path_flag & PATH_RAY_DIFFUSE)) {
        break;
      }
      /* fall through */
    case CLOSURE_BSDF_DIFFUSE_TOON_ID: {
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *b = bsdf_alloc(sd, weight);
      if (b) {
        b->N = N;
        b->alpha_x = param1;
        b->alpha_y = param2;
        sd->flag |= bsdf_toon_setup(b, (int)type);
      }
      break;
    }
    case CLOSURE_BSDF_HAIR_PRINCIPLED_ID: {
      /* svm_closure.h:735-844 (Principled Hair BSDF node) */
      const hc_uint4 data_node2 = kg->__svm_nodes[(*offset)++];
      const hc_uint4 data_node3 = kg->__svm_nodes[(*offset)++];
      const hc_uint4 data_node4 = kg->__svm_nodes[(*offset)++];
      const cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      const uint offset_ofs = data_node.y & 0xFF, ior_ofs = (data_node.y >> 8) & 0xFF;
      const uint color_ofs = (data_node.y >> 16) & 0xFF, parametrization = data_node.y >> 24;
      const float alpha = svm_load_default(stack, offset_ofs, data_node.z, err);
      const float ior = svm_load_default(stack, ior_ofs, data_node.w, err);
      const uint coat_ofs = data_node2.x & 0xFF, melanin_ofs = (data_node2.x >> 8) & 0xFF;
      const uint melanin_redness_ofs = (data_node2.x >> 16) & 0xFF, absorption_ofs = data_node2.x >> 24;
      const uint tint_ofs = data_node3.x & 0xFF, random_ofs = (data_node3.x >> 8) & 0xFF;
      const uint random_color_ofs = (data_node3.x >> 16) & 0xFF, random_roughness_ofs = data_node3.x >> 24;
      float random = 0.0f;
      const CyAttr attr_random = (data_node4.y != SVM_STACK_INVALID) ?
                                     find_attribute(kg, sd->object, sd->prim, data_node4.y) :
                                     attribute_not_found();
      if (attr_random.offset != (int)ATTR_STD_NOT_FOUND) {
        cy_set_error(err, CY_ERR_FEATURE, 11); /* curve attributes are not packed */
      }
      else {
        random = svm_load_default(stack, random_ofs, data_node3.y, err);
      }
      CyClosure *b = bsdf_alloc(sd, weight);
      if (b) {
        const int extra = closure_alloc_extra(sd);
        if (extra < 0) {
          break;
        }
        CyClosure *ex = &sd->closure[extra];
        const float random_roughness = svm_load_default(stack, random_roughness_ofs, data_node3.w, err);
        const float factor_random_roughness = 1.0f + 2.0f * (random - 0.5f) * random_roughness;
        const float roughness = param1 * factor_random_roughness;
        const float radial_roughness = param2 * factor_random_roughness;
        const float coat = svm_load_default(stack, coat_ofs, data_node2.y, err);
        const float m0_roughness = 1.0f - cclamp(coat, 0.0f, 1.0f);
        b->N = N;
        b->alpha_x = roughness;
        b->alpha_y = radial_roughness;
        b->ior = ior;
        b->extra = extra;
        ex->ior = m0_roughness;
        ex->alpha_y = alpha;
        ex->T = mk3(KD->film.rgb_to_y.x, KD->film.rgb_to_y.y, KD->film.rgb_to_y.z);
        switch (parametrization) {
          case 2: /* NODE_PRINCIPLED_HAIR_DIRECT_ABSORPTION */
            b->T = svm_load3(stack, absorption_ofs, err);
            break;
          case 1: { /* NODE_PRINCIPLED_HAIR_PIGMENT_CONCENTRATION */
            float melanin = svm_load_default(stack, melanin_ofs, data_node2.z, err);
            const float melanin_redness = svm_load_default(stack, melanin_redness_ofs, data_node2.w, err);
            float random_color = svm_load_default(stack, random_color_ofs, data_node3.z, err);
            random_color = cclamp(random_color, 0.0f, 1.0f);
            const float factor_random_color = 1.0f + 2.0f * (random - 0.5f) * random_color;
            melanin *= factor_random_color;
            melanin = -cy_logf(fmaxf(1.0f - melanin, 0.0001f));
            const float eumelanin = melanin * (1.0f - melanin_redness);
            const float pheomelanin = melanin * melanin_redness;
            const cfloat3 melanin_sigma = bsdf_principled_hair_sigma_from_concentration(eumelanin, pheomelanin);
            const cfloat3 tint = svm_load3(stack, tint_ofs, err);
            const cfloat3 tint_sigma = bsdf_principled_hair_sigma_from_reflectance(tint, radial_roughness);
            b->T = add3(melanin_sigma, tint_sigma);
            break;
          }
          case 0: /* NODE_PRINCIPLED_HAIR_REFLECTANCE */
            b->T = bsdf_principled_hair_sigma_from_reflectance(svm_load3(stack, color_ofs, err), radial_roughness);
            break;
          default:
            b->T = bsdf_principled_hair_sigma_from_concentration(0.0f, 0.8054375f);
            break;
        }
        sd->flag |= bsdf_principled_hair_setup(sd, b, ex);
      }
      break;
    }
    case CLOSURE_BSDF_HAIR_REFLECTION_ID:
    case CLOSURE_BSDF_HAIR_TRANSMISSION_ID: {
      /* svm_closure.h:846-877 (Hair BSDF node) */
      CyClosure *b = bsdf_alloc(sd, mul3f(sd->svm_closure_weight, mix_weight));
      if (b) {
        b->N = N;
        b->alpha_x = param1;
        b->alpha_y = param2;
        b->ior = -svm_load(stack, data_node.z, err);
        if (data_node.y != SVM_STACK_INVALID) {
          b->T = normalize3(svm_load3(stack, data_node.y, err));
        }
        else if (!(sd->type & PRIMITIVE_ALL_CURVE)) {
          b->T = normalize3(sd->dPdv);
          b->ior = 0.0f;
        }
        else {
          b->T = normalize3(sd->dPdu);
        }
        sd->flag |= bsdf_hair_setup(b, (int)type);
      }
      break;
    }
    case CLOSURE_BSSRDF_CUBIC_ID:
    case CLOSURE_BSSRDF_GAUSSIAN_ID:
    case CLOSURE_BSSRDF_BURLEY_ID:
    case CLOSURE_BSSRDF_RANDOM_WALK_ID: {
      /* svm_closure.h:880-905 (Subsurface Scattering node) */
      cfloat3 weight = mul3f(sd->svm_closure_weight, mix_weight);
      CyClosure *bssrdf = bssrdf_alloc(sd, weight);
      if (bssrdf) {
        if (path_flag & PATH_RAY_DIFFUSE_ANCESTOR) {
          param1 = 0.0f;
        }
        bssrdf->N = N;
        sd->flag |= bssrdf_setup(sd, bssrdf, (int)type, mul3f(svm_load3(stack, data_node.z, err), param1),
                                 sd->svm_closure_weight, 0.0f, svm_load(stack, data_node.w, err), param2);
      }
      break;
    }
#endif
    default:
      cy_set_error(err, CY_ERR_CLOSURE, type);
      break;
  }
}

CY_FN void emission_setup(CySD *sd, cfloat3 weight)
{
  if (sd->flag & SD_EMISSION) {
    sd->closure_emission_background = add3(sd->closure_emission_background, weight);
  }
  else {
    sd->flag |= SD_EMISSION;
    sd->closure_emission_background = weight;
  }
}

/* Texture / converter / input nodes (cy_svm_nodes.h).  Compiled only into the
 * kernels built with CY_SVM_TEX=1: the shading kernel exists in a variant
 * without them (picked at load_kernels when no shader uses them), whose
 * register allocation they would otherwise burden.  Returns the next node
 * offset, or -1 for an unknown node. */
#include "cy_svm_image.h"
#include "cy_svm_sky.h"
#include "cy_svm_ies.h"
#include "cy_svm_spectral.h"

typedef struct CySvmTexIn {
  cfloat3 P, N, Ng, I;
  float u, v, ray_length;
  int object, flag;
  int lamp; /* light index of a PRIMITIVE_LAMP point, else -1 */
  int bounce, diffuse_bounce, glossy_bounce, transparent_bounce, transmission_bounce;
} CySvmTexIn;

#if CY_SVM_TEX
/* svm_voxel.h:22-55 svm_node_tex_voxel (the Point Density node's dense grid):
 * the input point in object space (volume_normalized_position,
 * geom_volume.h:32-48: the object's inverse transform, then the mesh's
 * ATTR_STD_GENERATED_TRANSFORM when it has one) or through the node's own
 * world-space transform (three data nodes), then the 3D texture at its own
 * interpolation; density = alpha, colour = rgb.  Returns the next node. */
CY_NOINLINE int svm_node_tex_voxel(const hc_uint4 *svm_nodes, const hc_KernelObject *objects,
                                   const hc_uint4 *attributes_map, const hc_float4 *attributes_float3,
                                   const hc_TextureInfo *texture_info, int object, int prim, CySvmStack stack,
                                   hc_uint4 node, int offset, uint *err)
{
  CyGlobals kgv;
  kgv.__objects = objects;
  kgv.__attributes_map = attributes_map;
  kgv.__attributes_float3 = attributes_float3;
  const CyGlobals *kg = &kgv;
  uint co_offset, density_out_offset, color_out_offset, space;
  svm_unpack4(node.z, &co_offset, &density_out_offset, &color_out_offset, &space);
  cfloat3 co = svm_load3(stack, co_offset, err);
  if (space == 0u) { /* NODE_TEX_VOXEL_SPACE_OBJECT */
    if (object == OBJECT_NONE) {
      /* the reference reads an unset object transform here (world volume) */
      cy_set_error(err, CY_ERR_FEATURE, 12);
    }
    else {
      const CyAttr desc = find_attribute(kg, object, prim, 8u /* ATTR_STD_GENERATED_TRANSFORM */);
      co = transform_point(object_itfm(kg, object), co);
      if (desc.offset != (int)ATTR_STD_NOT_FOUND) {
        /* primitive_attribute_matrix (geom_attribute.h:93-103) */
        struct cy_tfm t;
        const hc_float4 r0 = kg->__attributes_float3[desc.offset + 0];
        const hc_float4 r1 = kg->__attributes_float3[desc.offset + 1];
        const hc_float4 r2 = kg->__attributes_float3[desc.offset + 2];
        t.x = {r0.x, r0.y, r0.z, r0.w};
        t.y = {r1.x, r1.y, r1.z, r1.w};
        t.z = {r2.x, r2.y, r2.z, r2.w};
        co = transform_point(&t, co);
      }
    }
  }
  else { /* NODE_TEX_VOXEL_SPACE_WORLD: read_node_float x 3 */
    struct cy_tfm t;
    const hc_uint4 a = svm_nodes[offset++], b = svm_nodes[offset++], c = svm_nodes[offset++];
    t.x = {as_float(a.x), as_float(a.y), as_float(a.z), as_float(a.w)};
    t.y = {as_float(b.x), as_float(b.y), as_float(b.z), as_float(b.w)};
    t.z = {as_float(c.x), as_float(c.y), as_float(c.z), as_float(c.w)};
    co = transform_point(&t, co);
  }
  const hc_float4 r = kernel_tex_image_interp_3d(texture_info, (int)node.y, co);
  if (density_out_offset != SVM_STACK_INVALID) {
    svm_store(stack, density_out_offset, r.w, err);
  }
  if (color_out_offset != SVM_STACK_INVALID) {
    svm_store3(stack, color_out_offset, mk3(r.x, r.y, r.z), err);
  }
  return offset;
}
#endif

CY_NOINLINE int svm_eval_texture_node(const hc_KernelData *data,
                                      const hc_uint4 *svm_nodes,
                                      const hc_KernelObject *objects,
                                      const hc_TextureInfo *texture_info,
                                      const float *ies,
                                      const hc_KernelLight *lights,
                                      CySvmTexIn in,
                                      CySvmStack stack,
                                      hc_uint4 node,
                                      int path_flag,
                                      int offset,
                                      uint *err)
{
  /* the three arrays the nodes read, in a local CyGlobals (registers) */
  CyGlobals kgv;
  kgv.data = data;
  kgv.__svm_nodes = svm_nodes;
  kgv.__objects = objects;
  const CyGlobals *kg = &kgv;
  CySD sdv;
  CySD *sd = &sdv;
  sdv.P = in.P;
  sdv.N = in.N;
  sdv.Ng = in.Ng;
  sdv.I = in.I;
  sdv.u = in.u;
  sdv.v = in.v;
  sdv.ray_length = in.ray_length;
  sdv.object = in.object;
  sdv.flag = in.flag;
  sdv.lamp = in.lamp;
  sdv.type = (in.lamp >= 0) ? (1 << 6) /* PRIMITIVE_LAMP */ : 0;
  kgv.__lights = lights;
  CyPathState stv;
  const CyPathState *state = &stv;
  stv.bounce = in.bounce;
  stv.diffuse_bounce = in.diffuse_bounce;
  stv.glossy_bounce = in.glossy_bounce;
  stv.transparent_bounce = in.transparent_bounce;
  stv.transmission_bounce = in.transmission_bounce;
  switch (node.x) {
      case NODE_GEOMETRY:
        svm_node_geometry(sd, stack, node.y, node.z, err);
        break;
      case NODE_CONVERT:
        svm_node_convert(kg, stack, node.y, node.z, node.w, err);
        break;
      case NODE_TEX_COORD:
        svm_node_tex_coord(kg, sd, path_flag, stack, node, &offset, err);
        break;
      case NODE_HSV:
        svm_node_hsv(stack, node, err);
        break;
      case NODE_MATH:
        svm_node_math(stack, node.y, node.z, node.w, err);
        break;
      case NODE_VECTOR_MATH:
        svm_node_vector_math(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_RGB_RAMP:
        svm_node_rgb_ramp(kg, stack, node, &offset, err);
        break;
      case NODE_GAMMA:
        svm_node_gamma(stack, node.y, node.z, node.w, err);
        break;
      case NODE_BRIGHTCONTRAST:
        svm_node_brightness(stack, node.y, node.z, node.w, err);
        break;
      case NODE_LIGHT_PATH:
        svm_node_light_path(sd, state, stack, node.y, node.z, path_flag, err);
        break;
      case NODE_MAPPING:
        svm_node_mapping(stack, node.y, node.z, node.w, err);
        break;
      case NODE_CAMERA:
        svm_node_camera(kg, sd, stack, node.y, node.z, node.w, err);
        break;
      case NODE_NORMAL:
        svm_node_normal(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_RGB_CURVES:
      case NODE_VECTOR_CURVES:
        svm_node_curves(kg, stack, node, &offset, err);
        break;
      case NODE_VECTOR_ROTATE:
        svm_node_vector_rotate(stack, node.y, node.z, node.w, err);
        break;
      case NODE_VECTOR_TRANSFORM:
        svm_node_vector_transform(kg, sd, stack, node, err);
        break;
      case NODE_TEX_GRADIENT:
        svm_node_tex_gradient(stack, node, err);
        break;
      case NODE_TEX_CHECKER:
        svm_node_tex_checker(stack, node, err);
        break;
      case NODE_LIGHT_FALLOFF:
        svm_node_light_falloff(sd, stack, node, err);
        break;
      case NODE_INVERT:
        svm_node_invert(stack, node.y, node.z, node.w, err);
        break;
      case NODE_MIX:
        svm_node_mix(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_SEPARATE_VECTOR:
        svm_node_separate_vector(stack, node.y, node.z, node.w, err);
        break;
      case NODE_COMBINE_VECTOR:
        svm_node_combine_vector(stack, node.y, node.z, node.w, err);
        break;
      case NODE_SEPARATE_HSV:
        svm_node_separate_hsv(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_COMBINE_HSV:
        svm_node_combine_hsv(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_MAP_RANGE:
        svm_node_map_range(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_CLAMP:
        svm_node_clamp(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_TEX_IMAGE:
        svm_node_tex_image(kg, texture_info, stack, node, &offset, err);
        break;
      case NODE_TEX_ENVIRONMENT:
        svm_node_tex_environment(texture_info, stack, node, err);
        break;
      case NODE_TEX_SKY:
        svm_node_tex_sky(kg, texture_info, stack, node, &offset, err);
        break;
      case NODE_IES:
        svm_node_ies(ies, stack, node, err);
        break;
      case NODE_WAVELENGTH:
        svm_node_wavelength(kg, stack, node.y, node.z, err);
        break;
      case NODE_BLACKBODY:
        svm_node_blackbody(stack, node.y, node.z, err);
        break;
      case NODE_TEX_NOISE:
        svm_node_tex_noise(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_TEX_WAVE:
        svm_node_tex_wave(kg, stack, node, &offset, err);
        break;
      case NODE_TEX_MAGIC:
        svm_node_tex_magic(kg, stack, node, &offset, err);
        break;
      case NODE_TEX_BRICK:
        svm_node_tex_brick(kg, stack, node, &offset, err);
        break;
      case NODE_TEX_WHITE_NOISE:
        svm_node_tex_white_noise(stack, node.y, node.z, node.w, err);
        break;
      case NODE_TEX_MUSGRAVE:
        svm_node_tex_musgrave(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      case NODE_TEX_VORONOI:
        svm_node_tex_voronoi(kg, stack, node.y, node.z, node.w, &offset, err);
        break;
      default:
        return -1;
  }
  return offset;
}

#if CY_CLOSURE_EXT
/* svm_closure.h:912-962 svm_node_closure_volume: absorption (extinction of
 * 1 - color) or Henyey-Greenstein scattering (a phase closure with its g in
 * alpha_x) times density; both add to the extinction. */
CY_FN void svm_node_closure_volume(CySD *sd, CySvmStack stack, hc_uint4 node, int shader_type, uint *err)
{
  if (shader_type != 1) {
    return;
  }
  const uint type = node.y & 0xFF, density_offset = (node.y >> 8) & 0xFF;
  const uint anisotropy_offset = (node.y >> 16) & 0xFF, mix_weight_offset = (node.y >> 24) & 0xFF;
  const float mix_weight = (mix_weight_offset != SVM_STACK_INVALID) ? svm_load(stack, mix_weight_offset, err) : 1.0f;
  if (mix_weight == 0.0f) {
    return;
  }
  float density = (density_offset != SVM_STACK_INVALID) ? svm_load(stack, density_offset, err) : as_float(node.z);
  density = mix_weight * fmaxf(density, 0.0f);
  cfloat3 weight = sd->svm_closure_weight;
  if (type == CLOSURE_VOLUME_ABSORPTION_ID) {
    weight = sub3(mk3(1.0f, 1.0f, 1.0f), weight);
  }
  weight = mul3f(weight, density);
  if (type == CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID) {
    CyClosure *volume = bsdf_alloc(sd, weight);
    if (volume) {
      const float g = (anisotropy_offset != SVM_STACK_INVALID) ? svm_load(stack, anisotropy_offset, err) :
                                                                 as_float(node.w);
      /* volume_henyey_greenstein_setup (closure/volume.h:54-62) */
      volume->type = CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID;
      volume->alpha_x = ((g < 0.0f) ? -1.0f : 1.0f) * fminf(fabsf(g), 1.0f - 1e-3f);
      sd->flag |= SD_SCATTER;
    }
  }
  /* volume_extinction_setup (closure/volume.h:24-34) */
  if (sd->flag & SD_EXTINCTION) {
    sd->closure_transparent_extinction = add3(sd->closure_transparent_extinction, weight);
  }
  else {
    sd->flag |= SD_EXTINCTION;
    sd->closure_transparent_extinction = weight;
  }
}

/* svm_closure.h:964-1075 svm_node_principled_volume without volume attributes
 * (the host packs none: find_attribute finds nothing) and without blackbody
 * (hipcy_load_kernels refuses a blackbody intensity). */
CY_FN void svm_node_principled_volume(const CyGlobals *kg, CySD *sd, CySvmStack stack, hc_uint4 node, int shader_type,
                                      int path_flag, int *offset, uint *err)
{
  const hc_uint4 value_node = kg->__svm_nodes[*offset];
  *offset += 2; /* value node, attribute node */
  if (shader_type != 1) {
    return;
  }
  const uint density_offset = node.y & 0xFF, anisotropy_offset = (node.y >> 8) & 0xFF;
  const uint absorption_color_offset = (node.y >> 16) & 0xFF, mix_weight_offset = (node.y >> 24) & 0xFF;
  const float mix_weight = (mix_weight_offset != SVM_STACK_INVALID) ? svm_load(stack, mix_weight_offset, err) : 1.0f;
  if (mix_weight == 0.0f) {
    return;
  }
  float density = (density_offset != SVM_STACK_INVALID) ? svm_load(stack, density_offset, err) :
                                                         as_float(value_node.x);
  density = mix_weight * fmaxf(density, 0.0f);
  if (density > CLOSURE_WEIGHT_CUTOFF) {
    const cfloat3 color = sd->svm_closure_weight;
    CyClosure *volume = bsdf_alloc(sd, mul3f(color, density));
    if (volume) {
      const float g = (anisotropy_offset != SVM_STACK_INVALID) ? svm_load(stack, anisotropy_offset, err) :
                                                                 as_float(value_node.y);
      volume->type = CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID;
      volume->alpha_x = ((g < 0.0f) ? -1.0f : 1.0f) * fminf(fabsf(g), 1.0f - 1e-3f);
      sd->flag |= SD_SCATTER;
    }
    const cfloat3 zero = mk3(0.0f, 0.0f, 0.0f);
    const cfloat3 one = mk3(1.0f, 1.0f, 1.0f);
    const cfloat3 ac = svm_load3(stack, absorption_color_offset, err);
    const cfloat3 absorption_color = max3v(mk3(sqrtf(ac.x), sqrtf(ac.y), sqrtf(ac.z)), zero);
    const cfloat3 absorption = mul3(max3v(sub3(one, color), zero), max3v(sub3(one, absorption_color), zero));
    const cfloat3 weight = mul3f(add3(color, absorption), density);
    if (sd->flag & SD_EXTINCTION) {
      sd->closure_transparent_extinction = add3(sd->closure_transparent_extinction, weight);
    }
    else {
      sd->flag |= SD_EXTINCTION;
      sd->closure_transparent_extinction = weight;
    }
  }
  if (path_flag & PATH_RAY_SHADOW) {
    return;
  }
  const uint emission_offset = node.z & 0xFF, emission_color_offset = (node.z >> 8) & 0xFF;
  const float emission = (emission_offset != SVM_STACK_INVALID) ? svm_load(stack, emission_offset, err) :
                                                                 as_float(value_node.z);
  if (emission > CLOSURE_WEIGHT_CUTOFF) {
    const cfloat3 emission_color = svm_load3(stack, emission_color_offset, err);
    emission_setup(sd, mul3f(emission_color, emission));
  }
}
#endif

/* type: SHADER_TYPE_SURFACE (0), SHADER_TYPE_VOLUME (1) or SHADER_TYPE_DISPLACEMENT (2), svm.h:236-246 */
#if CY_SVM_TEX && CY_CLOSURE_EXT
/* svm_wireframe.h:39-88: 1 when P lies within size / 2 (times the pixel's
 * footprint from the ray differentials with use_pixel_size) of an edge of
 * the shading point's triangle */
CY_FN float wireframe(const CyGlobals *kg, const CySD *sd, float size, int pixel_size, cfloat3 P)
{
  if (sd->prim != PRIM_NONE && (sd->type & PRIMITIVE_ALL_TRIANGLE)) {
    cfloat3 Co[3];
    float pixelwidth = 1.0f;
    const int np = 3;
    triangle_verts(kg, sd->prim, Co);
    if (!(sd->object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
      const struct cy_tfm *tfm = object_tfm(kg, sd->object);
      Co[0] = transform_point(tfm, Co[0]);
      Co[1] = transform_point(tfm, Co[1]);
      Co[2] = transform_point(tfm, Co[2]);
    }
    if (pixel_size) {
      /* the differentials of P projected on the plane across I */
      const float pixelwidth_x = len3(sub3(sd->dP.dx, mul3f(sd->I, dot3(sd->dP.dx, sd->I))));
      const float pixelwidth_y = len3(sub3(sd->dP.dy, mul3f(sd->I, dot3(sd->dP.dy, sd->I))));
      pixelwidth = (pixelwidth_x + pixelwidth_y) * 0.5f;
    }
    /* half the width (the neighbouring face renders the other half), squared */
    pixelwidth *= 0.5f * size;
    pixelwidth *= pixelwidth;
    for (int i = 0; i < np; i++) {
      const int i2 = i ? i - 1 : np - 1;
      const cfloat3 dir = sub3(P, Co[i]);
      const cfloat3 edge = sub3(Co[i], Co[i2]);
      const cfloat3 crs = cross3(edge, dir);
      /* dot(crs, crs) / dot(edge, edge): the squared distance to the edge */
      if (dot3(crs, crs) < (dot3(edge, edge) * pixelwidth)) {
        return 1.0f;
      }
    }
  }
  return 0.0f;
}

/* svm_wireframe.h:90-127; the bump forms add a one-sided difference */
CY_FN void svm_node_wireframe(const CyGlobals *kg, const CySD *sd, CySvmStack stack, hc_uint4 node, uint *err)
{
  const uint in_size = node.y, out_fac = node.z;
  const uint use_pixel_size = node.w & 0xFF, bump_offset = (node.w >> 8) & 0xFF;
  const float size = svm_load(stack, in_size, err);
  const int pixel_size = (int)use_pixel_size;
  float f = wireframe(kg, sd, size, pixel_size, sd->P);
  if (bump_offset == 1) { /* NODE_BUMP_OFFSET_DX */
    const cfloat3 Px = sub3(sd->P, sd->dP.dx);
    f += (f - wireframe(kg, sd, size, pixel_size, Px)) / len3(sd->dP.dx);
  }
  else if (bump_offset == 2) { /* NODE_BUMP_OFFSET_DY */
    const cfloat3 Py = sub3(sd->P, sd->dP.dy);
    f += (f - wireframe(kg, sd, size, pixel_size, Py)) / len3(sd->dP.dy);
  }
  if (out_fac != SVM_STACK_INVALID) {
    svm_store(stack, out_fac, f, err);
  }
}

/* the ray-tracing nodes (cy_svm_raytrace.h, after the local traversals) */
CY_FN void svm_node_ao(const CyGlobals *kg, CySD *sd, const CyPathState *state, CySvmStack stack, hc_uint4 node,
                       uint *err);
CY_FN void svm_node_bevel(const CyGlobals *kg, CySD *sd, const CyPathState *state, CySvmStack stack, hc_uint4 node,
                          uint *err);
#endif

/* buffer: the camera path's render-buffer pixel (kernel_path_integrate passes
 * it to every surface evaluation of the path, kernel_path.h:569), written by
 * the AOV output nodes; nullptr elsewhere */
CY_FN void svm_eval_nodes(const CyGlobals *kg, CySD *sd, const CyPathState *state, int path_flag, uint *err,
                          int type = 0, float *buffer = nullptr)
{
  CySvmStack stack;
  stack.p = sd->svm_stack;
  stack.stride = sd->svm_stride;
  stack.fast = sd->svm_fast;
  stack.spill = sd->svm_spill;
  int offset = (int)((uint)sd->shader & SHADER_MASK);
  for (int guard = 0; guard < 4096; guard++) {
    hc_uint4 node = kg->__svm_nodes[offset];
    offset++;
    switch (node.x) {
      case NODE_END:
        return;
      case NODE_SHADER_JUMP:
        offset = (int)(type == 2 ? node.w : type == 1 ? node.z : node.y);
        break;
#if CY_CLOSURE_EXT
      case NODE_CLOSURE_VOLUME:
        svm_node_closure_volume(sd, stack, node, type, err);
        break;
      case NODE_PRINCIPLED_VOLUME:
        svm_node_principled_volume(kg, sd, stack, node, type, path_flag, &offset, err);
        break;
#endif
      case NODE_CLOSURE_BSDF:
        svm_node_closure_bsdf(kg, sd, stack, node, path_flag, &offset, err);
        break;
      case NODE_CLOSURE_EMISSION:
      case NODE_CLOSURE_BACKGROUND: {
        uint mix_weight_offset = node.y;
        cfloat3 weight = sd->svm_closure_weight;
        if (mix_weight_offset != SVM_STACK_INVALID) {
          float mix_weight = svm_load(stack, mix_weight_offset, err);
          if (mix_weight == 0.0f) {
            break;
          }
          weight = mul3f(weight, mix_weight);
        }
        emission_setup(sd, weight);
        break;
      }
      case NODE_CLOSURE_SET_WEIGHT:
        sd->svm_closure_weight = mk3(as_float(node.y), as_float(node.z), as_float(node.w));
        break;
      case NODE_CLOSURE_WEIGHT:
        sd->svm_closure_weight = svm_load3(stack, node.y, err);
        break;
      case NODE_EMISSION_WEIGHT: {
        float strength = svm_load(stack, node.z, err);
        sd->svm_closure_weight = mul3f(svm_load3(stack, node.y, err), strength);
        break;
      }
      case NODE_MIX_CLOSURE: {
        uint weight_offset = node.y & 0xFF, in_weight_offset = (node.y >> 8) & 0xFF;
        uint weight1_offset = (node.y >> 16) & 0xFF, weight2_offset = (node.y >> 24) & 0xFF;
        float weight = saturate(svm_load(stack, weight_offset, err));
        float in_weight = (in_weight_offset != SVM_STACK_INVALID) ?
                              svm_load(stack, in_weight_offset, err) :
                              1.0f;
        if (weight1_offset != SVM_STACK_INVALID) {
          svm_store(stack, weight1_offset, in_weight * (1.0f - weight), err);
        }
        if (weight2_offset != SVM_STACK_INVALID) {
          svm_store(stack, weight2_offset, in_weight * weight, err);
        }
        break;
      }
      case NODE_JUMP_IF_ZERO:
        if (svm_load(stack, node.z, err) == 0.0f) {
          offset += (int)node.y;
        }
        break;
      case NODE_JUMP_IF_ONE:
        if (svm_load(stack, node.z, err) == 1.0f) {
          offset += (int)node.y;
        }
        break;
      case NODE_VALUE_F:
        svm_store(stack, node.z, as_float(node.y), err);
        break;
      case NODE_VALUE_V: {
        hc_uint4 node1 = kg->__svm_nodes[offset];
        offset++;
        svm_store3(stack, node.y, mk3(as_float(node1.y), as_float(node1.z), as_float(node1.w)), err);
        break;
      }
      case NODE_FRESNEL: {
        uint normal_offset = node.w & 0xFF, out_offset = (node.w >> 8) & 0xFF;
        float eta = (node.y != SVM_STACK_INVALID) ? svm_load(stack, node.y, err) : as_float(node.z);
        cfloat3 normal_in = (normal_offset != SVM_STACK_INVALID) ?
                                svm_load3(stack, normal_offset, err) :
                                sd->N;
        eta = fmaxf(eta, 1e-5f);
        eta = (sd->flag & SD_BACKFACING) ? 1.0f / eta : eta;
        svm_store(stack, out_offset, fresnel_dielectric_cos(dot3(sd->I, normal_in), eta), err);
        break;
      }
      case NODE_LAYER_WEIGHT: {
        uint ltype = node.w & 0xFF, normal_offset = (node.w >> 8) & 0xFF;
        uint out_offset = (node.w >> 16) & 0xFF;
        float blend = (node.y != SVM_STACK_INVALID) ? svm_load(stack, node.y, err) :
                                                      as_float(node.z);
        cfloat3 normal_in = (normal_offset != SVM_STACK_INVALID) ?
                                svm_load3(stack, normal_offset, err) :
                                sd->N;
        float f;
        if (ltype == NODE_LAYER_WEIGHT_FRESNEL) {
          float eta = fmaxf(1.0f - blend, 1e-5f);
          eta = (sd->flag & SD_BACKFACING) ? eta : 1.0f / eta;
          f = fresnel_dielectric_cos(dot3(sd->I, normal_in), eta);
        }
        else {
          f = fabsf(dot3(sd->I, normal_in));
          if (blend != 0.5f) {
            blend = cclamp(blend, 0.0f, 1.0f - 1e-5f);
            blend = (blend < 0.5f) ? 2.0f * blend : 0.5f / (1.0f - blend);
            CY_DBG3(sd, "lw dot blend", mk3(f, blend, 0.0f));
            f = cy_powf(f, blend); /* glibc powf, restated (cy_math.h) */
          }
          CY_DBG3(sd, "lw pow N", mk3(f, normal_in.x, normal_in.z));
          f = 1.0f - f;
        }
        svm_store(stack, out_offset, f, err);
        break;
      }
#if CY_SVM_TEX
#if CY_CLOSURE_EXT
      case NODE_WIREFRAME:
        svm_node_wireframe(kg, sd, stack, node, err);
        break;
      /* svm_ao.h, svm_bevel.h: rays traced from the shader */
      case NODE_AMBIENT_OCCLUSION:
        svm_node_ao(kg, sd, state, stack, node, err);
        break;
      case NODE_BEVEL:
        svm_node_bevel(kg, sd, state, stack, node, err);
        break;
#endif
      /* svm_closure.h:1113-1129: a holdout closure of the mix weight */
      case NODE_CLOSURE_HOLDOUT: {
        const uint mix_weight_offset = node.y;
        cfloat3 weight = sd->svm_closure_weight;
        if (mix_weight_offset != SVM_STACK_INVALID) {
          const float mix_weight = svm_load(stack, mix_weight_offset, err);
          if (mix_weight == 0.0f) {
            break;
          }
          weight = mul3f(weight, mix_weight);
        }
        closure_alloc(sd, CLOSURE_HOLDOUT_ID, weight);
        sd->flag |= SD_HOLDOUT;
        break;
      }
      /* svm_mapping.h:47-59: a texture node's TextureMapping matrix */
      case NODE_TEXTURE_MAPPING: {
        const cfloat3 v = svm_load3(stack, node.y, err);
        struct cy_tfm tfm;
        struct cy_f4 *rows[3] = {&tfm.x, &tfm.y, &tfm.z};
        for (int r = 0; r < 3; r++) {
          const hc_uint4 row = kg->__svm_nodes[offset];
          offset++;
          rows[r]->x = as_float(row.x);
          rows[r]->y = as_float(row.y);
          rows[r]->z = as_float(row.z);
          rows[r]->w = as_float(row.w);
        }
        svm_store3(stack, node.z, transform_point(&tfm, v), err);
        break;
      }
      /* svm_mapping.h:61-71: min(max(mn, v), mx) per component */
      case NODE_MIN_MAX: {
        const cfloat3 v = svm_load3(stack, node.y, err);
        const hc_uint4 a = kg->__svm_nodes[offset], b = kg->__svm_nodes[offset + 1];
        offset += 2;
        const cfloat3 r = mk3(cy_min(cy_max(as_float(a.x), v.x), as_float(b.x)),
                              cy_min(cy_max(as_float(a.y), v.y), as_float(b.y)),
                              cy_min(cy_max(as_float(a.z), v.z), as_float(b.z)));
        svm_store3(stack, node.z, r, err);
        break;
      }
      /* svm_closure.h:1188-1194: the bump program's normal becomes the
       * shading normal (displacement method "bump") */
      case NODE_CLOSURE_SET_NORMAL: {
        const cfloat3 normal = svm_load3(stack, node.y, err);
        sd->N = normal;
        svm_store3(stack, node.z, normal, err);
        break;
      }
      /* svm_displace.h:86-167 (displacement programs, SHADER_EVAL_DISPLACE) */
      case NODE_SET_DISPLACEMENT:
        sd->P = add3(sd->P, svm_load3(stack, node.y, err));
        break;
      case NODE_DISPLACEMENT: {
        const uint height_off = node.y & 0xFF, mid_off = (node.y >> 8) & 0xFF;
        const uint scale_off = (node.y >> 16) & 0xFF, normal_off = (node.y >> 24) & 0xFF;
        const float height = svm_load(stack, height_off, err);
        const float midlevel = svm_load(stack, mid_off, err);
        const float scale = svm_load(stack, scale_off, err);
        cfloat3 dP = (normal_off != SVM_STACK_INVALID) ? svm_load3(stack, normal_off, err) : sd->N;
        if (node.w == NODE_NORMAL_MAP_OBJECT) {
          if (sd->object != OBJECT_NONE) {
            dP = normalize3(transform_direction_transposed(object_tfm(kg, sd->object), dP));
          }
          dP = mul3f(dP, (height - midlevel) * scale);
          dP = transform_direction(object_tfm(kg, sd->object), dP);
        }
        else {
          dP = mul3f(dP, (height - midlevel) * scale);
        }
        svm_store3(stack, node.z, dP, err);
        break;
      }
      case NODE_VECTOR_DISPLACEMENT: {
        const hc_uint4 data = kg->__svm_nodes[offset];
        offset++;
        const uint space = data.x;
        const uint vector_off = node.y & 0xFF, mid_off = (node.y >> 8) & 0xFF;
        const uint scale_off = (node.y >> 16) & 0xFF, disp_off = (node.y >> 24) & 0xFF;
        const cfloat3 vec = svm_load3(stack, vector_off, err);
        const float midlevel = svm_load(stack, mid_off, err);
        const float scale = svm_load(stack, scale_off, err);
        cfloat3 dP = mul3f(sub3(vec, mk3(midlevel, midlevel, midlevel)), scale);
        if (space == NODE_NORMAL_MAP_TANGENT) {
          /* tangent space needs the tangent attributes: rejected at load_kernels */
          cy_set_error(err, CY_ERR_SVM_NODE, NODE_VECTOR_DISPLACEMENT);
          return;
        }
        if (space != NODE_NORMAL_MAP_WORLD) {
          dP = transform_direction(object_tfm(kg, sd->object), dP);
        }
        svm_store3(stack, disp_off, dP, err);
        break;
      }
#endif
      default:
#if !CY_SVM_TEX
        cy_set_error(err, CY_ERR_SVM_NODE, node.x);
        return;
#else
      {
        if (node.x == NODE_AOV_START) {
          /* svm_aov.h:21-27 svm_node_aov_check: only the camera path's first
           * (non-transparent) hit writes AOVs; otherwise the nodes after this
           * one, which only feed the AOV outputs, are skipped */
          if (!(buffer != nullptr && (path_flag & PATH_RAY_CAMERA) && !(path_flag & PATH_RAY_SINGLE_PASS_DONE))) {
            return;
          }
          break;
        }
        if (node.x == NODE_AOV_COLOR) {
          /* svm_aov.h:29-39: kernel_write_pass_float4, an atomic add on GPU
           * devices (kernel_write_passes.h:49-65) */
          const cfloat3 val = svm_load3(stack, node.y, err);
          if (buffer) {
            float *p = buffer + KD->film.pass_aov_color + 4 * (int)node.z;
            cy_pass_add(p + 0, val.x);
            cy_pass_add(p + 1, val.y);
            cy_pass_add(p + 2, val.z);
            cy_pass_add(p + 3, 1.0f);
          }
          break;
        }
        if (node.x == NODE_AOV_VALUE) {
          /* svm_aov.h:41-50 */
          const float val = svm_load(stack, node.y, err);
          if (buffer) {
            cy_pass_add(buffer + KD->film.pass_aov_value + (int)node.z, val);
          }
          break;
        }
        if (node.x == NODE_TEX_VOXEL) {
          offset = svm_node_tex_voxel(kg->__svm_nodes, kg->__objects, kg->__attributes_map, kg->__attributes_float3,
                                      kg->__texture_info, sd->object, sd->prim, stack, node, offset, err);
          break;
        }
#if CY_CLOSURE_EXT
        if (node.x == NODE_ENTER_BUMP_EVAL) {
          /* svm_bump.h:21-46: save P, dP.dx, dP.dy, then evaluate the bump
           * program at the undisplaced position */
          svm_store3(stack, node.y + 0, sd->P, err);
          svm_store3(stack, node.y + 3, sd->dP.dx, err);
          svm_store3(stack, node.y + 6, sd->dP.dy, err);
          CyAttrIn bin;
          bin.P = sd->P;
          bin.N = sd->N;
          bin.Ng = sd->Ng;
          bin.I = sd->I;
          bin.u = sd->u;
          bin.v = sd->v;
          bin.object = sd->object;
          bin.prim = sd->prim;
          bin.type = sd->type;
          bin.flag = sd->flag;
          bin.shader = sd->shader;
          bin.dPdu = sd->dPdu;
          bin.dPdx = sd->dP.dx;
          bin.dPdy = sd->dP.dy;
          bin.bump = 0;
          bin.bump_du = bin.bump_dv = 0.0f;
          const CyBumpEval be = svm_bump_undisplaced(kg->__objects, kg->__attributes_map, kg->__attributes_float3,
                                                     kg->__tri_vindex, bin, sd->du.dx, sd->du.dy, sd->dv.dx,
                                                     sd->dv.dy);
          if (be.found) {
            sd->P = be.P;
            sd->dP.dx = be.dPdx;
            sd->dP.dy = be.dPdy;
          }
          break;
        }
        if (node.x == NODE_LEAVE_BUMP_EVAL) {
          /* svm_bump.h:48-60: restore the state */
          sd->P = svm_load3(stack, node.y + 0, err);
          sd->dP.dx = svm_load3(stack, node.y + 3, err);
          sd->dP.dy = svm_load3(stack, node.y + 6, err);
          break;
        }
        /* the bump forms (svm.h:298-345) read their centre node at
         * P + dP.dx (.dy), u + du.dx, v + dv.dx (svm_geometry.h:54-100,
         * svm_tex_coord.h:97-255), attributes plus their derivative
         * (svm_attribute.h:92-188, svm_vertex_color.h:38-90) */
        int bump = 0;
        switch (node.x) {
          case NODE_GEOMETRY_BUMP_DX:
          case NODE_GEOMETRY_BUMP_DY:
            bump = (node.x == NODE_GEOMETRY_BUMP_DX) ? 1 : 2;
            node.x = NODE_GEOMETRY;
            break;
          case NODE_ATTR_BUMP_DX:
          case NODE_ATTR_BUMP_DY:
            bump = (node.x == NODE_ATTR_BUMP_DX) ? 1 : 2;
            node.x = NODE_ATTR;
            break;
          case NODE_VERTEX_COLOR_BUMP_DX:
          case NODE_VERTEX_COLOR_BUMP_DY:
            bump = (node.x == NODE_VERTEX_COLOR_BUMP_DX) ? 1 : 2;
            node.x = NODE_VERTEX_COLOR;
            break;
          case NODE_TEX_COORD_BUMP_DX:
          case NODE_TEX_COORD_BUMP_DY:
            bump = (node.x == NODE_TEX_COORD_BUMP_DX) ? 1 : 2;
            node.x = NODE_TEX_COORD;
            break;
        }
#endif
        if (node.x == NODE_ATTR || node.x == NODE_VERTEX_COLOR || node.x == NODE_NORMAL_MAP ||
            node.x == NODE_TANGENT || node.x == NODE_OBJECT_INFO || node.x == NODE_PARTICLE_INFO ||
            (node.x == NODE_GEOMETRY && node.y == 2u)
#if CY_CLOSURE_EXT
            || node.x == NODE_SET_BUMP || node.x == NODE_HAIR_INFO
#endif
        ) {
          CyAttrIn ain;
          ain.P = sd->P;
          ain.N = sd->N;
          ain.Ng = sd->Ng;
          ain.I = sd->I;
          ain.u = sd->u;
          ain.v = sd->v;
          ain.object = sd->object;
          ain.prim = sd->prim;
          ain.type = sd->type;
          ain.flag = sd->flag;
          ain.shader = sd->shader;
#if CY_CLOSURE_EXT
          ain.dPdu = sd->dPdu;
          ain.dPdx = sd->dP.dx;
          ain.dPdy = sd->dP.dy;
          ain.bump = bump;
#ifdef CY_DBG_X
          ain.dbg = sd->dbg;
#endif
          ain.bump_du = (bump == 2) ? sd->du.dy : sd->du.dx;
          ain.bump_dv = (bump == 2) ? sd->dv.dy : sd->dv.dx;
#endif
          svm_eval_attribute_node(kg->__objects, kg->__shaders, kg->__attributes_map, kg->__attributes_float,
                                  kg->__attributes_float2, kg->__attributes_float3, kg->__attributes_uchar4,
                                  kg->__tri_vindex, kg->__curves, kg->__curve_keys, kg->__particles, ain, stack,
                                  node, err);
          break;
        }
        CySvmTexIn in;
        in.P = sd->P;
        in.N = sd->N;
        in.Ng = sd->Ng;
        in.I = sd->I;
        in.u = sd->u;
        in.v = sd->v;
        in.ray_length = sd->ray_length;
        in.object = sd->object;
        in.flag = sd->flag;
        in.lamp = (sd->type == (1 << 6) /* PRIMITIVE_LAMP */) ? sd->lamp : -1;
        in.bounce = state ? state->bounce : 0; /* background SHADER task: PathState {0} */
        in.diffuse_bounce = state ? state->diffuse_bounce : 0;
        in.glossy_bounce = state ? state->glossy_bounce : 0;
        in.transparent_bounce = state ? state->transparent_bounce : 0;
        in.transmission_bounce = state ? state->transmission_bounce : 0;
#if CY_CLOSURE_EXT
        if (bump) {
          /* only the position-based outputs read P, u, v */
          in.P = add3(sd->P, (bump == 2) ? sd->dP.dy : sd->dP.dx);
          in.u = sd->u + ((bump == 2) ? sd->du.dy : sd->du.dx);
          in.v = sd->v + ((bump == 2) ? sd->dv.dy : sd->dv.dx);
        }
#endif
        offset = svm_eval_texture_node(kg->data, kg->__svm_nodes, kg->__objects, kg->__texture_info, kg->__ies, kg->__lights, in,
                                       stack, node, path_flag, offset, err);
        if (offset < 0) {
          cy_set_error(err, CY_ERR_SVM_NODE, node.x);
          return;
        }
        break;
      }
#endif
    }
  }
}

/* kernel_shader.h:1057-1112 */
CY_FN void shader_eval_surface(
    const CyGlobals *kg, CySD *sd, const CyPathState *state, int path_flag, uint *err, float *buffer = nullptr)
{
  int max_closures;
  if (path_flag & (PATH_RAY_TERMINATE | PATH_RAY_SHADOW | PATH_RAY_EMISSION)) {
    max_closures = 0;
  }
  else {
    max_closures = KD->integrator.max_closures;
  }
  sd->num_closure = 0;
  /* the closure array holds CY_MAX_CLOSURE (the variant load_kernels picked
   * holds every closure the shaders allocate, so allocations succeed exactly
   * as with the reference's budget; the clamp keeps extras in the array) */
  sd->num_closure_left = (max_closures < CY_MAX_CLOSURE) ? max_closures : CY_MAX_CLOSURE;
  svm_eval_nodes(kg, sd, state, path_flag, err, 0, buffer);
#if CY_CLOSURE_EXT
  if ((sd->flag & SD_BSDF_NEEDS_LCG) && state) {
    /* kernel_shader.h:1109-1111: lcg_state_init_addrspace(state, 0xb4bc3953) */
    sd->lcg_state = lcg_init(state->rng_hash + (uint)state->rng_offset + (uint)state->sample * 0xb4bc3953u);
  }
#endif
}

/* SHADER_EVAL_DISPLACE for one (object, prim, u, v): kernel_displace_evaluate
 * (kernel_bake.h:446-472).  shader_setup_from_displace (kernel_shader.h:367-393)
 * = triangle_point_normal (geom_triangle.h:44-66) + shader_setup_from_sample
 * (kernel_shader.h:244-360) with I = 0, t = 0, the smooth normal forced and the
 * object transform applied when the mesh is not pre-transformed; then the
 * displacement program moves sd->P and D = P' - P goes to object space. */
CY_FN cfloat3 displace_evaluate(const CyGlobals *kg, int object, int prim, float u, float v, CyShadeMem mem,
                                uint *err)
{
  CySD sd;
  sd.closure = mem.closure;
  sd.svm_stack = mem.svm_stack;
  sd.svm_stride = mem.svm_stride;
  sd.svm_fast = mem.svm_fast;
  sd.svm_spill = mem.svm_spill;
  cfloat3 V[3];
  triangle_verts(kg, prim, V);
  const float t = 1.0f - u - v;
  const cfloat3 P = add3(add3(mul3f(V[0], u), mul3f(V[1], v)), mul3f(V[2], t));
  const int object_flag = (int)kg->__object_flag[object];
  cfloat3 Ng = (object_flag & SD_OBJECT_NEGATIVE_SCALE_APPLIED) ?
                   normalize3(cross3(sub3(V[2], V[0]), sub3(V[1], V[0]))) :
                   normalize3(cross3(sub3(V[1], V[0]), sub3(V[2], V[0])));
  sd.shader = (int)(kg->__tri_shader[prim] | SHADER_SMOOTH_NORMAL);
  sd.P = P;
  sd.N = Ng;
  sd.Ng = Ng;
  sd.I = mk3(0.0f, 0.0f, 0.0f);
  sd.type = PRIMITIVE_TRIANGLE;
  sd.object = object;
  sd.prim = prim;
  sd.u = u;
  sd.v = v;
  sd.ray_length = 0.0f;
  sd.flag = kg->__shaders[(uint)sd.shader & SHADER_MASK].flags;
  sd.object_flag = object_flag;
  if (!(object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
    sd.P = transform_point(object_tfm(kg, object), sd.P);
    sd.Ng = object_normal_transform(kg, object, sd.Ng);
    sd.N = sd.Ng;
    sd.I = transform_direction(object_tfm(kg, object), sd.I);
  }
  sd.N = triangle_smooth_normal(kg, Ng, prim, u, v);
  if (!(object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
    sd.N = object_normal_transform(kg, object, sd.N);
  }
#if CY_CLOSURE_EXT
  triangle_dPdudv(kg, prim, &sd.dPdu, &sd.dPdv);
  if (!(object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
    sd.dPdu = transform_direction(object_tfm(kg, object), sd.dPdu);
    sd.dPdv = transform_direction(object_tfm(kg, object), sd.dPdv);
  }
  sd_zero_differentials(&sd); /* shader_setup_from_sample: no ray differentials */
#endif
  /* backfacing test: dot(Ng, I) with I = 0 is never negative */
  sd.num_closure = 0;
  sd.num_closure_left = 0;
  sd.svm_closure_weight = mk3(0.0f, 0.0f, 0.0f);
  const cfloat3 P0 = sd.P;
  svm_eval_nodes(kg, &sd, nullptr, 0, err, 2);
  return transform_direction(object_itfm(kg, object), sub3(sd.P, P0));
}

/* kernel_shader.h:527-551 */
CY_FN void shader_prepare_closures(CySD *sd, const CyPathState *state)
{
  if (state->bounce + state->transparent_bounce == 0 && sd->num_closure > 1) {
    float sum = 0.0f;
    for (int i = 0; i < sd->num_closure; i++) {
      CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_BSDF_OR_BSSRDF(sc->type)) {
        sum += sc->sample_weight;
      }
    }
    for (int i = 0; i < sd->num_closure; i++) {
      CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_BSDF_OR_BSSRDF(sc->type)) {
        sc->sample_weight = cmax(sc->sample_weight, 0.125f * sum);
      }
    }
  }
}

/* kernel_shader.h:553-582 (use_light_pass == 0: only eval->diffuse accumulates). */
CY_FN void shader_bsdf_multi_eval(const CySD *sd,
                                  const cfloat3 omega_in,
                                  float *pdf,
                                  int skip_sc,
                                  cfloat3 *result_eval,
                                  float sum_pdf,
                                  float sum_sample_weight)
{
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    if (i != skip_sc && CLOSURE_IS_BSDF(sc->type)) {
      float bsdf_pdf = 0.0f;
      cfloat3 eval = bsdf_eval(sd, sc, omega_in, &bsdf_pdf);
      if (bsdf_pdf != 0.0f) {
        /* bsdf_eval_accum(..., mis_weight 1.0): value *= 1.0f, then diffuse += */
        cfloat3 value = mul3(eval, sc->weight);
        value = mul3f(value, 1.0f);
        *result_eval = add3(*result_eval, value);
        sum_pdf += bsdf_pdf * sc->sample_weight;
      }
      sum_sample_weight += sc->sample_weight;
    }
  }
  *pdf = (sum_sample_weight > 0.0f) ? sum_pdf / sum_sample_weight : 0.0f;
}

/* _shader_bsdf_multi_eval_branched (kernel_shader.h:583-601), which
 * shader_bsdf_eval runs whenever KernelIntegrator.branched is set: every BSDF
 * closure MIS-weighted against the light on its own pdf; *eval_no_mis the
 * unweighted sum (BsdfEval.sum_no_mis) */
CY_FN void shader_bsdf_eval_branched(const CySD *sd, cfloat3 omega_in, float light_pdf, bool use_mis, cfloat3 *eval,
                                     cfloat3 *eval_no_mis)
{
  *eval = mk3(0.0f, 0.0f, 0.0f);
  *eval_no_mis = mk3(0.0f, 0.0f, 0.0f);
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    if (CLOSURE_IS_BSDF(sc->type)) {
      float bsdf_pdf = 0.0f;
      const cfloat3 e = bsdf_eval(sd, sc, omega_in, &bsdf_pdf);
      if (bsdf_pdf != 0.0f) {
        const float mis_weight = use_mis ? power_heuristic(light_pdf, bsdf_pdf) : 1.0f;
        const cfloat3 value = mul3(e, sc->weight);
        *eval_no_mis = add3(*eval_no_mis, value);
        *eval = add3(*eval, mul3f(value, mis_weight));
      }
    }
  }
}

/* BsdfEval with light passes (kernel_types.h:565-581, kernel_accumulate.h:
 * 24-98): the BSDF value per closure component */
#define CLOSURE_IS_BSDF_GLOSSY(type) \
  (((type) >= CLOSURE_BSDF_REFLECTION_ID && (type) <= CLOSURE_BSDF_HAIR_REFLECTION_ID) || \
   (type) == CLOSURE_BSDF_HAIR_PRINCIPLED_ID)
#define CLOSURE_IS_BSDF_TRANSMISSION(type) \
  ((type) >= CLOSURE_BSDF_REFRACTION_ID && (type) <= CLOSURE_BSDF_HAIR_TRANSMISSION_ID)
#define CLOSURE_IS_BSDF_BSSRDF(type) \
  ((type) == CLOSURE_BSDF_BSSRDF_ID || (type) == CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID)
typedef struct CyBsdfEvalLP {
  cfloat3 diffuse, glossy, transmission, transparent, volume;
} CyBsdfEvalLP;

CY_FN void bsdf_eval_lp_zero(CyBsdfEvalLP *e)
{
  e->diffuse = e->glossy = e->transmission = e->transparent = e->volume = mk3(0.0f, 0.0f, 0.0f);
}

/* bsdf_eval_accum's component (transparent closures add nothing there) */
CY_FN cfloat3 *bsdf_eval_lp_component(CyBsdfEvalLP *e, int type)
{
  if (CLOSURE_IS_BSDF_DIFFUSE(type) || CLOSURE_IS_BSDF_BSSRDF(type)) {
    return &e->diffuse;
  }
  if (CLOSURE_IS_BSDF_GLOSSY(type)) {
    return &e->glossy;
  }
  if (CLOSURE_IS_BSDF_TRANSMISSION(type)) {
    return &e->transmission;
  }
  if (CLOSURE_IS_PHASE(type)) {
    return &e->volume;
  }
  return nullptr;
}

CY_FN cfloat3 bsdf_eval_lp_sum(const CyBsdfEvalLP *e)
{
  return add3(add3(add3(e->diffuse, e->glossy), e->transmission), e->volume);
}

CY_FN bool bsdf_eval_lp_is_zero(const CyBsdfEvalLP *e)
{
  return is_zero3(e->diffuse) && is_zero3(e->glossy) && is_zero3(e->transmission) && is_zero3(e->transparent) &&
         is_zero3(e->volume);
}

/* bsdf_eval_mis / bsdf_eval_mul3: every component but the transparent one */
CY_FN void bsdf_eval_lp_mul3(CyBsdfEvalLP *e, cfloat3 v)
{
  e->diffuse = mul3(e->diffuse, v);
  e->glossy = mul3(e->glossy, v);
  e->transmission = mul3(e->transmission, v);
  e->volume = mul3(e->volume, v);
}

CY_FN void bsdf_eval_lp_mul(CyBsdfEvalLP *e, float v)
{
  e->diffuse = mul3f(e->diffuse, v);
  e->glossy = mul3f(e->glossy, v);
  e->transmission = mul3f(e->transmission, v);
  e->volume = mul3f(e->volume, v);
}

/* _shader_bsdf_multi_eval with light passes (kernel_shader.h:553-581) */
CY_FN void shader_bsdf_multi_eval_lp(const CySD *sd, const cfloat3 omega_in, float *pdf, int skip_sc,
                                     CyBsdfEvalLP *result_eval, float sum_pdf, float sum_sample_weight)
{
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    if (i != skip_sc && CLOSURE_IS_BSDF(sc->type)) {
      float bsdf_pdf = 0.0f;
      cfloat3 eval = bsdf_eval(sd, sc, omega_in, &bsdf_pdf);
      if (bsdf_pdf != 0.0f) {
        cfloat3 *c = bsdf_eval_lp_component(result_eval, sc->type);
        if (c) {
          *c = add3(*c, mul3f(mul3(eval, sc->weight), 1.0f));
        }
        sum_pdf += bsdf_pdf * sc->sample_weight;
      }
      sum_sample_weight += sc->sample_weight;
    }
  }
  *pdf = (sum_sample_weight > 0.0f) ? sum_pdf / sum_sample_weight : 0.0f;
}

/* kernel_shader.h:638-680 */
CY_FN int shader_bsdf_pick(const CySD *sd, float *randu)
{
  int sampled = 0;
  if (sd->num_closure > 1) {
    float sum = 0.0f;
    for (int i = 0; i < sd->num_closure; i++) {
      const CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_BSDF_OR_BSSRDF(sc->type)) {
        sum += sc->sample_weight;
      }
    }
    float r = (*randu) * sum;
    float partial_sum = 0.0f;
    for (int i = 0; i < sd->num_closure; i++) {
      const CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_BSDF_OR_BSSRDF(sc->type)) {
        float next_sum = partial_sum + sc->sample_weight;
        if (r < next_sum) {
          sampled = i;
          *randu = (r - partial_sum) / sc->sample_weight;
          break;
        }
        partial_sum = next_sum;
      }
    }
  }
  return CLOSURE_IS_BSDF(sd->closure[sampled].type) ? sampled : -1;
}

/* kernel_shader.h:739-775 */
CY_FN int shader_bsdf_sample(const CyGlobals *kg,
                             const CySD *sd,
                             float randu,
                             float randv,
                             cfloat3 *bsdf_eval_out,
                             cfloat3 *omega_in,
                             float *pdf,
                             uint *err,
                             CyDiff3 *domega_in = nullptr)
{
  int sci = shader_bsdf_pick(sd, &randu);
  if (sci < 0) {
    *pdf = 0.0f;
    return LABEL_NONE;
  }
  const CyClosure *sc = &sd->closure[sci];
  int label;
  cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
  *pdf = 0.0f;
#if CY_CLOSURE_EXT
  if (domega_in) {
    CyDiffRule rule;
    rule.kind = CY_DIFF_ZERO;
    label = bsdf_sample(kg, sd, sc, randu, randv, &eval, omega_in, pdf, err, &rule);
    domega_in->dx = diff_rule_apply(rule, sd->dI.dx);
    domega_in->dy = diff_rule_apply(rule, sd->dI.dy);
  }
  else
#endif
  {
    label = bsdf_sample(kg, sd, sc, randu, randv, &eval, omega_in, pdf, err);
  }
  if (*pdf != 0.0f) {
    *bsdf_eval_out = mul3(eval, sc->weight);
    if (sd->num_closure > 1) {
      float sweight = sc->sample_weight;
      shader_bsdf_multi_eval(sd, *omega_in, pdf, sci, bsdf_eval_out, *pdf * sweight, sweight);
    }
  }
  return label;
}

#if CY_CLOSURE_EXT
/* shader_bsdf_sample (kernel_shader.h:683-720) with light passes: the sampled
 * closure's value in its component (bsdf_eval_init), the others' added by
 * theirs */
CY_FN int shader_bsdf_sample_lp(const CyGlobals *kg, const CySD *sd, float randu, float randv, CyBsdfEvalLP *ev,
                                cfloat3 *omega_in, float *pdf, uint *err, CyDiff3 *domega_in)
{
  bsdf_eval_lp_zero(ev);
  int sci = shader_bsdf_pick(sd, &randu);
  if (sci < 0) {
    *pdf = 0.0f;
    return LABEL_NONE;
  }
  const CyClosure *sc = &sd->closure[sci];
  int label;
  cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
  *pdf = 0.0f;
  if (domega_in) {
    CyDiffRule rule;
    rule.kind = CY_DIFF_ZERO;
    label = bsdf_sample(kg, sd, sc, randu, randv, &eval, omega_in, pdf, err, &rule);
    domega_in->dx = diff_rule_apply(rule, sd->dI.dx);
    domega_in->dy = diff_rule_apply(rule, sd->dI.dy);
  }
  else {
    label = bsdf_sample(kg, sd, sc, randu, randv, &eval, omega_in, pdf, err);
  }
  if (*pdf != 0.0f) {
    /* bsdf_eval_init (kernel_accumulate.h:26-61) */
    const cfloat3 value = mul3(eval, sc->weight);
    if (sc->type == CLOSURE_BSDF_TRANSPARENT_ID) {
      ev->transparent = value;
    }
    else {
      cfloat3 *c = bsdf_eval_lp_component(ev, sc->type);
      if (c) {
        *c = value;
      }
    }
    if (sd->num_closure > 1) {
      float sweight = sc->sample_weight;
      shader_bsdf_multi_eval_lp(sd, *omega_in, pdf, sci, ev, *pdf * sweight, sweight);
    }
  }
  return label;
}
#endif

/* ---------------------------------------------------------------------------
 * Lights: kernel_light.h:331-617 (mesh lights with constant emission).
 */
typedef struct CyLightSample {
  cfloat3 P, Ng, D;
  float t, u, v, pdf, eval_fac;
  int object, prim, shader, lamp, type;
} CyLightSample;

CY_FN float triangle_light_pdf_area(const CyGlobals *kg, cfloat3 Ng, cfloat3 I, float t)
{
  float pdf = KD->integrator.pdf_triangles;
  float cos_pi = fabsf(dot3(Ng, I));
  if (cos_pi == 0.0f) {
    return 0.0f;
  }
  return t * t * pdf / cos_pi;
}

/* triangle_world_space_vertices (kernel_light.h:302-329), static objects:
 * true when the vertices were transformed (the reference's has_motion) */
CY_FN bool triangle_world_space_vertices(const CyGlobals *kg, int object, int prim, cfloat3 V[3])
{
  triangle_verts(kg, prim, V);
  if (kg->have_instancing && !(kg->__object_flag[object] & SD_OBJECT_TRANSFORM_APPLIED)) {
    const struct cy_tfm *tfm = object_tfm(kg, object);
    V[0] = transform_point(tfm, V[0]);
    V[1] = transform_point(tfm, V[1]);
    V[2] = transform_point(tfm, V[2]);
    return true;
  }
  return false;
}

/* util_math.h triangle_area */
CY_FN float triangle_area(cfloat3 v1, cfloat3 v2, cfloat3 v3)
{
  return len3(cross3(sub3(v3, v2), sub3(v1, v2))) * 0.5f;
}

CY_FN float triangle_light_pdf(const CyGlobals *kg, const CySD *sd, float t)
{
  cfloat3 V[3];
  const bool has_motion = triangle_world_space_vertices(kg, sd->object, sd->prim, V);
  const cfloat3 e0 = sub3(V[1], V[0]);
  const cfloat3 e1 = sub3(V[2], V[0]);
  const cfloat3 e2 = sub3(V[2], V[1]);
  const float longest_edge_squared = cmax(len_squared3(e0), cmax(len_squared3(e1), len_squared3(e2)));
  const cfloat3 N = cross3(e0, e1);
  const float distance_to_plane = fabsf(dot3(N, mul3f(sd->I, t))) / dot3(N, N);
  if (longest_edge_squared > distance_to_plane * distance_to_plane) {
    const cfloat3 Px = add3(sd->P, mul3f(sd->I, t));
    const cfloat3 v0_p = sub3(V[0], Px);
    const cfloat3 v1_p = sub3(V[1], Px);
    const cfloat3 v2_p = sub3(V[2], Px);
    const cfloat3 u01 = safe_normalize3(cross3(v0_p, v1_p));
    const cfloat3 u02 = safe_normalize3(cross3(v0_p, v2_p));
    const cfloat3 u12 = safe_normalize3(cross3(v1_p, v2_p));
    const float alpha = fast_acosf(dot3(u02, u01));
    const float beta = fast_acosf(-dot3(u01, u12));
    const float gamma = fast_acosf(dot3(u02, u12));
    const float solid_angle = alpha + beta + gamma - CY_PI_F;
    if (solid_angle == 0.0f) {
      return 0.0f;
    }
    float area = has_motion ? triangle_area(V[0], V[1], V[2]) : 0.5f * len3(N);
    const float pdf = area * KD->integrator.pdf_triangles;
    return pdf / solid_angle;
  }
  float pdf = triangle_light_pdf_area(kg, sd->Ng, sd->I, t);
  if (has_motion) {
    const float area = 0.5f * len3(N);
    if (area == 0.0f) {
      return 0.0f;
    }
    const float area_pre = triangle_area(V[0], V[1], V[2]);
    pdf = pdf * area_pre / area;
  }
  return pdf;
}

CY_FN void triangle_light_sample(const CyGlobals *kg,
                                 int prim,
                                 int object,
                                 float randu,
                                 float randv,
                                 CyLightSample *ls,
                                 const cfloat3 P)
{
  cfloat3 V[3];
  const bool has_motion = triangle_world_space_vertices(kg, object, prim, V);
  const cfloat3 e0 = sub3(V[1], V[0]);
  const cfloat3 e1 = sub3(V[2], V[0]);
  const cfloat3 e2 = sub3(V[2], V[1]);
  const float longest_edge_squared = cmax(len_squared3(e0), cmax(len_squared3(e1), len_squared3(e2)));
  const cfloat3 N0 = cross3(e0, e1);
  float Nl = 0.0f;
  ls->Ng = safe_normalize_len3(N0, &Nl);
  float area = 0.5f * Nl;
  const int object_flag = (int)kg->__object_flag[object];
  if (object_flag & SD_OBJECT_NEGATIVE_SCALE_APPLIED) {
    ls->Ng = neg3(ls->Ng);
  }
  ls->eval_fac = 1.0f;
  ls->shader = (int)kg->__tri_shader[prim];
  ls->object = object;
  ls->prim = prim;
  ls->lamp = LAMP_NONE;
  ls->shader |= (int)SHADER_USE_MIS;
  ls->type = 5; /* LIGHT_TRIANGLE */

  float distance_to_plane = fabsf(dot3(N0, sub3(V[0], P)) / dot3(N0, N0));
  if (longest_edge_squared > distance_to_plane * distance_to_plane) {
    const cfloat3 v0_p = sub3(V[0], P);
    const cfloat3 v1_p = sub3(V[1], P);
    const cfloat3 v2_p = sub3(V[2], P);
    const cfloat3 u01 = safe_normalize3(cross3(v0_p, v1_p));
    const cfloat3 u02 = safe_normalize3(cross3(v0_p, v2_p));
    const cfloat3 u12 = safe_normalize3(cross3(v1_p, v2_p));
    const cfloat3 A = safe_normalize3(v0_p);
    const cfloat3 B = safe_normalize3(v1_p);
    const cfloat3 C = safe_normalize3(v2_p);
    const float cos_alpha = dot3(u02, u01);
    const float cos_beta = -dot3(u01, u12);
    const float cos_gamma = dot3(u02, u12);
    const float alpha = fast_acosf(cos_alpha);
    const float beta = fast_acosf(cos_beta);
    const float gamma = fast_acosf(cos_gamma);
    const float solid_angle = alpha + beta + gamma - CY_PI_F;
    const float cos_c = dot3(A, B);
    const float sin_alpha = fast_sinf(alpha);
    const float product = sin_alpha * cos_c;
    const float phi = randu * solid_angle - alpha;
    float s, t;
    fast_sincosf(phi, &s, &t);
    const float u = t - cos_alpha;
    const float v = s + product;
    const cfloat3 U = safe_normalize3(sub3(C, mul3f(A, dot3(C, A))));
    float q = 1.0f;
    const float det = ((v * s + u * t) * sin_alpha);
    if (det != 0.0f) {
      q = ((v * t - u * s) * cos_alpha - v) / det;
    }
    const float temp = cmax(1.0f - q * q, 0.0f);
    const cfloat3 C_ = safe_normalize3(add3(mul3f(A, q), mul3f(U, sqrtf(temp))));
    const float z = 1.0f - randv * (1.0f - dot3(C_, B));
    ls->D = add3(mul3f(B, z), mul3f(safe_normalize3(sub3(C_, mul3f(B, dot3(C_, B)))),
                                    safe_sqrtf(1.0f - z * z)));
    if (!ray_triangle_intersect(P, ls->D, CY_FLT_MAX, V[0], V[1], V[2], &ls->u, &ls->v, &ls->t)) {
      ls->pdf = 0.0f;
      return;
    }
    ls->P = add3(P, mul3f(ls->D, ls->t));
    if (solid_angle == 0.0f) {
      ls->pdf = 0.0f;
      return;
    }
    if (has_motion) {
      area = triangle_area(V[0], V[1], V[2]);
    }
    const float pdf = area * KD->integrator.pdf_triangles;
    ls->pdf = pdf / solid_angle;
  }
  else {
    float u = randu;
    float v = randv;
    if (v > u) {
      u *= 0.5f;
      v -= u;
    }
    else {
      v *= 0.5f;
      u -= v;
    }
    const float t = 1.0f - u - v;
    ls->P = add3(add3(mul3f(V[0], u), mul3f(V[1], v)), mul3f(V[2], t));
    ls->D = normalize_len3(sub3(ls->P, P), &ls->t);
    ls->pdf = triangle_light_pdf_area(kg, ls->Ng, neg3(ls->D), ls->t);
    if (has_motion && area != 0.0f) {
      const float area_pre = triangle_area(V[0], V[1], V[2]);
      ls->pdf = ls->pdf * area_pre / area;
    }
    ls->u = u;
    ls->v = v;
  }
}

/* ---------------------------------------------------------------------------
 * Lamps: kernel_light.h:38-258 (lamp_light_sample / lamp_light_eval) with the
 * helpers of kernel_light_common.h and util_math_intersect.h.  KernelLight's
 * union (kernel_types.h:1489-1534) is read from hc_KernelLight.uni:
 *   spot/point: radius, invarea, spot_angle, spot_smooth, dir[3]
 *   area:       axisu[3], invarea, axisv[3], pad, dir[3]
 *   distant:    radius, cosangle, invarea
 */
#define LIGHT_POINT 0
#define LIGHT_DISTANT 1
#define LIGHT_BACKGROUND 2
#define LIGHT_AREA 3
#define LIGHT_SPOT 4
#define LIGHT_TRIANGLE 5

/* kernel_montecarlo.h:39-46 */
CY_FN void to_unit_disk(float *x, float *y)
{
  float phi = CY_2PI_F * (*x);
  float r = sqrtf(*y);
  *x = r * cy_cosf(phi);
  *y = r * cy_sinf(phi);
}

/* kernel_light_common.h:106-130 */
CY_FN cfloat3 ellipse_sample(cfloat3 ru, cfloat3 rv, float randu, float randv)
{
  to_unit_disk(&randu, &randv);
  return add3(mul3f(ru, randu), mul3f(rv, randv));
}
CY_FN cfloat3 disk_light_sample(cfloat3 v, float randu, float randv)
{
  cfloat3 ru, rv;
  make_orthonormals(v, &ru, &rv);
  return ellipse_sample(ru, rv, randu, randv);
}
CY_FN cfloat3 distant_light_sample(cfloat3 D, float radius, float randu, float randv)
{
  return normalize3(add3(D, mul3f(disk_light_sample(D, randu, randv), radius)));
}
CY_FN cfloat3 sphere_light_sample(cfloat3 P, cfloat3 center, float radius, float randu, float randv)
{
  return mul3f(disk_light_sample(normalize3(sub3(P, center)), randu, randv), radius);
}

/* kernel_light_common.h:132-157; util_math.h:399-403 */
CY_FN float spot_light_attenuation(cfloat3 dir, float spot_angle, float spot_smooth, cfloat3 N)
{
  float attenuation = dot3(dir, N);
  if (attenuation <= spot_angle) {
    attenuation = 0.0f;
  }
  else {
    float t = attenuation - spot_angle;
    if (t < spot_smooth && spot_smooth != 0.0f) {
      const float f = t / spot_smooth;
      const float ff = f * f;
      attenuation *= (3.0f * ff - 2.0f * ff * f);
    }
  }
  return attenuation;
}
CY_FN float lamp_light_pdf(cfloat3 Ng, cfloat3 I, float t)
{
  float cos_pi = dot3(Ng, I);
  if (cos_pi <= 0.0f) {
    return 0.0f;
  }
  return t * t / cos_pi;
}

/* kernel_light_common.h:30-104: solid-angle sampling of a rectangle */
CY_FN float rect_light_sample(
    cfloat3 P, cfloat3 *light_p, cfloat3 axisu, cfloat3 axisv, float randu, float randv, bool sample_coord)
{
  cfloat3 corner = sub3(sub3(*light_p, mul3f(axisu, 0.5f)), mul3f(axisv, 0.5f));
  float axisu_len, axisv_len;
  cfloat3 x = normalize_len3(axisu, &axisu_len);
  cfloat3 y = normalize_len3(axisv, &axisv_len);
  cfloat3 z = cross3(x, y);
  cfloat3 dir = sub3(corner, P);
  float z0 = dot3(dir, z);
  if (z0 > 0.0f) {
    z = mul3f(z, -1.0f);
    z0 *= -1.0f;
  }
  float x0 = dot3(dir, x);
  float y0 = dot3(dir, y);
  float x1 = x0 + axisu_len;
  float y1 = y0 + axisv_len;
  /* float4 diff = (x0, y1, x1, y0) - (x1, y0, x0, y1); nz = (y0, x1, y1, x0) * diff */
  const float d0 = x0 - x1, d1 = y1 - y0, d2 = x1 - x0, d3 = y0 - y1;
  float n0 = y0 * d0, n1 = x1 * d1, n2 = y1 * d2, n3 = x0 * d3;
  const float zz = z0 * z0;
  /* nz / sqrt(z0 * z0 * diff * diff + nz * nz), component-wise */
  n0 = n0 / sqrtf(zz * d0 * d0 + n0 * n0);
  n1 = n1 / sqrtf(zz * d1 * d1 + n1 * n1);
  n2 = n2 / sqrtf(zz * d2 * d2 + n2 * n2);
  n3 = n3 / sqrtf(zz * d3 * d3 + n3 * n3);
  float g0 = safe_acosf(-n0 * n1);
  float g1 = safe_acosf(-n1 * n2);
  float g2 = safe_acosf(-n2 * n3);
  float g3 = safe_acosf(-n3 * n0);
  float b0 = n0;
  float b1 = n2;
  float b0sq = b0 * b0;
  float k = CY_2PI_F - g2 - g3;
  float S = g0 + g1 - k;
  if (sample_coord) {
    float au = randu * S + k;
    float fu = (cy_cosf(au) * b0 - b1) / cy_sinf(au);
    float cu = 1.0f / sqrtf(fu * fu + b0sq) * (fu > 0.0f ? 1.0f : -1.0f);
    cu = cclamp(cu, -1.0f, 1.0f);
    float xu = -(cu * z0) / cmax(sqrtf(1.0f - cu * cu), 1e-7f);
    xu = cclamp(xu, x0, x1);
    float z0sq = z0 * z0;
    float y0sq = y0 * y0;
    float y1sq = y1 * y1;
    float d = sqrtf(xu * xu + z0sq);
    float h0 = y0 / sqrtf(d * d + y0sq);
    float h1 = y1 / sqrtf(d * d + y1sq);
    float hv = h0 + randv * (h1 - h0), hv2 = hv * hv;
    float yv = (hv2 < 1.0f - 1e-6f) ? (hv * d) / sqrtf(1.0f - hv2) : y1;
    *light_p = add3(add3(add3(P, mul3f(x, xu)), mul3f(y, yv)), mul3f(z, z0));
  }
  if (S != 0.0f) {
    return 1.0f / S;
  }
  return 0.0f;
}

/* util_math_intersect.h:58-86 */
CY_FN bool ray_aligned_disk_intersect(
    cfloat3 ray_P, cfloat3 ray_D, float ray_t, cfloat3 disk_P, float disk_radius, cfloat3 *isect_P, float *isect_t)
{
  float disk_t;
  const cfloat3 disk_N = normalize_len3(sub3(ray_P, disk_P), &disk_t);
  const float div = dot3(ray_D, disk_N);
  if (div == 0.0f) {
    return false;
  }
  const float t = -disk_t / div;
  if (t < 0.0f || t > ray_t) {
    return false;
  }
  cfloat3 P = add3(ray_P, mul3f(ray_D, t));
  if (len_squared3(sub3(P, disk_P)) > disk_radius * disk_radius) {
    return false;
  }
  *isect_P = P;
  *isect_t = t;
  return true;
}

/* util_math_intersect.h:202-245 */
CY_FN bool ray_quad_intersect(cfloat3 ray_P,
                              cfloat3 ray_D,
                              float ray_mint,
                              float ray_maxt,
                              cfloat3 quad_P,
                              cfloat3 quad_u,
                              cfloat3 quad_v,
                              cfloat3 quad_n,
                              cfloat3 *isect_P,
                              float *isect_t,
                              float *isect_u,
                              float *isect_v,
                              bool ellipse)
{
  float t = -(dot3(ray_P, quad_n) - dot3(quad_P, quad_n)) / dot3(ray_D, quad_n);
  if (t < ray_mint || t > ray_maxt) {
    return false;
  }
  const cfloat3 hit = add3(ray_P, mul3f(ray_D, t));
  const cfloat3 inplane = sub3(hit, quad_P);
  const float u = dot3(inplane, quad_u) / dot3(quad_u, quad_u);
  if (u < -0.5f || u > 0.5f) {
    return false;
  }
  const float v = dot3(inplane, quad_v) / dot3(quad_v, quad_v);
  if (v < -0.5f || v > 0.5f) {
    return false;
  }
  if (ellipse && (u * u + v * v > 0.25f)) {
    return false;
  }
  *isect_P = hit;
  *isect_t = t;
  *isect_u = u + 0.5f;
  *isect_v = v + 0.5f;
  return true;
}

CY_FN cfloat3 klight_vec(const float *f)
{
  return mk3(f[0], f[1], f[2]);
}

/* ---------------------------------------------------------------------------
 * Background light: importance sampling of the world through the
 * equirectangular luminance map built at scene upload
 * (kernel_light_background.h:24-131 map, 302-447 strategy mix).  Portals and
 * the sky texture's sun strategy are rejected at load_kernels, so their
 * weights are zero here; the weights are still normalised as the reference
 * does. */

/* direction_to_equirectangular: cy_svm_image.h */

/* kernel_montecarlo.h:112-121 */
CY_FN cfloat3 sample_uniform_sphere(float u1, float u2)
{
  const float z = 1.0f - 2.0f * u1;
  const float r = sqrtf(fmaxf(0.0f, 1.0f - z * z));
  const float phi = CY_2PI_F * u2;
  return mk3(r * cy_cosf(phi), r * cy_sinf(phi), z);
}

CY_FN hc_float4 mkf4_bg(float x, float y, float z, float w)
{
  hc_float4 r;
  r.x = x;
  r.y = y;
  r.z = z;
  r.w = w;
  return r;
}

/* util_math.h:425-428 */
CY_FN float inverse_lerp(float a, float b, float x)
{
  return (x - a) / (b - a);
}

/* kernel_light_background.h:26-100 */
CY_FN cfloat3 background_map_sample(const CyGlobals *kg, float randu, float randv, float *pdf)
{
  const int res_x = KD->background.map_res_x;
  const int res_y = KD->background.map_res_y;
  const int cdf_width = res_x + 1;
  const hc_float2 *marg = kg->__light_background_marginal_cdf;
  const hc_float2 *cond = kg->__light_background_conditional_cdf;
  /* std::lower_bound over the marginal CDF */
  int first = 0;
  int count = res_y;
  while (count > 0) {
    const int step = count >> 1;
    const int middle = first + step;
    if (marg[middle].y < randv) {
      first = middle + 1;
      count -= step + 1;
    }
    else {
      count = step;
    }
  }
  const int index_v = (first - 1 > 0) ? first - 1 : 0;
  const hc_float2 cdf_v = marg[index_v];
  const hc_float2 cdf_next_v = marg[index_v + 1];
  const hc_float2 cdf_last_v = marg[res_y];
  const float dv = inverse_lerp(cdf_v.y, cdf_next_v.y, randv);
  const float v = ((float)index_v + dv) / (float)res_y;

  first = 0;
  count = res_x;
  while (count > 0) {
    const int step = count >> 1;
    const int middle = first + step;
    if (cond[index_v * cdf_width + middle].y < randu) {
      first = middle + 1;
      count -= step + 1;
    }
    else {
      count = step;
    }
  }
  const int index_u = (first - 1 > 0) ? first - 1 : 0;
  const hc_float2 cdf_u = cond[index_v * cdf_width + index_u];
  const hc_float2 cdf_next_u = cond[index_v * cdf_width + index_u + 1];
  const hc_float2 cdf_last_u = cond[index_v * cdf_width + res_x];
  const float du = inverse_lerp(cdf_u.y, cdf_next_u.y, randu);
  const float u = ((float)index_u + du) / (float)res_x;

  const float sin_theta = cy_sinf(CY_PI_F * v);
  const float denom = (CY_2PI_F * CY_PI_F * sin_theta) * cdf_last_u.x * cdf_last_v.x;
  if (sin_theta == 0.0f || denom == 0.0f) {
    *pdf = 0.0f;
  }
  else {
    *pdf = (cdf_u.x * cdf_v.x) / denom;
  }
  return equirectangular_range_to_direction(u, v, mkf4_bg(-CY_2PI_F, CY_PI_F, -CY_PI_F, CY_PI_F));
}

/* kernel_light_background.h:105-131 */
CY_FN float background_map_pdf(const CyGlobals *kg, cfloat3 direction)
{
  float u, v;
  direction_to_equirectangular(direction, &u, &v);
  const int res_x = KD->background.map_res_x;
  const int res_y = KD->background.map_res_y;
  const int cdf_width = res_x + 1;
  const float sin_theta = cy_sinf(v * CY_PI_F);
  if (sin_theta == 0.0f) {
    return 0.0f;
  }
  int index_u = (int)(u * (float)res_x);
  index_u = index_u < 0 ? 0 : (index_u > res_x - 1 ? res_x - 1 : index_u);
  int index_v = (int)(v * (float)res_y);
  index_v = index_v < 0 ? 0 : (index_v > res_y - 1 ? res_y - 1 : index_v);
  const hc_float2 cdf_last_u = kg->__light_background_conditional_cdf[index_v * cdf_width + res_x];
  const hc_float2 cdf_last_v = kg->__light_background_marginal_cdf[res_y];
  const float denom = (CY_2PI_F * CY_PI_F * sin_theta) * cdf_last_u.x * cdf_last_v.x;
  if (denom == 0.0f) {
    return 0.0f;
  }
  const hc_float2 cdf_u = kg->__light_background_conditional_cdf[index_v * cdf_width + index_u];
  const hc_float2 cdf_v = kg->__light_background_marginal_cdf[index_v];
  return (cdf_u.x * cdf_v.x) / denom;
}

/* kernel_light_background.h:302-405 with no portals and no sun */
CY_FN cfloat3 background_light_sample(const CyGlobals *kg, float randu, float randv, float *pdf)
{
  float map_method_pdf = KD->background.map_weight;
  const float pdf_fac = map_method_pdf;
  if (pdf_fac == 0.0f) {
    *pdf = 1.0f / (4.0f * CY_PI_F);
    return sample_uniform_sphere(randu, randv);
  }
  map_method_pdf *= 1.0f / pdf_fac;
  /* sun_method_cdf = portal + sun = 0: the map is sampled */
  if (map_method_pdf != 1.0f) {
    randu = (randu - 0.0f) / map_method_pdf;
  }
  const cfloat3 D = background_map_sample(kg, randu, randv, pdf);
  if (map_method_pdf != 1.0f) {
    *pdf *= map_method_pdf;
  }
  return D;
}

/* kernel_light_background.h:407-445 */
CY_FN float background_light_pdf(const CyGlobals *kg, cfloat3 direction)
{
  float map_method_pdf = KD->background.map_weight;
  float pdf_fac = map_method_pdf;
  if (pdf_fac == 0.0f) {
    return KD->integrator.pdf_lights / (4.0f * CY_PI_F);
  }
  pdf_fac = 1.0f / pdf_fac;
  map_method_pdf *= pdf_fac;
  float pdf = 0.0f * 0.0f; /* portal_pdf * portal_method_pdf */
  if (map_method_pdf != 0.0f) {
    pdf += background_map_pdf(kg, direction) * map_method_pdf;
  }
  return pdf * KD->integrator.pdf_lights;
}

/* kernel_light.h:38-158.  u/v (texture coordinates of the lamp) are only read
 * by non-constant lamp shaders, which the device rejects; they are not set. */
CY_FN bool lamp_light_sample(const CyGlobals *kg, int lamp, float randu, float randv, cfloat3 P, CyLightSample *ls,
                             uint *err)
{
  const hc_KernelLight *klight = &kg->__lights[lamp];
  const float *uni = klight->uni;
  const int type = klight->type;
  ls->type = type;
  ls->shader = klight->shader_id;
  ls->object = PRIM_NONE;
  ls->prim = PRIM_NONE;
  ls->lamp = lamp;
  ls->u = randu;
  ls->v = randv;

  if (type == LIGHT_DISTANT) {
    cfloat3 lightD = klight_vec(klight->co);
    cfloat3 D = lightD;
    float radius = uni[0];
    float invarea = uni[2];
    if (radius > 0.0f) {
      D = distant_light_sample(D, radius, randu, randv);
    }
    ls->P = D;
    ls->Ng = D;
    ls->D = neg3(D);
    ls->t = CY_FLT_MAX;
    float costheta = dot3(lightD, D);
    ls->pdf = invarea / (costheta * costheta * costheta);
    ls->eval_fac = ls->pdf;
  }
  else if (type == LIGHT_BACKGROUND) {
    /* infinite area light (world importance sampling) */
    const cfloat3 D = neg3(background_light_sample(kg, randu, randv, &ls->pdf));
    ls->P = D;
    ls->Ng = D;
    ls->D = neg3(D);
    ls->t = CY_FLT_MAX;
    ls->eval_fac = 1.0f;
  }
  else {
    ls->P = klight_vec(klight->co);
    if (type == LIGHT_POINT || type == LIGHT_SPOT) {
      float radius = uni[0];
      if (radius > 0.0f) {
        ls->P = add3(ls->P, sphere_light_sample(P, ls->P, radius, randu, randv));
      }
      ls->D = normalize_len3(sub3(ls->P, P), &ls->t);
      ls->Ng = neg3(ls->D);
      float invarea = uni[1];
      ls->eval_fac = (0.25f * CY_1_PI_F) * invarea;
      ls->pdf = invarea;
      if (type == LIGHT_SPOT) {
        ls->eval_fac *= spot_light_attenuation(klight_vec(uni + 4), uni[2], uni[3], ls->Ng);
        if (ls->eval_fac == 0.0f) {
          return false;
        }
      }
      ls->pdf *= lamp_light_pdf(ls->Ng, neg3(ls->D), ls->t);
    }
    else {
      cfloat3 axisu = klight_vec(uni + 0);
      cfloat3 axisv = klight_vec(uni + 4);
      cfloat3 D = klight_vec(uni + 8);
      float invarea = fabsf(uni[3]);
      bool is_round = (uni[3] < 0.0f);
      if (dot3(sub3(ls->P, P), D) > 0.0f) {
        return false;
      }
      if (is_round) {
        ls->P = add3(ls->P, ellipse_sample(mul3f(axisu, 0.5f), mul3f(axisv, 0.5f), randu, randv));
        ls->pdf = invarea;
      }
      else {
        ls->pdf = rect_light_sample(P, &ls->P, axisu, axisv, randu, randv, true);
      }
      ls->Ng = D;
      ls->D = normalize_len3(sub3(ls->P, P), &ls->t);
      ls->eval_fac = 0.25f * invarea;
      if (is_round) {
        ls->pdf *= lamp_light_pdf(D, neg3(ls->D), ls->t);
      }
    }
  }
  ls->pdf *= KD->integrator.pdf_lights;
  return (ls->pdf > 0.0f);
}

/* kernel_light.h:160-258 */
CY_FN bool lamp_light_eval(const CyGlobals *kg, int lamp, cfloat3 P, cfloat3 D, float t, CyLightSample *ls)
{
  const hc_KernelLight *klight = &kg->__lights[lamp];
  const float *uni = klight->uni;
  const int type = klight->type;
  ls->type = type;
  ls->shader = klight->shader_id;
  ls->object = PRIM_NONE;
  ls->prim = PRIM_NONE;
  ls->lamp = lamp;
  ls->u = 0.0f;
  ls->v = 0.0f;
  if (!((uint)ls->shader & SHADER_USE_MIS)) {
    return false;
  }
  if (type == LIGHT_DISTANT) {
    float radius = uni[0];
    if (radius == 0.0f) {
      return false;
    }
    if (t != CY_FLT_MAX) {
      return false;
    }
    cfloat3 lightD = klight_vec(klight->co);
    float costheta = dot3(neg3(lightD), D);
    float cosangle = uni[1];
    if (costheta < cosangle) {
      return false;
    }
    ls->P = neg3(D);
    ls->Ng = neg3(D);
    ls->D = D;
    ls->t = CY_FLT_MAX;
    float invarea = uni[2];
    ls->pdf = invarea / (costheta * costheta * costheta);
    ls->eval_fac = ls->pdf;
  }
  else if (type == LIGHT_POINT || type == LIGHT_SPOT) {
    cfloat3 lightP = klight_vec(klight->co);
    float radius = uni[0];
    if (radius == 0.0f) {
      return false;
    }
    if (!ray_aligned_disk_intersect(P, D, t, lightP, radius, &ls->P, &ls->t)) {
      return false;
    }
    ls->Ng = neg3(D);
    ls->D = D;
    float invarea = uni[1];
    ls->eval_fac = (0.25f * CY_1_PI_F) * invarea;
    ls->pdf = invarea;
    if (type == LIGHT_SPOT) {
      ls->eval_fac *= spot_light_attenuation(klight_vec(uni + 4), uni[2], uni[3], ls->Ng);
      if (ls->eval_fac == 0.0f) {
        return false;
      }
    }
    if (ls->t != CY_FLT_MAX) {
      ls->pdf *= lamp_light_pdf(ls->Ng, neg3(ls->D), ls->t);
    }
  }
  else if (type == LIGHT_AREA) {
    float invarea = fabsf(uni[3]);
    bool is_round = (uni[3] < 0.0f);
    if (invarea == 0.0f) {
      return false;
    }
    cfloat3 axisu = klight_vec(uni + 0);
    cfloat3 axisv = klight_vec(uni + 4);
    cfloat3 Ng = klight_vec(uni + 8);
    if (dot3(D, Ng) >= 0.0f) {
      return false;
    }
    cfloat3 light_P = klight_vec(klight->co);
    if (!ray_quad_intersect(P, D, 0.0f, t, light_P, axisu, axisv, Ng, &ls->P, &ls->t, &ls->u, &ls->v, is_round)) {
      return false;
    }
    ls->D = D;
    ls->Ng = Ng;
    if (is_round) {
      ls->pdf = invarea * lamp_light_pdf(Ng, neg3(D), ls->t);
    }
    else {
      ls->pdf = rect_light_sample(P, &light_P, axisu, axisv, 0.0f, 0.0f, false);
    }
    ls->eval_fac = 0.25f * invarea;
  }
  else {
    return false;
  }
  ls->pdf *= KD->integrator.pdf_lights;
  return true;
}

CY_FN int light_distribution_sample(const CyGlobals *kg, float *randu)
{
  int first = 0;
  int len = KD->integrator.num_distribution + 1;
  float r = *randu;
  do {
    int half_len = len >> 1;
    int middle = first + half_len;
    if (r < kg->__light_distribution[middle].totarea) {
      len = half_len;
    }
    else {
      first = middle + 1;
      len = len - half_len - 1;
    }
  } while (len > 0);
  int index = iclamp(first - 1, 0, KD->integrator.num_distribution - 1);
  float distr_min = kg->__light_distribution[index].totarea;
  float distr_max = kg->__light_distribution[index + 1].totarea;
  *randu = (r - distr_min) / (distr_max - distr_min);
  return index;
}

/* kernel_light.h:628-661 */
CY_FN bool light_sample(
    const CyGlobals *kg, float randu, float randv, cfloat3 P, int bounce, CyLightSample *ls, uint *err)
{
  int index = light_distribution_sample(kg, &randu);
  const hc_KernelLightDistribution *kd = &kg->__light_distribution[index];
  int prim = kd->prim;
  if (prim >= 0) {
    triangle_light_sample(kg, prim, kd->object_id, randu, randv, ls, P);
    ls->shader |= kd->shader_flag;
    return (ls->pdf > 0.0f);
  }
  const int lamp = -prim - 1;
  /* light_select_reached_max_bounces: max_bounces is stored as a float */
  if ((float)bounce > kg->__lights[lamp].max_bounces) {
    return false;
  }
  return lamp_light_sample(kg, lamp, randu, randv, P, ls, err);
}

/* kernel_shader.h:978-992 */
CY_FN bool shader_constant_emission_eval(const CyGlobals *kg, int shader, cfloat3 *eval)
{
  int shader_index = (int)((uint)shader & SHADER_MASK);
  const hc_KernelShader *ks = &kg->__shaders[shader_index];
  if (ks->flags & SD_HAS_CONSTANT_EMISSION) {
    *eval = mk3(ks->constant_emission[0], ks->constant_emission[1], ks->constant_emission[2]);
    return true;
  }
  return false;
}

#endif /* CY_PATH_H */
