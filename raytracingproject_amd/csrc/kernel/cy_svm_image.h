/*
 * cy_svm_image.h — image textures: the reference CPU kernel's texture
 * interpolation (kernel/kernels/cpu/kernel_cpu_image.h:26-200, 471-500) and
 * the image / environment texture nodes (kernel/svm/svm_image.h:19-112,
 * 218-245), evaluated with the reference's arithmetic.
 *
 * Textures live in device memory the host allocates per image
 * (hipcy_tex_alloc, the analogue of CUDADevice::tex_alloc); __texture_info
 * holds one hc_TextureInfo per SVM image slot with the image's device
 * address in `data` (on the host emulator and the reference: a host pointer).
 * 2D images only; all eight ImageDataTypes; closest / linear / cubic (smart
 * = cubic, as on the CPU device) interpolation; repeat / extend / clip.
 *
 * Also here: direction_to_equirectangular (kernel_projection.h:56-78), which
 * the environment node and the background light share.
 */
#ifndef CY_SVM_IMAGE_H
#define CY_SVM_IMAGE_H

#define CY_IMAGE_DATA_TYPE_FLOAT4 0
#define CY_IMAGE_DATA_TYPE_BYTE4 1
#define CY_IMAGE_DATA_TYPE_HALF4 2
#define CY_IMAGE_DATA_TYPE_FLOAT 3
#define CY_IMAGE_DATA_TYPE_BYTE 4
#define CY_IMAGE_DATA_TYPE_HALF 5
#define CY_IMAGE_DATA_TYPE_USHORT4 6
#define CY_IMAGE_DATA_TYPE_USHORT 7
#define CY_INTERPOLATION_LINEAR 0
#define CY_INTERPOLATION_CLOSEST 1
#define CY_EXTENSION_REPEAT 0
#define CY_EXTENSION_EXTEND 1
#define CY_EXTENSION_CLIP 2
#define CY_NODE_IMAGE_PROJ_SPHERE 2
#define CY_NODE_IMAGE_PROJ_TUBE 3
#define CY_NODE_IMAGE_COMPRESS_AS_SRGB 1
#define CY_NODE_IMAGE_ALPHA_UNASSOCIATE 2

/* kernel_projection.h:56-78 direction_to_equirectangular (default range) */
CY_FN void direction_to_equirectangular(cfloat3 dir, float *u, float *v)
{
  if (dir.x == 0.0f && dir.y == 0.0f && dir.z == 0.0f) {
    *u = 0.0f;
    *v = 0.0f;
    return;
  }
  *u = (cy_atan2f(dir.y, dir.x) - CY_PI_F) / -CY_2PI_F;
  *v = (cy_acosf(dir.z / len3(dir)) - CY_PI_F) / -CY_PI_F;
}

/* kernel_projection.h:171-184 */
CY_FN void direction_to_mirrorball(cfloat3 dir, float *u, float *v)
{
  dir.y -= 1.0f;
  float div = 2.0f * sqrtf(cmax(-0.5f * dir.y, 0.0f));
  if (div > 0.0f) {
    dir = div3f(dir, div);
  }
  *u = 0.5f * (dir.x + 1.0f);
  *v = 0.5f * (dir.z + 1.0f);
}

/* util_math.h:737-768 */
CY_FN void map_to_tube(cfloat3 co, float *u, float *v)
{
  float len = sqrtf(co.x * co.x + co.y * co.y);
  if (len > 0.0f) {
    *u = (1.0f - (cy_atan2f(co.x / len, co.y / len) / CY_PI_F)) * 0.5f;
    *v = (co.z + 1.0f) * 0.5f;
  }
  else {
    *u = *v = 0.0f;
  }
}
CY_FN void map_to_sphere(cfloat3 co, float *u, float *v)
{
  float l = len3(co);
  if (l > 0.0f) {
    if (co.x == 0.0f && co.y == 0.0f) {
      *u = 0.0f;
    }
    else {
      *u = (1.0f - cy_atan2f(co.x, co.y) / CY_PI_F) / 2.0f;
    }
    *v = 1.0f - safe_acosf(co.z / l) / CY_PI_F;
  }
  else {
    *u = *v = 0.0f;
  }
}

/* util_half.h:120-127 (the CPU device's conversion: no denormal / inf handling) */
CY_FN float cy_half_to_float(uint16_t h)
{
  const uint hh = h;
  return as_float(((hh & 0x8000u) << 16) | (((hh & 0x7c00u) + 0x1C000u) << 13) | ((hh & 0x03FFu) << 13));
}

/* TextureInterpolator<T>::read(data, x, y, ...) per data type */
CY_FN hc_float4 cy_tex_read(const hc_TextureInfo *info, int idx)
{
  hc_float4 r;
  switch (info->data_type) {
    case CY_IMAGE_DATA_TYPE_FLOAT4:
      r = ((const hc_float4 *)info->data)[idx];
      break;
    case CY_IMAGE_DATA_TYPE_BYTE4: {
      const uint8_t *p = ((const uint8_t *)info->data) + 4 * (size_t)idx;
      float f = 1.0f / 255.0f;
      r.x = p[0] * f;
      r.y = p[1] * f;
      r.z = p[2] * f;
      r.w = p[3] * f;
      break;
    }
    case CY_IMAGE_DATA_TYPE_HALF4: {
      const uint16_t *p = ((const uint16_t *)info->data) + 4 * (size_t)idx;
      r.x = cy_half_to_float(p[0]);
      r.y = cy_half_to_float(p[1]);
      r.z = cy_half_to_float(p[2]);
      r.w = cy_half_to_float(p[3]);
      break;
    }
    case CY_IMAGE_DATA_TYPE_FLOAT: {
      float f = ((const float *)info->data)[idx];
      r.x = r.y = r.z = f;
      r.w = 1.0f;
      break;
    }
    case CY_IMAGE_DATA_TYPE_BYTE: {
      float f = ((const uint8_t *)info->data)[idx] * (1.0f / 255.0f);
      r.x = r.y = r.z = f;
      r.w = 1.0f;
      break;
    }
    case CY_IMAGE_DATA_TYPE_HALF: {
      float f = cy_half_to_float(((const uint16_t *)info->data)[idx]);
      r.x = r.y = r.z = f;
      r.w = 1.0f;
      break;
    }
    case CY_IMAGE_DATA_TYPE_USHORT4: {
      const uint16_t *p = ((const uint16_t *)info->data) + 4 * (size_t)idx;
      float f = 1.0f / 65535.0f;
      r.x = p[0] * f;
      r.y = p[1] * f;
      r.z = p[2] * f;
      r.w = p[3] * f;
      break;
    }
    default: { /* USHORT */
      float f = ((const uint16_t *)info->data)[idx] * (1.0f / 65535.0f);
      r.x = r.y = r.z = f;
      r.w = 1.0f;
      break;
    }
  }
  return r;
}

CY_FN hc_float4 cy_f4(float x, float y, float z, float w)
{
  hc_float4 r;
  r.x = x;
  r.y = y;
  r.z = z;
  r.w = w;
  return r;
}
CY_FN hc_float4 cy_f4_scale(float s, hc_float4 a)
{
  return cy_f4(s * a.x, s * a.y, s * a.z, s * a.w);
}
CY_FN hc_float4 cy_f4_add(hc_float4 a, hc_float4 b)
{
  return cy_f4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

/* read(data, x, y, width, height): zero outside the image (clip extension) */
CY_FN hc_float4 cy_tex_read_xy(const hc_TextureInfo *info, int x, int y, int width, int height)
{
  if (x < 0 || y < 0 || x >= width || y >= height) {
    return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  return cy_tex_read(info, y * width + x);
}

CY_FN int cy_wrap_periodic(int x, int width)
{
  x %= width;
  if (x < 0) {
    x += width;
  }
  return x;
}
CY_FN int cy_wrap_clamp(int x, int width)
{
  return iclamp(x, 0, width - 1);
}
CY_FN float cy_tex_frac(float x, int *ix)
{
  int i = (int)((uint)cy_ftoi(x) - ((x < 0.0f) ? 1u : 0u)); /* wrapping, as x86 */
  *ix = i;
  return x - (float)i;
}

/* kernel_cpu_image.h:111-137 */
CY_FN hc_float4 cy_interp_closest(const hc_TextureInfo *info, float x, float y)
{
  const int width = (int)info->width;
  const int height = (int)info->height;
  int ix, iy;
  cy_tex_frac(x * (float)width, &ix);
  cy_tex_frac(y * (float)height, &iy);
  switch (info->extension) {
    case CY_EXTENSION_REPEAT:
      ix = cy_wrap_periodic(ix, width);
      iy = cy_wrap_periodic(iy, height);
      break;
    case CY_EXTENSION_CLIP:
      if (x < 0.0f || y < 0.0f || x > 1.0f || y > 1.0f) {
        return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
      }
      /* fall through */
    case CY_EXTENSION_EXTEND:
      ix = cy_wrap_clamp(ix, width);
      iy = cy_wrap_clamp(iy, height);
      break;
    default:
      return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  return cy_tex_read(info, ix + iy * width);
}

/* kernel_cpu_image.h:139-170: ((1-ty)(1-tx)) p00 + ((1-ty) tx) p10 + ... summed left to right */
CY_FN hc_float4 cy_interp_linear(const hc_TextureInfo *info, float x, float y)
{
  const int width = (int)info->width;
  const int height = (int)info->height;
  int ix, iy, nix, niy;
  const float tx = cy_tex_frac(x * (float)width - 0.5f, &ix);
  const float ty = cy_tex_frac(y * (float)height - 0.5f, &iy);
  switch (info->extension) {
    case CY_EXTENSION_REPEAT:
      ix = cy_wrap_periodic(ix, width);
      iy = cy_wrap_periodic(iy, height);
      nix = cy_wrap_periodic(ix + 1, width);
      niy = cy_wrap_periodic(iy + 1, height);
      break;
    case CY_EXTENSION_CLIP:
      nix = ix + 1;
      niy = iy + 1;
      break;
    case CY_EXTENSION_EXTEND:
      nix = cy_wrap_clamp(ix + 1, width);
      niy = cy_wrap_clamp(iy + 1, height);
      ix = cy_wrap_clamp(ix, width);
      iy = cy_wrap_clamp(iy, height);
      break;
    default:
      return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  hc_float4 r = cy_f4_scale((1.0f - ty) * (1.0f - tx), cy_tex_read_xy(info, ix, iy, width, height));
  r = cy_f4_add(r, cy_f4_scale((1.0f - ty) * tx, cy_tex_read_xy(info, nix, iy, width, height)));
  r = cy_f4_add(r, cy_f4_scale(ty * (1.0f - tx), cy_tex_read_xy(info, ix, niy, width, height)));
  r = cy_f4_add(r, cy_f4_scale(ty * tx, cy_tex_read_xy(info, nix, niy, width, height)));
  return r;
}

/* kernel_cpu_image.h:27-34 SET_CUBIC_SPLINE_WEIGHTS */
CY_FN void cy_cubic_weights(float *u, float t)
{
  u[0] = (((-1.0f / 6.0f) * t + 0.5f) * t - 0.5f) * t + (1.0f / 6.0f);
  u[1] = ((0.5f * t - 1.0f) * t) * t + (2.0f / 3.0f);
  u[2] = ((-0.5f * t + 0.5f) * t + 0.5f) * t + (1.0f / 6.0f);
  u[3] = (1.0f / 6.0f) * t * t * t;
}

/* kernel_cpu_image.h:172-236 (bicubic B-spline) */
CY_FN hc_float4 cy_interp_cubic(const hc_TextureInfo *info, float x, float y)
{
  const int width = (int)info->width;
  const int height = (int)info->height;
  int ix, iy, nix, niy;
  const float tx = cy_tex_frac(x * (float)width - 0.5f, &ix);
  const float ty = cy_tex_frac(y * (float)height - 0.5f, &iy);
  int pix, piy, nnix, nniy;
  switch (info->extension) {
    case CY_EXTENSION_REPEAT:
      ix = cy_wrap_periodic(ix, width);
      iy = cy_wrap_periodic(iy, height);
      pix = cy_wrap_periodic(ix - 1, width);
      piy = cy_wrap_periodic(iy - 1, height);
      nix = cy_wrap_periodic(ix + 1, width);
      niy = cy_wrap_periodic(iy + 1, height);
      nnix = cy_wrap_periodic(ix + 2, width);
      nniy = cy_wrap_periodic(iy + 2, height);
      break;
    case CY_EXTENSION_CLIP:
      pix = ix - 1;
      piy = iy - 1;
      nix = ix + 1;
      niy = iy + 1;
      nnix = ix + 2;
      nniy = iy + 2;
      break;
    case CY_EXTENSION_EXTEND:
      pix = cy_wrap_clamp(ix - 1, width);
      piy = cy_wrap_clamp(iy - 1, height);
      nix = cy_wrap_clamp(ix + 1, width);
      niy = cy_wrap_clamp(iy + 1, height);
      nnix = cy_wrap_clamp(ix + 2, width);
      nniy = cy_wrap_clamp(iy + 2, height);
      ix = cy_wrap_clamp(ix, width);
      iy = cy_wrap_clamp(iy, height);
      break;
    default:
      return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  const int xc[4] = {pix, ix, nix, nnix};
  const int yc[4] = {piy, iy, niy, nniy};
  float u[4], v[4];
  cy_cubic_weights(u, tx);
  cy_cubic_weights(v, ty);
  /* TERM(col) = v[col] * (u0 D(0,col) + u1 D(1,col) + u2 D(2,col) + u3 D(3,col)); sum of TERM(0..3) */
  hc_float4 r;
  for (int col = 0; col < 4; col++) {
    hc_float4 s = cy_f4_scale(u[0], cy_tex_read_xy(info, xc[0], yc[col], width, height));
    s = cy_f4_add(s, cy_f4_scale(u[1], cy_tex_read_xy(info, xc[1], yc[col], width, height)));
    s = cy_f4_add(s, cy_f4_scale(u[2], cy_tex_read_xy(info, xc[2], yc[col], width, height)));
    s = cy_f4_add(s, cy_f4_scale(u[3], cy_tex_read_xy(info, xc[3], yc[col], width, height)));
    s = cy_f4_scale(v[col], s);
    r = (col == 0) ? s : cy_f4_add(r, s);
  }
  return r;
}

/* kernel_cpu_image.h:238-250, 471-500 kernel_tex_image_interp */
CY_FN hc_float4 kernel_tex_image_interp(const hc_TextureInfo *texture_info, int id, float x, float y)
{
  const hc_TextureInfo *info = &texture_info[id];
  if (info->data == 0) {
    return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  switch (info->interpolation) {
    case CY_INTERPOLATION_CLOSEST:
      return cy_interp_closest(info, x, y);
    case CY_INTERPOLATION_LINEAR:
      return cy_interp_linear(info, x, y);
    default:
      return cy_interp_cubic(info, x, y);
  }
}

/* ---- 3D textures (kernel_cpu_image.h:254-469 TextureInterpolator::interp_3d):
 * dense voxel grids, e.g. the Point Density node's.  Unlike the 2D reader the
 * clip extension returns zero only outside [0, 1]^3 and otherwise clamps like
 * extend (ATTR_FALLTHROUGH); the voxel reads themselves are unchecked. */
CY_FN int cy_tex3_index(const hc_TextureInfo *info, int x, int y, int z)
{
  return x + y * (int)info->width + z * (int)info->width * (int)info->height;
}

CY_FN bool cy_tex3_outside(float x, float y, float z)
{
  return x < 0.0f || y < 0.0f || z < 0.0f || x > 1.0f || y > 1.0f || z > 1.0f;
}

/* kernel_cpu_image.h:256-293 */
CY_FN hc_float4 cy_interp_3d_closest(const hc_TextureInfo *info, float x, float y, float z)
{
  const int width = (int)info->width, height = (int)info->height, depth = (int)info->depth;
  int ix, iy, iz;
  cy_tex_frac(x * (float)width, &ix);
  cy_tex_frac(y * (float)height, &iy);
  cy_tex_frac(z * (float)depth, &iz);
  switch (info->extension) {
    case CY_EXTENSION_REPEAT:
      ix = cy_wrap_periodic(ix, width);
      iy = cy_wrap_periodic(iy, height);
      iz = cy_wrap_periodic(iz, depth);
      break;
    case CY_EXTENSION_CLIP:
      if (cy_tex3_outside(x, y, z)) {
        return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
      }
      /* fall through */
    case CY_EXTENSION_EXTEND:
      ix = cy_wrap_clamp(ix, width);
      iy = cy_wrap_clamp(iy, height);
      iz = cy_wrap_clamp(iz, depth);
      break;
    default:
      return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  return cy_tex_read(info, cy_tex3_index(info, ix, iy, iz));
}

/* kernel_cpu_image.h:295-358: eight weighted voxels summed in order, each
 * weight the product of its three factors left to right */
CY_FN hc_float4 cy_interp_3d_linear(const hc_TextureInfo *info, float x, float y, float z)
{
  const int width = (int)info->width, height = (int)info->height, depth = (int)info->depth;
  int ix, iy, iz, nix, niy, niz;
  const float tx = cy_tex_frac(x * (float)width - 0.5f, &ix);
  const float ty = cy_tex_frac(y * (float)height - 0.5f, &iy);
  const float tz = cy_tex_frac(z * (float)depth - 0.5f, &iz);
  switch (info->extension) {
    case CY_EXTENSION_REPEAT:
      ix = cy_wrap_periodic(ix, width);
      iy = cy_wrap_periodic(iy, height);
      iz = cy_wrap_periodic(iz, depth);
      nix = cy_wrap_periodic(ix + 1, width);
      niy = cy_wrap_periodic(iy + 1, height);
      niz = cy_wrap_periodic(iz + 1, depth);
      break;
    case CY_EXTENSION_CLIP:
      if (cy_tex3_outside(x, y, z)) {
        return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
      }
      /* fall through */
    case CY_EXTENSION_EXTEND:
      nix = cy_wrap_clamp(ix + 1, width);
      niy = cy_wrap_clamp(iy + 1, height);
      niz = cy_wrap_clamp(iz + 1, depth);
      ix = cy_wrap_clamp(ix, width);
      iy = cy_wrap_clamp(iy, height);
      iz = cy_wrap_clamp(iz, depth);
      break;
    default:
      return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  hc_float4 r = cy_f4_scale((1.0f - tz) * (1.0f - ty) * (1.0f - tx), cy_tex_read(info, cy_tex3_index(info, ix, iy, iz)));
  r = cy_f4_add(r, cy_f4_scale((1.0f - tz) * (1.0f - ty) * tx, cy_tex_read(info, cy_tex3_index(info, nix, iy, iz))));
  r = cy_f4_add(r, cy_f4_scale((1.0f - tz) * ty * (1.0f - tx), cy_tex_read(info, cy_tex3_index(info, ix, niy, iz))));
  r = cy_f4_add(r, cy_f4_scale((1.0f - tz) * ty * tx, cy_tex_read(info, cy_tex3_index(info, nix, niy, iz))));
  r = cy_f4_add(r, cy_f4_scale(tz * (1.0f - ty) * (1.0f - tx), cy_tex_read(info, cy_tex3_index(info, ix, iy, niz))));
  r = cy_f4_add(r, cy_f4_scale(tz * (1.0f - ty) * tx, cy_tex_read(info, cy_tex3_index(info, nix, iy, niz))));
  r = cy_f4_add(r, cy_f4_scale(tz * ty * (1.0f - tx), cy_tex_read(info, cy_tex3_index(info, ix, niy, niz))));
  r = cy_f4_add(r, cy_f4_scale(tz * ty * tx, cy_tex_read(info, cy_tex3_index(info, nix, niy, niz))));
  return r;
}

/* kernel_cpu_image.h:368-453 (tricubic B-spline):
 * ROW_TERM(row) = w[row] * (COL_TERM(0, row) + ... + COL_TERM(3, row)),
 * COL_TERM(col, row) = v[col] * (u0 D(0, col, row) + ... + u3 D(3, col, row)),
 * the four row terms summed left to right */
CY_FN hc_float4 cy_interp_3d_tricubic(const hc_TextureInfo *info, float x, float y, float z)
{
  const int width = (int)info->width, height = (int)info->height, depth = (int)info->depth;
  int ix, iy, iz, nix, niy, niz, pix, piy, piz, nnix, nniy, nniz;
  const float tx = cy_tex_frac(x * (float)width - 0.5f, &ix);
  const float ty = cy_tex_frac(y * (float)height - 0.5f, &iy);
  const float tz = cy_tex_frac(z * (float)depth - 0.5f, &iz);
  switch (info->extension) {
    case CY_EXTENSION_REPEAT:
      ix = cy_wrap_periodic(ix, width);
      iy = cy_wrap_periodic(iy, height);
      iz = cy_wrap_periodic(iz, depth);
      pix = cy_wrap_periodic(ix - 1, width);
      piy = cy_wrap_periodic(iy - 1, height);
      piz = cy_wrap_periodic(iz - 1, depth);
      nix = cy_wrap_periodic(ix + 1, width);
      niy = cy_wrap_periodic(iy + 1, height);
      niz = cy_wrap_periodic(iz + 1, depth);
      nnix = cy_wrap_periodic(ix + 2, width);
      nniy = cy_wrap_periodic(iy + 2, height);
      nniz = cy_wrap_periodic(iz + 2, depth);
      break;
    case CY_EXTENSION_CLIP:
      if (cy_tex3_outside(x, y, z)) {
        return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
      }
      /* fall through */
    case CY_EXTENSION_EXTEND:
      pix = cy_wrap_clamp(ix - 1, width);
      piy = cy_wrap_clamp(iy - 1, height);
      piz = cy_wrap_clamp(iz - 1, depth);
      nix = cy_wrap_clamp(ix + 1, width);
      niy = cy_wrap_clamp(iy + 1, height);
      niz = cy_wrap_clamp(iz + 1, depth);
      nnix = cy_wrap_clamp(ix + 2, width);
      nniy = cy_wrap_clamp(iy + 2, height);
      nniz = cy_wrap_clamp(iz + 2, depth);
      ix = cy_wrap_clamp(ix, width);
      iy = cy_wrap_clamp(iy, height);
      iz = cy_wrap_clamp(iz, depth);
      break;
    default:
      return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  const int xc[4] = {pix, ix, nix, nnix};
  const int yc[4] = {width * piy, width * iy, width * niy, width * nniy};
  const int zc[4] = {width * height * piz, width * height * iz, width * height * niz, width * height * nniz};
  float u[4], v[4], w[4];
  cy_cubic_weights(u, tx);
  cy_cubic_weights(v, ty);
  cy_cubic_weights(w, tz);
  hc_float4 r;
  for (int row = 0; row < 4; row++) {
    hc_float4 rt;
    for (int col = 0; col < 4; col++) {
      const int yz = yc[col] + zc[row];
      hc_float4 c = cy_f4_scale(u[0], cy_tex_read(info, xc[0] + yz));
      c = cy_f4_add(c, cy_f4_scale(u[1], cy_tex_read(info, xc[1] + yz)));
      c = cy_f4_add(c, cy_f4_scale(u[2], cy_tex_read(info, xc[2] + yz)));
      c = cy_f4_add(c, cy_f4_scale(u[3], cy_tex_read(info, xc[3] + yz)));
      c = cy_f4_scale(v[col], c);
      rt = (col == 0) ? c : cy_f4_add(rt, c);
    }
    rt = cy_f4_scale(w[row], rt);
    r = (row == 0) ? rt : cy_f4_add(r, rt);
  }
  return r;
}

/* kernel_cpu_image.h:501-531 kernel_tex_image_interp_3d with
 * INTERPOLATION_NONE: the texture's own interpolation; the optional 3D
 * transform first (TextureInfo::use_transform_3d) */
CY_FN hc_float4 kernel_tex_image_interp_3d(const hc_TextureInfo *texture_info, int id, cfloat3 P)
{
  const hc_TextureInfo *info = &texture_info[id];
  if (info->use_transform_3d) {
    const hc_Transform &t = info->transform_3d;
    P = mk3(t.x.x * P.x + t.x.y * P.y + t.x.z * P.z + t.x.w, t.y.x * P.x + t.y.y * P.y + t.y.z * P.z + t.y.w,
            t.z.x * P.x + t.z.y * P.y + t.z.z * P.z + t.z.w);
  }
  if (info->data == 0) {
    return cy_f4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  switch (info->interpolation) {
    case CY_INTERPOLATION_CLOSEST:
      return cy_interp_3d_closest(info, P.x, P.y, P.z);
    case CY_INTERPOLATION_LINEAR:
      return cy_interp_3d_linear(info, P.x, P.y, P.z);
    default:
      return cy_interp_3d_tricubic(info, P.x, P.y, P.z);
  }
}

/* util_color.h:185-242: the reference CPU kernel is built with __KERNEL_SSE2__,
 * so color_srgb_to_linear_v4 takes the SSE path: powf(x, 2.4) by fastpow24
 * (a float-bits initial guess refined by three Newton steps on the fifth
 * root), madd without FMA.  The int conversions are cvtepi32_ps and
 * cvtps_epi32 (round to nearest even). */
CY_FN float cy_srgb_to_linear_sse(float c)
{
  const float lt = cmax(c * (1.0f / 12.92f), 0.0f);
  if (c < 0.04045f) {
    return lt;
  }
  const float arg = (c + 0.055f) * (1.0f / 1.055f);
  float x = arg * as_float(0x4F55A7FBu);
  x = (float)(int)as_uint(x);
  x = x * as_float(0x3F4CCCCDu);
  x = as_float((uint)(int)rintf(x));
  const float arg2 = arg * arg;
  const float arg4 = arg2 * arg2;
  for (int i = 0; i < 3; i++) {
    const float approx2 = x * x;
    const float approx4 = approx2 * approx2;
    const float t = arg4 / approx4;
    const float summ = 4.0f * x + t;
    x = summ * (1.0f / 5.0f);
  }
  return x * (x * x);
}

/* svm_image.h:19-39 svm_image_texture */
CY_FN hc_float4 svm_image_texture(const hc_TextureInfo *texture_info, int id, float x, float y, uint flags)
{
  if (id == -1) {
    return cy_f4(1.0f, 0.0f, 1.0f, 1.0f); /* TEX_IMAGE_MISSING_R/G/B/A */
  }
  hc_float4 r = kernel_tex_image_interp(texture_info, id, x, y);
  const float alpha = r.w;
  if ((flags & CY_NODE_IMAGE_ALPHA_UNASSOCIATE) && alpha != 1.0f && alpha != 0.0f) {
    /* float4 /= float: multiply by the reciprocal (util_math_float4.h) */
    const float inv = 1.0f / alpha;
    r = cy_f4(r.x * inv, r.y * inv, r.z * inv, r.w * inv);
    r.w = alpha;
  }
  if (flags & CY_NODE_IMAGE_COMPRESS_AS_SRGB) {
    r = cy_f4(cy_srgb_to_linear_sse(r.x), cy_srgb_to_linear_sse(r.y), cy_srgb_to_linear_sse(r.z), r.w);
  }
  return r;
}

/* svm_image.h:43-112 svm_node_tex_image (flat, sphere and tube projection;
 * UDIM tiles as tile nodes after the image node).  Box projection is
 * NODE_TEX_IMAGE_BOX, rejected at load_kernels. */
CY_FN void svm_node_tex_image(const CyGlobals *kg,
                              const hc_TextureInfo *texture_info,
                              CySvmStack stack,
                              hc_uint4 node,
                              int *offset,
                              uint *err)
{
  const uint co_offset = node.z & 0xFF, out_offset = (node.z >> 8) & 0xFF;
  const uint alpha_offset = (node.z >> 16) & 0xFF, flags = (node.z >> 24) & 0xFF;
  cfloat3 co = svm_load3(stack, co_offset, err);
  float tu, tv;
  if (node.w == CY_NODE_IMAGE_PROJ_SPHERE) {
    co = mul3f(sub3(co, mk3(0.5f, 0.5f, 0.5f)), 2.0f);
    map_to_sphere(co, &tu, &tv);
  }
  else if (node.w == CY_NODE_IMAGE_PROJ_TUBE) {
    co = mul3f(sub3(co, mk3(0.5f, 0.5f, 0.5f)), 2.0f);
    map_to_tube(co, &tu, &tv);
  }
  else {
    tu = co.x;
    tv = co.y;
  }
  int id = -1;
  const int num_nodes = (int)node.y;
  if (num_nodes > 0) {
    const int next_offset = (*offset) + num_nodes;
    const int tx = cy_ftoi(tu);
    const int ty = cy_ftoi(tv);
    if (tx >= 0 && ty >= 0 && tx < 10) {
      const int tile = 1001 + 10 * ty + tx;
      for (int i = 0; i < num_nodes; i++) {
        const hc_uint4 tile_node = kg->__svm_nodes[(*offset)++];
        if ((int)tile_node.x == tile) {
          id = (int)tile_node.y;
          break;
        }
        if ((int)tile_node.z == tile) {
          id = (int)tile_node.w;
          break;
        }
      }
      if (id != -1) {
        tu -= tx;
        tv -= ty;
      }
    }
    *offset = next_offset;
  }
  else {
    id = -num_nodes;
  }
  const hc_float4 f = svm_image_texture(texture_info, id, tu, tv, flags);
  if (out_offset != SVM_STACK_INVALID) {
    svm_store3(stack, out_offset, mk3(f.x, f.y, f.z), err);
  }
  if (alpha_offset != SVM_STACK_INVALID) {
    svm_store(stack, alpha_offset, f.w, err);
  }
}

/* svm_image.h:218-245 svm_node_tex_environment */
CY_FN void svm_node_tex_environment(const hc_TextureInfo *texture_info, CySvmStack stack, hc_uint4 node,
                                    uint *err)
{
  const uint id = node.y;
  const uint co_offset = node.z & 0xFF, out_offset = (node.z >> 8) & 0xFF;
  const uint alpha_offset = (node.z >> 16) & 0xFF, flags = (node.z >> 24) & 0xFF;
  cfloat3 co = safe_normalize3(svm_load3(stack, co_offset, err));
  float u, v;
  if (node.w == 0) {
    direction_to_equirectangular(co, &u, &v);
  }
  else {
    direction_to_mirrorball(co, &u, &v);
  }
  const hc_float4 f = svm_image_texture(texture_info, (int)id, u, v, flags);
  if (out_offset != SVM_STACK_INVALID) {
    svm_store3(stack, out_offset, mk3(f.x, f.y, f.z), err);
  }
  if (alpha_offset != SVM_STACK_INVALID) {
    svm_store(stack, alpha_offset, f.w, err);
  }
}

#endif /* CY_SVM_IMAGE_H */
