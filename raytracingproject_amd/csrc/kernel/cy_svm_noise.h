/*
 * cy_svm_noise.h — the procedural noise textures of the SVM (Noise, Wave,
 * Magic, Brick, White Noise, Musgrave), restated in the arithmetic of the
 * reference CPU kernel's x86-64 build:
 *   Jenkins lookup3 hashes, hash-to-float          util/util_hash.h:30-220
 *   Perlin noise 1D (scalar), 2D/3D/4D (the SSE2
 *     branch the x86-64 kernel compiles:
 *     __KERNEL_SSE2__ without __KERNEL_AVX__)      kernel/svm/svm_noise.h:41-70, 265-560, 667-742
 *   fractal_noise_1d..4d                           kernel/svm/svm_fractal_noise.h
 *   noise_texture_*d, svm_node_tex_noise           kernel/svm/svm_noisetex.h
 *   svm_wave, svm_node_tex_wave                    kernel/svm/svm_wave.h
 *   svm_magic, svm_node_tex_magic                  kernel/svm/svm_magic.h
 *   svm_brick, svm_node_tex_brick                  kernel/svm/svm_brick.h
 *   svm_node_tex_white_noise                       kernel/svm/svm_white_noise.h
 *   noise_musgrave_* (all types, 1D..4D)           kernel/svm/svm_musgrave.h
 * The SSE2 Perlin code differs from the scalar one in two roundings, both
 * kept here: fade is (t*t) * (t * (t*(t*6-15) + 10)) and the interpolation
 * is t*b + (1-t)*a (util_ssef.h mix/madd without FMA), where the scalar
 * branch computes t*t*t*(...) and a + t*(b-a).  The four dimensions of each
 * Musgrave type are one template over the coordinate type, as the reference's
 * four copies differ only in it.  The noise functions and the node bodies
 * are out-of-line calls (CY_NOINLINE, as the reference marks them
 * ccl_device_noinline): inlined into every shading kernel they multiply the
 * code size and compile time for shaders that rarely use them.
 */
#ifndef CY_SVM_NOISE_H
#define CY_SVM_NOISE_H

enum {
  NODE_TEX_NOISE = 25,
  NODE_TEX_MUSGRAVE = 59,
  NODE_TEX_WAVE = 60,
  NODE_TEX_MAGIC = 61,
  NODE_TEX_BRICK = 63,
  NODE_TEX_WHITE_NOISE = 64
};

typedef struct cyf2 {
  float x, y;
} cyf2;
typedef struct cyf4 {
  float x, y, z, w;
} cyf4;

CY_FN cyf2 mkf2(float x, float y)
{
  cyf2 r;
  r.x = x;
  r.y = y;
  return r;
}
CY_FN cyf4 mkf4v(float x, float y, float z, float w)
{
  cyf4 r;
  r.x = x;
  r.y = y;
  r.z = z;
  r.w = w;
  return r;
}
/* elementwise p * s and p + q for the four coordinate types */
CY_FN float nmul(float p, float s)
{
  return p * s;
}
CY_FN cyf2 nmul(cyf2 p, float s)
{
  return mkf2(p.x * s, p.y * s);
}
CY_FN cfloat3 nmul(cfloat3 p, float s)
{
  return mk3(p.x * s, p.y * s, p.z * s);
}
CY_FN cyf4 nmul(cyf4 p, float s)
{
  return mkf4v(p.x * s, p.y * s, p.z * s, p.w * s);
}
CY_FN float nadd(float p, float q)
{
  return p + q;
}
CY_FN cyf2 nadd(cyf2 p, cyf2 q)
{
  return mkf2(p.x + q.x, p.y + q.y);
}
CY_FN cfloat3 nadd(cfloat3 p, cfloat3 q)
{
  return mk3(p.x + q.x, p.y + q.y, p.z + q.z);
}
CY_FN cyf4 nadd(cyf4 p, cyf4 q)
{
  return mkf4v(p.x + q.x, p.y + q.y, p.z + q.z, p.w + q.w);
}

/* ---- util_hash.h --------------------------------------------------------- */
#define CY_ROT(x, k) (((x) << (k)) | ((x) >> (32 - (k))))
#define CY_HASH_MIX(a, b, c) \
  { \
    a -= c; \
    a ^= CY_ROT(c, 4); \
    c += b; \
    b -= a; \
    b ^= CY_ROT(a, 6); \
    a += c; \
    c -= b; \
    c ^= CY_ROT(b, 8); \
    b += a; \
    a -= c; \
    a ^= CY_ROT(c, 16); \
    c += b; \
    b -= a; \
    b ^= CY_ROT(a, 19); \
    a += c; \
    c -= b; \
    c ^= CY_ROT(b, 4); \
    b += a; \
  }
#define CY_HASH_FINAL(a, b, c) \
  { \
    c ^= b; \
    c -= CY_ROT(b, 14); \
    a ^= c; \
    a -= CY_ROT(c, 11); \
    b ^= a; \
    b -= CY_ROT(a, 25); \
    c ^= b; \
    c -= CY_ROT(b, 16); \
    a ^= c; \
    a -= CY_ROT(c, 4); \
    b ^= a; \
    b -= CY_ROT(a, 14); \
    c ^= b; \
    c -= CY_ROT(b, 24); \
  }

CY_FN uint hash_uint(uint kx)
{
  uint a, b, c;
  a = b = c = 0xdeadbeefu + (1u << 2) + 13u;
  a += kx;
  CY_HASH_FINAL(a, b, c);
  return c;
}
CY_FN uint hash_uint3(uint kx, uint ky, uint kz)
{
  uint a, b, c;
  a = b = c = 0xdeadbeefu + (3u << 2) + 13u;
  c += kz;
  b += ky;
  a += kx;
  CY_HASH_FINAL(a, b, c);
  return c;
}
CY_FN uint hash_uint4(uint kx, uint ky, uint kz, uint kw)
{
  uint a, b, c;
  a = b = c = 0xdeadbeefu + (4u << 2) + 13u;
  a += kx;
  b += ky;
  c += kz;
  CY_HASH_MIX(a, b, c);
  a += kw;
  CY_HASH_FINAL(a, b, c);
  return c;
}
#undef CY_HASH_MIX
#undef CY_HASH_FINAL
#undef CY_ROT

CY_FN float hash_uint_to_float(uint kx)
{
  return (float)hash_uint(kx) / (float)0xFFFFFFFFu;
}
CY_FN float hash_uint2_to_float(uint kx, uint ky)
{
  return (float)hash_uint2(kx, ky) / (float)0xFFFFFFFFu;
}
CY_FN float hash_uint3_to_float(uint kx, uint ky, uint kz)
{
  return (float)hash_uint3(kx, ky, kz) / (float)0xFFFFFFFFu;
}
CY_FN float hash_uint4_to_float(uint kx, uint ky, uint kz, uint kw)
{
  return (float)hash_uint4(kx, ky, kz, kw) / (float)0xFFFFFFFFu;
}
CY_FN float hash_float_to_float(float k)
{
  return hash_uint_to_float(as_uint(k));
}
CY_FN float hash_float2_to_float(float x, float y)
{
  return hash_uint2_to_float(as_uint(x), as_uint(y));
}
CY_FN float hash_float3_to_float(float x, float y, float z)
{
  return hash_uint3_to_float(as_uint(x), as_uint(y), as_uint(z));
}
CY_FN float hash_float4_to_float(float x, float y, float z, float w)
{
  return hash_uint4_to_float(as_uint(x), as_uint(y), as_uint(z), as_uint(w));
}

/* ---- Perlin noise (svm_noise.h) ------------------------------------------ */
CY_FN float negate_if(float val, int condition)
{
  return condition ? -val : val;
}

/* scalar branch, 1D */
CY_NOINLINE float perlin_1d(float x)
{
  const int X = (int)((uint)cy_ftoi(x) - ((x < 0.0f) ? 1u : 0u)); /* quick_floor_to_int (wrapping, as x86) */
  const float fx = x - (float)X;
  const float u = fx * fx * fx * (fx * (fx * 6.0f - 15.0f) + 10.0f);
  const int h0 = (int)hash_uint((uint)X) & 15;
  const int h1 = (int)hash_uint(((uint)X + (uint)1)) & 15;
  const float a = negate_if((float)(1 + (h0 & 7)), h0 & 8) * fx;
  const float b = negate_if((float)(1 + (h1 & 7)), h1 & 8) * (fx - 1.0f);
  return a + u * (b - a);
}

/* SSE2 branch helpers: ssef floorfrac (truncate + (x < 0 ? -1 : 0)), fade and mix */
CY_FN float sse_floorfrac(float x, int *i)
{
  *i = (int)((uint)cy_ftoi(x) - ((x < 0.0f) ? 1u : 0u)); /* wrapping, as x86 */
  return x - (float)(*i);
}
CY_FN float sse_fade(float t)
{
  const float a = t * 6.0f + -15.0f;
  const float b = t * a + 10.0f;
  return (t * t) * (t * b);
}
CY_FN float sse_mix(float a, float b, float t)
{
  return t * b + (1.0f - t) * a;
}
CY_FN float grad2(uint hash, float x, float y)
{
  const int h = (int)(hash & 7u);
  const float u = h < 4 ? x : y;
  const float v = 2.0f * (h < 4 ? y : x);
  return negate_if(u, h & 1) + negate_if(v, h & 2);
}
CY_FN float grad3(uint hash, float x, float y, float z)
{
  const int h = (int)(hash & 15u);
  const float u = h < 8 ? x : y;
  const float vt = ((h == 12) || (h == 14)) ? x : z;
  const float v = h < 4 ? y : vt;
  return negate_if(u, h & 1) + negate_if(v, h & 2);
}
CY_FN float grad4(uint hash, float x, float y, float z, float w)
{
  const int h = (int)(hash & 31u);
  const float u = h < 24 ? x : y;
  const float v = h < 16 ? y : z;
  const float s = h < 8 ? z : w;
  return negate_if(u, h & 1) + negate_if(v, h & 2) + negate_if(s, h & 4);
}

CY_NOINLINE float perlin_2d(float x, float y)
{
  int X, Y;
  const float fx = sse_floorfrac(x, &X);
  const float fy = sse_floorfrac(y, &Y);
  const float u = sse_fade(fx), v = sse_fade(fy);
  /* lanes (X, Y), (X, Y+1), (X+1, Y), (X+1, Y+1) */
  const float g0 = grad2(hash_uint2((uint)X, (uint)Y), fx, fy);
  const float g1 = grad2(hash_uint2((uint)X, ((uint)Y + (uint)1)), fx, fy - 1.0f);
  const float g2 = grad2(hash_uint2(((uint)X + (uint)1), (uint)Y), fx - 1.0f, fy);
  const float g3 = grad2(hash_uint2(((uint)X + (uint)1), ((uint)Y + (uint)1)), fx - 1.0f, fy - 1.0f);
  return sse_mix(sse_mix(g0, g2, u), sse_mix(g1, g3, u), v);
}

/* tri_mix of the lanes p (x) and q (x + 1): (y, z), (y, z+1), (y+1, z), (y+1, z+1) */
CY_FN float sse_tri_mix(const float p[4], const float q[4], float u, float v, float w)
{
  const float s0 = sse_mix(p[0], q[0], u), s1 = sse_mix(p[1], q[1], u);
  const float s2 = sse_mix(p[2], q[2], u), s3 = sse_mix(p[3], q[3], u);
  return sse_mix(sse_mix(s0, s2, v), sse_mix(s1, s3, v), w);
}

CY_NOINLINE float perlin_3d(float x, float y, float z)
{
  int X, Y, Z;
  const float fx = sse_floorfrac(x, &X);
  const float fy = sse_floorfrac(y, &Y);
  const float fz = sse_floorfrac(z, &Z);
  const float u = sse_fade(fx), v = sse_fade(fy), w = sse_fade(fz);
  float g1[4], g2[4];
  for (int k = 0; k < 4; k++) {
    const int dy = k >> 1, dz = k & 1;
    const float gy = dy ? fy - 1.0f : fy, gz = dz ? fz - 1.0f : fz;
    g1[k] = grad3(hash_uint3((uint)X, ((uint)Y + (uint)dy), ((uint)Z + (uint)dz)), fx, gy, gz);
    g2[k] = grad3(hash_uint3(((uint)X + (uint)1), ((uint)Y + (uint)dy), ((uint)Z + (uint)dz)), fx - 1.0f, gy, gz);
  }
  return sse_tri_mix(g1, g2, u, v, w);
}

CY_NOINLINE float perlin_4d(float x, float y, float z, float w)
{
  int X, Y, Z, W;
  const float fx = sse_floorfrac(x, &X);
  const float fy = sse_floorfrac(y, &Y);
  const float fz = sse_floorfrac(z, &Z);
  const float fw = sse_floorfrac(w, &W);
  const float u = sse_fade(fx), v = sse_fade(fy), t = sse_fade(fz), s = sse_fade(fw);
  float g1[4], g2[4], g3[4], g4[4];
  for (int k = 0; k < 4; k++) {
    const int dy = k >> 1, dz = k & 1;
    const float gy = dy ? fy - 1.0f : fy, gz = dz ? fz - 1.0f : fz;
    const uint yy = ((uint)Y + (uint)dy), zz = ((uint)Z + (uint)dz);
    g1[k] = grad4(hash_uint4((uint)X, yy, zz, (uint)W), fx, gy, gz, fw);
    g2[k] = grad4(hash_uint4(((uint)X + (uint)1), yy, zz, (uint)W), fx - 1.0f, gy, gz, fw);
    g3[k] = grad4(hash_uint4((uint)X, yy, zz, ((uint)W + (uint)1)), fx, gy, gz, fw - 1.0f);
    g4[k] = grad4(hash_uint4(((uint)X + (uint)1), yy, zz, ((uint)W + (uint)1)), fx - 1.0f, gy, gz, fw - 1.0f);
  }
  return sse_mix(sse_tri_mix(g1, g2, u, v, t), sse_tri_mix(g3, g4, u, v, t), s);
}

CY_FN float ensure_finite(float v)
{
  return isfinite_safe(v) ? v : 0.0f;
}

/* signed noise remapped to [-1, 1] (noise_scale1..4) and unsigned [0, 1] */
CY_FN float snoise(float p)
{
  return 0.2500f * ensure_finite(perlin_1d(p));
}
CY_FN float snoise(cyf2 p)
{
  return 0.6616f * ensure_finite(perlin_2d(p.x, p.y));
}
CY_FN float snoise(cfloat3 p)
{
  return 0.9820f * ensure_finite(perlin_3d(p.x, p.y, p.z));
}
CY_FN float snoise(cyf4 p)
{
  return 0.8344f * ensure_finite(perlin_4d(p.x, p.y, p.z, p.w));
}
template<typename V> CY_FN float unoise(V p)
{
  return 0.5f * snoise(p) + 0.5f;
}

/* svm_fractal_noise.h fractal_noise_1d..4d */
template<typename V> CY_NOINLINE float fractal_noise(V p, float octaves, float roughness)
{
  float fscale = 1.0f;
  float amp = 1.0f;
  float maxamp = 0.0f;
  float sum = 0.0f;
  octaves = cy_clampf(octaves, 0.0f, 16.0f);
  const int n = (int)octaves;
  for (int i = 0; i <= n; i++) {
    const float t = unoise(nmul(p, fscale));
    sum += t * amp;
    maxamp += amp;
    amp *= cy_clampf(roughness, 0.0f, 1.0f);
    fscale *= 2.0f;
  }
  const float rmd = octaves - floorf(octaves);
  if (rmd != 0.0f) {
    const float t = unoise(nmul(p, fscale));
    float sum2 = sum + t * amp;
    sum /= maxamp;
    sum2 /= maxamp + amp;
    return (1.0f - rmd) * sum + rmd * sum2;
  }
  return sum / maxamp;
}

/* svm_noisetex.h random offsets: components in [100, 200] */
CY_FN float random_float_offset(float seed)
{
  return 100.0f + hash_float_to_float(seed) * 100.0f;
}
CY_FN float random_offset_component(float seed, float k)
{
  return 100.0f + hash_float2_to_float(seed, k) * 100.0f;
}
CY_FN float noise_offset(float seed, float)
{
  return random_float_offset(seed);
}
CY_FN cyf2 noise_offset(float seed, cyf2)
{
  return mkf2(random_offset_component(seed, 0.0f), random_offset_component(seed, 1.0f));
}
CY_FN cfloat3 noise_offset(float seed, cfloat3)
{
  return mk3(random_offset_component(seed, 0.0f), random_offset_component(seed, 1.0f),
             random_offset_component(seed, 2.0f));
}
CY_FN cyf4 noise_offset(float seed, cyf4)
{
  return mkf4v(random_offset_component(seed, 0.0f), random_offset_component(seed, 1.0f),
               random_offset_component(seed, 2.0f), random_offset_component(seed, 3.0f));
}

/* noise_texture_*d: distortion by signed noise at seeded offsets (seeds
 * 0..D-1), then the fractal noise value and (seeds D, D+1) two more channels */
CY_FN float noise_distort(float p, float distortion)
{
  return p + snoise(p + random_float_offset(0.0f)) * distortion;
}
CY_FN cyf2 noise_distort(cyf2 p, float distortion)
{
  return nadd(p, mkf2(snoise(nadd(p, noise_offset(0.0f, p))) * distortion,
                      snoise(nadd(p, noise_offset(1.0f, p))) * distortion));
}
CY_FN cfloat3 noise_distort(cfloat3 p, float distortion)
{
  return nadd(p, mk3(snoise(nadd(p, noise_offset(0.0f, p))) * distortion,
                     snoise(nadd(p, noise_offset(1.0f, p))) * distortion,
                     snoise(nadd(p, noise_offset(2.0f, p))) * distortion));
}
CY_FN cyf4 noise_distort(cyf4 p, float distortion)
{
  return nadd(p, mkf4v(snoise(nadd(p, noise_offset(0.0f, p))) * distortion,
                       snoise(nadd(p, noise_offset(1.0f, p))) * distortion,
                       snoise(nadd(p, noise_offset(2.0f, p))) * distortion,
                       snoise(nadd(p, noise_offset(3.0f, p))) * distortion));
}

template<typename V>
CY_FN void noise_texture(V co, float color_seed, float detail, float roughness, float distortion,
                         bool color_is_needed, float *value, cfloat3 *color)
{
  V p = co;
  if (distortion != 0.0f) {
    p = noise_distort(p, distortion);
  }
  *value = fractal_noise(p, detail, roughness);
  if (color_is_needed) {
    *color = mk3(*value, fractal_noise(nadd(p, noise_offset(color_seed, p)), detail, roughness),
                 fractal_noise(nadd(p, noise_offset(color_seed + 1.0f, p)), detail, roughness));
  }
}

CY_NOINLINE void svm_node_tex_noise(const CyGlobals *kg, CySvmStack stack, uint dimensions, uint offsets1, uint offsets2,
                              int *offset, uint *err)
{
  uint vector_off, w_off, scale_off, detail_off, roughness_off, distortion_off, value_off, color_off;
  svm_unpack4(offsets1, &vector_off, &w_off, &scale_off, &detail_off);
  svm_unpack4(offsets2, &roughness_off, &distortion_off, &value_off, &color_off);
  const hc_uint4 defaults1 = kg->__svm_nodes[*offset];
  const hc_uint4 defaults2 = kg->__svm_nodes[*offset + 1];
  *offset += 2;
  cfloat3 vector = svm_load3(stack, vector_off, err);
  float w = svm_load_default(stack, w_off, defaults1.x, err);
  const float scale = svm_load_default(stack, scale_off, defaults1.y, err);
  const float detail = svm_load_default(stack, detail_off, defaults1.z, err);
  const float roughness = svm_load_default(stack, roughness_off, defaults1.w, err);
  const float distortion = svm_load_default(stack, distortion_off, defaults2.x, err);
  vector = mul3f(vector, scale);
  w *= scale;
  float value = 0.0f;
  cfloat3 color = mk3(0.0f, 0.0f, 0.0f);
  const bool need_color = color_off != SVM_STACK_INVALID;
  switch (dimensions) {
    case 1:
      noise_texture(w, 1.0f, detail, roughness, distortion, need_color, &value, &color);
      break;
    case 2:
      noise_texture(mkf2(vector.x, vector.y), 2.0f, detail, roughness, distortion, need_color, &value, &color);
      break;
    case 3:
      noise_texture(vector, 3.0f, detail, roughness, distortion, need_color, &value, &color);
      break;
    case 4:
      noise_texture(mkf4v(vector.x, vector.y, vector.z, w), 4.0f, detail, roughness, distortion, need_color, &value,
                    &color);
      break;
    default:
      cy_set_error(err, CY_ERR_SVM_NODE, NODE_TEX_NOISE);
      return;
  }
  if (value_off != SVM_STACK_INVALID) {
    svm_store(stack, value_off, value, err);
  }
  if (need_color) {
    svm_store3(stack, color_off, color, err);
  }
}

/* ---- Wave (svm_wave.h) --------------------------------------------------- */
CY_NOINLINE float svm_wave(uint type, uint bands_dir, uint rings_dir, uint profile, cfloat3 p, float distortion,
                     float detail, float dscale, float droughness, float phase)
{
  p = mul3f(add3(p, mk3(0.000001f, 0.000001f, 0.000001f)), 0.999999f);
  float n;
  if (type == 0) { /* NODE_WAVE_BANDS */
    if (bands_dir == 0) {
      n = p.x * 20.0f;
    }
    else if (bands_dir == 1) {
      n = p.y * 20.0f;
    }
    else if (bands_dir == 2) {
      n = p.z * 20.0f;
    }
    else { /* diagonal */
      n = (p.x + p.y + p.z) * 10.0f;
    }
  }
  else { /* NODE_WAVE_RINGS */
    cfloat3 rp = p;
    if (rings_dir == 0) {
      rp = mul3(rp, mk3(0.0f, 1.0f, 1.0f));
    }
    else if (rings_dir == 1) {
      rp = mul3(rp, mk3(1.0f, 0.0f, 1.0f));
    }
    else if (rings_dir == 2) {
      rp = mul3(rp, mk3(1.0f, 1.0f, 0.0f));
    }
    n = len3(rp) * 20.0f;
  }
  n += phase;
  if (distortion != 0.0f) {
    n += distortion * (fractal_noise(mul3f(p, dscale), detail, droughness) * 2.0f - 1.0f);
  }
  if (profile == 0) { /* sine */
    return 0.5f + 0.5f * cy_sinf(n - CY_PI_2_F);
  }
  else if (profile == 1) { /* saw */
    n /= CY_2PI_F;
    return n - floorf(n);
  }
  n /= CY_2PI_F; /* triangle */
  return fabsf(n - floorf(n + 0.5f)) * 2.0f;
}

CY_NOINLINE void svm_node_tex_wave(const CyGlobals *kg, CySvmStack stack, hc_uint4 node, int *offset, uint *err)
{
  const hc_uint4 node2 = kg->__svm_nodes[*offset];
  const hc_uint4 node3 = kg->__svm_nodes[*offset + 1];
  *offset += 2;
  uint type, bands_dir, rings_dir, profile, co_off, scale_off, distortion_off, detail_off, dscale_off, droughness_off,
      phase_off, color_off, fac_off, unused;
  svm_unpack4(node.y, &type, &bands_dir, &rings_dir, &profile);
  svm_unpack3(node.z, &co_off, &scale_off, &distortion_off);
  svm_unpack4(node.w, &detail_off, &dscale_off, &droughness_off, &phase_off);
  svm_unpack3(node2.x, &color_off, &fac_off, &unused);
  const cfloat3 co = svm_load3(stack, co_off, err);
  const float scale = svm_load_default(stack, scale_off, node2.y, err);
  const float distortion = svm_load_default(stack, distortion_off, node2.z, err);
  const float detail = svm_load_default(stack, detail_off, node2.w, err);
  const float dscale = svm_load_default(stack, dscale_off, node3.x, err);
  const float droughness = svm_load_default(stack, droughness_off, node3.y, err);
  const float phase = svm_load_default(stack, phase_off, node3.z, err);
  const float f = svm_wave(type, bands_dir, rings_dir, profile, mul3f(co, scale), distortion, detail, dscale,
                           droughness, phase);
  if (fac_off != SVM_STACK_INVALID) {
    svm_store(stack, fac_off, f, err);
  }
  if (color_off != SVM_STACK_INVALID) {
    svm_store3(stack, color_off, mk3(f, f, f), err);
  }
}

/* ---- Magic (svm_magic.h) ------------------------------------------------- */
CY_NOINLINE cfloat3 svm_magic(cfloat3 p, int n, float distortion)
{
  float x = cy_sinf((p.x + p.y + p.z) * 5.0f);
  float y = cy_cosf((-p.x + p.y - p.z) * 5.0f);
  float z = -cy_cosf((-p.x - p.y + p.z) * 5.0f);
  if (n > 0) {
    x *= distortion;
    y *= distortion;
    z *= distortion;
    y = -cy_cosf(x - y + z);
    y *= distortion;
    if (n > 1) {
      x = cy_cosf(x - y - z);
      x *= distortion;
      if (n > 2) {
        z = cy_sinf(-x - y - z);
        z *= distortion;
        if (n > 3) {
          x = -cy_cosf(-x + y - z);
          x *= distortion;
          if (n > 4) {
            y = -cy_sinf(-x + y + z);
            y *= distortion;
            if (n > 5) {
              y = -cy_cosf(-x + y + z);
              y *= distortion;
              if (n > 6) {
                x = cy_cosf(x + y + z);
                x *= distortion;
                if (n > 7) {
                  z = cy_sinf(x + y - z);
                  z *= distortion;
                  if (n > 8) {
                    x = -cy_cosf(-x - y + z);
                    x *= distortion;
                    if (n > 9) {
                      y = -cy_sinf(x - y + z);
                      y *= distortion;
                    }
                  }
                }
              }
            }
          }
        }
      }
    }
  }
  if (distortion != 0.0f) {
    distortion *= 2.0f;
    x /= distortion;
    y /= distortion;
    z /= distortion;
  }
  return mk3(0.5f - x, 0.5f - y, 0.5f - z);
}

CY_NOINLINE void svm_node_tex_magic(const CyGlobals *kg, CySvmStack stack, hc_uint4 node, int *offset, uint *err)
{
  uint depth, color_off, fac_off, co_off, scale_off, distortion_off;
  svm_unpack3(node.y, &depth, &color_off, &fac_off);
  svm_unpack3(node.z, &co_off, &scale_off, &distortion_off);
  const hc_uint4 node2 = kg->__svm_nodes[*offset];
  *offset += 1;
  const cfloat3 co = svm_load3(stack, co_off, err);
  const float scale = svm_load_default(stack, scale_off, node2.x, err);
  const float distortion = svm_load_default(stack, distortion_off, node2.y, err);
  const cfloat3 color = svm_magic(mul3f(co, scale), (int)depth, distortion);
  if (fac_off != SVM_STACK_INVALID) {
    svm_store(stack, fac_off, average3(color), err);
  }
  if (color_off != SVM_STACK_INVALID) {
    svm_store3(stack, color_off, color, err);
  }
}

/* ---- Brick (svm_brick.h) ------------------------------------------------- */
CY_FN float brick_noise(uint n)
{
  uint nn;
  n = (n + 1013u) & 0x7fffffffu;
  n = (n >> 13) ^ n;
  nn = (n * (n * n * 60493u + 19990303u) + 1376312589u) & 0x7fffffffu;
  return 0.5f * ((float)nn / 1073741824.0f);
}

CY_NOINLINE void svm_brick(cfloat3 p, float mortar_size, float mortar_smooth, float bias, float brick_width,
                     float row_height, float offset_amount, int offset_frequency, float squash_amount,
                     int squash_frequency, float *tint_out, float *mortar_out)
{
  float offset = 0.0f;
  const int rownum = cy_ftoi(floorf(p.y / row_height));
  if (offset_frequency && squash_frequency) {
    brick_width *= (rownum % squash_frequency) ? 1.0f : squash_amount;
    offset = (rownum % offset_frequency) ? 0.0f : (brick_width * offset_amount);
  }
  const int bricknum = cy_ftoi(floorf((p.x + offset) / brick_width));
  const float x = (p.x + offset) - brick_width * bricknum;
  const float y = p.y - row_height * rownum;
  const float tint = saturate((brick_noise(((uint)rownum << 16) + (uint)(bricknum & 0xFFFF)) + bias));
  float min_dist = cy_min(cy_min(x, y), cy_min(brick_width - x, row_height - y));
  float mortar;
  if (min_dist >= mortar_size) {
    mortar = 0.0f;
  }
  else if (mortar_smooth == 0.0f) {
    mortar = 1.0f;
  }
  else {
    min_dist = 1.0f - min_dist / mortar_size;
    if (min_dist < mortar_smooth) {
      const float f = min_dist / mortar_smooth;
      const float ff = f * f;
      mortar = 3.0f * ff - 2.0f * ff * f; /* smoothstepf */
    }
    else {
      mortar = 1.0f;
    }
  }
  *tint_out = tint;
  *mortar_out = mortar;
}

CY_NOINLINE void svm_node_tex_brick(const CyGlobals *kg, CySvmStack stack, hc_uint4 node, int *offset, uint *err)
{
  const hc_uint4 node2 = kg->__svm_nodes[*offset];
  const hc_uint4 node3 = kg->__svm_nodes[*offset + 1];
  const hc_uint4 node4 = kg->__svm_nodes[*offset + 2];
  *offset += 3;
  uint co_off, color1_off, color2_off, mortar_off, scale_off, mortar_size_off, bias_off, brick_width_off;
  uint row_height_off, color_off, fac_off, mortar_smooth_off, offset_frequency, squash_frequency, unused;
  svm_unpack4(node.y, &co_off, &color1_off, &color2_off, &mortar_off);
  svm_unpack4(node.z, &scale_off, &mortar_size_off, &bias_off, &brick_width_off);
  svm_unpack4(node.w, &row_height_off, &color_off, &fac_off, &mortar_smooth_off);
  svm_unpack3(node2.x, &offset_frequency, &squash_frequency, &unused);
  const cfloat3 co = svm_load3(stack, co_off, err);
  cfloat3 color1 = svm_load3(stack, color1_off, err);
  const cfloat3 color2 = svm_load3(stack, color2_off, err);
  const cfloat3 mortar = svm_load3(stack, mortar_off, err);
  const float scale = svm_load_default(stack, scale_off, node2.y, err);
  const float mortar_size = svm_load_default(stack, mortar_size_off, node2.z, err);
  const float mortar_smooth = svm_load_default(stack, mortar_smooth_off, node4.x, err);
  const float bias = svm_load_default(stack, bias_off, node2.w, err);
  const float brick_width = svm_load_default(stack, brick_width_off, node3.x, err);
  const float row_height = svm_load_default(stack, row_height_off, node3.y, err);
  const float offset_amount = as_float(node3.z);
  const float squash_amount = as_float(node3.w);
  float tint, f;
  svm_brick(mul3f(co, scale), mortar_size, mortar_smooth, bias, brick_width, row_height, offset_amount,
            (int)offset_frequency, squash_amount, (int)squash_frequency, &tint, &f);
  if (f != 1.0f) {
    const float facm = 1.0f - tint;
    color1 = add3(mul3f(color1, facm), mul3f(color2, tint));
  }
  if (color_off != SVM_STACK_INVALID) {
    svm_store3(stack, color_off, add3(mul3f(color1, 1.0f - f), mul3f(mortar, f)), err);
  }
  if (fac_off != SVM_STACK_INVALID) {
    svm_store(stack, fac_off, f, err);
  }
}

/* ---- White noise (svm_white_noise.h) ------------------------------------- */
CY_NOINLINE void svm_node_tex_white_noise(CySvmStack stack, uint dimensions, uint inputs, uint outputs, uint *err)
{
  const uint vector_off = inputs & 0xFF, w_off = (inputs >> 8) & 0xFF;
  const uint value_off = outputs & 0xFF, color_off = (outputs >> 8) & 0xFF;
  const cfloat3 v = svm_load3(stack, vector_off, err);
  const float w = svm_load(stack, w_off, err);
  if (color_off != SVM_STACK_INVALID) {
    cfloat3 color;
    switch (dimensions) {
      case 1:
        color = mk3(hash_float_to_float(w), hash_float2_to_float(w, 1.0f), hash_float2_to_float(w, 2.0f));
        break;
      case 2:
        color = mk3(hash_float2_to_float(v.x, v.y), hash_float3_to_float(v.x, v.y, 1.0f),
                    hash_float3_to_float(v.x, v.y, 2.0f));
        break;
      case 3:
        color = mk3(hash_float3_to_float(v.x, v.y, v.z), hash_float4_to_float(v.x, v.y, v.z, 1.0f),
                    hash_float4_to_float(v.x, v.y, v.z, 2.0f));
        break;
      case 4:
        color = mk3(hash_float4_to_float(v.x, v.y, v.z, w), hash_float4_to_float(v.z, v.x, w, v.y),
                    hash_float4_to_float(w, v.z, v.y, v.x));
        break;
      default:
        cy_set_error(err, CY_ERR_SVM_NODE, NODE_TEX_WHITE_NOISE);
        return;
    }
    svm_store3(stack, color_off, color, err);
  }
  if (value_off != SVM_STACK_INVALID) {
    float value;
    switch (dimensions) {
      case 1:
        value = hash_float_to_float(w);
        break;
      case 2:
        value = hash_float2_to_float(v.x, v.y);
        break;
      case 3:
        value = hash_float3_to_float(v.x, v.y, v.z);
        break;
      case 4:
        value = hash_float4_to_float(v.x, v.y, v.z, w);
        break;
      default:
        cy_set_error(err, CY_ERR_SVM_NODE, NODE_TEX_WHITE_NOISE);
        return;
    }
    svm_store(stack, value_off, value, err);
  }
}

/* ---- Musgrave (svm_musgrave.h) ------------------------------------------- */
template<typename V> CY_NOINLINE float musgrave_fBm(V p, float H, float lacunarity, float octaves)
{
  float value = 0.0f;
  float pwr = 1.0f;
  const float pwHL = cy_powf(lacunarity, -H);
  for (int i = 0; i < (int)octaves; i++) {
    value += snoise(p) * pwr;
    pwr *= pwHL;
    p = nmul(p, lacunarity);
  }
  const float rmd = octaves - floorf(octaves);
  if (rmd != 0.0f) {
    value += rmd * snoise(p) * pwr;
  }
  return value;
}

template<typename V> CY_NOINLINE float musgrave_multi_fractal(V p, float H, float lacunarity, float octaves)
{
  float value = 1.0f;
  float pwr = 1.0f;
  const float pwHL = cy_powf(lacunarity, -H);
  for (int i = 0; i < (int)octaves; i++) {
    value *= (pwr * snoise(p) + 1.0f);
    pwr *= pwHL;
    p = nmul(p, lacunarity);
  }
  const float rmd = octaves - floorf(octaves);
  if (rmd != 0.0f) {
    value *= (rmd * pwr * snoise(p) + 1.0f);
  }
  return value;
}

template<typename V>
CY_NOINLINE float musgrave_hetero_terrain(V p, float H, float lacunarity, float octaves, float offset)
{
  const float pwHL = cy_powf(lacunarity, -H);
  float pwr = pwHL;
  float value = offset + snoise(p);
  p = nmul(p, lacunarity);
  for (int i = 1; i < (int)octaves; i++) {
    const float increment = (snoise(p) + offset) * pwr * value;
    value += increment;
    pwr *= pwHL;
    p = nmul(p, lacunarity);
  }
  const float rmd = octaves - floorf(octaves);
  if (rmd != 0.0f) {
    const float increment = (snoise(p) + offset) * pwr * value;
    value += rmd * increment;
  }
  return value;
}

template<typename V>
CY_NOINLINE float musgrave_hybrid_multi_fractal(V p, float H, float lacunarity, float octaves, float offset, float gain)
{
  const float pwHL = cy_powf(lacunarity, -H);
  float pwr = pwHL;
  float value = snoise(p) + offset;
  float weight = gain * value;
  p = nmul(p, lacunarity);
  for (int i = 1; (weight > 0.001f) && (i < (int)octaves); i++) {
    if (weight > 1.0f) {
      weight = 1.0f;
    }
    const float signal = (snoise(p) + offset) * pwr;
    pwr *= pwHL;
    value += weight * signal;
    weight *= gain * signal;
    p = nmul(p, lacunarity);
  }
  const float rmd = octaves - floorf(octaves);
  if (rmd != 0.0f) {
    value += rmd * ((snoise(p) + offset) * pwr);
  }
  return value;
}

template<typename V>
CY_NOINLINE float musgrave_ridged_multi_fractal(V p, float H, float lacunarity, float octaves, float offset, float gain)
{
  const float pwHL = cy_powf(lacunarity, -H);
  float pwr = pwHL;
  float signal = offset - fabsf(snoise(p));
  signal *= signal;
  float value = signal;
  float weight = 1.0f;
  for (int i = 1; i < (int)octaves; i++) {
    p = nmul(p, lacunarity);
    weight = saturate(signal * gain);
    signal = offset - fabsf(snoise(p));
    signal *= signal;
    signal *= weight;
    value += signal * pwr;
    pwr *= pwHL;
  }
  return value;
}

/* NodeMusgraveType (svm_types.h): multifractal, fBm, hybrid, ridged, hetero terrain */
template<typename V>
CY_FN float musgrave(uint type, V p, float dimension, float lacunarity, float detail, float foffset, float gain)
{
  switch (type) {
    case 0:
      return musgrave_multi_fractal(p, dimension, lacunarity, detail);
    case 1:
      return musgrave_fBm(p, dimension, lacunarity, detail);
    case 2:
      return musgrave_hybrid_multi_fractal(p, dimension, lacunarity, detail, foffset, gain);
    case 3:
      return musgrave_ridged_multi_fractal(p, dimension, lacunarity, detail, foffset, gain);
    case 4:
      return musgrave_hetero_terrain(p, dimension, lacunarity, detail, foffset);
    default:
      return 0.0f;
  }
}

CY_NOINLINE void svm_node_tex_musgrave(const CyGlobals *kg, CySvmStack stack, uint offsets1, uint offsets2, uint offsets3,
                                 int *offset, uint *err)
{
  uint type, dimensions, co_off, w_off, scale_off, detail_off, dimension_off, lacunarity_off;
  uint offset_off, gain_off, fac_off;
  svm_unpack4(offsets1, &type, &dimensions, &co_off, &w_off);
  svm_unpack4(offsets2, &scale_off, &detail_off, &dimension_off, &lacunarity_off);
  svm_unpack3(offsets3, &offset_off, &gain_off, &fac_off);
  const hc_uint4 defaults1 = kg->__svm_nodes[*offset];
  const hc_uint4 defaults2 = kg->__svm_nodes[*offset + 1];
  *offset += 2;
  const cfloat3 co = svm_load3(stack, co_off, err);
  const float w = svm_load_default(stack, w_off, defaults1.x, err);
  const float scale = svm_load_default(stack, scale_off, defaults1.y, err);
  float detail = svm_load_default(stack, detail_off, defaults1.z, err);
  float dimension = svm_load_default(stack, dimension_off, defaults1.w, err);
  float lacunarity = svm_load_default(stack, lacunarity_off, defaults2.x, err);
  const float foffset = svm_load_default(stack, offset_off, defaults2.y, err);
  const float gain = svm_load_default(stack, gain_off, defaults2.z, err);
  dimension = fmaxf(dimension, 1e-5f);
  detail = cy_clampf(detail, 0.0f, 16.0f);
  lacunarity = fmaxf(lacunarity, 1e-5f);
  float fac;
  switch (dimensions) {
    case 1:
      fac = musgrave(type, w * scale, dimension, lacunarity, detail, foffset, gain);
      break;
    case 2:
      fac = musgrave(type, mkf2(co.x * scale, co.y * scale), dimension, lacunarity, detail, foffset, gain);
      break;
    case 3:
      fac = musgrave(type, mul3f(co, scale), dimension, lacunarity, detail, foffset, gain);
      break;
    case 4:
      fac = musgrave(type, mkf4v(co.x * scale, co.y * scale, co.z * scale, w * scale), dimension, lacunarity, detail,
                     foffset, gain);
      break;
    default:
      fac = 0.0f;
  }
  svm_store(stack, fac_off, fac, err);
}

/* ---- Voronoi (svm_voronoi.h) --------------------------------------------- */
/* NodeVoronoiDistanceMetric / NodeVoronoiFeature (svm_types.h:429-442) */
enum { NODE_TEX_VORONOI = 58 };
enum { VORONOI_EUCLIDEAN = 0, VORONOI_MANHATTAN = 1, VORONOI_CHEBYCHEV = 2, VORONOI_MINKOWSKI = 3 };
enum { VORONOI_F1 = 0, VORONOI_F2 = 1, VORONOI_SMOOTH_F1 = 2, VORONOI_DISTANCE_TO_EDGE = 3, VORONOI_N_SPHERE_RADIUS = 4 };

/* smoothstep (util_math.h:298-310) */
CY_FN float cy_smoothstep(float edge0, float edge1, float x)
{
  if (x < edge0) {
    return 0.0f;
  }
  if (x >= edge1) {
    return 1.0f;
  }
  const float t = (x - edge0) / (edge1 - edge0);
  return (3.0f - 2.0f * t) * (t * t);
}

/* 1D (svm_voronoi.h:32-193): distances are fabsf */
CY_FN cfloat3 hash_float_to_float3(float k)
{
  return mk3(hash_float_to_float(k), hash_float2_to_float(k, 1.0f), hash_float2_to_float(k, 2.0f));
}

CY_NOINLINE void voronoi_1d(uint feature, float w, float smoothness, float randomness, float *out_distance,
                            cfloat3 *out_color, float *out_w, float *out_radius)
{
  const float cellPosition = floorf(w);
  const float localPosition = w - cellPosition;
  if (feature == VORONOI_F1) {
    float minDistance = 8.0f, targetOffset = 0.0f, targetPosition = 0.0f;
    for (int i = -1; i <= 1; i++) {
      const float cellOffset = (float)i;
      const float pointPosition = cellOffset + hash_float_to_float(cellPosition + cellOffset) * randomness;
      const float distanceToPoint = fabsf(localPosition - pointPosition);
      if (distanceToPoint < minDistance) {
        targetOffset = cellOffset;
        minDistance = distanceToPoint;
        targetPosition = pointPosition;
      }
    }
    *out_distance = minDistance;
    *out_color = hash_float_to_float3(cellPosition + targetOffset);
    *out_w = targetPosition + cellPosition;
  }
  else if (feature == VORONOI_SMOOTH_F1) {
    float smoothDistance = 8.0f, smoothPosition = 0.0f;
    cfloat3 smoothColor = mk3(0.0f, 0.0f, 0.0f);
    for (int i = -2; i <= 2; i++) {
      const float cellOffset = (float)i;
      const float pointPosition = cellOffset + hash_float_to_float(cellPosition + cellOffset) * randomness;
      const float distanceToPoint = fabsf(localPosition - pointPosition);
      const float h = cy_smoothstep(0.0f, 1.0f, 0.5f + 0.5f * (smoothDistance - distanceToPoint) / smoothness);
      float correctionFactor = smoothness * h * (1.0f - h);
      smoothDistance = (smoothDistance + h * (distanceToPoint - smoothDistance)) - correctionFactor;
      correctionFactor /= 1.0f + 3.0f * smoothness;
      const cfloat3 cellColor = hash_float_to_float3(cellPosition + cellOffset);
      smoothColor = sub3(add3(smoothColor, mul3f(sub3(cellColor, smoothColor), h)),
                         mk3(correctionFactor, correctionFactor, correctionFactor));
      smoothPosition = (smoothPosition + h * (pointPosition - smoothPosition)) - correctionFactor;
    }
    *out_distance = smoothDistance;
    *out_color = smoothColor;
    *out_w = cellPosition + smoothPosition;
  }
  else if (feature == VORONOI_F2) {
    float distanceF1 = 8.0f, distanceF2 = 8.0f, offsetF1 = 0.0f, positionF1 = 0.0f, offsetF2 = 0.0f,
          positionF2 = 0.0f;
    for (int i = -1; i <= 1; i++) {
      const float cellOffset = (float)i;
      const float pointPosition = cellOffset + hash_float_to_float(cellPosition + cellOffset) * randomness;
      const float distanceToPoint = fabsf(localPosition - pointPosition);
      if (distanceToPoint < distanceF1) {
        distanceF2 = distanceF1;
        distanceF1 = distanceToPoint;
        offsetF2 = offsetF1;
        offsetF1 = cellOffset;
        positionF2 = positionF1;
        positionF1 = pointPosition;
      }
      else if (distanceToPoint < distanceF2) {
        distanceF2 = distanceToPoint;
        offsetF2 = cellOffset;
        positionF2 = pointPosition;
      }
    }
    *out_distance = distanceF2;
    *out_color = hash_float_to_float3(cellPosition + offsetF2);
    *out_w = positionF2 + cellPosition;
  }
  else if (feature == VORONOI_DISTANCE_TO_EDGE) {
    float minDistance = 8.0f;
    for (int i = -1; i <= 1; i++) {
      const float cellOffset = (float)i;
      const float pointPosition = cellOffset + hash_float_to_float(cellPosition + cellOffset) * randomness;
      minDistance = cy_min(fabsf(pointPosition - localPosition), minDistance);
    }
    *out_distance = minDistance;
  }
  else if (feature == VORONOI_N_SPHERE_RADIUS) {
    float closestPoint = 0.0f, closestPointOffset = 0.0f, minDistance = 8.0f;
    for (int i = -1; i <= 1; i++) {
      const float cellOffset = (float)i;
      const float pointPosition = cellOffset + hash_float_to_float(cellPosition + cellOffset) * randomness;
      const float distanceToPoint = fabsf(pointPosition - localPosition);
      if (distanceToPoint < minDistance) {
        minDistance = distanceToPoint;
        closestPoint = pointPosition;
        closestPointOffset = cellOffset;
      }
    }
    minDistance = 8.0f;
    float closestPointToClosestPoint = 0.0f;
    for (int i = -1; i <= 1; i++) {
      if (i == 0) {
        continue;
      }
      const float cellOffset = (float)i + closestPointOffset;
      const float pointPosition = cellOffset + hash_float_to_float(cellPosition + cellOffset) * randomness;
      const float distanceToPoint = fabsf(closestPoint - pointPosition);
      if (distanceToPoint < minDistance) {
        minDistance = distanceToPoint;
        closestPointToClosestPoint = pointPosition;
      }
    }
    *out_radius = fabsf(closestPointToClosestPoint - closestPoint) / 2.0f;
  }
}

/* 2D..4D: one template over the dimension; float2/float3/float4 operators of
 * util_math_float{2,3,4}.h (componentwise; dot pairs (xx + yy) + (zz + ww) in
 * 4D; a / f multiplies by 1 / f). */
template<int D> struct vv {
  float c[D];
};
template<int D> CY_FN vv<D> vv_add(vv<D> a, vv<D> b)
{
  vv<D> r;
  for (int i = 0; i < D; i++) {
    r.c[i] = a.c[i] + b.c[i];
  }
  return r;
}
template<int D> CY_FN vv<D> vv_sub(vv<D> a, vv<D> b)
{
  vv<D> r;
  for (int i = 0; i < D; i++) {
    r.c[i] = a.c[i] - b.c[i];
  }
  return r;
}
template<int D> CY_FN vv<D> vv_mul(vv<D> a, float s)
{
  vv<D> r;
  for (int i = 0; i < D; i++) {
    r.c[i] = a.c[i] * s;
  }
  return r;
}
template<int D> CY_FN vv<D> vv_subf(vv<D> a, float s)
{
  vv<D> r;
  for (int i = 0; i < D; i++) {
    r.c[i] = a.c[i] - s;
  }
  return r;
}
/* mix(a, b, t) = a + t * (b - a) */
template<int D> CY_FN vv<D> vv_mix(vv<D> a, vv<D> b, float t)
{
  vv<D> r;
  for (int i = 0; i < D; i++) {
    r.c[i] = a.c[i] + t * (b.c[i] - a.c[i]);
  }
  return r;
}
template<int D> CY_FN float vv_dot(vv<D> a, vv<D> b)
{
  if constexpr (D == 2) {
    return a.c[0] * b.c[0] + a.c[1] * b.c[1];
  }
  else if constexpr (D == 3) {
    return a.c[0] * b.c[0] + a.c[1] * b.c[1] + a.c[2] * b.c[2];
  }
  else {
    return (a.c[0] * b.c[0] + a.c[1] * b.c[1]) + (a.c[2] * b.c[2] + a.c[3] * b.c[3]);
  }
}
template<int D> CY_FN float vv_len(vv<D> a)
{
  return sqrtf(vv_dot(a, a));
}
template<int D> CY_FN vv<D> vv_floor(vv<D> a)
{
  vv<D> r;
  for (int i = 0; i < D; i++) {
    r.c[i] = floorf(a.c[i]);
  }
  return r;
}
/* hash_float{2,3,4}_to_float{2,3,4} (util_hash.h:175-193) */
template<int D> CY_FN vv<D> vv_hash(vv<D> k)
{
  vv<D> r;
  if constexpr (D == 2) {
    r.c[0] = hash_float2_to_float(k.c[0], k.c[1]);
    r.c[1] = hash_float3_to_float(k.c[0], k.c[1], 1.0f);
  }
  else if constexpr (D == 3) {
    r.c[0] = hash_float3_to_float(k.c[0], k.c[1], k.c[2]);
    r.c[1] = hash_float4_to_float(k.c[0], k.c[1], k.c[2], 1.0f);
    r.c[2] = hash_float4_to_float(k.c[0], k.c[1], k.c[2], 2.0f);
  }
  else {
    r.c[0] = hash_float4_to_float(k.c[0], k.c[1], k.c[2], k.c[3]);
    r.c[1] = hash_float4_to_float(k.c[3], k.c[0], k.c[1], k.c[2]);
    r.c[2] = hash_float4_to_float(k.c[2], k.c[3], k.c[0], k.c[1]);
    r.c[3] = hash_float4_to_float(k.c[1], k.c[2], k.c[3], k.c[0]);
  }
  return r;
}
/* hash_float{2,3,4}_to_float3 (util_hash.h:180-215) */
template<int D> CY_FN cfloat3 vv_hash_color(vv<D> k)
{
  if constexpr (D == 2) {
    return mk3(hash_float2_to_float(k.c[0], k.c[1]), hash_float3_to_float(k.c[0], k.c[1], 1.0f),
               hash_float3_to_float(k.c[0], k.c[1], 2.0f));
  }
  else if constexpr (D == 3) {
    return mk3(hash_float3_to_float(k.c[0], k.c[1], k.c[2]), hash_float4_to_float(k.c[0], k.c[1], k.c[2], 1.0f),
               hash_float4_to_float(k.c[0], k.c[1], k.c[2], 2.0f));
  }
  else {
    return mk3(hash_float4_to_float(k.c[0], k.c[1], k.c[2], k.c[3]),
               hash_float4_to_float(k.c[2], k.c[0], k.c[3], k.c[1]),
               hash_float4_to_float(k.c[3], k.c[2], k.c[1], k.c[0]));
  }
}
/* voronoi_distance_{2,3,4}d */
template<int D> CY_FN float vv_distance(vv<D> a, vv<D> b, uint metric, float exponent)
{
  if (metric == VORONOI_EUCLIDEAN) {
    return vv_len(vv_sub(a, b));
  }
  if (metric == VORONOI_MANHATTAN) {
    float r = fabsf(a.c[0] - b.c[0]);
    for (int i = 1; i < D; i++) {
      r = r + fabsf(a.c[i] - b.c[i]);
    }
    return r;
  }
  if (metric == VORONOI_CHEBYCHEV) {
    float r = fabsf(a.c[D - 1] - b.c[D - 1]);
    for (int i = D - 2; i >= 0; i--) {
      r = cy_max(fabsf(a.c[i] - b.c[i]), r);
    }
    return r;
  }
  if (metric == VORONOI_MINKOWSKI) {
    float r = cy_powf(fabsf(a.c[0] - b.c[0]), exponent);
    for (int i = 1; i < D; i++) {
      r = r + cy_powf(fabsf(a.c[i] - b.c[i]), exponent);
    }
    return cy_powf(r, 1.0f / exponent);
  }
  return 0.0f;
}
/* the neighbour cell offsets in the reference's loop order (x innermost) */
template<int D> CY_FN vv<D> vv_offset(int n, int range)
{
  vv<D> r;
  const int side = 2 * range + 1;
  for (int i = 0; i < D; i++) {
    r.c[i] = (float)(n % side - range);
    n /= side;
  }
  return r;
}
template<int D> CY_FN int vv_cells(int range)
{
  int n = 1;
  for (int i = 0; i < D; i++) {
    n *= 2 * range + 1;
  }
  return n;
}

template<int D>
CY_NOINLINE void voronoi_nd(uint feature, vv<D> coord, float smoothness, float exponent, float randomness,
                            uint metric, float *out_distance, cfloat3 *out_color, vv<D> *out_position,
                            float *out_radius)
{
  const vv<D> cellPosition = vv_floor(coord);
  const vv<D> localPosition = vv_sub(coord, cellPosition);
  if (feature == VORONOI_F1) {
    float minDistance = 8.0f;
    vv<D> targetOffset = vv_mul(cellPosition, 0.0f), targetPosition = targetOffset;
    for (int n = 0; n < vv_cells<D>(1); n++) {
      const vv<D> cellOffset = vv_offset<D>(n, 1);
      const vv<D> pointPosition = vv_add(cellOffset, vv_mul(vv_hash(vv_add(cellPosition, cellOffset)), randomness));
      const float distanceToPoint = vv_distance(pointPosition, localPosition, metric, exponent);
      if (distanceToPoint < minDistance) {
        targetOffset = cellOffset;
        minDistance = distanceToPoint;
        targetPosition = pointPosition;
      }
    }
    *out_distance = minDistance;
    *out_color = vv_hash_color(vv_add(cellPosition, targetOffset));
    *out_position = vv_add(targetPosition, cellPosition);
  }
  else if (feature == VORONOI_SMOOTH_F1) {
    float smoothDistance = 8.0f;
    cfloat3 smoothColor = mk3(0.0f, 0.0f, 0.0f);
    vv<D> smoothPosition = vv_offset<D>(0, 0);
    for (int n = 0; n < vv_cells<D>(2); n++) {
      const vv<D> cellOffset = vv_offset<D>(n, 2);
      const vv<D> pointPosition = vv_add(cellOffset, vv_mul(vv_hash(vv_add(cellPosition, cellOffset)), randomness));
      const float distanceToPoint = vv_distance(pointPosition, localPosition, metric, exponent);
      const float h = cy_smoothstep(0.0f, 1.0f, 0.5f + 0.5f * (smoothDistance - distanceToPoint) / smoothness);
      float correctionFactor = smoothness * h * (1.0f - h);
      smoothDistance = (smoothDistance + h * (distanceToPoint - smoothDistance)) - correctionFactor;
      correctionFactor /= 1.0f + 3.0f * smoothness;
      const cfloat3 cellColor = vv_hash_color(vv_add(cellPosition, cellOffset));
      smoothColor = sub3(add3(smoothColor, mul3f(sub3(cellColor, smoothColor), h)),
                         mk3(correctionFactor, correctionFactor, correctionFactor));
      smoothPosition = vv_subf(vv_mix(smoothPosition, pointPosition, h), correctionFactor);
    }
    *out_distance = smoothDistance;
    *out_color = smoothColor;
    *out_position = vv_add(cellPosition, smoothPosition);
  }
  else if (feature == VORONOI_F2) {
    float distanceF1 = 8.0f, distanceF2 = 8.0f;
    vv<D> offsetF1 = vv_offset<D>(0, 0), positionF1 = offsetF1, offsetF2 = offsetF1, positionF2 = offsetF1;
    for (int n = 0; n < vv_cells<D>(1); n++) {
      const vv<D> cellOffset = vv_offset<D>(n, 1);
      const vv<D> pointPosition = vv_add(cellOffset, vv_mul(vv_hash(vv_add(cellPosition, cellOffset)), randomness));
      const float distanceToPoint = vv_distance(pointPosition, localPosition, metric, exponent);
      if (distanceToPoint < distanceF1) {
        distanceF2 = distanceF1;
        distanceF1 = distanceToPoint;
        offsetF2 = offsetF1;
        offsetF1 = cellOffset;
        positionF2 = positionF1;
        positionF1 = pointPosition;
      }
      else if (distanceToPoint < distanceF2) {
        distanceF2 = distanceToPoint;
        offsetF2 = cellOffset;
        positionF2 = pointPosition;
      }
    }
    *out_distance = distanceF2;
    *out_color = vv_hash_color(vv_add(cellPosition, offsetF2));
    *out_position = vv_add(positionF2, cellPosition);
  }
  else if (feature == VORONOI_DISTANCE_TO_EDGE) {
    vv<D> vectorToClosest = vv_offset<D>(0, 0);
    float minDistance = 8.0f;
    for (int n = 0; n < vv_cells<D>(1); n++) {
      const vv<D> cellOffset = vv_offset<D>(n, 1);
      const vv<D> vectorToPoint = vv_sub(
          vv_add(cellOffset, vv_mul(vv_hash(vv_add(cellPosition, cellOffset)), randomness)), localPosition);
      const float distanceToPoint = vv_dot(vectorToPoint, vectorToPoint);
      if (distanceToPoint < minDistance) {
        minDistance = distanceToPoint;
        vectorToClosest = vectorToPoint;
      }
    }
    minDistance = 8.0f;
    for (int n = 0; n < vv_cells<D>(1); n++) {
      const vv<D> cellOffset = vv_offset<D>(n, 1);
      const vv<D> vectorToPoint = vv_sub(
          vv_add(cellOffset, vv_mul(vv_hash(vv_add(cellPosition, cellOffset)), randomness)), localPosition);
      const vv<D> perpendicularToEdge = vv_sub(vectorToPoint, vectorToClosest);
      if (vv_dot(perpendicularToEdge, perpendicularToEdge) > 0.0001f) {
        const vv<D> half = vv_mul(vv_add(vectorToClosest, vectorToPoint), 1.0f / 2.0f);
        const vv<D> dir = vv_mul(perpendicularToEdge, 1.0f / vv_len(perpendicularToEdge));
        minDistance = cy_min(minDistance, vv_dot(half, dir));
      }
    }
    *out_distance = minDistance;
  }
  else if (feature == VORONOI_N_SPHERE_RADIUS) {
    vv<D> closestPoint = vv_offset<D>(0, 0), closestPointOffset = closestPoint;
    float minDistance = 8.0f;
    for (int n = 0; n < vv_cells<D>(1); n++) {
      const vv<D> cellOffset = vv_offset<D>(n, 1);
      const vv<D> pointPosition = vv_add(cellOffset, vv_mul(vv_hash(vv_add(cellPosition, cellOffset)), randomness));
      const float distanceToPoint = vv_len(vv_sub(pointPosition, localPosition));
      if (distanceToPoint < minDistance) {
        minDistance = distanceToPoint;
        closestPoint = pointPosition;
        closestPointOffset = cellOffset;
      }
    }
    minDistance = 8.0f;
    vv<D> closestPointToClosestPoint = vv_offset<D>(0, 0);
    for (int n = 0; n < vv_cells<D>(1); n++) {
      const vv<D> unit = vv_offset<D>(n, 1);
      bool centre = true;
      for (int i = 0; i < D; i++) {
        centre &= unit.c[i] == 0.0f;
      }
      if (centre) {
        continue;
      }
      const vv<D> cellOffset = vv_add(unit, closestPointOffset);
      const vv<D> pointPosition = vv_add(cellOffset, vv_mul(vv_hash(vv_add(cellPosition, cellOffset)), randomness));
      const float distanceToPoint = vv_len(vv_sub(closestPoint, pointPosition));
      if (distanceToPoint < minDistance) {
        minDistance = distanceToPoint;
        closestPointToClosestPoint = pointPosition;
      }
    }
    *out_radius = vv_len(vv_sub(closestPointToClosestPoint, closestPoint)) / 2.0f;
  }
}

CY_NOINLINE void svm_node_tex_voronoi(const CyGlobals *kg, CySvmStack stack, uint dimensions, uint feature,
                                      uint metric, int *offset, uint *err)
{
  const hc_uint4 stack_offsets = kg->__svm_nodes[*offset];
  const hc_uint4 defaults = kg->__svm_nodes[*offset + 1];
  *offset += 2;
  uint coord_off, w_off, scale_off, smoothness_off, exponent_off, randomness_off, distance_out, color_out;
  uint position_out, w_out_off, radius_out_off;
  svm_unpack4(stack_offsets.x, &coord_off, &w_off, &scale_off, &smoothness_off);
  svm_unpack4(stack_offsets.y, &exponent_off, &randomness_off, &distance_out, &color_out);
  svm_unpack3(stack_offsets.z, &position_out, &w_out_off, &radius_out_off);
  cfloat3 coord = svm_load3(stack, coord_off, err);
  float w = svm_load_default(stack, w_off, stack_offsets.w, err);
  const float scale = svm_load_default(stack, scale_off, defaults.x, err);
  float smoothness = svm_load_default(stack, smoothness_off, defaults.y, err);
  const float exponent = svm_load_default(stack, exponent_off, defaults.z, err);
  float randomness = svm_load_default(stack, randomness_off, defaults.w, err);
  float distance_v = 0.0f, w_v = 0.0f, radius_v = 0.0f;
  cfloat3 color_v = mk3(0.0f, 0.0f, 0.0f), position_v = mk3(0.0f, 0.0f, 0.0f);
  randomness = cy_clampf(randomness, 0.0f, 1.0f);
  smoothness = cy_clampf(smoothness / 2.0f, 0.0f, 0.5f);
  w *= scale;
  coord = mul3f(coord, scale);
  switch (dimensions) {
    case 1:
      voronoi_1d(feature, w, smoothness, randomness, &distance_v, &color_v, &w_v, &radius_v);
      w_v = (scale != 0.0f) ? w_v / scale : 0.0f; /* safe_divide */
      break;
    case 2: {
      vv<2> c, pos = vv_offset<2>(0, 0);
      c.c[0] = coord.x;
      c.c[1] = coord.y;
      voronoi_nd<2>(feature, c, smoothness, exponent, randomness, metric, &distance_v, &color_v, &pos, &radius_v);
      pos = (scale != 0.0f) ? vv_mul(pos, 1.0f / scale) : vv_offset<2>(0, 0);
      position_v = mk3(pos.c[0], pos.c[1], 0.0f);
      break;
    }
    case 3: {
      vv<3> c, pos = vv_offset<3>(0, 0);
      c.c[0] = coord.x;
      c.c[1] = coord.y;
      c.c[2] = coord.z;
      voronoi_nd<3>(feature, c, smoothness, exponent, randomness, metric, &distance_v, &color_v, &pos, &radius_v);
      position_v = (scale != 0.0f) ? mk3(pos.c[0], pos.c[1], pos.c[2]) : mk3(0.0f, 0.0f, 0.0f);
      if (scale != 0.0f) {
        position_v = div3f(position_v, scale);
      }
      break;
    }
    case 4: {
      vv<4> c, pos = vv_offset<4>(0, 0);
      c.c[0] = coord.x;
      c.c[1] = coord.y;
      c.c[2] = coord.z;
      c.c[3] = w;
      voronoi_nd<4>(feature, c, smoothness, exponent, randomness, metric, &distance_v, &color_v, &pos, &radius_v);
      pos = (scale != 0.0f) ? vv_mul(pos, 1.0f / scale) : vv_offset<4>(0, 0);
      position_v = mk3(pos.c[0], pos.c[1], pos.c[2]);
      w_v = pos.c[3];
      break;
    }
    default:
      cy_set_error(err, CY_ERR_SVM_NODE, NODE_TEX_VORONOI);
      return;
  }
  if (distance_out != SVM_STACK_INVALID) {
    svm_store(stack, distance_out, distance_v, err);
  }
  if (color_out != SVM_STACK_INVALID) {
    svm_store3(stack, color_out, color_v, err);
  }
  if (position_out != SVM_STACK_INVALID) {
    svm_store3(stack, position_out, position_v, err);
  }
  if (w_out_off != SVM_STACK_INVALID) {
    svm_store(stack, w_out_off, w_v, err);
  }
  if (radius_out_off != SVM_STACK_INVALID) {
    svm_store(stack, radius_out_off, radius_v, err);
  }
}

#endif /* CY_SVM_NOISE_H */
