/*
 * cy_math.h — scalar float math of the path-tracing hot path, restated for gfx950.
 *
 * Every operation keeps the exact operand order and rounding steps of the
 * reference's *scalar* (non-SSE) code path, which is what the reference CPU
 * kernel compiles on x86-64 without __KERNEL_SSE__ and what CUDA compiles:
 *   util/util_math.h            min/max/clamp/saturate/safe_sqrtf/make_orthonormals (112-130, 283-318, 477-499, 586)
 *   util/util_math_float3.h     float3 operators, dot, cross, normalize, len (90-480)
 *   util/util_math_float4.h:243 dot(float4) = (x*x + y*y) + (z*z + w*w)
 *   util/util_math_fast.h       madd, fast_rint, fast_sinf/cosf/sincosf, fast_acosf (50-293)
 *   util/util_transform.h:56-110, util/util_projection.h:48-55 transforms
 *   util/util_hash.h:28-93      rot / final / hash_uint2
 *   kernel/kernel_jitter.h:106-129 cmj_hash / cmj_hash_simple
 * The HIP build uses -ffp-contract=off and correctly rounded f32 div/sqrt so that
 * every value is bit-identical to the reference CPU kernel.  Transcendentals that
 * the reference takes from libm (sinf/cosf in to_unit_disk, kernel_montecarlo.h:39-46)
 * are evaluated in double and rounded once (cy_sinf/cy_cosf): glibc's sinf/cosf are
 * correctly rounded on all but rare inputs, so this matches them except at those.
 */
#ifndef CY_MATH_H
#define CY_MATH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#  include <hip/hip_runtime.h>
#  define CY_FN __device__ __forceinline__
#  define CY_NOINLINE __device__ __noinline__ /* a real call: large, rarely used code */
#  define CY_MFN __device__ __forceinline__
#  define CY_CONST __constant__
#else
#  include <math.h>
#  include <string.h>
#  define CY_FN static inline
#  define CY_NOINLINE static
#  define CY_MFN inline
#  define CY_CONST static const
#endif

#define CY_PI_F 3.14159265358979323846f
#define CY_PI_2_F 1.57079632679489661923f
#define CY_2PI_F 6.2831853071795864f
#define CY_1_PI_F 0.318309886183790671538f
#define CY_FLT_MAX 3.402823466e+38f
#define CY_INF __builtin_inff()

typedef unsigned int uint;

struct float3c {
  float x, y, z;
};
typedef struct float3c cfloat3;

CY_FN cfloat3 mk3(float x, float y, float z)
{
  cfloat3 r;
  r.x = x;
  r.y = y;
  r.z = z;
  return r;
}

CY_FN float as_float(uint i)
{
#if defined(__HIP_DEVICE_COMPILE__)
  return __uint_as_float(i);
#else
  float f;
  memcpy(&f, &i, 4);
  return f;
#endif
}
CY_FN uint as_uint(float f)
{
#if defined(__HIP_DEVICE_COMPILE__)
  return __float_as_uint(f);
#else
  uint i;
  memcpy(&i, &f, 4);
  return i;
#endif
}
CY_FN int as_int(float f)
{
  return (int)as_uint(f);
}
CY_FN float int_as_float(int i)
{
  return as_float((uint)i);
}

/* float_to_int (util_math.h: (int)f) as the reference's x86 CPU kernel
 * computes it: truncation toward zero, and for NaN or a value outside the int
 * range cvttss2si's "integer indefinite" 0x80000000, where C leaves the
 * conversion undefined and the GPU's v_cvt_i32_f32 saturates instead.  Texture
 * nodes meet such values at the huge offsets of a Bump node's differentials
 * (a checker at 1e11: x86 gives INT_MIN, the saturating conversion INT_MAX, and
 * the parity of the cell flips). */
CY_FN int cy_ftoi(float f)
{
#if defined(__HIP_DEVICE_COMPILE__)
  return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000u;
#else
  return (int)f; /* cvttss2si */
#endif
}

/* kernel_write_pass_float (kernel_write_passes.h:21-30): an atomic add on GPU
 * devices; the host emulation renders one path at a time */
CY_FN void cy_pass_add(float *p, float v)
{
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}

/* util_math.h:112-130 (ternary forms: NaN handling matches the reference). */
CY_FN float cmin(float a, float b)
{
  return (a < b) ? a : b;
}
CY_FN float cmax(float a, float b)
{
  return (a > b) ? a : b;
}
CY_FN int imin(int a, int b)
{
  return (a < b) ? a : b;
}
CY_FN int imax(int a, int b)
{
  return (a > b) ? a : b;
}
CY_FN float cclamp(float a, float mn, float mx)
{
  return cmin(cmax(a, mn), mx);
}
CY_FN int iclamp(int a, int mn, int mx)
{
  return imin(imax(a, mn), mx);
}
CY_FN float saturate(float a)
{
  return cclamp(a, 0.0f, 1.0f);
}
CY_FN float min4(float a, float b, float c, float d)
{
  return cmin(cmin(a, b), cmin(c, d));
}
CY_FN float max4(float a, float b, float c, float d)
{
  return cmax(cmax(a, b), cmax(c, d));
}
CY_FN float sqr(float a)
{
  return a * a;
}
CY_FN float safe_sqrtf(float f)
{
  return sqrtf(cmax(f, 0.0f));
}
/* util_math.h:591 */
CY_FN float inversesqrtf(float f)
{
  return (f > 0.0f) ? 1.0f / sqrtf(f) : 0.0f;
}
CY_FN float xor_signmask(float x, int y)
{
  return int_as_float(as_int(x) ^ y);
}
/* glibc 2.35 acosf (sysdeps/ieee754/flt-32/e_acosf.c, the fdlibm algorithm in
 * float arithmetic), which the reference reaches through safe_acosf
 * (util_math.h:601).  Bit-identical to the host libm for every float in
 * [-1, 1] (checked exhaustively, tests/test_kernel_math.py samples it). */
CY_FN float cy_acosf(float x)
{
  const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
  const float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f,
              pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f;
  const float qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f,
              qS4 = 7.7038154006e-02f;
  const int hx = as_int(x);
  const int ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) {
    return (hx > 0) ? 0.0f : pi + 2.0f * pio2_lo;
  }
  if (ix > 0x3f800000) {
    return (x - x) / (x - x);
  }
  if (ix < 0x3f000000) {
    if (ix <= 0x32800000) {
      return pio2_hi + pio2_lo;
    }
    const float z = x * x;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  }
  if (hx < 0) {
    const float z = (one + x) * 0.5f;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float s = sqrtf(z);
    const float r = p / q;
    const float w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  }
  const float z = (one - x) * 0.5f;
  const float s = sqrtf(z);
  const float df = int_as_float(as_int(s) & (int)0xfffff000);
  const float c = (z - df * df) / (s + df);
  const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  const float r = p / q;
  const float w = r * s + c;
  return 2.0f * (df + w);
}

CY_FN float safe_acosf(float a)
{
  return cy_acosf(cclamp(a, -1.0f, 1.0f));
}

/* glibc 2.35 asinf (sysdeps/ieee754/flt-32/e_asinf.c: odd polynomial below
 * 0.5, half-angle reduction above, split sqrt in the middle band), which the
 * reference reaches through fisheye_equisolid_to_direction
 * (kernel_projection.h:118).  Checked against the host libm over [-1, 1]
 * (tests/test_kernel_math.py). */
CY_FN float cy_asinf(float x)
{
  const float one = 1.0f, pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
              pio4_hi = 0.785398185253143310546875f;
  const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
              p4 = 4.216630880e-2f;
  const int hx = as_int(x);
  const int ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) {
    return x * pio2_hi + x * pio2_lo;
  }
  if (ix > 0x3f800000) {
    return (x - x) / (x - x);
  }
  if (ix < 0x3f000000) {
    if (ix < 0x32000000) {
      return x;
    }
    const float t = x * x;
    const float w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    return x + x * w;
  }
  float w = one - fabsf(x);
  float t = w * 0.5f;
  float p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  const float s = sqrtf(t);
  if (ix >= 0x3F79999A) {
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  }
  else {
    w = int_as_float(as_int(s) & (int)0xfffff000);
    const float c = (t - w * w) / (s + w);
    const float r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    const float q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return (hx > 0) ? t : -t;
}

CY_FN float power_heuristic(float a, float b)
{
  return (a * a) / (a * a + b * b);
}

/* float3 operators (util_math_float3.h, scalar branch). */
CY_FN cfloat3 neg3(cfloat3 a)
{
  return mk3(-a.x, -a.y, -a.z);
}
CY_FN cfloat3 add3(cfloat3 a, cfloat3 b)
{
  return mk3(a.x + b.x, a.y + b.y, a.z + b.z);
}
CY_FN cfloat3 sub3(cfloat3 a, cfloat3 b)
{
  return mk3(a.x - b.x, a.y - b.y, a.z - b.z);
}
CY_FN cfloat3 mul3(cfloat3 a, cfloat3 b)
{
  return mk3(a.x * b.x, a.y * b.y, a.z * b.z);
}
/* float3 * float and float * float3 both compute a.x * f (operand order kept). */
CY_FN cfloat3 mul3f(cfloat3 a, float f)
{
  return mk3(a.x * f, a.y * f, a.z * f);
}
CY_FN cfloat3 div3(cfloat3 a, cfloat3 b)
{
  return mk3(a.x / b.x, a.y / b.y, a.z / b.z);
}
/* operator/(float3, float): multiplies by the reciprocal. */
CY_FN cfloat3 div3f(cfloat3 a, float f)
{
  float invf = 1.0f / f;
  return mul3f(a, invf);
}
CY_FN float dot3(cfloat3 a, cfloat3 b)
{
  return a.x * b.x + a.y * b.y + a.z * b.z;
}
CY_FN cfloat3 cross3(cfloat3 a, cfloat3 b)
{
  return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
CY_FN float len3(cfloat3 a)
{
  return sqrtf(dot3(a, a));
}
CY_FN float len_squared3(cfloat3 a)
{
  return dot3(a, a);
}
CY_FN cfloat3 normalize3(cfloat3 a)
{
  return div3f(a, len3(a));
}
CY_FN cfloat3 normalize_len3(cfloat3 a, float *t)
{
  *t = len3(a);
  float x = 1.0f / *t;
  return mul3f(a, x);
}
CY_FN cfloat3 safe_normalize3(cfloat3 a)
{
  float t = len3(a);
  return (t != 0.0f) ? mul3f(a, 1.0f / t) : a;
}
CY_FN cfloat3 safe_normalize_len3(cfloat3 a, float *t)
{
  *t = len3(a);
  return (*t != 0.0f) ? div3f(a, *t) : a;
}
/* util_math.h:514 safe_divide_color */
CY_FN cfloat3 safe_divide_color(cfloat3 a, cfloat3 b)
{
  return mk3((b.x != 0.0f) ? a.x / b.x : 0.0f, (b.y != 0.0f) ? a.y / b.y : 0.0f, (b.z != 0.0f) ? a.z / b.z : 0.0f);
}
CY_FN cfloat3 fabs3(cfloat3 a)
{
  return mk3(fabsf(a.x), fabsf(a.y), fabsf(a.z));
}
CY_FN cfloat3 rcp3(cfloat3 a)
{
  return mk3(1.0f / a.x, 1.0f / a.y, 1.0f / a.z);
}
CY_FN float reduce_add3(cfloat3 a)
{
  return (a.x + a.y + a.z);
}
CY_FN float average3(cfloat3 a)
{
  return reduce_add3(a) * (1.0f / 3.0f);
}
CY_FN float max3f(cfloat3 a)
{
  return cmax(cmax(a.x, a.y), a.z);
}
CY_FN bool is_zero3(cfloat3 a)
{
  return (a.x == 0.0f && a.y == 0.0f && a.z == 0.0f);
}
CY_FN bool isequal3(cfloat3 a, cfloat3 b)
{
  return (a.x == b.x && a.y == b.y && a.z == b.z);
}
CY_FN bool isfinite_safe(float f)
{
  /* util_math.h:isfinite_safe — exponent bits test, immune to fast-math. */
  uint x = as_uint(f);
  return (f == f) && (x == 0 || x == (1u << 31) || (f != 2.0f * f)) && !((x << 1) > 0xff000000u);
}

/* util_math.h:477-499 */
CY_FN void make_orthonormals(cfloat3 N, cfloat3 *a, cfloat3 *b)
{
  if (N.x != N.y || N.x != N.z) {
    *a = mk3(N.z - N.y, N.x - N.z, N.y - N.x);
  }
  else {
    *a = mk3(N.z - N.y, N.x + N.z, -N.y - N.x);
  }
  *a = normalize3(*a);
  *b = cross3(N, *a);
}

/* util_math_fast.h */
CY_FN float madd(float a, float b, float c)
{
  return a * b + c;
}
CY_FN int fast_rint(float x)
{
  return (int)(x + copysignf(0.5f, x));
}
CY_FN float fast_sinf(float x)
{
  int q = fast_rint(x * CY_1_PI_F);
  float qf = (float)q;
  x = madd(qf, -0.78515625f * 4, x);
  x = madd(qf, -0.00024187564849853515625f * 4, x);
  x = madd(qf, -3.7747668102383613586e-08f * 4, x);
  x = madd(qf, -1.2816720341285448015e-12f * 4, x);
  x = CY_PI_2_F - (CY_PI_2_F - x);
  float s = x * x;
  if ((q & 1) != 0) {
    x = -x;
  }
  float u = 2.6083159809786593541503e-06f;
  u = madd(u, s, -0.0001981069071916863322258f);
  u = madd(u, s, +0.00833307858556509017944336f);
  u = madd(u, s, -0.166666597127914428710938f);
  u = madd(s, u * x, x);
  if (fabsf(u) > 1.0f) {
    u = 0.0f;
  }
  return u;
}
CY_FN void fast_sincosf(float x, float *sine, float *cosine)
{
  int q = fast_rint(x * CY_1_PI_F);
  float qf = (float)q;
  x = madd(qf, -0.78515625f * 4, x);
  x = madd(qf, -0.00024187564849853515625f * 4, x);
  x = madd(qf, -3.7747668102383613586e-08f * 4, x);
  x = madd(qf, -1.2816720341285448015e-12f * 4, x);
  x = CY_PI_2_F - (CY_PI_2_F - x);
  float s = x * x;
  if ((q & 1) != 0) {
    x = -x;
  }
  float su = 2.6083159809786593541503e-06f;
  su = madd(su, s, -0.0001981069071916863322258f);
  su = madd(su, s, +0.00833307858556509017944336f);
  su = madd(su, s, -0.166666597127914428710938f);
  su = madd(s, su * x, x);
  float cu = -2.71811842367242206819355e-07f;
  cu = madd(cu, s, +2.47990446951007470488548e-05f);
  cu = madd(cu, s, -0.00138888787478208541870117f);
  cu = madd(cu, s, +0.0416666641831398010253906f);
  cu = madd(cu, s, -0.5f);
  cu = madd(cu, s, +1.0f);
  if ((q & 1) != 0) {
    cu = -cu;
  }
  if (fabsf(su) > 1.0f) {
    su = 0.0f;
  }
  if (fabsf(cu) > 1.0f) {
    cu = 0.0f;
  }
  *sine = su;
  *cosine = cu;
}
CY_FN float fast_acosf(float x)
{
  const float f = fabsf(x);
  const float m = (f < 1.0f) ? 1.0f - (1.0f - f) : 1.0f;
  const float a = sqrtf(1.0f - m) *
                  (1.5707963267f + m * (-0.213300989f + m * (0.077980478f + m * -0.02164095f)));
  return x < 0 ? CY_PI_F - a : a;
}

/* libm sinf/cosf as the reference CPU kernel calls them (glibc): correctly rounded
 * double evaluation. */
#if defined(CY_HOST_LIBM_SINCOS)
/* host emulation build: call the same libm entry points as the reference */
CY_FN float cy_sinf(float x)
{
  return sinf(x);
}
CY_FN float cy_cosf(float x)
{
  return cosf(x);
}
#else
/* The reference CPU kernel takes sinf/cosf from glibc 2.35, whose single-precision
 * sin/cos are NOT correctly rounded (a double-evaluated sin differs from them on
 * ~1.3 % of inputs).  For bit parity the device evaluates glibc's own algorithm
 * (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h: double-precision
 * polynomial after a single-multiply range reduction, valid for |x| < 120):
 * restated from its published form and checked exhaustively against the
 * container's libm over all 2.17e9 floats in [-2pi, 2pi] (tests/test_sincos.py). */
struct cy_sincos_t {
  double sign[4];
  double hpi_inv, hpi;
  double c0, c1, c2, c3, c4, s1, s2, s3;
};
CY_CONST struct cy_sincos_t cy_sincosf_table[2] = {
    {{1.0, -1.0, -1.0, 1.0},
     0x1.45F306DC9C883p+23,
     0x1.921FB54442D18p0,
     0x1p0,
     -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5,
     -0x1.6c087e89a359dp-10,
     0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7,
     -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0},
     0x1.45F306DC9C883p+23,
     0x1.921FB54442D18p0,
     -0x1p0,
     0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5,
     0x1.6c087e89a359dp-10,
     -0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7,
     -0x1.994eb3774cf24p-13}};

CY_FN uint cy_abstop12(float x)
{
  return (as_uint(x) >> 20) & 0x7ff;
}
CY_FN float cy_sincos_poly(double x, double x2, const struct cy_sincos_t *p, int n)
{
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = fma(x2, p->s3, p->s2);
    double x7 = x3 * x2;
    double s = fma(x3, p->s1, x);
    return (float)fma(x7, s1, s);
  }
  double x4 = x2 * x2;
  double c2 = fma(x2, p->c4, p->c3);
  double c1 = fma(x2, p->c1, p->c0);
  double x6 = x4 * x2;
  double c = fma(x4, p->c2, c1);
  return (float)fma(x6, c2, c);
}
CY_FN double cy_sincos_reduce(double x, const struct cy_sincos_t *p, int *np)
{
  double r = x * p->hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fma(-(double)n, p->hpi, x);
}
/* glibc's large-argument reduction (sincosf.h reduce_large): x * 4/pi from the
 * bits of 4/pi (__inv_pio4) in 64-bit integer arithmetic.  With it cy_sinf /
 * cy_cosf match the container's libm on every float (checked exhaustively). */
CY_CONST uint32_t cy_inv_pio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
CY_FN double cy_sincos_reduce_large(uint xi, int *np)
{
  const uint32_t *arr = &cy_inv_pio4[(xi >> 26) & 15];
  const int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
  const uint64_t res1 = (uint64_t)xi * arr[4];
  const uint64_t res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  const uint64_t n = (res0 + (1ull << 61)) >> 62;
  res0 -= n << 62;
  const double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * 0x1.921FB54442D18p-62;
}
CY_FN float cy_sinf(float y)
{
  double x = y;
  int n;
  const struct cy_sincos_t *p = &cy_sincosf_table[0];
  if (cy_abstop12(y) < cy_abstop12(0x1.921FB6p-1f)) {
    double s = x * x;
    if (cy_abstop12(y) < cy_abstop12(0x1p-12f)) {
      return y;
    }
    return cy_sincos_poly(x, s, p, 0);
  }
  else if (cy_abstop12(y) < cy_abstop12(120.0f)) {
    x = cy_sincos_reduce(x, p, &n);
    double s = p->sign[n & 3];
    if (n & 2) {
      p = &cy_sincosf_table[1];
    }
    return cy_sincos_poly(x * s, x * x, p, n);
  }
  else if (cy_abstop12(y) < cy_abstop12(CY_INF)) {
    const uint sign = as_uint(y) >> 31;
    x = cy_sincos_reduce_large(as_uint(y), &n);
    const double s = p->sign[(n + sign) & 3];
    if ((n + sign) & 2) {
      p = &cy_sincosf_table[1];
    }
    return cy_sincos_poly(x * s, x * x, p, n);
  }
  return (y - y) / (y - y);
}
CY_FN float cy_cosf(float y)
{
  double x = y;
  int n;
  const struct cy_sincos_t *p = &cy_sincosf_table[0];
  if (cy_abstop12(y) < cy_abstop12(0x1.921FB6p-1f)) {
    double x2 = x * x;
    if (cy_abstop12(y) < cy_abstop12(0x1p-12f)) {
      return 1.0f;
    }
    return cy_sincos_poly(x, x2, p, 1);
  }
  else if (cy_abstop12(y) < cy_abstop12(120.0f)) {
    x = cy_sincos_reduce(x, p, &n);
    double s = p->sign[n & 3];
    if (n & 2) {
      p = &cy_sincosf_table[1];
    }
    return cy_sincos_poly(x * s, x * x, p, n ^ 1);
  }
  else if (cy_abstop12(y) < cy_abstop12(CY_INF)) {
    const uint sign = as_uint(y) >> 31;
    x = cy_sincos_reduce_large(as_uint(y), &n);
    const double s = p->sign[(n + sign) & 3];
    if ((n + sign) & 2) {
      p = &cy_sincosf_table[1];
    }
    return cy_sincos_poly(x * s, x * x, p, n ^ 1);
  }
  return (y - y) / (y - y);
}
#endif

/* Transform = 3 rows of float4, ProjectionTransform = 4 rows. */
struct cy_f4 {
  float x, y, z, w;
};
struct cy_tfm {
  struct cy_f4 x, y, z;
};
struct cy_ptfm {
  struct cy_f4 x, y, z, w;
};

CY_FN cfloat3 transform_point(const struct cy_tfm *t, cfloat3 a)
{
  return mk3(a.x * t->x.x + a.y * t->x.y + a.z * t->x.z + t->x.w,
             a.x * t->y.x + a.y * t->y.y + a.z * t->y.z + t->y.w,
             a.x * t->z.x + a.y * t->z.y + a.z * t->z.z + t->z.w);
}
CY_FN cfloat3 transform_direction(const struct cy_tfm *t, cfloat3 a)
{
  return mk3(a.x * t->x.x + a.y * t->x.y + a.z * t->x.z,
             a.x * t->y.x + a.y * t->y.y + a.z * t->y.z,
             a.x * t->z.x + a.y * t->z.y + a.z * t->z.z);
}
/* util_transform.h transform_direction_transposed: dot products with the columns */
CY_FN cfloat3 transform_direction_transposed(const struct cy_tfm *t, cfloat3 a)
{
  return mk3(dot3(mk3(t->x.x, t->y.x, t->z.x), a), dot3(mk3(t->x.y, t->y.y, t->z.y), a),
             dot3(mk3(t->x.z, t->y.z, t->z.z), a));
}
CY_FN float dot4(struct cy_f4 a, struct cy_f4 b)
{
  return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w);
}
CY_FN cfloat3 transform_perspective(const struct cy_ptfm *t, cfloat3 a)
{
  struct cy_f4 b;
  b.x = a.x;
  b.y = a.y;
  b.z = a.z;
  b.w = 1.0f;
  cfloat3 c = mk3(dot4(t->x, b), dot4(t->y, b), dot4(t->z, b));
  float w = dot4(t->w, b);
  return (w != 0.0f) ? div3f(c, w) : mk3(0.0f, 0.0f, 0.0f);
}

/* util_hash.h */
#define CY_ROT(x, k) (((x) << (k)) | ((x) >> (32 - (k))))
CY_FN uint hash_uint2(uint kx, uint ky)
{
  uint a, b, c;
  a = b = c = 0xdeadbeef + (2 << 2) + 13;
  b += ky;
  a += kx;
  c ^= b;
  c -= CY_ROT(b, 14);
  a ^= c;
  a -= CY_ROT(c, 11);
  b ^= a;
  b -= CY_ROT(a, 25);
  c ^= b;
  c -= CY_ROT(b, 16);
  a ^= c;
  a -= CY_ROT(c, 4);
  b ^= a;
  b -= CY_ROT(a, 14);
  c ^= b;
  c -= CY_ROT(b, 24);
  return c;
}

/* kernel_jitter.h:106-129 */
CY_FN uint cmj_hash(uint i, uint p)
{
  i ^= p;
  i ^= i >> 17;
  i ^= i >> 10;
  i *= 0xb36534e5;
  i ^= i >> 12;
  i ^= i >> 21;
  i *= 0x93fc4795;
  i ^= 0xdf6e307f;
  i ^= i >> 17;
  i *= 1 | p >> 18;
  return i;
}
CY_FN uint cmj_hash_simple(uint i, uint p)
{
  i = (i ^ 61) ^ p;
  i += i << 3;
  i ^= i >> 4;
  i *= 0x27d4eb2d;
  return i;
}

CY_FN uint find_first_set(uint x)
{
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint)__ffs(x);
#else
  return (uint)__builtin_ffs((int)x);
#endif
}

/* libm powf as the reference calls it in color_linear_to_srgb
 * (util/util_color.h:77-83, film convert).  glibc 2.35 powf
 * (sysdeps/ieee754/flt-32/e_powf.c, e_powf_log2_data.c, e_exp2f_data.c; the
 * FMA ifunc variant x86-64 selects on FMA hardware) is not correctly rounded:
 * a double-evaluated pow differs from it on 0.06 % of inputs.  The device
 * evaluates glibc's algorithm: log2(x) from a 16-entry (1/c, log2 c) table and a
 * degree-5 polynomial, y*log2(x) in double, 2^t from a 32-entry table and a
 * cubic.  Table values are glibc's published data; the restatement matches the
 * container's libm on every float x in [0.0031308, 65504] for y = 1/2.4
 * (tests/test_kernel_math.py).  Positive normal finite x only (x = +inf gives
 * +inf, NaN gives NaN): the film never passes anything else here. */
#if defined(CY_HOST_LIBM_SINCOS)
CY_FN float cy_powf(float x, float y)
{
  return powf(x, y);
}
CY_FN float cy_expf(float x)
{
  return expf(x);
}
CY_FN float cy_logf(float x)
{
  return logf(x);
}
#else
struct cy_powf_t {
  double invc[16], logc[16];
  double A[5];
  uint64_t E[32];
  double C[3];
};
CY_CONST struct cy_powf_t cy_powf_table = {
    {0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010b0p+0, 0x1.3c995b0b80385p+0,
     0x1.30d190c8864a5p+0, 0x1.25e227b0b8ea0p+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
     0x1.0953f419900a7p+0, 0x1.0000000000000p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aa0p-1,
     0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1},
    {-0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
     -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7af0p-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
     -0x1.a6f9db6475fcep-5, 0x0.0p+0, 0x1.338ca9f24f53dp-4, 0x1.476a9543891bap-3,
     0x1.e840b4ac4e4d2p-3, 0x1.40645f0c6651cp-2, 0x1.88e9c2c1b9ff8p-2, 0x1.ce0a44eb17bccp-2},
    {0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2, 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1,
     0x1.71547652ab82bp+0},
    {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
     0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
     0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
     0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
     0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
     0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
     0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
     0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull},
    {0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3, 0x1.62e42ff0c52d6p-1},
};

CY_FN double cy_as_double(uint64_t u)
{
  double d;
  memcpy(&d, &u, 8);
  return d;
}

CY_FN uint64_t cy_as_u64(double d)
{
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}

/* glibc powf's classification of y (e_powf.c checkint): 0 not an integer,
 * 1 odd integer, 2 even integer */
CY_FN int cy_powf_checkint(uint iy)
{
  const int e = (int)(iy >> 23 & 0xff);
  if (e < 0x7f) {
    return 0;
  }
  if (e > 0x7f + 23) {
    return 2;
  }
  if (iy & ((1u << (0x7f + 23 - e)) - 1u)) {
    return 0;
  }
  if (iy & (1u << (0x7f + 23 - e))) {
    return 1;
  }
  return 2;
}
CY_FN bool cy_powf_zeroinfnan(uint ix)
{
  return 2u * ix - 1u >= 2u * 0x7f800000u - 1u;
}

/* glibc 2.35 powf (e_powf.c, FMA variant), every special case included:
 * zero / inf / nan operands, negative x with integer y, subnormal x,
 * overflow and underflow (the math node's POWER, svm_math_util.h). */
CY_FN float cy_powf(float x, float y)
{
  const struct cy_powf_t *T = &cy_powf_table;
  uint sign_bias = 0;
  uint ix = as_uint(x);
  const uint iy = as_uint(y);
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || cy_powf_zeroinfnan(iy)) {
    if (cy_powf_zeroinfnan(iy)) {
      /* issignalingf_inline: a signaling NaN operand propagates */
      if (2u * iy == 0u) {
        return (2u * (ix ^ 0x00400000u) > 2u * 0x7fc00000u) ? x + y : 1.0f;
      }
      if (ix == 0x3f800000u) {
        return (2u * (iy ^ 0x00400000u) > 2u * 0x7fc00000u) ? x + y : 1.0f;
      }
      if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) {
        return x + y;
      }
      if (2u * ix == 2u * 0x3f800000u) {
        return 1.0f;
      }
      if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) {
        return 0.0f;
      }
      return y * y;
    }
    if (cy_powf_zeroinfnan(ix)) {
      float x2 = x * x;
      if ((ix & 0x80000000u) && cy_powf_checkint(iy) == 1) {
        x2 = -x2;
      }
      return (iy & 0x80000000u) ? 1.0f / x2 : x2;
    }
    if (ix & 0x80000000u) {
      const int yint = cy_powf_checkint(iy);
      if (yint == 0) {
        return (x - x) / (x - x);
      }
      if (yint == 1) {
        sign_bias = 1u << 16;
      }
      ix &= 0x7fffffffu;
    }
    if (ix < 0x00800000u) {
      ix = as_uint(as_float(ix) * 0x1p23f);
      ix &= 0x7fffffffu;
      ix -= 23u << 23;
    }
  }
  /* log2_inline */
  const uint tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16u);
  const uint top = tmp & 0xff800000u;
  const uint iz = ix - top;
  const int k = (int)top >> 23;
  const double z = (double)as_float(iz);
  const double r = fma(z, T->invc[i], -1.0);
  const double y0 = T->logc[i] + (double)k;
  const double r2 = r * r;
  double p5 = fma(T->A[0], r, T->A[1]);
  const double p3 = fma(T->A[2], r, T->A[3]);
  const double r4 = r2 * r2;
  double q = fma(T->A[4], r, y0);
  q = fma(p3, r2, q);
  p5 = fma(p5, r4, q);
  const double xd = (double)y * p5;
  if (((cy_as_u64(xd) >> 47) & 0xffff) >= (cy_as_u64(126.0) >> 47)) {
    if (xd > 0x1.fffffffd1d571p+6) {
      return sign_bias ? -CY_INF : CY_INF;
    }
    if (xd <= -150.0) {
      return sign_bias ? as_float(0x80000000u) : 0.0f; /* signed underflow */
    }
  }
  /* exp2_inline */
  const double shift = 0x1.8p+47;
  double kd = xd + shift;
  const uint64_t ki = cy_as_u64(kd);
  kd -= shift;
  const double rr = xd - kd;
  const uint64_t t = T->E[ki % 32u] + ((ki + sign_bias) << 47);
  const double s = cy_as_double(t);
  const double zz = fma(T->C[0], rr, T->C[1]);
  const double rr2 = rr * rr;
  double e = fma(T->C[2], rr, 1.0);
  e = fma(zz, rr2, e);
  return (float)(e * s);
}

/* glibc 2.35 expf (e_expf.c, FMA variant): 2^(k/32) from the exp2f table and
 * a cubic in the remainder; matches the container's libm on every float. */
CY_FN float cy_expf(float x)
{
  const struct cy_powf_t *T = &cy_powf_table;
  const uint abstop = (as_uint(x) >> 20) & 0x7ff;
  if (abstop >= ((as_uint(88.0f) >> 20) & 0x7ff)) {
    if (as_uint(x) == as_uint(-CY_INF)) {
      return 0.0f;
    }
    if (abstop >= ((as_uint(CY_INF) >> 20) & 0x7ff)) {
      return x + x;
    }
    if (x > 0x1.62e42ep6f) {
      return CY_INF;
    }
    if (x < -0x1.9fe368p6f) {
      return 0.0f;
    }
  }
  const double N = 32.0;
  const double InvLn2N = 0x1.71547652b82fep+0 * N;
  const double xd = (double)x;
  const double z = InvLn2N * xd;
  const double shift = 0x1.8p+52;
  double kd = z + shift;
  const uint64_t ki = cy_as_u64(kd);
  kd -= shift;
  const double r = fma(InvLn2N, xd, -kd);
  const uint64_t t = T->E[ki % 32u] + (ki << 47);
  const double s = cy_as_double(t);
  const double zz = fma(T->C[0] / (N * N * N), r, T->C[1] / (N * N));
  const double r2 = r * r;
  double y = fma(T->C[2] / N, r, 1.0);
  y = fma(zz, r2, y);
  return (float)(y * s);
}

/* glibc 2.35 logf (e_logf.c): log(c) table over 16 subintervals of [0.7, 1.4]
 * (the same 1/c as powf's log2 table) and a cubic; matches the container's
 * libm on every float. */
CY_CONST double cy_logf_logc[16] = {
    -0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3,
    -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3,   -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611ccp-4,
    -0x1.252f438e10c1ep-5, 0x0p+0,                0x1.aa5aa5df25984p-5,  0x1.c5e53aa362eb4p-4,
    0x1.526e57720db08p-3,  0x1.bc2860d22477p-3,   0x1.1058bc8a07ee1p-2,  0x1.4043057b6ee09p-2};
CY_FN float cy_logf(float x)
{
  const struct cy_powf_t *T = &cy_powf_table;
  uint ix = as_uint(x);
  if (ix == 0x3f800000u) {
    return 0.0f;
  }
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2u == 0u) {
      return -CY_INF;
    }
    if (ix == 0x7f800000u) {
      return x;
    }
    if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u) {
      return (x - x) / (x - x);
    }
    ix = as_uint(x * 0x1p23f);
    ix -= 23u << 23;
  }
  const uint tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16u);
  const int k = (int)tmp >> 23;
  const uint iz = ix - (tmp & 0xff800000u);
  const double z = (double)as_float(iz);
  const double r = z * T->invc[i] - 1.0;
  const double y0 = cy_logf_logc[i] + (double)k * 0x1.62e42fefa39efp-1;
  const double r2 = r * r;
  double y = 0x1.5575b0be00b6ap-2 * r + -0x1.ffffef20a4123p-2;
  y = -0x1.00ea348b88334p-2 * r2 + y;
  y = y * r2 + (y0 + r);
  return (float)y;
}
#endif

/* libm lgammaf as the reference reaches it through beta() (util_math.h:
 * expf(lgammaf(x) + lgammaf(y) - lgammaf(x + y))) in the multiscatter GGX
 * glass closure (bsdf_microfacet_multi_impl.h mf_eval, MF_MULTI_GLASS).
 * glibc 2.35's lgammaf is fdlibm's float algorithm
 * (sysdeps/ieee754/flt-32/e_lgammaf_r.c): rational / polynomial fits around
 * the minimum (tc), on [0.9, 2), the recurrence lgamma(x) = log((x-1)(x-2)..)
 * + lgamma(frac) on [2, 8) and Stirling's series above; its published
 * coefficients are restated here in its evaluation order (float, no FMA), with
 * logf from cy_logf.  Positive x only (beta's arguments are >= 0.9999 there);
 * every float of [2^-40, 2^26] agrees with the container's libm
 * (tests/test_kernel_math.py). */
#if defined(CY_HOST_LIBM_SINCOS)
CY_FN float cy_lgammaf(float x)
{
  return lgammaf(x);
}
#else
CY_FN float cy_lgammaf_poly(float x, int i, float y, float r)
{
  if (i == 0) {
    const float z = y * y;
    const float p1 = 0.0772156641f +
                     z * (0.0673523024f +
                          z * (0.007385551f + z * (0.00119270768f + z * (0.000220862785f + z * 2.52144564e-05f))));
    const float p2 = z * (0.322467029f +
                          z * (0.0205808077f +
                               z * (0.00289051374f + z * (0.000510069774f + z * (0.000108011569f + z * 4.48640967e-05f)))));
    const float p = y * p1 + p2;
    return r + (p - 0.5f * y);
  }
  if (i == 1) {
    const float z = y * y;
    const float w = z * y;
    const float p1 = 0.483836114f + w * (-0.0327885412f + w * (0.00610053865f + w * (-0.0014034647f + w * 0.00031563206f)));
    const float p2 = -0.147587717f + w * (0.0179706756f + w * (-0.00368452026f + w * (0.000881081854f + w * -0.000312754157f)));
    const float p3 = 0.0646249428f + w * (-0.0103142243f + w * (0.00225964771f + w * (-0.000538595312f + w * 0.000335529185f)));
    const float p = z * p1 - (6.69710065e-09f - w * (p2 + y * p3));
    return r + (-0.121486284f + p);
  }
  const float p1 = y * (-0.0772156641f +
                        y * (0.632827044f + y * (1.45492256f + y * (0.977717519f + y * (0.228963733f + y * 0.0133810919f)))));
  const float p2 = 1.0f + y * (2.45597792f + y * (2.12848973f + y * (0.769285142f + y * (0.104222648f + y * 0.00321709248f))));
  return r + (-0.5f * y + p1 / p2);
}

CY_FN float cy_lgammaf(float x)
{
  const int hx = as_int(x);
  const int ix = hx & 0x7fffffff;
  if (ix >= 0x7f800000) {
    return x * x;
  }
  if (hx <= 0) {
    return (x - x) / (x - x); /* x <= 0: not reached by beta() */
  }
  const float tc = 1.46163213f; /* 0x3fbb16c3, the minimum of gamma */
  if (ix < 0x30800000) {
    return -cy_logf(x); /* |x| < 2^-30 */
  }
  if (ix == 0x3f800000 || ix == 0x40000000) {
    return 0.0f;
  }
  if (ix < 0x40000000) {
    /* x < 2 */
    if (ix <= 0x3f666666) {
      /* lgamma(x) = lgamma(x+1) - log(x) */
      const float r = -cy_logf(x);
      if (ix >= 0x3f3b4a20) {
        return cy_lgammaf_poly(x, 0, 1.0f - x, r);
      }
      if (ix >= 0x3e6d3308) {
        return cy_lgammaf_poly(x, 1, x - (tc - 1.0f), r);
      }
      return cy_lgammaf_poly(x, 2, x, r);
    }
    if (ix >= 0x3fdda618) {
      return cy_lgammaf_poly(x, 0, 2.0f - x, 0.0f);
    }
    if (ix >= 0x3f9da620) {
      return cy_lgammaf_poly(x, 1, x - tc, 0.0f);
    }
    return cy_lgammaf_poly(x, 2, x - 1.0f, 0.0f);
  }
  if (ix < 0x41000000) {
    /* 2 <= x < 8: lgamma(i + y) = lgamma(1 + y) + log((y+1)(y+2)..(y+i-1)) */
    const int i = (int)x;
    const float y = x - (float)i;
    const float p = y * (-0.0772156641f +
                         y * (0.21498242f +
                              y * (0.325778782f + y * (0.146350473f + y * (0.0266422704f + y * (0.00184028456f +
                                                                                                  y * 3.1947533e-05f))))));
    const float q = 1.0f + y * (1.39200532f +
                                y * (0.72193557f +
                                     y * (0.17193386f + y * (0.0186459199f + y * (0.000777942478f + y * 7.32668423e-06f)))));
    float r = 0.5f * y + p / q;
    float z = 1.0f;
    switch (i) {
      case 7:
        z *= (y + 6.0f);
        /* fall through */
      case 6:
        z *= (y + 5.0f);
        /* fall through */
      case 5:
        z *= (y + 4.0f);
        /* fall through */
      case 4:
        z *= (y + 3.0f);
        /* fall through */
      case 3:
        z *= (y + 2.0f);
        r += cy_logf(z);
        break;
    }
    return r;
  }
  if (ix < 0x4c800000) {
    /* 8 <= x < 2^26: Stirling */
    const float t = cy_logf(x);
    const float z = 1.0f / x;
    const float y = z * z;
    const float w = 0.418938547f +
                    z * (0.0833333358f +
                         y * (-0.00277777785f +
                              y * (0.000793650572f + y * (-0.000595187536f + y * (0.000836339896f + y * -0.0016309293f)))));
    return (x - 0.5f) * (t - 1.0f) + w;
  }
  return x * (cy_logf(x) - 1.0f);
}
#endif

/* util_math.h beta(): the reference's expf / lgammaf (glibc) */
CY_FN float cy_beta(float x, float y)
{
  return cy_expf(cy_lgammaf(x) + cy_lgammaf(y) - cy_lgammaf(x + y));
}

/* libm atan2f as the reference calls it in direction_to_equirectangular
 * (kernel_projection.h:56-65, background MIS pdf).  glibc 2.35 atan2f/atanf are
 * fdlibm's float algorithms (sysdeps/ieee754/flt-32/e_atan2f.c, s_atanf.c),
 * restated here with their published constants; agreement with the
 * container's libm on 20M random argument pairs (0 differ) was checked during
 * development and is sampled by tests/test_kernel_math.py. */
#if defined(CY_HOST_LIBM_SINCOS)
CY_FN float cy_atan2f(float y, float x)
{
  return atan2f(y, x);
}
CY_FN float cy_atanf(float x)
{
  return atanf(x);
}
#else
struct cy_atanf_t {
  float hi[4], lo[4], aT[11];
};
CY_CONST struct cy_atanf_t cy_atanf_table = {
    {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f},
    {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f},
    {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f, 9.0908870101e-02f,
     -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f, 4.9768779427e-02f, -3.6531571299e-02f,
     1.6285819933e-02f},
};

CY_FN float cy_atanf(float x)
{
  const struct cy_atanf_t *T = &cy_atanf_table;
  const int hx = (int)as_uint(x);
  const int ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) { /* |x| >= 2^25 */
    if (ix > 0x7f800000) {
      return x + x;
    }
    return (hx > 0) ? T->hi[3] + T->lo[3] : -T->hi[3] - T->lo[3];
  }
  if (ix < 0x3ee00000) { /* |x| < 0.4375 */
    if (ix < 0x31000000) {
      return x;
    }
    id = -1;
  }
  else {
    x = fabsf(x);
    if (ix < 0x3f980000) {
      if (ix < 0x3f300000) {
        id = 0;
        x = (2.0f * x - 1.0f) / (2.0f + x);
      }
      else {
        id = 1;
        x = (x - 1.0f) / (x + 1.0f);
      }
    }
    else {
      if (ix < 0x401c0000) {
        id = 2;
        x = (x - 1.5f) / (1.0f + 1.5f * x);
      }
      else {
        id = 3;
        x = -1.0f / x;
      }
    }
  }
  const float *aT = T->aT;
  const float z = x * x;
  const float w = z * z;
  const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) {
    return x - x * (s1 + s2);
  }
  const float r = T->hi[id] - ((x * (s1 + s2) - T->lo[id]) - x);
  return (hx < 0) ? -r : r;
}

CY_FN float cy_atan2f(float y, float x)
{
  const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f;
  const float pi_lo = -8.7422776573e-08f, tiny = 1.0e-30f;
  const int hx = (int)as_uint(x), ix = hx & 0x7fffffff;
  const int hy = (int)as_uint(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) {
    return x + y;
  }
  if (hx == 0x3f800000) {
    return cy_atanf(y);
  }
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    switch (m) {
      case 0:
      case 1:
        return y;
      case 2:
        return pi + tiny;
      default:
        return -pi - tiny;
    }
  }
  if (ix == 0) {
    return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  }
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0:
          return pi_o_4 + tiny;
        case 1:
          return -pi_o_4 - tiny;
        case 2:
          return 3.0f * pi_o_4 + tiny;
        default:
          return -3.0f * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0:
        return 0.0f;
      case 1:
        return -0.0f;
      case 2:
        return pi + tiny;
      default:
        return -pi - tiny;
    }
  }
  if (iy == 0x7f800000) {
    return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  }
  const int k = (iy - ix) >> 23;
  float z;
  if (k > 60) {
    z = pi_o_2 + 0.5f * pi_lo;
  }
  else if (hx < 0 && k < -60) {
    z = 0.0f;
  }
  else {
    z = cy_atanf(fabsf(y / x));
  }
  switch (m) {
    case 0:
      return z;
    case 1:
      return as_float(as_uint(z) ^ 0x80000000u);
    case 2:
      return pi - (z - pi_lo);
    default:
      return (z - pi_lo) - pi;
  }
}
#endif

/* libm tanf, expm1f and sinhf as the reference's hair closures call them
 * (closure/bsdf_hair.h sample: tanf; bsdf_hair_principled.h
 * longitudinal_scattering: sinhf).  glibc 2.35's are fdlibm's float
 * algorithms (sysdeps/ieee754/flt-32/k_tanf.c, s_expm1f.c, e_sinhf.c),
 * restated with their published constants in their evaluation order (float,
 * no FMA); tanf's range reduction is glibc's own (e_rem_pio2f.c, the sinf /
 * cosf reduction in double) and its tiny-argument cotangent is a plain
 * -1 / x.  Every float of both signs agrees with the container's libm for all
 * three (tests/test_kernel_math.py samples it). */
#if defined(CY_HOST_LIBM_SINCOS)
CY_FN float cy_tanf(float x)
{
  return tanf(x);
}
CY_FN float cy_expm1f(float x)
{
  return expm1f(x);
}
CY_FN float cy_sinhf(float x)
{
  return sinhf(x);
}
CY_FN float cy_coshf(float x)
{
  return coshf(x);
}
CY_FN float cy_tanhf(float x)
{
  return tanhf(x);
}
#else
CY_FN float cy_kernel_tanf(float x, float y, int iy)
{
  const float one = 1.0f, pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
  const float T0 = 3.3333334327e-01f, T1 = 1.3333334029e-01f, T2 = 5.3968254477e-02f, T3 = 2.1869488060e-02f,
              T4 = 8.8632395491e-03f, T5 = 3.5920790397e-03f, T6 = 1.4562094584e-03f, T7 = 5.8804126456e-04f,
              T8 = 2.4646313977e-04f, T9 = 7.8179444245e-05f, T10 = 7.1407252108e-05f, T11 = -1.8558637748e-05f,
              T12 = 2.5907305826e-05f;
  float z, r, v, w, s;
  const int hx = as_int(x);
  const int ix = hx & 0x7fffffff;
  if (ix < 0x39000000) { /* |x| < 2^-13 */
    if ((int)x == 0) {
      if ((ix | (iy + 1)) == 0) {
        return one / fabsf(x);
      }
      else if (iy == 1) {
        return x;
      }
      else {
        return -one / x;
      }
    }
  }
  if (ix >= 0x3f2ca140) { /* |x| >= 0.6744 */
    if (hx < 0) {
      x = -x;
      y = -y;
    }
    z = pio4 - x;
    w = pio4lo - y;
    x = z + w;
    y = 0.0f;
    if (fabsf(x) < 0x1p-13f) {
      return (float)(1 - ((hx >> 30) & 2)) * (float)iy * (1.0f - 2.0f * (float)iy * x);
    }
  }
  z = x * x;
  w = z * z;
  r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
  v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
  s = z * x;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  w = x + r;
  if (ix >= 0x3f2ca140) {
    v = (float)iy;
    return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
  }
  if (iy == 1) {
    return w;
  }
  /* -1.0 / (x + r) accurately */
  z = w;
  z = int_as_float(as_int(z) & 0xfffff000);
  v = r - (z - x);
  float t, a;
  t = a = -1.0f / w;
  t = int_as_float(as_int(t) & 0xfffff000);
  s = 1.0f + t * z;
  return t + a * (s + t * v);
}

/* __ieee754_rem_pio2f (glibc 2.35 e_rem_pio2f.c): the sinf / cosf range
 * reduction (sincosf.h reduce_fast below 120, reduce_large above) in double,
 * split into y[0] + y[1]; compiled without FMA (not a multiarch routine), so
 * the fast step is a separate multiply and subtract. */
CY_FN int cy_rem_pio2f(float x, float *y)
{
  const struct cy_sincos_t *p = &cy_sincosf_table[0];
  double dx = x;
  int n;
  if (cy_abstop12(x) < cy_abstop12(120.0f)) {
    const double r = dx * p->hpi_inv;
    n = ((int32_t)r + 0x800000) >> 24;
    const double nh = (double)n * p->hpi;
    dx = dx - nh;
  }
  else {
    const uint xi = as_uint(x);
    dx = cy_sincos_reduce_large(xi, &n);
    dx = (xi >> 31) ? -dx : dx;
  }
  y[0] = (float)dx;
  y[1] = (float)(dx - (double)y[0]);
  return n;
}

CY_FN float cy_tanf(float x)
{
  const int ix = as_int(x) & 0x7fffffff;
  if (ix <= 0x3f490fda) {
    return cy_kernel_tanf(x, 0.0f, 1);
  }
  if (ix >= 0x7f800000) {
    return x - x;
  }
  float y[2];
  const int n = cy_rem_pio2f(x, y);
  return cy_kernel_tanf(y[0], y[1], 1 - ((n & 1) << 1));
}

CY_FN float cy_expm1f(float x)
{
  const float one = 1.0f, huge = 1.0e+30f, tiny = 1.0e-30f, o_threshold = 8.8721679688e+01f,
              ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f, invln2 = 1.4426950216e+00f,
              Q1 = -3.3333335072e-02f, Q2 = 1.5873016091e-03f, Q3 = -7.9365076090e-05f, Q4 = 4.0082177293e-06f,
              Q5 = -2.0109921195e-07f;
  float y, hi, lo, c = 0.0f, t, e, hxs, hfx, r1;
  int k;
  uint hx = as_uint(x);
  const uint xsb = hx & 0x80000000u;
  hx &= 0x7fffffffu;
  if (hx == 0u) {
    return x; /* +-0 */
  }
  if (hx >= 0x4195b844u) { /* |x| >= 27 ln2 */
    if (hx >= 0x42b17218u) {
      if (hx > 0x7f800000u) {
        return x + x;
      }
      if (hx == 0x7f800000u) {
        return (xsb == 0) ? x : -1.0f;
      }
      if (x > o_threshold) {
        return huge * huge;
      }
    }
    if (xsb != 0) {
      return tiny - one;
    }
  }
  if (hx > 0x3eb17218u) { /* |x| > 0.5 ln2 */
    if (hx < 0x3F851592u) {
      if (xsb == 0) {
        hi = x - ln2_hi;
        lo = ln2_lo;
        k = 1;
      }
      else {
        hi = x + ln2_hi;
        lo = -ln2_lo;
        k = -1;
      }
    }
    else {
      k = (int)(invln2 * x + ((xsb == 0) ? 0.5f : -0.5f));
      t = (float)k;
      hi = x - t * ln2_hi;
      lo = t * ln2_lo;
    }
    x = hi - lo;
    c = (hi - x) - lo;
  }
  else if (hx < 0x33000000u) { /* |x| < 2^-25 */
    t = huge + x;
    return x - (t - (huge + x));
  }
  else {
    k = 0;
  }
  hfx = 0.5f * x;
  hxs = x * hfx;
  r1 = one + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
  t = 3.0f - r1 * hfx;
  e = hxs * ((r1 - t) / (6.0f - x * t));
  if (k == 0) {
    return x - (x * e - hxs);
  }
  e = (x * (e - c) - c);
  e -= hxs;
  if (k == -1) {
    return 0.5f * (x - e) - 0.5f;
  }
  if (k == 1) {
    if (x < -0.25f) {
      return -2.0f * (e - (x + 0.5f));
    }
    return one + 2.0f * (x - e);
  }
  if (k <= -2 || k > 56) {
    y = one - (e - x);
    y = int_as_float(as_int(y) + (k << 23));
    return y - one;
  }
  if (k < 23) {
    t = int_as_float(0x3f800000 - (0x1000000 >> k)); /* 1 - 2^-k */
    y = t - (e - x);
    y = int_as_float(as_int(y) + (k << 23));
  }
  else {
    t = int_as_float((0x7f - k) << 23); /* 2^-k */
    y = x - (e + t);
    y += one;
    y = int_as_float(as_int(y) + (k << 23));
  }
  return y;
}

CY_FN float cy_sinhf(float x)
{
  const float one = 1.0f, shuge = 1.0e37f;
  const int jx = as_int(x);
  const int ix = jx & 0x7fffffff;
  if (ix >= 0x7f800000) {
    return x + x;
  }
  const float h = (jx < 0) ? -0.5f : 0.5f;
  if (ix < 0x41b00000) { /* |x| < 22 */
    if (ix < 0x31800000) { /* |x| < 2^-28 */
      if (shuge + x > one) {
        return x;
      }
    }
    const float t = cy_expm1f(fabsf(x));
    if (ix < 0x3f800000) {
      return h * (2.0f * t - t * t / (t + one));
    }
    return h * (t + t / (t + one));
  }
  if (ix < 0x42b17180) {
    return h * cy_expf(fabsf(x));
  }
  if (ix <= 0x42b2d4fc) {
    const float w = cy_expf(0.5f * fabsf(x));
    const float t = h * w;
    return t * w;
  }
  return x * shuge;
}

/* e_coshf.c */
CY_FN float cy_coshf(float x)
{
  const float one = 1.0f, half = 0.5f, huge = 1.0e30f;
  const int ix = as_int(x) & 0x7fffffff;
  if (ix < 0x41b00000) { /* |x| < 22 */
    if (ix < 0x3eb17218) { /* |x| < 0.5 ln2 */
      const float t = cy_expm1f(fabsf(x));
      const float w = one + t;
      if (ix < 0x24000000) {
        return w;
      }
      return one + (t * t) / (w + w);
    }
    const float t = cy_expf(fabsf(x));
    return half * t + half / t;
  }
  if (ix < 0x42b17180) {
    return half * cy_expf(fabsf(x));
  }
  if (ix <= 0x42b2d4fc) {
    const float w = cy_expf(half * fabsf(x));
    const float t = half * w;
    return t * w;
  }
  if (ix >= 0x7f800000) {
    return x * x;
  }
  return huge * huge;
}

/* s_tanhf.c */
CY_FN float cy_tanhf(float x)
{
  const float one = 1.0f, two = 2.0f, tiny = 1.0e-30f;
  const int jx = as_int(x);
  const int ix = jx & 0x7fffffff;
  float t, z;
  if (ix >= 0x7f800000) {
    return (jx >= 0) ? one / x + one : one / x - one;
  }
  if (ix < 0x41b00000) { /* |x| < 22 */
    if (ix == 0) {
      return x;
    }
    if (ix < 0x24000000) {
      return x * (one + x);
    }
    if (ix >= 0x3f800000) {
      t = cy_expm1f(two * fabsf(x));
      z = one - two / (t + two);
    }
    else {
      t = cy_expm1f(-two * fabsf(x));
      z = -t / (t + two);
    }
  }
  else {
    z = one - tiny;
  }
  return (jx >= 0) ? z : -z;
}
#endif

/* util/util_color.h:77-83 */
CY_FN float color_linear_to_srgb(float c)
{
  if (c < 0.0031308f) {
    return (c < 0.0f) ? 0.0f : c * 12.92f;
  }
  return 1.055f * cy_powf(c, 1.0f / 2.4f) - 0.055f;
}

#endif /* CY_MATH_H */
