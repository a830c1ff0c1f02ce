/* Host build of the device's sinf/cosf restatement (csrc/kernel/cy_math.h)
 * next to libm's, for tests/test_kernel_math.py. */
#include <cmath>

#include "../../raytracingproject_amd/csrc/kernel/cy_math.h"

extern "C" void sincos_eval(const float *x, long n, float *s_dev, float *c_dev, float *s_libm, float *c_libm)
{
  for (long i = 0; i < n; i++) {
    s_dev[i] = cy_sinf(x[i]);
    c_dev[i] = cy_cosf(x[i]);
    s_libm[i] = sinf(x[i]);
    c_libm[i] = cosf(x[i]);
  }
}

extern "C" void acos_eval(const float *x, long n, float *dev, float *libm)
{
  for (long i = 0; i < n; i++) {
    dev[i] = cy_acosf(x[i]);
    libm[i] = acosf(x[i]);
  }
}

extern "C" long asin_sweep(uint32_t lo, uint32_t hi, uint32_t step)
{
  long bad = 0;
  for (uint64_t u = lo; u <= hi; u += step) {
    const float x = as_float((uint32_t)u);
    volatile float vx = x;
    if (as_uint(cy_asinf(x)) != as_uint(asinf(vx))) {
      bad++;
    }
  }
  return bad;
}

/* cy_powf (glibc powf restatement) and libm powf over [lo, hi] bit patterns,
 * with y = 1/2.4 (color_linear_to_srgb); returns the number of mismatches. */
extern "C" long powf_sweep(uint32_t lo, uint32_t hi, uint32_t step)
{
  long bad = 0;
  const float y = 1.0f / 2.4f;
  for (uint64_t u = lo; u <= hi; u += step) {
    const float x = as_float((uint32_t)u);
    volatile float vx = x;
    if (as_uint(cy_powf(x, y)) != as_uint(powf(vx, y))) {
      bad++;
    }
  }
  return bad;
}

extern "C" void srgb_eval(const float *x, long n, float *dev)
{
  for (long i = 0; i < n; i++) {
    dev[i] = color_linear_to_srgb(x[i]);
  }
}

extern "C" void atan2_eval(const float *y, const float *x, long n, float *dev, float *libm)
{
  for (long i = 0; i < n; i++) {
    dev[i] = cy_atan2f(y[i], x[i]);
    volatile float vy = y[i], vx = x[i];
    libm[i] = atan2f(vy, vx);
  }
}

/* cy_lgammaf (glibc lgammaf restatement) and libm lgammaf over [lo, hi] bit
 * patterns; returns the number of mismatches (and the first one in *first). */
extern "C" long lgammaf_sweep(uint32_t lo, uint32_t hi, uint32_t step, uint32_t *first)
{
  long bad = 0;
  for (uint64_t u = lo; u <= hi; u += step) {
    const float x = as_float((uint32_t)u);
    volatile float vx = x;
    if (as_uint(cy_lgammaf(x)) != as_uint(lgammaf(vx))) {
      if (!bad && first) {
        *first = (uint32_t)u;
      }
      bad++;
    }
  }
  return bad;
}

/* cy_tanf / cy_expm1f / cy_sinhf (glibc restatements) against libm over [lo, hi]
 * bit patterns: which = 0 tanf, 1 expm1f, 2 sinhf, 3 coshf, 4 tanhf; returns the
 * mismatches. */
extern "C" long libm_sweep(int which, uint32_t lo, uint32_t hi, uint32_t step, uint32_t *first)
{
  long bad = 0;
  for (uint64_t u = lo; u <= hi; u += step) {
    const float x = as_float((uint32_t)u);
    volatile float vx = x;
    float a, b;
    if (which == 0) {
      a = cy_tanf(x);
      b = tanf(vx);
    }
    else if (which == 1) {
      a = cy_expm1f(x);
      b = expm1f(vx);
    }
    else if (which == 2) {
      a = cy_sinhf(x);
      b = sinhf(vx);
    }
    else if (which == 3) {
      a = cy_coshf(x);
      b = coshf(vx);
    }
    else {
      a = cy_tanhf(x);
      b = tanhf(vx);
    }
    if (as_uint(a) != as_uint(b) && !(a != a && b != b)) {
      if (!bad && first) {
        *first = (uint32_t)u;
      }
      bad++;
    }
  }
  return bad;
}
