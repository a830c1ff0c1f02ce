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
