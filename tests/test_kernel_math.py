"""Host checks of the device math that parity depends on (no GPU).

cy_sinf/cy_cosf restate glibc 2.35's sinf/cosf (sysdeps/ieee754/flt-32/s_sinf.c
algorithm, which the reference CPU kernel calls through util/util_math.h) for
|x| < 120; the path tracer only takes sines of angles in [-2*pi, 2*pi].
"""
import numpy as np
import pytest

import native_build as nb


def _eval(x):
    lib = nb.sincos()
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = [np.zeros_like(x) for _ in range(4)]
    lib.sincos_eval(x.ctypes.data, len(x), *[a.ctypes.data for a in out])
    return out


def test_sincos_bit_exact_vs_libm_random():
    rng = np.random.default_rng(0)
    x = rng.uniform(-119.0, 119.0, 1 << 20).astype(np.float32)
    s, c, s_ref, c_ref = _eval(x)
    assert np.array_equal(s.view(np.uint32), s_ref.view(np.uint32))
    assert np.array_equal(c.view(np.uint32), c_ref.view(np.uint32))


def test_sincos_bit_exact_vs_libm_path_tracer_range():
    # every float in a slice of [0, 2*pi] (the integrator's angle range), strided
    lo = np.float32(0.0).view(np.uint32)
    hi = np.float32(2 * np.pi).view(np.uint32)
    x = np.arange(lo, hi, 997, dtype=np.uint32).view(np.float32)
    x = np.concatenate([x, -x])
    s, c, s_ref, c_ref = _eval(x)
    assert np.array_equal(s.view(np.uint32), s_ref.view(np.uint32))
    assert np.array_equal(c.view(np.uint32), c_ref.view(np.uint32))


@pytest.mark.parametrize("v", [0.0, -0.0, 1e-45, 1e-30, 3.1415927, -3.1415927, 1.5707964, 6.2831855, 119.9])
def test_sincos_special_values(v):
    s, c, s_ref, c_ref = _eval(np.array([v], dtype=np.float32))
    assert s.view(np.uint32)[0] == s_ref.view(np.uint32)[0]
    assert c.view(np.uint32)[0] == c_ref.view(np.uint32)[0]


def test_acosf_bit_exact_vs_libm():
    """cy_acosf restates glibc's acosf (fdlibm e_acosf.c); the reference reaches
    it through safe_acosf in rect_light_sample (kernel_light_common.h:64-67).
    Exhaustive agreement over [-1, 1] was checked during development; here a
    strided sweep of the float range plus random values."""
    lib = nb.sincos()
    one = np.float32(1.0).view(np.uint32)
    x = np.arange(0, one + 1, 251, dtype=np.uint32).view(np.float32)
    rng = np.random.default_rng(4)
    x = np.concatenate([x, -x, rng.uniform(-1, 1, 1 << 18).astype(np.float32),
                        np.array([1.0, -1.0, 0.5, -0.5, 0.49999997, -0.49999997, 1e-30], dtype=np.float32)])
    x = np.ascontiguousarray(x)
    dev, ref = np.zeros_like(x), np.zeros_like(x)
    lib.acos_eval(x.ctypes.data, len(x), dev.ctypes.data, ref.ctypes.data)
    assert np.array_equal(dev.view(np.uint32), ref.view(np.uint32))


def test_powf_bit_exact_vs_libm():
    """cy_powf restates glibc 2.35 powf (FMA variant) for the film's sRGB
    transform (util_color.h:77-83).  Exhaustive agreement over every float in
    [0.0031308, 65504] was checked during development (0 of 237M differ); here
    every 7th float of that range plus [65504, 1e30] strided."""
    lib = nb.sincos()
    lo = int(np.float32(0.0031308).view(np.uint32))
    hi = int(np.float32(65504.0).view(np.uint32))
    assert lib.powf_sweep(lo, hi, 7) == 0
    assert lib.powf_sweep(hi, int(np.float32(1e30).view(np.uint32)), 101) == 0
    assert lib.powf_sweep(int(np.float32(1e-30).view(np.uint32)), lo, 1009) == 0


def test_atan2f_bit_exact_vs_libm():
    """cy_atan2f restates glibc's fdlibm atan2f/atanf (direction_to_equirectangular,
    kernel_projection.h:56-65): random directions, axis-aligned and special values."""
    lib = nb.sincos()
    rng = np.random.default_rng(8)
    n = 1 << 20
    y = rng.standard_normal(n).astype(np.float32)
    x = rng.standard_normal(n).astype(np.float32)
    x[::5] *= np.float32(1e-4)
    y[::7] *= np.float32(1e5)
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 1e-38, 3e38, 1e-45], dtype=np.float32)
    yy, xx = np.meshgrid(sp, sp)
    y = np.ascontiguousarray(np.concatenate([y, yy.ravel()]))
    x = np.ascontiguousarray(np.concatenate([x, xx.ravel()]))
    dev, ref = np.zeros_like(x), np.zeros_like(x)
    lib.atan2_eval(y.ctypes.data, x.ctypes.data, len(x), dev.ctypes.data, ref.ctypes.data)
    assert np.array_equal(dev.view(np.uint32), ref.view(np.uint32))


def test_asinf_bit_exact_vs_libm():
    """cy_asinf restates glibc's asinf (flt-32 e_asinf.c); the reference reaches
    it through fisheye_equisolid_to_direction (kernel_projection.h:118).  Every
    7th float of [0, 1] and of [-1, 0] (the full range was checked exhaustively
    during development: 0 mismatches)."""
    lib = nb.sincos()
    assert lib.asin_sweep(0, 0x3F800000, 7) == 0
    assert lib.asin_sweep(0x80000000, 0xBF800000, 7) == 0


def test_lgammaf_bit_exact_vs_libm():
    """cy_lgammaf restates glibc 2.35's lgammaf (fdlibm flt-32 e_lgammaf_r.c)
    for beta() in the multiscatter GGX glass closure.  Every float of
    [2^-40, 2^26] agreed during development (0 of 1.15e9 differ); here every
    13th float of that range and every float of [0.9, 8] (the branches the
    closure's arguments reach)."""
    import ctypes

    lib = nb.sincos()
    lib.lgammaf_sweep.restype = ctypes.c_long
    lib.lgammaf_sweep.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    assert lib.lgammaf_sweep(0x2B800000, 0x4C800000, 13, None) == 0
    lo, hi = int(np.float32(0.9).view(np.uint32)), int(np.float32(8.0).view(np.uint32))
    assert lib.lgammaf_sweep(lo, hi, 1, None) == 0


def test_tanf_expm1f_sinhf_coshf_tanhf_bit_exact_vs_libm():
    """cy_tanf / cy_expm1f / cy_sinhf / cy_coshf / cy_tanhf restate glibc 2.35
    (fdlibm k_tanf.c with glibc's double-precision rem_pio2f, s_expm1f.c,
    e_sinhf.c, e_coshf.c, s_tanhf.c) for the hair closures and the Math node.  Every float of both signs agreed during development (0 of
    4.3e9 differ for each); here every 997th float of the whole range and
    every 13th of [-4, 4] (tanf) / [-12, 12] (expm1f, sinhf), both of which
    walk every exponent and branch."""
    import ctypes

    lib = nb.sincos()
    lib.libm_sweep.restype = ctypes.c_long
    lib.libm_sweep.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    for which, dense in ((0, 4.0), (1, 12.0), (2, 12.0), (3, 12.0), (4, 12.0)):
        top = int(np.float32(dense).view(np.uint32))
        assert lib.libm_sweep(which, 0, 0x7F800000, 997, None) == 0, which
        assert lib.libm_sweep(which, 0x80000000, 0xFF800000, 997, None) == 0, which
        assert lib.libm_sweep(which, 0, top, 13, None) == 0, which
        assert lib.libm_sweep(which, 0x80000000, 0x80000000 | top, 13, None) == 0, which
