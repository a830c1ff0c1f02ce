"""Sobol direction vectors for ``__sample_pattern_lut``.

The reference host fills the LUT with Joe-Kuo direction numbers
(render/integrator.cpp:235-243 -> render/sobol.cpp).  That table is data of the
host scene compiler, not of the hot path: the kernel only XORs LUT entries
(kernel_random.h:40-49).  This module builds a valid Sobol table of its own:
dimension 0 is the van der Corput sequence (identical to the reference's
dimension 0), dimension d >= 1 uses the d-th primitive polynomial over GF(2) in
(degree, coefficient) order with odd initial direction numbers from a fixed
seed.  Parity tests feed the same LUT to both kernels, so the table's origin
does not affect them.
"""
from __future__ import annotations

import numpy as np

SOBOL_BITS = 32
SOBOL_MAX_DIMENSIONS = 21201


def _is_primitive(poly: int, degree: int) -> bool:
    """poly includes the x^degree and constant terms."""
    order = (1 << degree) - 1
    # x has order dividing 2^d - 1; primitive iff order is exactly 2^d - 1
    def mulmod(a: int, b: int) -> int:
        r = 0
        while b:
            if b & 1:
                r ^= a
            b >>= 1
            a <<= 1
            if a >> degree & 1:
                a ^= poly
        return r

    def powmod(e: int) -> int:
        r, base = 1, 2
        while e:
            if e & 1:
                r = mulmod(r, base)
            base = mulmod(base, base)
            e >>= 1
        return r

    if powmod(order) != 1:
        return False
    n, p = order, 2
    factors = set()
    while p * p <= n:
        while n % p == 0:
            factors.add(p)
            n //= p
        p += 1
    if n > 1:
        factors.add(n)
    return all(powmod(order // f) != 1 for f in factors)


def primitive_polynomials(count: int):
    out = []
    degree = 1
    while len(out) < count:
        for a in range(1 << max(degree - 1, 0)):
            poly = (1 << degree) | (a << 1) | 1
            if degree == 1:
                poly = 0b11
            if _is_primitive(poly, degree):
                out.append((degree, a))
                if len(out) == count:
                    break
            if degree == 1:
                break
        degree += 1
    return out


def direction_vectors(dimensions: int, seed: int = 0x5EED) -> np.ndarray:
    """Return uint32 array [dimensions, 32] (LUT layout: 32 * dimension + bit)."""
    dims = min(dimensions, SOBOL_MAX_DIMENSIONS)
    v = np.zeros((dims, SOBOL_BITS), dtype=np.uint64)
    for i in range(SOBOL_BITS):
        v[0, i] = 1 << (31 - i)
    if dims == 1:
        return v.astype(np.uint32)
    rng = np.random.default_rng(seed)
    polys = primitive_polynomials(dims - 1)
    L = SOBOL_BITS
    for d in range(1, dims):
        s, a = polys[d - 1]
        # odd initial direction numbers m_i < 2^(i+1)
        m = [int(rng.integers(0, 1 << i)) * 2 + 1 for i in range(s)]
        vd = [0] * L
        if L <= s:
            for i in range(L):
                vd[i] = m[i] << (31 - i)
        else:
            for i in range(s):
                vd[i] = m[i] << (31 - i)
            for i in range(s, L):
                x = vd[i - s] ^ (vd[i - s] >> s)
                for k in range(1, s):
                    x ^= ((a >> (s - 1 - k)) & 1) * vd[i - k]
                vd[i] = x & 0xFFFFFFFF
        v[d, :] = vd
    return v.astype(np.uint32)


def sample_pattern_lut(dimensions: int, generated: int = 256) -> np.ndarray:
    """LUT of `dimensions` dims; the first `generated` dims are distinct Sobol
    dimensions, later ones (only reached by volume-bound / SSS bounces, which the
    HIP device rejects) repeat them cyclically so the array has the size the host
    integrator allocates (integrator.cpp:230-238)."""
    base = direction_vectors(min(generated, dimensions))
    reps = -(-dimensions // base.shape[0])
    full = np.concatenate([base] * reps, axis=0)[:dimensions]
    return np.ascontiguousarray(full.reshape(-1))
