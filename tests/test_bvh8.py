"""The device's 8-wide BVH (csrc/host/cy_bvh8_collapse.h + csrc/kernel/cy_bvh8.h)
on CPU: structure and conservative quantization checked against the bound
BVH2, and the traversal (the device code compiled for the host) against the
reference's golden hits and renders.

The wide traversal reaches every triangle the BVH2 traversal accepts, so hit
flags and any-hit (shadow) results are identical; the closest primitive can
differ only where two candidates' distances agree to a few ulp, because the
visiting order decides such ties (bvh/bvh_traversal.h:34-227 visits BVH2
children near-first; util/util_math_intersect.h:178 accepts T <= ray_t*den).
Renders are held to the north-star bar, film RMSE <= 1e-4.
"""
import numpy as np
import pytest

import native_build as nb
from parity_cases import CASES, PATH_RAY_SHADOW_OPAQUE, compile_case, load_golden

RMSE_TOL = 1e-4


@pytest.fixture(scope="module")
def emu():
    return nb.host_emu(libm_sincos=True)


@pytest.fixture(scope="module", params=list(CASES))
def case(request, emu):
    ds = compile_case(request.param)
    return request.param, ds, load_golden(request.param), nb.EmuScene(emu, ds, bvh_width=8)


def _decode(words):
    """(n, 8 slots) child words, meta words and decoded float32 boxes."""
    w = words.reshape(-1, 32)
    origin = w[:, 0:3].view(np.float32)
    eb = np.stack([(w[:, 3] >> (8 * a)) & 0xFF for a in range(3)], axis=1)
    scale = (eb.astype(np.uint32) << 23).view(np.float32)
    b = w[:, 4:16].copy().view(np.uint8).reshape(-1, 3, 16)
    qlo = b[:, :, 0:8].astype(np.float32)
    qhi = b[:, :, 8:16].astype(np.float32)
    lo = origin[:, :, None] + qlo * scale[:, :, None]
    hi = origin[:, :, None] + qhi * scale[:, :, None]
    return w[:, 16:24].view(np.int32), w[:, 24:32], lo, hi


def _bvh2_leaf_boxes(ds):
    """exact child boxes of every BVH2 leaf, keyed by its first primitive"""
    nodes = ds.arrays["__bvh_nodes"].reshape(-1, 4)
    leaves = ds.arrays["__bvh_leaf_nodes"].reshape(-1, 4)
    out = {}
    for a in range(0, len(nodes), 4):
        c = nodes[a].view(np.int32)
        for k in range(2):
            if c[2 + k] < 0:
                leaf = leaves[-c[2 + k] - 1].view(np.int32)
                lo = np.array([nodes[a + 1][k], nodes[a + 2][k], nodes[a + 3][k]], dtype=np.float32)
                hi = np.array([nodes[a + 1][2 + k], nodes[a + 2][2 + k], nodes[a + 3][2 + k]], dtype=np.float32)
                out[int(leaf[0])] = (int(leaf[1] - leaf[0]), lo, hi)
    return out


def test_collapse_structure(case):
    name, ds, g, es = case
    child, meta, lo, hi = _decode(es.bvh8)
    n = len(child)
    valid = (meta & 0x0FFFFFFF) != 0
    inner = valid & (child >= 0)
    leaf = valid & (child < 0)
    # every wide node except the root is referenced exactly once
    refs = np.bincount(child[inner], minlength=n)
    assert refs[0] == 0 and np.all(refs[1:] == 1)
    # every BVH2 leaf appears exactly once, with its primitive count
    want = _bvh2_leaf_boxes(ds)
    starts = ~child[leaf]
    counts = meta[leaf] >> 28
    assert sorted(starts.tolist()) == sorted(want)
    for s, c in zip(starts.tolist(), counts.tolist()):
        assert want[s][0] == c
    # 8-wide: far fewer nodes than BVH2 inner nodes
    assert n * 2 < ds.arrays["__bvh_nodes"].reshape(-1, 4).shape[0] // 4


def test_quantized_boxes_contain_exact_boxes(case):
    name, ds, g, es = case
    child, meta, lo, hi = _decode(es.bvh8)
    want = _bvh2_leaf_boxes(ds)
    for node, slot in zip(*np.nonzero(((meta & 0x0FFFFFFF) != 0) & (child < 0))):
        _, elo, ehi = want[int(~child[node, slot])]
        assert np.all(lo[node, :, slot] <= elo) and np.all(hi[node, :, slot] >= ehi)


def test_wide_closest_hit_vs_reference(case):
    name, ds, g, es = case
    of, oi, cnt = es.intersect(g["rays"], any_hit=False)
    hf, hi = g["hit_f"], g["hit_i"]
    assert np.array_equal(oi[:, 0], hi[:, 0])
    # rays carrying the opaque-shadow bits are any-hit queries: the primitive
    # reported is whichever the traversal meets first, only the flag is defined
    closest = (g["rays"][:, 7].view(np.uint32) & PATH_RAY_SHADOW_OPAQUE) == 0
    hit = (hi[:, 0] == 1) & closest
    same = oi[hit, 1] == hi[hit, 1]
    # the Cornell boxes stand on the floor: coplanar faces give exact t ties
    assert same.mean() >= 0.995, same.mean()
    assert np.array_equal(of[hit][same].view(np.uint32), hf[hit][same].view(np.uint32))
    t, tr = of[hit][~same, 0], hf[hit][~same, 0]
    assert np.all(np.abs(t - tr) <= 1e-6 * np.abs(tr))


def test_wide_shadow_any_hit_vs_reference(case):
    name, ds, g, es = case
    of, oi, cnt = es.intersect(g["shadow_rays"], any_hit=True)
    assert np.array_equal(oi[:, 0], g["shadow_i"][:, 0])


def test_wide_visits_fewer_nodes(case, emu):
    name, ds, g, es = case
    narrow = nb.EmuScene(emu, ds, bvh_width=2)
    _, _, c8 = es.intersect(g["rays"])
    _, _, c2 = narrow.intersect(g["rays"])
    assert c8[0] * 2 < c2[0], (c8, c2)
    # bytes: 128 per wide node (leaves inline) vs 64 per BVH2 node + 16 per leaf
    assert 128 * c8[0] < 64 * c2[0] + 16 * c2[1]


def test_wide_render_vs_reference(case):
    name, ds, g, es = case
    buf = es.render()
    s = int(g["samples"])
    film, ref = buf[..., :3] / s, g["buffer"][..., :3] / s
    rmse = float(np.sqrt(np.mean((film - ref) ** 2)))
    assert rmse <= RMSE_TOL, rmse
    assert np.array_equal(buf[..., 3], g["buffer"][..., 3])
