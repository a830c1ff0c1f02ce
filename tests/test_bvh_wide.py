"""The device's wide BVH (csrc/host/cy_bvhw_collapse.h + csrc/kernel/cy_bvhw.h)
on CPU: structure checked against the bound BVH2, and the traversal (the
device code compiled for the host) against the reference's golden hits and
renders, for 4- and 8-wide nodes with and without leaf merging.

The wide nodes carry the exact BVH2 child boxes and the traversal applies the
reference's slab test to them, so it reaches every triangle the BVH2 traversal
accepts: hit flags and any-hit (shadow) results are identical.  Where two
candidates' distances tie, the reference's visiting order decides
(bvh/bvh_traversal.h:34-227 visits BVH2 children near-first;
util/util_math_intersect.h:178 accepts T <= ray_t*den); the wide traversal
flags such rays and they are re-traced in the reference's order, so closest
hits and renders are bit-identical to the reference.
"""
import numpy as np
import pytest

import native_build as nb
from parity_cases import CURVE_CASES, EMU_CASES, PATH_RAY_SHADOW_OPAQUE, compile_case, load_golden, with_background_golden

RMSE_TOL = 1e-4
VARIANTS = [(4, 0), (8, 0), (4, 4), (8, 8)]


@pytest.fixture(scope="module")
def emu():
    return nb.host_emu(libm_sincos=True)


@pytest.fixture(scope="module", params=[(n, w, m) for n in EMU_CASES if n not in CURVE_CASES for w, m in VARIANTS],
                ids=lambda p: f"{p[0]}-w{p[1]}-m{p[2]}")
def case(request, emu):
    name, width, merge = request.param
    g = load_golden(name)
    ds = with_background_golden(compile_case(name), g)
    return name, ds, g, nb.EmuScene(emu, ds, width, merge), merge


def _decode(es):
    W = es.width
    w = es.wide.reshape(-1, 8, W)
    f = w.view(np.float32)
    lo = np.stack([f[:, 0], f[:, 2], f[:, 4]], axis=1)
    hi = np.stack([f[:, 1], f[:, 3], f[:, 5]], axis=1)
    return w[:, 6].view(np.int32), w[:, 7], lo, hi


def _bvh2_leaves(ds):
    leaves = ds.arrays["__bvh_leaf_nodes"].reshape(-1, 4).view(np.int32)
    return {int(l[0]): int(l[1] - l[0]) for l in leaves}


def test_collapse_structure(case):
    name, ds, g, es, merge = case
    child, meta, lo, hi = _decode(es)
    n = len(child)
    valid = (meta & 0x0FFFFFFF) != 0
    inner = valid & (child >= 0)
    leaf = valid & (child < 0)
    # every wide node except the roots (top level, each instanced geometry's
    # own BVH) is referenced exactly once
    refs = np.bincount(child[inner], minlength=n)
    onode = ds.arrays["__object_node"].view(np.int32)
    inst_objects = np.nonzero(ds.arrays["__object_flag"] & 4 == 0)[0]  # not SD_OBJECT_TRANSFORM_APPLIED
    roots = {0} | {int(es.object_root[o]) for o in inst_objects}
    assert all(es.object_root[o] >= 0 for o in inst_objects)
    assert len(roots) == 1 + len({int(onode[o]) for o in inst_objects})
    is_root = np.zeros(n, dtype=bool)
    is_root[list(roots)] = True
    assert np.all(refs[is_root] == 0) and np.all(refs[~is_root] == 1)
    # the leaf ranges tile the primitive array exactly once (instance slots,
    # prim_type 0, are entered through count-0 instance leaves instead)
    starts, counts = (~child[leaf]) >> 4, meta[leaf] >> 28
    assert np.array_equal((~child[leaf]) & 15, counts)
    tri_leaf = counts > 0
    assert set(((~child[leaf]) >> 4)[~tri_leaf].tolist()) == set(inst_objects.tolist())
    starts, counts = starts[tri_leaf], counts[tri_leaf]
    cover = np.zeros(len(ds.arrays["__prim_index"]), dtype=np.int32)
    for s, c in zip(starts.tolist(), counts.tolist()):
        cover[s:s + c] += 1
    assert np.all(cover == (ds.arrays["__prim_type"] != 0))
    if merge == 0:
        bvh2 = {k: v for k, v in _bvh2_leaves(ds).items() if k >= 0}
        assert dict(zip(starts.tolist(), counts.tolist())) == bvh2
    else:
        assert np.all(counts <= max(merge, 8))
    leaf = leaf & ((meta >> 28) > 0)
    # leaf boxes contain their triangles
    verts = ds.arrays["__prim_tri_verts"].reshape(-1, 4)[:, :3]
    tri_index = ds.arrays["__prim_tri_index"].astype(np.int64)
    for (node, slot), s, c in zip(zip(*np.nonzero(leaf)), starts.tolist(), counts.tolist()):
        v = np.concatenate([verts[tri_index[k]:tri_index[k] + 3] for k in range(s, s + c)])
        assert np.all(v >= lo[node, :, slot]) and np.all(v <= hi[node, :, slot])


def test_wide_closest_hit_vs_reference(case):
    name, ds, g, es, merge = case
    of, oi, cnt = es.intersect(g["rays"], any_hit=False)
    hf, hi = g["hit_f"], g["hit_i"]
    assert np.array_equal(oi[:, 0], hi[:, 0])
    # rays carrying the opaque-shadow bits are any-hit queries: the primitive
    # reported is whichever the traversal meets first, only the flag is defined
    closest = (g["rays"][:, 7].view(np.uint32) & PATH_RAY_SHADOW_OPAQUE) == 0
    hit = (hi[:, 0] == 1) & closest
    # the reference's closest hit bit for bit (near-ties re-traced in its order)
    assert np.array_equal(oi[hit, 1], hi[hit, 1])
    assert np.array_equal(of[hit].view(np.uint32), hf[hit].view(np.uint32))


def test_wide_shadow_any_hit_vs_reference(case):
    name, ds, g, es, merge = case
    of, oi, cnt = es.intersect(g["shadow_rays"], any_hit=True)
    assert np.array_equal(oi[:, 0], g["shadow_i"][:, 0])


def test_wide_visits_fewer_nodes(case, emu):
    name, ds, g, es, merge = case
    narrow = nb.EmuScene(emu, ds, 2)
    _, _, cw = es.intersect(g["rays"])
    _, _, c2 = narrow.intersect(g["rays"])
    assert cw[0] < c2[0], (cw, c2)


def test_wide_render_vs_reference(case):
    name, ds, g, es, merge = case
    buf = es.render()
    s = int(g["samples"])
    film, ref = buf[..., :3] / s, g["buffer"][..., :3] / s
    rmse = float(np.sqrt(np.mean((film - ref) ** 2)))
    assert rmse <= RMSE_TOL, rmse
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32))
