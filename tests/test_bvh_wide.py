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

Ribbon hair scenes use the wide layout too: the BVH2's unaligned nodes are
kept as oriented two-child nodes (the reference's test on its own
transforms, on every unaligned node of a path), and a ribbon the ray crosses in two subdivision steps (whose
result depends on the bound it is tested with) is re-traced in the
reference's order like a near-tie.  Thick
curves keep the BVH2 (cy_bvhw.h, hipcycles.hip pick_width).
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


# hair scenes whose curves are all ribbons (the wide layout serves them)
RIBBON_CASES = ["hair_ribbon", "hair_principled", "hair_info_ribbon"]
WIDE_CASES = [n for n in EMU_CASES if n not in CURVE_CASES or n in RIBBON_CASES]


@pytest.fixture(scope="module", params=[(n, w, m) for n in WIDE_CASES for w, m in VARIANTS],
                ids=lambda p: f"{p[0]}-w{p[1]}-m{p[2]}")
def case(request, emu):
    name, width, merge = request.param
    g = load_golden(name)
    ds = with_background_golden(compile_case(name), g)
    return name, ds, g, nb.EmuScene(emu, ds, width, merge), merge


def _bvh2_leaves(ds):
    leaves = ds.arrays["__bvh_leaf_nodes"].reshape(-1, 4).view(np.int32)
    return {int(l[0]): int(l[1] - l[0]) for l in leaves}


OBB = 1 << 30  # child code bit of an oriented-box node (hair scenes)


def _walk(es, roots):
    """Every node reachable from the roots: per node its kind and child codes
    (wide node: (code, meta, lo, hi) per valid slot; OBB node: two codes)."""
    W = es.width
    words = es.wide.reshape(-1, 8 * W)
    out, todo = {}, [(r, False) for r in roots]
    while todo:
        idx, obb = todo.pop()
        if idx in out:
            continue
        w = words[idx]
        if obb:
            # OBB node: two stored visibilities, two codes, two transforms
            kids = [(int(np.int32(np.uint32(w[2 + k]))), None, None, None) for k in range(2)]
        else:
            f = w.view(np.float32).reshape(8, W)
            m = w.reshape(8, W)
            kids = [(int(np.int32(m[6, j])), int(m[7, j]), f[0:6:2, j], f[1:6:2, j])
                    for j in range(W) if (m[7, j] & 0x0FFFFFFF) != 0]
        out[idx] = (obb, kids)
        for code, *_ in kids:
            if code >= 0:
                todo.append((code & ~OBB, bool(code & OBB)))
    return out


def test_collapse_structure(case):
    name, ds, g, es, merge = case
    onode = ds.arrays["__object_node"].view(np.int32)
    inst_objects = np.nonzero(ds.arrays["__object_flag"] & 4 == 0)[0]  # not SD_OBJECT_TRANSFORM_APPLIED
    roots = {0} | {int(es.object_root[o]) for o in inst_objects}
    assert all(es.object_root[o] >= 0 for o in inst_objects)
    assert len(roots) == 1 + len({int(onode[o]) for o in inst_objects})
    nodes = _walk(es, sorted(roots))
    # every node of the array is reached, each non-root node from exactly one
    # parent slot
    n = len(es.wide) // (8 * es.width)
    assert set(nodes) == set(range(n))
    refs = np.zeros(n, dtype=np.int64)
    for obb, kids in nodes.values():
        for code, *_ in kids:
            if code >= 0:
                refs[code & ~OBB] += 1
    is_root = np.zeros(n, dtype=bool)
    is_root[list(roots)] = True
    nodes_mask = np.zeros(n, dtype=bool)
    nodes_mask[list(nodes)] = True
    assert np.all(refs[is_root] == 0) and np.all(refs[~is_root & nodes_mask] == 1)
    assert np.all(refs[~nodes_mask] == 0)
    if name not in CURVE_CASES:
        assert not any(obb for obb, _ in nodes.values())
    # the leaf ranges tile the primitive array exactly once (instance slots,
    # prim_type 0, are entered through count-0 instance leaves instead)
    leaves = [(~code >> 4, ~code & 15, lo, hi) for obb, kids in nodes.values() for code, meta, lo, hi in kids
              if code < 0]
    counts = np.array([c for _, c, _, _ in leaves])
    starts = np.array([s for s, _, _, _ in leaves])
    assert set(starts[counts == 0].tolist()) == set(inst_objects.tolist())
    cover = np.zeros(len(ds.arrays["__prim_index"]), dtype=np.int32)
    for st, c in zip(starts[counts > 0].tolist(), counts[counts > 0].tolist()):
        cover[st:st + c] += 1
    assert np.all(cover == (ds.arrays["__prim_type"] != 0))
    if merge == 0 or name in CURVE_CASES:
        # hair scenes never merge (a merged leaf could mix primitive types)
        bvh2 = {k: v for k, v in _bvh2_leaves(ds).items() if k >= 0}
        got = {int(st): int(c) for st, c in zip(starts.tolist(), counts.tolist()) if c > 0}
        assert got == bvh2
    else:
        assert np.all(counts <= max(merge, 8))
    # wide-node leaf boxes (exact BVH2 boxes) contain their triangles
    ptype = ds.arrays["__prim_type"].astype(np.uint32)
    verts = ds.arrays["__prim_tri_verts"].reshape(-1, 4)[:, :3]
    tri_index = ds.arrays["__prim_tri_index"].astype(np.int64)
    for st, c, lo, hi in leaves:
        if c == 0 or lo is None or ptype[st] & 0x3C:
            continue
        v = np.concatenate([verts[tri_index[k]:tri_index[k] + 3] for k in range(st, st + c)])
        assert np.all(v >= lo) and np.all(v <= hi)


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
