"""Scene compiler and host BVH2 builder (no GPU): determinism and the packed
layout invariants the traversal kernels rely on (bvh/bvh2.cpp:40-163 layout:
4 float4 per inner node, 1 float4 per leaf, leaf address ~i)."""
import numpy as np
import pytest

from parity_cases import CASES, compile_case, scene_digest
from raytracingproject_amd import scene as sc
from raytracingproject_amd import scenes


def _walk(ds):
    """Walk the two-level BVH2: the top level from KernelBVH.root, each
    instanced object's own BVH once from __object_node (bvh.cpp:323-520)."""
    nodes = ds.arrays["__bvh_nodes"].reshape(-1, 4)
    leaves = ds.arrays["__bvh_leaf_nodes"].reshape(-1, 4)
    verts = ds.arrays["__prim_tri_verts"].reshape(-1, 4)[:, :3]
    tri_index = ds.arrays["__prim_tri_index"].astype(np.int64)
    n_prims = len(ds.arrays["__prim_type"])
    seen = np.zeros(n_prims, dtype=np.int32)
    stack = [(int(ds.data.bvh.root), None)]
    entered = set()
    n_inner = 0
    while stack:
        addr, box = stack.pop()
        if addr < 0:
            leaf = leaves[-addr - 1].view(np.int32)
            lo, hi = int(leaf[0]), int(leaf[1])
            if lo < 0:  # instance leaf: ~slot, 0, visibility, type 0
                slot = ~lo
                assert hi == 0 and ds.arrays["__prim_type"][slot] == 0
                seen[slot] += 1
                root = int(ds.arrays["__object_node"].view(np.int32)[ds.arrays["__prim_object"][slot]])
                if root not in entered:
                    entered.add(root)
                    stack.append((root, None))
                continue
            assert 0 <= lo < hi <= n_prims
            seen[lo:hi] += 1
            if box is not None:
                v = np.concatenate([verts[tri_index[k]:tri_index[k] + 3] for k in range(lo, hi)])
                assert np.all(v >= box[0]) and np.all(v <= box[1])
            continue
        n_inner += 1
        c = nodes[addr].view(np.int32)
        n0, n1, n2 = nodes[addr + 1], nodes[addr + 2], nodes[addr + 3]
        for k, child in ((0, int(c[2])), (1, int(c[3]))):
            cbox = (np.array([n0[k], n1[k], n2[k]]), np.array([n0[2 + k], n1[2 + k], n2[2 + k]]))
            assert np.all(cbox[0] <= cbox[1])
            if box is not None:
                assert np.all(cbox[0] >= box[0]) and np.all(cbox[1] <= box[1])
            stack.append((child, cbox))
    return seen, n_inner


@pytest.mark.parametrize("name", list(CASES))
def test_bvh2_covers_every_primitive_once(name):
    ds = compile_case(name)
    seen, n_inner = _walk(ds)
    assert np.all(seen == 1)
    assert 4 * n_inner == ds.arrays["__bvh_nodes"].reshape(-1, 4).shape[0]


@pytest.mark.parametrize("name", list(CASES))
def test_compile_is_deterministic(name):
    assert scene_digest(compile_case(name)) == scene_digest(compile_case(name))


def test_kernel_data_header():
    ds = compile_case("cornell_64")
    assert ds.data.film.pass_stride == 4 == ds.pass_stride
    assert ds.data.integrator.sampling_pattern == 0  # Sobol
    assert ds.data.bvh.bvh_layout == 1  # BVH_LAYOUT_BVH2
    assert ds.data.cam.width == 64 and ds.data.cam.height == 64


def test_bmw_standin_scale():
    """The bench workload: BMW27-class triangle count at the benchmark resolution."""
    s = scenes.bmw27_standin()
    assert (s.width, s.height, s.samples) == (1280, 720, 128)
    ntris = sum(np.asarray(m.tris).reshape(-1, 3).shape[0] for m in s.meshes)
    assert 5e5 < ntris < 2e6


def test_bvh_build_small_random():
    rng = np.random.default_rng(0)
    tv = rng.random((1000, 3, 3)).astype(np.float32)
    nodes, leaves, order, n_inner = sc.build_bvh2(tv, np.ones(1000, dtype=np.uint32))
    assert sorted(order.tolist()) == list(range(1000))
