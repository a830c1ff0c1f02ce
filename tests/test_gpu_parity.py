"""GPU parity: the HIP device against the reference Cycles CPU kernel.

Expected values come from tests/golden/*.npz, written by tests/golden/make_golden.py
with the reference kernel compiled from /root/reference (oracle/_ref).  The
inputs are recompiled here from the same deterministic scene generators and
checked against the recorded digest first, so a fixture can never be compared
with different inputs.

Bars (BASELINE.json north_star): integer results (hit flags, primitive ids,
rng hashes) bit-exact; camera rays and hit t/u/v bit-exact (IEEE f32, no
contraction); rendered film within 1e-4 RMSE of the reference.

Every test runs at three widths: the BVH2 exactly as bound (width 2, the
reference's visiting order) and the device's 4-wide (the default) and 8-wide
BVHs.  The wide traversals visit in another order but return the reference's
closest hit bit for bit: rays whose hits tie are re-traced in the reference's
order (cy_bvhw.h), and instanced scenes keep the reference's top-level order
(cy_path.h bvh2_intersect WI > 2), so renders are bit-identical at every width.
"""
import numpy as np
import pytest

from parity_cases import (CASES, HOST_LOOP_CASES, PATH_RAY_SHADOW_OPAQUE, atomic_pass_channels, buffers_match,
                          compile_case, load_golden, scene_digest)

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4

def assert_film_exact(name, buf, ref, *extra):
    """Bit-exact film (no tolerated deviations: the last one, shading_bump_paths
    pixel (23, 7) sample 4, was a float-to-int conversion of a checker
    coordinate beyond the int range, which x86 and the GPU round differently;
    cy_math.h cy_ftoi, found with tools/dbg_trace.py)."""
    a, b = buf.view(np.uint32), ref.view(np.uint32)
    if np.array_equal(a, b):
        return
    diff = a != b
    ulps = np.abs(a[diff].astype(np.int64) - b[diff].astype(np.int64))
    assert False, (name, int(diff.sum()), int(ulps.max()), *extra)


@pytest.fixture(scope="module")
def device():
    from raytracingproject_amd.device import HIPDevice

    dev = HIPDevice(0)
    yield dev
    dev.close()


@pytest.fixture(scope="module", params=[(n, w) for w in (2, 4, 8) for n in CASES], ids=lambda p: f"{p[0]}-bvh{p[1]}")
def case(request, device):
    name, width = request.param
    ds = compile_case(name)
    g = load_golden(name)
    assert str(g["digest"]) == scene_digest(ds), "scene generator drifted from the golden inputs"
    device.upload_scene(ds)
    device.set_bvh_width(width)
    # ribbon scenes on the wide layout at W = 4 / 8 (hipcy_set_curve_layout;
    # the device default, the BVH2, is the W = 2 traversal)
    device.set_curve_layout(width > 2)
    device.bvh_width_under_test = width
    return name, ds, g


def test_native_library_is_the_hip_device(device):
    from raytracingproject_amd import native

    assert device.lib._name == native.DEVICE_LIB
    devs = device.available_devices()
    assert devs and "gfx950" in devs[0]["name"]


def test_camera_rays_bit_exact(case, device):
    name, ds, g = case
    out = device.camera_rays(g["cam_xys"])
    ref = g["cam_out"]
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), (
        name, np.abs(out - ref).max())


def test_closest_hit_matches_reference(case, device):
    name, ds, g = case
    device.set_bvh_width(device.bvh_width_under_test)
    of, oi = device.intersect(g["rays"], any_hit=False)
    ref_f, ref_i = g["hit_f"], g["hit_i"]
    assert np.array_equal(oi[:, 0], ref_i[:, 0]), name
    hit = ref_i[:, 0] == 1
    # any-hit queries (opaque-shadow visibility) report whichever primitive the
    # traversal meets first: only their flag is defined
    hit &= (g["rays"][:, 7].view(np.uint32) & PATH_RAY_SHADOW_OPAQUE) == 0
    if device.bvh_width_under_test == 2:
        hit = ref_i[:, 0] == 1
    # closest hits: the reference's primitive and t, u, v bit for bit at every
    # width (the wide traversal re-traces near-ties in the reference's order)
    assert np.array_equal(oi[hit, 1], ref_i[hit, 1]), name
    assert np.array_equal(of[hit].view(np.uint32), ref_f[hit].view(np.uint32)), name


def test_shadow_any_hit_matches_reference(case, device):
    name, ds, g = case
    of, oi = device.intersect(g["shadow_rays"], any_hit=True)
    assert np.array_equal(oi[:, 0], g["shadow_i"][:, 0]), name


def test_background_map_matches_reference(case, device):
    """World importance sampling: the device's SHADER-task map and the host
    CDFs built from it equal the reference kernel's map and the oracle's CDFs."""
    name, ds, g = case
    if not ds.info.get("background_map"):
        pytest.skip("no background light")
    res_x, res_y = ds.info["background_map"]
    m = device.background_eval(res_x, res_y, 1)
    assert np.array_equal(m.view(np.uint32), g["bg_map"].view(np.uint32))
    marg, cond = device.background_cdfs
    assert np.array_equal(marg.view(np.uint32), g["bg_marg"].view(np.uint32))
    assert np.array_equal(cond.view(np.uint32), g["bg_cond"].view(np.uint32))


def test_render_matches_reference(case, device):
    name, ds, g = case
    buf = device.render()
    ref = g["buffer"]
    samples = int(g["samples"])
    assert np.isfinite(buf).all()
    film = buf[..., :3] / samples
    ref_film = ref[..., :3] / samples
    rmse = float(np.sqrt(np.mean((film - ref_film) ** 2)))
    exact = float(np.mean(buf.view(np.uint32) == ref.view(np.uint32)))
    print(f"{name}: film RMSE {rmse:.3e}, bit-exact fraction {exact:.4f}, max abs {np.abs(film - ref_film).max():.3e}")
    assert rmse <= RMSE_TOL, (name, rmse, exact)
    m = atomic_pass_channels(ds)
    assert_film_exact(name, buf[..., ~m].copy(), ref[..., ~m].copy(), exact)
    # AOV passes (atomic adds, parity_cases.atomic_pass_channels): to rounding
    assert buffers_match(ds, buf, ref), name
    # alpha is exactly the sample count for opaque scenes
    assert np.array_equal(buf[..., 3], ref[..., 3])


def test_render_is_deterministic(case, device):
    name, ds, g = case
    a = device.render()
    b = device.render()
    assert buffers_match(ds, a, b)


def test_tiles_and_sample_ranges_compose(case, device):
    """Rendering in two sample ranges and two tiles gives the full-frame buffer
    (Session tiles + progressive start_sample, tile.cpp / integrator.cpp:72)."""
    name, ds, g = case
    if name in HOST_LOOP_CASES:
        pytest.skip("adaptive sampling filters and rescales per RenderTile: tiles do not compose")
    full = device.render()
    h = ds.height
    w = ds.width
    half = h // 2
    s = ds.samples
    top = device.render(samples=s // 2, start_sample=0, tile=(0, 0, w, half)) + \
        device.render(samples=s - s // 2, start_sample=s // 2, tile=(0, 0, w, half))
    bot = device.render(tile=(0, half, w, h - half))
    comp = np.concatenate([top, bot], axis=0)
    # sample-range split changes the float summation grouping: compare in film space
    film = comp[..., :3] / s
    ref = full[..., :3] / s
    assert float(np.sqrt(np.mean((film - ref) ** 2))) < 1e-6
    assert buffers_match(ds, bot, full[half:])


def test_interleaved_rows(case, device):
    """Row-interleaved sharding (multi-GPU layout) reproduces the full frame."""
    from raytracingproject_amd.device import DeviceBuffer  # noqa: F401

    name, ds, g = case
    if name in HOST_LOOP_CASES:
        # device errors are sticky (Device::set_error): use a device of its own
        from raytracingproject_amd.device import HIPDevice

        dev2 = HIPDevice(0)
        try:
            dev2.upload_scene(ds)
            w, h = ds.width, ds.height
            rows = len(range(0, h, 2))
            buf = dev2.mem_alloc(w * rows * ds.pass_stride * 4)
            with pytest.raises(Exception, match="adaptive sampling needs whole tiles"):
                dev2.render_tile(buf, (0, 0, w, rows), 0, ds.samples, 0, w, y_step=2)
        finally:
            dev2.close()
        return
    full = device.render()
    w, h = ds.width, ds.height
    n = 3
    out = np.zeros_like(full)
    for r in range(n):
        rows = len(range(r, h, n))
        buf = device.mem_alloc(w * rows * ds.pass_stride * 4)
        buf.zero()
        device.render_tile(buf, (0, r, w, rows), 0, ds.samples, -(r * w), w, y_step=n)
        part = np.zeros((rows, w, ds.pass_stride), dtype=np.float32)
        buf.copy_from_device(part)
        buf.free()
        out[r::n] = part
    assert buffers_match(ds, out, full)


@pytest.mark.parametrize("mode", [3, 5, 8])
@pytest.mark.parametrize("name", ["cornell_64", "bmw_small", "cornell_instanced", "transparent_shadows",
                                  "closures_principled", "hair_principled", "sss_disk"])
def test_render_with_ray_sort_matches_reference(name, mode, device):
    """Wavefront ray sorting (hipcy_set_ray_sort) reorders the closest queue of
    every bounce iteration (modes 3, 5), or the shading queue by the hit's
    shader (mode 8); each path depends on its work item alone, so the film
    stays bit-identical to the reference."""
    if name not in CASES:
        pytest.skip(f"{name} not a parity case")
    ds = compile_case(name)
    g = load_golden(name)
    device.upload_scene(ds)
    device.set_bvh_width(4)
    device.set_ray_sort(mode)
    try:
        buf = device.render()
    finally:
        device.set_ray_sort(-1)
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32)), name


@pytest.mark.parametrize("mode", [3, 5])
@pytest.mark.parametrize("name", ["cornell_64", "bmw_small", "cornell_lamps", "cornell_instanced", "world_mis"])
def test_render_with_shadow_sort_matches_reference(name, mode, device):
    """Shadow-queue sort (hipcy_set_shadow_sort): the opaque-shadow queue of
    every iteration binned by shadow ray direction before its traversal; the
    light each path adds depends on its own shadow ray alone, so the film stays
    bit-identical to the reference."""
    if name not in CASES:
        pytest.skip(f"{name} not a parity case")
    ds = compile_case(name)
    g = load_golden(name)
    device.upload_scene(ds)
    device.set_bvh_width(4)
    device.set_shadow_sort(mode)
    try:
        buf = device.render()
    finally:
        device.set_shadow_sort(0)
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32)), name


@pytest.mark.parametrize("tail", [0, 1 << 40])
@pytest.mark.parametrize("width", [2, 4, 8])
@pytest.mark.parametrize("name", ["cornell_64", "bmw_small", "cornell_lamps", "cornell_instanced", "camera_dof",
                                  "camera_equirect", "cornell_joe_kuo"])
def test_render_with_fused_tail_matches_reference(name, width, tail, device):
    """Fused tail (hipcy_set_tail, k_shade.hip k_tail_*): once a lane's work
    items are all claimed, its live paths run to their ends in one launch
    (closest hit, shading and shadow per bounce) instead of one three-kernel
    iteration per bounce.  0 never takes it; 2^40 takes it right after the
    camera launch.  Each path runs the same per-slot functions in the same
    order, so the film is bit-identical to the reference; with the tail the
    pass needs two lane iterations (camera iteration + tail) on these scenes
    (plain shading kernel, opaque shadows, triangles)."""
    if name not in CASES:
        pytest.skip(f"{name} not a parity case")
    ds = compile_case(name)
    g = load_golden(name)
    device.upload_scene(ds)
    device.set_bvh_width(width)
    device.set_tail(tail)
    try:
        buf = device.render()
        st = device.stats()
    finally:
        device.set_tail(1 << 17)
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32)), name
    if tail:
        assert st["iterations"] <= 8, st
    else:
        assert st["iterations"] > 8, st


@pytest.mark.parametrize("budget", [(1, 2), (3, 5), (12, 24)])
@pytest.mark.parametrize("width", [4, 8])
@pytest.mark.parametrize("name", ["cornell_64", "bmw_small", "cornell_lamps", "world_mis", "closures_principled"])
def test_render_with_traversal_budget_matches_reference(name, width, budget, device):
    """Iteration budget (hipcy_set_traversal_budget): closest and shadow
    traversals stop after `budget[0]` iterations, are saved as continuation
    records and resumed in packed launches (again suspended after budget[1]).
    A resumed traversal continues with the same stack, hit and near-tie state,
    so the film is bit-identical to the reference; (1, 2) suspends almost every
    ray twice."""
    if name not in CASES:
        pytest.skip(f"{name} not a parity case")
    ds = compile_case(name)
    g = load_golden(name)
    device.upload_scene(ds)
    device.set_bvh_width(width)
    device.set_traversal_budget(*budget)
    try:
        buf = device.render()
        st = device.stats()
    finally:
        device.set_traversal_budget(0, 0)
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32)), (name, budget)
    assert st["closest_rays"] > 0


@pytest.mark.parametrize("refill", [(1, 1), (4, 16), (16, 64)])
@pytest.mark.parametrize("width", [4, 8])
@pytest.mark.parametrize("name", ["cornell_64", "bmw_small", "cornell_lamps", "closures_principled",
                                  "shading_bump_paths", "sss_disk"])
def test_render_with_lane_refill_matches_reference(name, width, refill, device):
    """Lane refill (hipcy_set_traversal_refill): persistent closest-hit waves
    traverse `refill[0]` iterations at a time and hand finished lanes the next
    rays of the queue once `refill[1]` lanes are idle; camera launches write
    their rays into the slots first.  Each ray's traversal is split into rounds
    of the resumable cursor, so the film is bit-identical; (1, 1) refills after
    every iteration."""
    if name not in CASES:
        pytest.skip(f"{name} not a parity case")
    ds = compile_case(name)
    g = load_golden(name)
    device.upload_scene(ds)
    device.set_bvh_width(width)
    device.set_traversal_refill(*refill)
    try:
        buf = device.render()
        st = device.stats()
    finally:
        device.set_traversal_refill(0, 16)
    assert_film_exact(name, buf, g["buffer"], refill)
    assert st["closest_rays"] > 0


@pytest.mark.parametrize("capacity", [1, 97])
@pytest.mark.parametrize("name", ["cornell_64", "bmw_small"])
def test_traversal_budget_with_full_continuation_buffer(name, capacity, device, monkeypatch):
    """Continuation buffers smaller than the suspended traversals
    (HIPCY_CONT_CAPACITY): lanes that find the buffer full finish their
    traversal in place (cont_suspend's fallback), still bit-exact."""
    monkeypatch.setenv("HIPCY_CONT_CAPACITY", str(capacity))
    ds = compile_case(name)
    g = load_golden(name)
    device.upload_scene(ds)
    device.set_bvh_width(4)
    device.set_traversal_budget(1, 2)
    try:
        buf = device.render()
    finally:
        device.set_traversal_budget(0, 0)
        monkeypatch.delenv("HIPCY_CONT_CAPACITY")
        device.render(samples=1)  # back to the default continuation buffers
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32)), (name, capacity)


def test_curve_scene_default_layout_is_the_bvh2(device):
    """Scenes with curves traverse the bound BVH2 unless hipcy_set_curve_layout
    asks for the wide layout: at W = 4 the default render equals the reference
    and the wide-layout render alike."""
    ds = compile_case("hair_ribbon")
    g = load_golden("hair_ribbon")
    device.upload_scene(ds)
    device.set_bvh_width(4)
    device.set_curve_layout(False)
    default = device.render()
    device.set_curve_layout(True)
    wide = device.render()
    device.set_curve_layout(False)
    assert_film_exact("hair_ribbon", default, g["buffer"], "default layout")
    assert_film_exact("hair_ribbon", wide, g["buffer"], "wide layout")
