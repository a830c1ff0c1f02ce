"""GPU parity at the BASELINE.json configs' full size.

The small golden cases (test_gpu_parity.py) pin the arithmetic; these pin the
same device path on the configs' own scenes, resolutions and sample counts:
  * crops of the full-size CB, BMW and BBS stand-ins rendered through the
    C-ABI tile entry (hipcy_path_trace with the crop as RenderTile) against the
    reference CPU kernel's render of the same crop (tests/golden/scale_*.npz);
  * whole frames of BMW (1280x720x128), BBS (1920x1080x512), CLS
    (1920x1080x256) and JNK (3840x2160 at 32 spp) against the sha256 of the
    reference kernel's float32 buffer of the same frame (full_<name>.npz);
  * the bench frame's 16x16 block means and determinism.
Bars: film RMSE <= 1e-4 (north_star); measured and asserted: bit-exact on
every crop for the BVH2 and the default 4-wide BVH, and on every full frame.
"""
import os

import numpy as np
import pytest

from parity_cases import (FULL_DIGEST_CASES, FULL_FRAME_BLOCK, FULL_FRAME_CASE, GOLDEN, SCALE_CASES, block_means,
                          buffer_sha256, scene_digest)
from raytracingproject_amd import scene as sc
from raytracingproject_amd import scenes

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4


@pytest.fixture(scope="module")
def device():
    from raytracingproject_amd.device import HIPDevice

    dev = HIPDevice(0)
    yield dev
    dev.close()


def _golden(name):
    return np.load(os.path.join(GOLDEN, f"scale_{name}.npz"), allow_pickle=False)


@pytest.fixture(scope="module", params=list(SCALE_CASES))
def scale_case(request, device):
    name = request.param
    fn, tile = SCALE_CASES[name]
    ds = sc.compile_scene(fn())
    g = _golden(name)
    assert str(g["digest"]) == scene_digest(ds), "scene generator drifted from the golden inputs"
    device.upload_scene(ds)
    return name, ds, g


@pytest.mark.parametrize("width", [2, 4])
def test_crop_matches_reference(scale_case, device, width):
    name, ds, g = scale_case
    device.set_bvh_width(width)
    device.set_curve_layout(width > 2)  # JNK's ribbons on the wide layout at W = 4
    x, y, w, h = (int(v) for v in g["tile"])
    buf = device.render(tile=(x, y, w, h))
    ref = g["buffer"]
    s = int(g["samples"])
    assert buf.shape == ref.shape
    assert np.isfinite(buf).all()
    film, ref_film = buf[..., :3] / s, ref[..., :3] / s
    rmse = float(np.sqrt(np.mean((film - ref_film) ** 2)))
    exact = float(np.mean(buf.view(np.uint32) == ref.view(np.uint32)))
    print(f"{name} bvh{width}: crop {w}x{h}x{s} film RMSE {rmse:.3e}, bit-exact fraction {exact:.4f}")
    assert rmse <= RMSE_TOL, (name, width, rmse, exact)
    assert np.array_equal(buf[..., 3], ref[..., 3])
    assert exact == 1.0, (name, width, exact)


@pytest.fixture(scope="module")
def bench_frame(device):
    ds = sc.compile_scene(scenes.CONFIGS[FULL_FRAME_CASE]())
    g = _golden("full_frame")
    assert str(g["digest"]) == scene_digest(ds)
    device.upload_scene(ds)
    device.set_bvh_width(4)
    return ds, g


def test_full_frame_matches_reference_block_means(bench_frame, device):
    ds, g = bench_frame
    buf = device.render()
    s = ds.samples
    assert buf.shape == (ds.height, ds.width, ds.pass_stride)
    assert np.isfinite(buf).all()
    # opaque scene, opaque background: every sample contributes alpha 1
    assert np.all(buf[..., 3] == np.float32(s))
    bm = block_means(buf, FULL_FRAME_BLOCK)
    ref = g["block_means"]
    rmse = float(np.sqrt(np.mean((bm[..., :3] / s - ref[..., :3] / s) ** 2)))
    print(f"full frame {ds.width}x{ds.height}x{s}: block-mean film RMSE {rmse:.3e}")
    assert rmse <= RMSE_TOL, rmse


def test_full_frame_deterministic(bench_frame, device):
    ds, g = bench_frame
    a = device.render()
    b = device.render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("name", list(FULL_DIGEST_CASES))
def test_full_frame_bit_exact(device, name):
    """Whole frames of the BASELINE configs at their full resolution and
    sample count (JNK at 32 spp), compared with the reference CPU kernel's
    render of the same scene through the sha256 of the float32 buffer
    (tests/golden/full_<name>.npz).  On a mismatch the 16x16 block-mean RMSE
    against the reference is reported."""
    path = os.path.join(GOLDEN, f"full_{name}.npz")
    if not os.path.exists(path):
        pytest.skip(f"full_{name}.npz not generated")
    g = np.load(path, allow_pickle=False)
    ds = sc.compile_scene(FULL_DIGEST_CASES[name]())
    assert str(g["digest"]) == scene_digest(ds), "scene generator drifted from the golden inputs"
    device.upload_scene(ds)
    device.set_bvh_width(4)
    buf = device.render()
    assert buf.shape == tuple(int(v) for v in g["shape"])
    assert np.isfinite(buf).all()
    digest = buffer_sha256(buf)
    if digest != str(g["sha256"]):
        s = int(g["samples"])
        bm = block_means(buf, int(g["block"]))
        rmse = float(np.sqrt(np.mean((bm[..., :3] / s - g["block_means"][..., :3] / s) ** 2)))
        pytest.fail(f"{name}: film differs from the reference (block-mean film RMSE {rmse:.3e})")
