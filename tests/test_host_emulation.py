"""The HIP device's per-path code (csrc/kernel/cy_integrator.h, cy_path.h)
compiled for the host and driven path by path (tools/host_emu.cpp) renders
bit-identically to the reference CPU kernel's golden buffers.  This pins the
device LOGIC on CPU; tests/test_gpu_parity.py pins the GPU arithmetic."""
import numpy as np
import pytest

import native_build as nb
from parity_cases import EMU_CASES, compile_case, load_golden, with_background_golden


def emu_render(lib, ds, tile=None, start_sample=0, samples=None, offset=None, out=None, bvh_width=2):
    return nb.EmuScene(lib, ds, bvh_width).render(tile, start_sample, samples, offset, out)


@pytest.fixture(scope="module")
def emu():
    return nb.host_emu(libm_sincos=True)


@pytest.mark.parametrize("name", list(EMU_CASES))
def test_device_logic_bit_exact_vs_reference(emu, name):
    g = load_golden(name)
    ds = with_background_golden(compile_case(name), g)
    buf = emu_render(emu, ds)
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32))


@pytest.mark.parametrize("name", ["cornell_64", "closures_diffuse", "closures_microfacet", "closures_principled",
                                  "shading_image", "shading_noise", "shading_voronoi", "shading_attributes", "shading_normals", "closures_multiscatter",
                                  "volume_cornell"])
def test_device_sincos_restatement_matches_on_host(name):
    """Same render with the device's own libm restatements (sinf/cosf, expf,
    logf, powf, acosf) instead of the host libm: still bit-exact."""
    lib = nb.host_emu(libm_sincos=False)
    g = load_golden(name)
    ds = with_background_golden(compile_case(name), g)
    assert np.array_equal(emu_render(lib, ds).view(np.uint32), g["buffer"].view(np.uint32))


def test_sample_ranges_compose(emu):
    """Rendering samples [0,k) then [k,n) into one buffer equals one pass
    (task.acquire_tile hands out sample ranges; device_cuda_impl.cpp:1895-1933)."""
    ds = compile_case("cornell_64")
    g = load_golden("cornell_64")
    buf = emu_render(emu, ds, samples=5)
    emu_render(emu, ds, start_sample=5, samples=ds.samples - 5, out=buf)
    assert np.array_equal(buf.view(np.uint32), g["buffer"].view(np.uint32))
