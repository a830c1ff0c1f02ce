"""Shader node graphs (raytracingproject_amd/nodes.py) compiled to SVM code.

The renders of the shading_* parity cases pin the node arithmetic against the
reference kernel (tests/golden/shading_*.npz, test_host_emulation.py on CPU,
test_gpu_parity.py on the GPU).  These tests pin the host side: the encodings
the kernel decoders expect (svm_*.h), stack-slot reuse within the device's 32
slots, implicit socket conversions, and constant-emission detection.
"""
import numpy as np
import pytest

from raytracingproject_amd import abi
from raytracingproject_amd import nodes as nd
from raytracingproject_amd import scene as sc
from raytracingproject_amd import scenes


def _program(closure):
    """SVM code of one surface shader (index 0), as a list of 4-tuples."""
    code = sc.SVMCompiler().compile([closure], sc.background((0.0, 0.0, 0.0)))
    start, end = int(code[0, 1]), int(code[1, 1])  # up to the world shader's code
    return [tuple(int(x) for x in row) for row in code[start:end]]


def _f(bits):
    return float(np.array([bits], dtype=np.uint32).view(np.float32)[0])


@pytest.mark.parametrize("fn", [scenes.shading_math, scenes.shading_vector, scenes.shading_color,
                                scenes.shading_coords])
def test_shading_scenes_fit_the_device_stack(fn):
    s = fn(8, 8, 1)
    comp = sc.SVMCompiler()
    comp.compile(s.materials, sc.background(s.world_color, s.world_strength))
    assert comp.stack_top <= sc.SVM_STACK_SIZE


def test_clamp_extra_node_holds_min_max():
    """svm_clamp.h: defaults = read_node() -> (min, max) in .x/.y."""
    v = nd.clamp(nd.separate_xyz(nd.geometry()["Position"])["X"], 0.25, 0.75, kind="range")
    prog = _program(sc.diffuse(nd.combine_xyz(v, 0.0, 0.0)))
    i = next(k for k, n in enumerate(prog) if n[0] == nd.NODE_CLAMP)
    assert (prog[i][2] >> 16) & 0xFF == 1  # NODE_CLAMP_RANGE
    assert (prog[i][2] & 0xFF, (prog[i][2] >> 8) & 0xFF) == (255, 255)  # unlinked -> defaults
    assert (_f(prog[i + 1][0]), _f(prog[i + 1][1])) == (0.25, 0.75)


def test_map_range_reads_two_default_nodes():
    v = nd.map_range(nd.separate_xyz(nd.geometry()["Position"])["Y"], 1.0, 2.0, 3.0, 4.0, steps=5.0,
                     kind="stepped")
    prog = _program(sc.diffuse(nd.combine_xyz(v, 0.0, 0.0)))
    i = next(k for k, n in enumerate(prog) if n[0] == nd.NODE_MAP_RANGE)
    assert [_f(x) for x in prog[i + 1]] == [1.0, 2.0, 3.0, 4.0]
    assert _f(prog[i + 2][0]) == 5.0
    assert prog[i][3] & 0xFF == 1  # NODE_MAP_RANGE_STEPPED


def test_vector_math_wrap_has_operand_node():
    vm = nd.vector_math("wrap", nd.geometry()["Position"], (1.0, 1.0, 1.0), (-1.0, -1.0, -1.0))
    prog = _program(sc.diffuse(vm["Vector"]))
    i = next(k for k, n in enumerate(prog) if n[0] == nd.NODE_VECTOR_MATH)
    assert prog[i][1] == nd.VECTOR_MATH_OPS.index("wrap")
    c = prog[i + 1][0]
    # the operand slot was filled by a NODE_VALUE_V before the vector math node
    assert any(n[0] == nd.NODE_VALUE_V and n[1] == c for n in prog[:i])


def test_vector_math_value_output_only_for_value_ops():
    vm = nd.vector_math("add", (1.0, 0.0, 0.0), (0.0, 1.0, 0.0))
    with pytest.raises(ValueError):
        _program(sc.diffuse(nd.combine_xyz(vm["Value"], 0.0, 0.0)))


def test_ramp_table_follows_size_node():
    r = nd.color_ramp(0.5, [(0.0, (0, 0, 0, 1)), (1.0, (1, 1, 1, 1))], table_size=16)
    prog = _program(sc.diffuse(r["Color"]))
    i = next(k for k, n in enumerate(prog) if n[0] == nd.NODE_RGB_RAMP)
    assert prog[i + 1][0] == 16
    table = np.array([[_f(x) for x in prog[i + 2 + j]] for j in range(16)])
    assert np.allclose(table[:, 0], np.linspace(0, 1, 16), atol=1e-6)


def test_float_into_color_converts():
    """A float socket linked into a color input goes through NODE_CONVERT FV;
    color into float through CF (film rgb_to_y)."""
    f = nd.separate_xyz(nd.geometry()["Normal"])["Z"]
    prog = _program(sc.diffuse(f))
    assert any(n[0] == nd.NODE_CONVERT and n[1] == nd.CONVERT_FV for n in prog)
    prog = _program(sc.glossy((0.8, 0.8, 0.8), nd.rgb((0.2, 0.3, 0.4))))
    assert any(n[0] == nd.NODE_CONVERT and n[1] == nd.CONVERT_CF for n in prog)


def test_linked_bsdf_inputs_use_stack():
    rough = nd.math("multiply", nd.separate_xyz(nd.geometry()["Position"])["X"], 0.1)
    prog = _program(sc.glossy(nd.rgb((0.5, 0.5, 0.5)), rough))
    w = next(n for n in prog if n[0] == sc.NODE_CLOSURE_WEIGHT)  # linked color
    b = next(n for n in prog if n[0] == sc.NODE_CLOSURE_BSDF)
    assert w[1] != nd.SVM_STACK_INVALID
    assert (b[1] >> 8) & 0xFF != nd.SVM_STACK_INVALID  # roughness from the stack


def test_slots_are_reused():
    """A long chain needs only a few live slots (svm.cpp stack_clear_users)."""
    v = nd.separate_xyz(nd.geometry()["Position"])["X"]
    for k in range(60):
        v = nd.math("add", v, float(k))
    comp = sc.SVMCompiler()
    comp.compile([sc.diffuse(nd.combine_xyz(v, v, v))], sc.background((0, 0, 0)))
    assert comp.stack_top <= 8


def test_constant_emission_detection():
    assert sc.emission((1.0, 2.0, 3.0), 2.0).constant_emission().tolist() == [2.0, 4.0, 6.0]
    assert sc.emission(nd.rgb((1.0, 1.0, 1.0)), 1.0).constant_emission() is None
    assert sc.background((0.5, 0.5, 0.5), nd.value(2.0)).constant_emission() is None
    ds = sc.compile_scene(scenes.shading_coords(8, 8, 1))
    # the node world is not a constant emitter: the kernels evaluate it per ray
    n = ds.info["shaders"]
    shaders = (abi.KernelShader * n).from_buffer_copy(ds.arrays["__shaders"].tobytes())
    assert not (shaders[n - 1].flags & sc.SD_HAS_CONSTANT_EMISSION)
    assert all(shaders[i].flags & sc.SD_USE_MIS for i in range(n))


@pytest.mark.gpu
def test_unimplemented_node_rejected_at_load_kernels():
    """A node the device does not run is rejected by the program scan before
    any render, naming the node.  Every node of svm_types.h runs since round 6
    (the last ones were NODE_TEX_VOXEL and the AOV / bump-eval nodes), so the
    program gets a node number past the reference's enum, patched over a Math
    node (a program from a newer or corrupt compiler)."""
    from raytracingproject_amd.device import DeviceError, HIPDevice

    s = scenes.shading_math(8, 8, 1)
    s.materials[0] = sc.diffuse(nd.combine_xyz(nd.math("sine", 0.3, 0.0), 0.0, 0.0))
    ds = sc.compile_scene(s)
    prog = ds.arrays["__svm_nodes"]
    k = int(np.flatnonzero(prog[:, 0] == 42)[0])  # NODE_MATH
    prog[k, 0] = 150  # past the last node number of svm_types.h
    dev = HIPDevice(0)
    try:
        with pytest.raises(DeviceError, match="SVM node 150 is not implemented"):
            dev.upload_scene(ds)
    finally:
        dev.close()
