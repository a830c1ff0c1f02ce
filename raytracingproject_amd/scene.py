"""Scene description + compiler into the Cycles device data (stand-in host).

The reference host (render/scene.cpp:193-310 Scene::device_update and the
managers it calls) turns a scene into KernelData plus the named device arrays of
kernel/kernel_textures.h.  The HIP path sits *below* that host, so tests and the
benchmark need a producer of the same data; this module is that producer for
the feature subset the HIP kernels implement (triangle meshes with transforms
applied, SVM diffuse / GGX glossy / GGX or sharp glass / emission / mix,
constant-emission mesh lights, constant world, perspective camera, combined pass).

Each step cites the host code whose output layout it reproduces.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field

import numpy as np

from . import abi, native, sobol

# ---------------------------------------------------------------------------
# constants of the device ABI (kernel_types.h / svm_types.h)
PATH_RAY_ALL_VISIBILITY = (1 << 14) - 1
PATH_RAY_SHADOW_OPAQUE_CATCHER = 1 << 8
PATH_RAY_SHADOW_TRANSPARENT_CATCHER = 1 << 10
PATH_RAY_NODE_UNALIGNED = 1 << 13
SHADER_SMOOTH_NORMAL = 1 << 31
SHADER_CAST_SHADOW = 1 << 30
SHADER_AREA_LIGHT = 1 << 29
SHADER_USE_MIS = 1 << 28
SD_USE_MIS = 1 << 16
SD_HAS_CONSTANT_EMISSION = 1 << 27
SD_OBJECT_TRANSFORM_APPLIED = 1 << 2
SD_OBJECT_NEGATIVE_SCALE_APPLIED = 1 << 3
PRIMITIVE_TRIANGLE = 1
PASSMASK_COMBINED = 1 << 1
BVH_LAYOUT_BVH2 = 1
FILTER_TABLE_SIZE = 1024
INT_MAX = 2**31 - 1
FLT_MAX = float(np.finfo(np.float32).max)
VOLUME_BOUNDS_MAX = 1024
BSSRDF_MAX_BOUNCES = 256
PRNG_BASE_NUM = 10
PRNG_BOUNCE_NUM = 8

NODE_END, NODE_SHADER_JUMP, NODE_CLOSURE_BSDF, NODE_CLOSURE_EMISSION = 0, 1, 2, 3
NODE_CLOSURE_BACKGROUND, NODE_CLOSURE_SET_WEIGHT = 4, 5
NODE_MIX_CLOSURE, NODE_JUMP_IF_ZERO, NODE_VALUE_F = 8, 9, 14
SVM_STACK_INVALID = 255

CLOSURE_BSDF_DIFFUSE_ID = 2
CLOSURE_BSDF_REFLECTION_ID = 9
CLOSURE_BSDF_MICROFACET_GGX_ID = 10
CLOSURE_BSDF_REFRACTION_ID = 22
CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID = 24
CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID = 27
CLOSURE_BSDF_SHARP_GLASS_ID = 29


def f32bits(x: float) -> int:
    return int(np.array([x], dtype=np.float32).view(np.uint32)[0])


# ---------------------------------------------------------------------------
# Shader description (a tiny node graph: one closure tree per material)


@dataclass
class Closure:
    kind: str  # diffuse | glossy | glass | sharp_glass | refraction | emission | mix
    color: tuple = (0.8, 0.8, 0.8)
    roughness: float = 0.0
    ior: float = 1.45
    strength: float = 1.0
    fac: float = 0.5
    a: "Closure | None" = None
    b: "Closure | None" = None

    def num_closures(self) -> int:
        """ShaderGraph::get_num_closures (render/graph.cpp:1130-1161)."""
        if self.kind == "mix":
            return self.a.num_closures() + self.b.num_closures()
        if self.kind in ("glass", "sharp_glass"):
            return 2
        return 1

    def has_emission(self) -> bool:
        if self.kind == "mix":
            return self.a.has_emission() or self.b.has_emission()
        return self.kind == "emission"


def diffuse(color, roughness=0.0):
    return Closure("diffuse", tuple(color), roughness=roughness)


def glossy(color, roughness):
    return Closure("glossy", tuple(color), roughness=roughness)


def glass(color, roughness, ior=1.45):
    return Closure("glass" if roughness > 0 else "sharp_glass", tuple(color), roughness=roughness, ior=ior)


def emission(color, strength):
    return Closure("emission", tuple(color), strength=strength)


def mix(fac, a, b):
    return Closure("mix", fac=fac, a=a, b=b)


class SVMCompiler:
    """Emits SVM bytecode with the node encodings of svm/svm.h + svm_closure.h
    (the reference host compiler is render/svm.cpp + nodes.cpp compile())."""

    def __init__(self):
        self.nodes: list[tuple[int, int, int, int]] = []
        self.stack_top = 0

    def alloc(self, n=1) -> int:
        off = self.stack_top
        self.stack_top += n
        if self.stack_top > 32:
            raise ValueError("SVM stack exceeds the HIP device's 32 slots")
        return off

    @staticmethod
    def uchar4(x, y, z, w) -> int:
        return (x & 0xFF) | ((y & 0xFF) << 8) | ((z & 0xFF) << 16) | ((w & 0xFF) << 24)

    def emit_closure(self, c: Closure, mix_weight: int) -> list:
        out = []
        if c.kind == "mix":
            fac_off = self.alloc()
            w1, w2 = self.alloc(), self.alloc()
            out.append((NODE_VALUE_F, f32bits(c.fac), fac_off, 0))
            out.append((NODE_MIX_CLOSURE, self.uchar4(fac_off, mix_weight, w1, w2), 0, 0))
            for sub, w in ((c.a, w1), (c.b, w2)):
                code = self.emit_closure(sub, w)
                out.append((NODE_JUMP_IF_ZERO, len(code), w, 0))
                out.extend(code)
            return out
        if c.kind == "emission":
            col = np.array(c.color, dtype=np.float32) * np.float32(c.strength)
            out.append((NODE_CLOSURE_SET_WEIGHT, *(f32bits(v) for v in col)))
            out.append((NODE_CLOSURE_EMISSION, mix_weight, 0, 0))
            return out
        ctype = {
            "diffuse": CLOSURE_BSDF_DIFFUSE_ID,
            "glossy": CLOSURE_BSDF_MICROFACET_GGX_ID if c.roughness > 0 else CLOSURE_BSDF_REFLECTION_ID,
            "glass": CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID,
            "sharp_glass": CLOSURE_BSDF_SHARP_GLASS_ID,
            "refraction": CLOSURE_BSDF_REFRACTION_ID,
        }[c.kind]
        out.append((NODE_CLOSURE_SET_WEIGHT, *(f32bits(v) for v in c.color)))
        out.append(
            (
                NODE_CLOSURE_BSDF,
                self.uchar4(ctype, SVM_STACK_INVALID, SVM_STACK_INVALID, mix_weight),
                f32bits(c.roughness),
                f32bits(c.ior),
            )
        )
        # data node: normal, tangent, rotation, extra — all default
        out.append((SVM_STACK_INVALID, SVM_STACK_INVALID, SVM_STACK_INVALID, SVM_STACK_INVALID))
        return out

    def compile(self, surfaces: list[Closure], world: Closure) -> np.ndarray:
        """Shader i's code starts with the jump node at index i (svm.cpp
        SVMShaderManager::device_update: shader ids index the jump table)."""
        shaders = list(surfaces) + [world]
        n = len(shaders)
        self.nodes = [(NODE_SHADER_JUMP, 0, 0, 0)] * n
        for i, sh in enumerate(shaders):
            self.stack_top = 0
            start = len(self.nodes)
            self.nodes[i] = (NODE_SHADER_JUMP, start, 0, 0)
            if i == n - 1:  # world background
                col = np.array(sh.color, dtype=np.float32) * np.float32(sh.strength)
                self.nodes.append((NODE_CLOSURE_SET_WEIGHT, *(f32bits(v) for v in col)))
                self.nodes.append((4, SVM_STACK_INVALID, 0, 0))  # NODE_CLOSURE_BACKGROUND
            else:
                self.nodes.extend(self.emit_closure(sh, SVM_STACK_INVALID))
            self.nodes.append((NODE_END, 0, 0, 0))
        return np.array(self.nodes, dtype=np.uint32).reshape(-1, 4)


# ---------------------------------------------------------------------------
# Geometry / camera


@dataclass
class Mesh:
    verts: np.ndarray  # (V, 3) float32, world space
    tris: np.ndarray  # (T, 3) int
    shader: np.ndarray | int = 0  # per-triangle material index, or one index
    smooth: bool = False
    normals: np.ndarray | None = None  # (V, 3) vertex normals for smooth shading


@dataclass
class Lamp:
    """A Cycles Light (render/light.h): point, spot, area or sun (distant)."""

    kind: str  # point | spot | area | sun
    co: tuple = (0.0, 0.0, 0.0)
    direction: tuple = (0.0, 0.0, -1.0)  # emission direction (spot, area normal, sun)
    size: float = 0.0  # point/spot radius, area size multiplier
    axisu: tuple = (1.0, 0.0, 0.0)  # area: unit axes, scaled by sizeu/sizev * size
    axisv: tuple = (0.0, 1.0, 0.0)
    sizeu: float = 1.0
    sizev: float = 1.0
    round: bool = False
    angle: float = 0.0  # sun: angular diameter
    spot_angle: float = math.radians(45.0)
    spot_smooth: float = 0.0
    color: tuple = (1.0, 1.0, 1.0)
    strength: float = 10.0
    use_mis: bool = True
    cast_shadow: bool = True
    max_bounces: int = 1024


@dataclass
class Camera:
    eye: tuple = (0.0, 0.0, -5.0)
    target: tuple = (0.0, 0.0, 0.0)
    up: tuple = (0.0, 1.0, 0.0)
    fov: float = math.radians(40.0)  # full vertical-or-horizontal fov as in Cycles
    nearclip: float = 1e-5
    farclip: float = 1e5


@dataclass
class Scene:
    width: int
    height: int
    camera: Camera
    meshes: list
    materials: list
    world_color: tuple = (0.05, 0.05, 0.05)
    world_strength: float = 1.0
    samples: int = 16
    max_bounce: int = 7
    max_diffuse_bounce: int = 7
    max_glossy_bounce: int = 7
    max_transmission_bounce: int = 7
    transparent_max_bounce: int = 7
    min_bounce: int = 0
    filter_type: str = "box"  # box | gaussian | blackman_harris
    filter_width: float = 1.0
    seed: int = 0
    light_sampling_threshold: float = 0.05
    filter_glossy: float = 0.0
    lamps: list = field(default_factory=list)
    caustics_reflective: bool = True
    caustics_refractive: bool = True
    name: str = "scene"


@dataclass
class DeviceScene:
    data: abi.KernelData
    arrays: dict
    width: int
    height: int
    samples: int
    info: dict = field(default_factory=dict)

    @property
    def pass_stride(self) -> int:
        return self.data.film.pass_stride


# ---------------------------------------------------------------------------
# camera matrices: render/camera.cpp:220-330 (perspective, no border, no motion)


def _look_at(eye, target, up) -> np.ndarray:
    eye, target, up = (np.asarray(v, dtype=np.float64) for v in (eye, target, up))
    fwd = target - eye
    fwd /= np.linalg.norm(fwd)
    right = np.cross(up, fwd)  # Cycles camera space: +x right, +y up, +z forward
    right /= np.linalg.norm(right)
    up2 = np.cross(fwd, right)
    m = np.eye(4)
    m[:3, 0] = right
    m[:3, 1] = up2
    m[:3, 2] = fwd
    m[:3, 3] = eye
    return m


def _viewplane(width, height):
    """Camera::compute_auto_viewplane (sensor fit AUTO)."""
    aspect = width / height
    if width >= height:
        return (-aspect, aspect, -1.0, 1.0)
    return (-1.0, 1.0, -1.0 / aspect, 1.0 / aspect)


def _from_viewplane(vp):
    l, r, b, t = vp
    s = np.diag([1.0 / (r - l), 1.0 / (t - b), 1.0, 1.0])
    tr = np.eye(4)
    tr[0, 3] = -l
    tr[1, 3] = -b
    return s @ tr


def _perspective(fov, n, f):
    persp = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, f / (f - n), -f * n / (f - n)], [0, 0, 1, 0]], dtype=np.float64)
    inv_angle = 1.0 / math.tan(0.5 * fov)
    return np.diag([inv_angle, inv_angle, 1.0, 1.0]) @ persp


def compile_camera(kcam, cam: Camera, width: int, height: int):
    screentondc = _from_viewplane(_viewplane(width, height))
    ndctoraster = np.diag([width, height, 1.0, 1.0])
    screentoraster = ndctoraster @ screentondc
    rastertoscreen = np.linalg.inv(screentoraster)
    cameratoscreen = _perspective(cam.fov, cam.nearclip, cam.farclip)
    screentocamera = np.linalg.inv(cameratoscreen)
    rastertocamera = screentocamera @ rastertoscreen
    cameratoworld = _look_at(cam.eye, cam.target, cam.up)
    worldtocamera = np.linalg.inv(cameratoworld)

    def persp(m, v):
        p = m @ np.array([v[0], v[1], v[2], 1.0])
        return p[:3] / p[3]

    dx = persp(rastertocamera, (1, 0, 0)) - persp(rastertocamera, (0, 0, 0))
    dy = persp(rastertocamera, (0, 1, 0)) - persp(rastertocamera, (0, 0, 0))
    dx = cameratoworld[:3, :3] @ dx
    dy = cameratoworld[:3, :3] @ dy

    kcam.type = 0
    kcam.panorama_type = 0
    abi.set_transform(kcam.cameratoworld, cameratoworld[:3])
    abi.set_transform(kcam.rastertocamera, rastertocamera)
    abi.set_transform(kcam.worldtocamera, worldtocamera[:3])
    abi.set_transform(kcam.screentoworld, cameratoworld @ screentocamera)
    abi.set_transform(kcam.rastertoworld, cameratoworld @ rastertocamera)
    abi.set_transform(kcam.ndctoworld, cameratoworld @ rastertocamera @ ndctoraster)
    abi.set_transform(kcam.worldtoscreen, cameratoscreen @ worldtocamera)
    abi.set_transform(kcam.worldtondc, screentondc @ cameratoscreen @ worldtocamera)
    abi.set_transform(kcam.worldtoraster, ndctoraster @ screentondc @ cameratoscreen @ worldtocamera)
    kcam.dx.x, kcam.dx.y, kcam.dx.z, kcam.dx.w = (*dx, 0.0)
    kcam.dy.x, kcam.dy.y, kcam.dy.z, kcam.dy.w = (*dy, 0.0)
    kcam.aperturesize = 0.0
    kcam.blades = 0.0
    kcam.focaldistance = 10.0
    kcam.shuttertime = -1.0
    kcam.num_motion_steps = 0
    kcam.have_perspective_motion = 0
    kcam.nearclip = cam.nearclip
    kcam.cliplength = cam.farclip - cam.nearclip
    kcam.sensorwidth = 36.0
    kcam.sensorheight = 24.0
    kcam.width = float(width)
    kcam.height = float(height)
    kcam.resolution = 1
    kcam.inv_aperture_ratio = 1.0
    kcam.interocular_offset = 0.0
    kcam.shutter_table_offset = 0


# ---------------------------------------------------------------------------
# film filter table: render/film.cpp:298-355 + util/util_math_cdf.{h,cpp}


def filter_table(ftype: str, width: float) -> np.ndarray:
    f32 = np.float32
    if ftype == "box":
        func = lambda v, w: f32(1.0)  # noqa: E731
    elif ftype == "gaussian":
        width *= 3.0

        def func(v, w):
            v = f32(v) * f32(6.0 / w)
            return f32(math.exp(-2.0 * float(v) * float(v)))
    elif ftype == "blackman_harris":
        width *= 2.0

        def func(v, w):
            v = f32(2.0 * math.pi) * (f32(v) / f32(w) + f32(0.5))
            v = float(v)
            return f32(0.35875 - 0.48829 * math.cos(v) + 0.14128 * math.cos(2 * v) - 0.01168 * math.cos(3 * v))
    else:
        raise ValueError(ftype)
    resolution = FILTER_TABLE_SIZE
    frm, to = f32(0.0), f32(width * 0.5)
    # util_cdf_evaluate(resolution - 1, ...)
    res = resolution - 1
    cdf = np.zeros(res + 1, dtype=np.float32)
    rng_ = to - frm
    for i in range(res):
        x = frm + rng_ * f32(i) / f32(res - 1)
        cdf[i + 1] = cdf[i] + abs(func(x, width))
    cdf = (cdf / cdf[res]).astype(np.float32)
    # util_cdf_invert(make_symmetric = true)
    inv = np.zeros(resolution, dtype=np.float32)
    half = (resolution - 1) // 2
    for i in range(half + 1):
        x = f32(i) / f32(half)
        index = int(np.searchsorted(cdf, x, side="right"))
        if index < len(cdf) - 1:
            t = (x - cdf[index]) / (cdf[index + 1] - cdf[index])
        else:
            t = f32(0.0)
            index = len(cdf) - 1
        y = ((f32(index) + t) / f32(resolution - 1)) * (f32(2.0) * rng_)
        inv[half + i] = f32(0.5) * (f32(1.0) + y)
        inv[half - i] = f32(0.5) * (f32(1.0) - y)
    return inv


# ---------------------------------------------------------------------------
# BVH build + pack (native stand-in for bvh/bvh2.cpp, bvh.cpp)


def build_bvh2(tri_verts: np.ndarray, visibility: np.ndarray, max_leaf: int = 8):
    lib = native.host_lib()
    n = tri_verts.shape[0]
    tv = np.ascontiguousarray(tri_verts.reshape(n, 9), dtype=np.float32)
    vis = np.ascontiguousarray(visibility, dtype=np.uint32)
    counts = np.zeros(3, dtype=np.int64)
    h = lib.hcb_build(n, tv.ctypes.data, vis.ctypes.data, max_leaf, counts.ctypes.data)
    try:
        nodes = np.zeros((max(int(counts[0]), 1), 4), dtype=np.float32)
        leaves = np.zeros((max(int(counts[1]), 1), 4), dtype=np.float32)
        order = np.zeros(n, dtype=np.int32)
        lib.hcb_pack(h, nodes.ctypes.data, leaves.ctypes.data, order.ctypes.data)
    finally:
        lib.hcb_free(h)
    return nodes[: int(counts[0])] if counts[0] else nodes, leaves, order, int(counts[2])


# ---------------------------------------------------------------------------


def compile_scene(scene: Scene) -> DeviceScene:
    f32 = np.float32
    kd = abi.KernelData()

    # --- geometry (render/geometry.cpp device_update_mesh + mesh.cpp pack_*)
    verts_all, tris_all, shader_all, smooth_all, norm_all, objid_all = [], [], [], [], [], []
    voff = 0
    for oi, m in enumerate(scene.meshes):
        v = np.asarray(m.verts, dtype=np.float32).reshape(-1, 3)
        t = np.asarray(m.tris, dtype=np.int64).reshape(-1, 3)
        sh = np.broadcast_to(np.asarray(m.shader, dtype=np.int64), (t.shape[0],))
        verts_all.append(v)
        tris_all.append(t + voff)
        shader_all.append(sh)
        smooth_all.append(np.full(t.shape[0], bool(m.smooth)))
        if m.normals is not None:
            norm_all.append(np.asarray(m.normals, dtype=np.float32).reshape(-1, 3))
        else:
            norm_all.append(_vertex_normals(v, t))
        objid_all.append(np.full(t.shape[0], oi, dtype=np.int64))
        voff += v.shape[0]
    verts = np.concatenate(verts_all)
    tris = np.concatenate(tris_all)
    tri_shader_idx = np.concatenate(shader_all)
    tri_smooth = np.concatenate(smooth_all)
    vnormals = np.concatenate(norm_all)
    tri_object = np.concatenate(objid_all)
    ntri = tris.shape[0]

    # object visibility_for_tracing (render/object.cpp): all rays, not a shadow catcher
    vis_obj = PATH_RAY_ALL_VISIBILITY & ~(PATH_RAY_SHADOW_OPAQUE_CATCHER | PATH_RAY_SHADOW_TRANSPARENT_CATCHER)
    tri_pos = verts[tris]  # (T, 3, 3)
    visibility = np.full(ntri, vis_obj, dtype=np.uint32)
    nodes, leaves, order, root = build_bvh2(tri_pos, visibility)

    # pack_primitives (bvh.cpp:279-321): BVH slot i -> triangle order[i]
    prim_index = order.astype(np.uint32)
    prim_object = tri_object[order].astype(np.uint32)
    prim_type = np.full(ntri, PRIMITIVE_TRIANGLE, dtype=np.uint32)
    prim_visibility = visibility[order]
    prim_tri_index = (3 * np.arange(ntri, dtype=np.uint32)).astype(np.uint32)
    prim_tri_verts = np.ones((ntri * 3, 4), dtype=np.float32)
    prim_tri_verts[:, :3] = tri_pos[order].reshape(-1, 3)
    slot_of_tri = np.empty(ntri, dtype=np.int64)
    slot_of_tri[order] = np.arange(ntri)
    tri_vindex = np.zeros((ntri, 4), dtype=np.uint32)
    tri_vindex[:, :3] = tris.astype(np.uint32)
    tri_vindex[:, 3] = (3 * slot_of_tri).astype(np.uint32)
    tri_vnormal = np.zeros((verts.shape[0], 4), dtype=np.float32)
    tri_vnormal[:, :3] = vnormals

    # --- shaders (render/shader.cpp:462-475, 508-581 + svm.cpp); lamps share
    # one emission shader (the default light shader: emission 1.0), their
    # color and power go to KernelLight.strength
    mats = list(scene.materials)
    lamp_shader = None
    if scene.lamps:
        lamp_shader = len(mats)
        mats.append(Closure("emission", (1.0, 1.0, 1.0), strength=1.0))
    world = Closure("background", tuple(scene.world_color), strength=scene.world_strength)
    svm = SVMCompiler().compile(mats, world)
    n_shaders = len(mats) + 1
    kshaders = (abi.KernelShader * n_shaders)()
    for i, m in enumerate(mats + [world]):
        flag = SD_USE_MIS
        const = None
        if m.kind == "emission":
            const = np.array(m.color, dtype=np.float32) * f32(m.strength)
        elif m.kind == "background":
            const = np.array(m.color, dtype=np.float32) * f32(m.strength)
        if const is not None:
            flag |= SD_HAS_CONSTANT_EMISSION
            kshaders[i].constant_emission[:] = [float(c) for c in const]
        kshaders[i].flags = flag
    tri_shader = tri_shader_idx.astype(np.uint32) | np.uint32(SHADER_CAST_SHADOW | SHADER_AREA_LIGHT)
    tri_shader = np.where(tri_smooth, tri_shader | np.uint32(SHADER_SMOOTH_NORMAL), tri_shader).astype(np.uint32)

    # --- objects (render/object.cpp device_update_object_transform; transforms applied)
    nobj = len(scene.meshes)
    kobjects = (abi.KernelObject * max(nobj, 1))()
    ident = np.eye(4)[:3]
    for i in range(nobj):
        abi.set_transform(kobjects[i].tfm, ident)
        abi.set_transform(kobjects[i].itfm, ident)
        kobjects[i].shadow_terminator_offset = 0.0
    object_flag = np.full(max(nobj, 1), SD_OBJECT_TRANSFORM_APPLIED, dtype=np.uint32)

    # --- lights (render/light.cpp:277-480, mesh lights only)
    emissive = np.array([m.has_emission() for m in mats], dtype=bool)
    light_tris = np.nonzero(emissive[tri_shader_idx])[0]
    dist = (abi.KernelLightDistribution * (len(light_tris) + 1))()
    totarea = f32(0.0)
    for k, ti in enumerate(light_tris):
        dist[k].totarea = float(totarea)
        dist[k].prim = int(ti)
        dist[k].shader_flag = 0
        dist[k].object_id = int(tri_object[ti])
        p1, p2, p3 = tri_pos[ti].astype(np.float32)
        area = f32(0.5) * f32(np.sqrt(np.sum(np.cross(p2 - p1, p3 - p1).astype(np.float32) ** 2, dtype=np.float32)))
        totarea = f32(totarea + area)
    nd = len(light_tris)
    trianglearea = totarea
    lamps = list(scene.lamps)
    num_lights = len(lamps)
    dist_all = (abi.KernelLightDistribution * (nd + num_lights + 1))()
    for k in range(nd):
        dist_all[k] = dist[k]
    dist = dist_all
    # lamps (light.cpp:404-433): equal share of the triangle area each
    lightarea = f32(totarea / f32(num_lights)) if (totarea > 0 and num_lights) else f32(1.0)
    use_lamp_mis = False
    klights = (abi.KernelLight * max(num_lights, 1))()
    for li, lamp in enumerate(lamps):
        e = dist[nd + li]
        e.totarea = float(totarea)
        e.prim = ~li
        e.shader_flag = f32bits_signed(1.0)  # lamp.pad
        e.object_id = f32bits_signed(lamp.size)  # lamp.size
        totarea = f32(totarea + lightarea)
        use_lamp_mis |= _pack_lamp(klights[li], lamp, lamp_shader)
    ntot = nd + num_lights
    dist[ntot].totarea = float(totarea)
    dist[ntot].prim = 0
    if totarea > 0:
        for k in range(ntot):
            dist[k].totarea = float(f32(dist[k].totarea) / totarea)
        dist[ntot].totarea = 1.0
    ki = kd.integrator
    ki.use_direct_light = int(totarea > 0)
    if ki.use_direct_light:
        ki.num_distribution = ntot
        ki.num_all_lights = num_lights
        ki.pdf_triangles = 0.0
        ki.pdf_lights = 0.0
        if trianglearea > 0:
            ki.pdf_triangles = float(f32(1.0) / trianglearea)
            if num_lights:
                ki.pdf_triangles = float(f32(ki.pdf_triangles) * f32(0.5))
        if num_lights:
            ki.pdf_lights = float(f32(1.0) / f32(num_lights))
            if trianglearea > 0:
                ki.pdf_lights = float(f32(ki.pdf_lights) * f32(0.5))
        ki.use_lamp_mis = int(use_lamp_mis)
    else:
        ki.use_lamp_mis = 0

    # --- integrator (render/integrator.cpp:103-245)
    ki.min_bounce = scene.min_bounce + 1
    ki.max_bounce = scene.max_bounce + 1
    ki.max_diffuse_bounce = scene.max_diffuse_bounce + 1
    ki.max_glossy_bounce = scene.max_glossy_bounce + 1
    ki.max_transmission_bounce = scene.max_transmission_bounce + 1
    ki.max_volume_bounce = 7 + 1
    ki.transparent_min_bounce = 0 + 1
    ki.transparent_max_bounce = scene.transparent_max_bounce + 1
    ki.ao_bounces = INT_MAX
    ki.transparent_shadows = 0
    ki.volume_max_steps = 1024
    ki.volume_step_rate = 1.0
    ki.caustics_reflective = int(scene.caustics_reflective)
    ki.caustics_refractive = int(scene.caustics_refractive)
    ki.filter_glossy = FLT_MAX if scene.filter_glossy == 0.0 else 1.0 / scene.filter_glossy
    ki.seed = native.hash_uint2(scene.seed, 0)
    ki.use_ambient_occlusion = 0
    ki.sample_clamp_direct = FLT_MAX
    ki.sample_clamp_indirect = FLT_MAX
    ki.branched = 0
    ki.volume_decoupled = 0
    ki.diffuse_samples = ki.glossy_samples = ki.transmission_samples = 1
    ki.ao_samples = ki.mesh_light_samples = ki.subsurface_samples = ki.volume_samples = 1
    ki.start_sample = 0
    ki.sample_all_lights_direct = 0
    ki.sample_all_lights_indirect = 0
    ki.sampling_pattern = 0
    ki.aa_samples = scene.samples
    ki.adaptive_min_samples = max(4, int(math.sqrt(scene.samples)))
    ki.adaptive_step = 4
    ki.adaptive_stop_per_sample = 0
    ki.adaptive_threshold = max(0.001, 1.0 / scene.samples)
    ki.light_inv_rr_threshold = (1.0 / scene.light_sampling_threshold) if scene.light_sampling_threshold > 0 else 0.0
    ki.use_volumes = 0
    ki.max_closures = max([m.num_closures() for m in mats] + [1])
    total_bounces = scene.max_bounce + scene.transparent_max_bounce + 3 + VOLUME_BOUNDS_MAX + BSSRDF_MAX_BOUNCES
    dims = min(PRNG_BASE_NUM + total_bounces * PRNG_BOUNCE_NUM, sobol.SOBOL_MAX_DIMENSIONS)
    lut = sobol.sample_pattern_lut(dims)

    # --- background (render/background.cpp:63-118)
    kb = kd.background
    kb.surface_shader = n_shaders - 1
    kb.volume_shader = -1
    kb.transparent = 0
    kb.transparent_roughness_squared_threshold = -1.0
    kb.ao_factor = 0.0
    kb.ao_bounces_factor = 0.0
    kb.ao_distance = FLT_MAX
    kb.use_mis = 0

    # --- film (render/film.cpp device_update, combined pass only)
    kf = kd.film
    kf.exposure = 1.0
    kf.pass_flag = PASSMASK_COMBINED
    kf.light_pass_flag = 0
    kf.pass_stride = 4
    kf.use_light_pass = 0
    kf.pass_combined = 0
    kf.pass_alpha_threshold = 0.5
    kf.filter_table_offset = 0
    lookup = filter_table(scene.filter_type, scene.filter_width)

    # --- camera
    compile_camera(kd.cam, scene.camera, scene.width, scene.height)

    # --- bvh
    kd.bvh.root = root
    kd.bvh.have_motion = 0
    kd.bvh.have_curves = 0
    kd.bvh.bvh_layout = BVH_LAYOUT_BVH2
    kd.bvh.use_bvh_steps = 0
    kd.bvh.curve_subdivisions = 4
    kd.tables.beckmann_offset = 0

    arrays = {
        "__bvh_nodes": nodes.astype(np.float32),
        "__bvh_leaf_nodes": leaves.astype(np.float32),
        "__prim_tri_verts": prim_tri_verts,
        "__prim_tri_index": prim_tri_index,
        "__prim_type": prim_type,
        "__prim_visibility": prim_visibility,
        "__prim_index": prim_index,
        "__prim_object": prim_object,
        "__object_node": np.zeros(max(nobj, 1), dtype=np.uint32),
        "__objects": np.frombuffer(abi.array_bytes(kobjects), dtype=np.uint8).copy(),
        "__object_flag": object_flag,
        "__tri_shader": tri_shader,
        "__tri_vnormal": tri_vnormal,
        "__tri_vindex": tri_vindex,
        "__light_distribution": np.frombuffer(abi.array_bytes(dist), dtype=np.uint8).copy(),
        "__lights": np.frombuffer(abi.array_bytes(klights), dtype=np.uint8).copy(),
        "__svm_nodes": svm,
        "__shaders": np.frombuffer(abi.array_bytes(kshaders), dtype=np.uint8).copy(),
        "__lookup_table": lookup,
        "__sample_pattern_lut": lut,
    }
    info = {
        "triangles": ntri,
        "bvh_inner_nodes": nodes.shape[0] // 4,
        "bvh_leaves": leaves.shape[0],
        "light_triangles": nd,
        "lamps": num_lights,
        "shaders": n_shaders,
        "name": scene.name,
    }
    return DeviceScene(kd, arrays, scene.width, scene.height, scene.samples, info)


def f32bits_signed(x: float) -> int:
    return int(np.array([x], dtype=np.float32).view(np.int32)[0])


def _f3(v) -> np.ndarray:
    return np.asarray(v, dtype=np.float32)


def _safe_normalize(v: np.ndarray) -> np.ndarray:
    t = np.float32(np.sqrt(np.float32(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])))
    return (v * (np.float32(1.0) / t)).astype(np.float32) if t != 0 else v


LIGHT_TYPES = {"point": 0, "sun": 1, "area": 3, "spot": 4}


def _pack_lamp(kl, lamp: Lamp, shader_index: int) -> bool:
    """LightManager::device_update_points (render/light.cpp:722-907); returns
    whether the lamp turns on lamp MIS (light.cpp:419-427)."""
    f32 = np.float32
    shader_id = shader_index | SHADER_CAST_SHADOW | SHADER_AREA_LIGHT
    if not lamp.cast_shadow:
        shader_id &= ~SHADER_CAST_SHADOW
    kl.type = LIGHT_TYPES[lamp.kind]
    kl.samples = 1
    strength = _f3(lamp.color) * f32(lamp.strength)
    kl.strength[:] = [float(c) for c in strength]
    uni = [0.0] * 12
    co = _f3(lamp.co)
    mis = False
    if lamp.kind in ("point", "spot"):
        shader_id &= ~SHADER_AREA_LIGHT
        radius = f32(lamp.size)
        invarea = f32(1.0) / (f32(math.pi) * radius * radius) if radius > 0 else f32(1.0)
        if lamp.use_mis and radius > 0:
            shader_id |= SHADER_USE_MIS
            mis = True
        kl.co[:] = [float(c) for c in co]
        uni[0], uni[1] = float(radius), float(invarea)
        if lamp.kind == "spot":
            spot_angle = f32(math.cos(f32(lamp.spot_angle) * f32(0.5)))
            spot_smooth = (f32(1.0) - spot_angle) * f32(lamp.spot_smooth)
            d = _safe_normalize(_f3(lamp.direction))
            uni[2], uni[3] = float(spot_angle), float(spot_smooth)
            uni[4:7] = [float(c) for c in d]
    elif lamp.kind == "sun":
        shader_id &= ~SHADER_AREA_LIGHT
        angle = f32(lamp.angle) / f32(2.0)
        radius = f32(math.tan(angle))
        cosangle = f32(math.cos(angle))
        area = f32(math.pi) * radius * radius
        invarea = f32(1.0) / area if area > 0 else f32(1.0)
        d = _safe_normalize(_f3(lamp.direction))
        if lamp.use_mis and area > 0:
            shader_id |= SHADER_USE_MIS
            mis = True
        kl.co[:] = [float(c) for c in d]
        uni[0], uni[1], uni[2] = float(radius), float(cosangle), float(invarea)
    elif lamp.kind == "area":
        axisu = (_f3(lamp.axisu) * (f32(lamp.sizeu) * f32(lamp.size))).astype(f32)
        axisv = (_f3(lamp.axisv) * (f32(lamp.sizev) * f32(lamp.size))).astype(f32)
        lu = f32(np.sqrt(np.float32(np.dot(axisu, axisu))))
        lv = f32(np.sqrt(np.float32(np.dot(axisv, axisv))))
        area = lu * lv
        if lamp.round:
            area = area * f32(-math.pi / 4)
        invarea = f32(1.0) / area if area != 0 else f32(1.0)
        d = _safe_normalize(_f3(lamp.direction))
        if lamp.use_mis and area != 0:
            shader_id |= SHADER_USE_MIS
        mis = lamp.use_mis
        kl.co[:] = [float(c) for c in co]
        uni[0:3] = [float(c) for c in axisu]
        uni[3] = float(invarea)
        uni[4:7] = [float(c) for c in axisv]
        uni[8:11] = [float(c) for c in d]
    else:
        raise ValueError(f"unsupported lamp kind {lamp.kind}")
    kl.uni[:] = uni
    kl.shader_id = int(np.array([shader_id], dtype=np.uint32).view(np.int32)[0])
    kl.max_bounces = float(lamp.max_bounces)
    kl.random = 0.0
    ident = np.eye(4)[:3]
    abi.set_transform(kl.tfm, ident)
    abi.set_transform(kl.itfm, ident)
    return mis


def _vertex_normals(v: np.ndarray, t: np.ndarray) -> np.ndarray:
    n = np.zeros_like(v, dtype=np.float64)
    fn = np.cross(v[t[:, 1]] - v[t[:, 0]], v[t[:, 2]] - v[t[:, 0]])
    for k in range(3):
        np.add.at(n, t[:, k], fn)
    ln = np.linalg.norm(n, axis=1, keepdims=True)
    ln[ln == 0] = 1.0
    return (n / ln).astype(np.float32)


# element counts as CPUDevice::global_alloc passes them (mem.data_size)
ELEMENT_BYTES = {
    "__bvh_nodes": 16, "__bvh_leaf_nodes": 16, "__prim_tri_verts": 16, "__prim_tri_index": 4,
    "__prim_type": 4, "__prim_visibility": 4, "__prim_index": 4, "__prim_object": 4,
    "__object_node": 4, "__objects": ctypes.sizeof(abi.KernelObject), "__object_flag": 4,
    "__tri_shader": 4, "__tri_vnormal": 16, "__tri_vindex": 16,
    "__light_distribution": ctypes.sizeof(abi.KernelLightDistribution),
    "__lights": ctypes.sizeof(abi.KernelLight), "__svm_nodes": 16,
    "__shaders": ctypes.sizeof(abi.KernelShader), "__lookup_table": 4, "__sample_pattern_lut": 4,
}
