"""Procedural stand-in scenes for BASELINE.json's configs.

The named .blend benchmarks are not available offline, so each config is a
procedural scene with the config's resolution and sample count:
  cornell_box()   CB : 256x256, 32 spp, diffuse + one emissive quad
  bmw27_standin() BMW: 1280x720, 128 spp, a tessellated car-like assembly with
                       car paint (diffuse/glossy mix), chrome, glass, tyres,
                       a studio floor and two emissive panels
Generator seeds are fixed (0x5EED + config index).
"""
from __future__ import annotations

import math

import numpy as np

from . import scene as sc


def _quad(p0, p1, p2, p3):
    v = np.array([p0, p1, p2, p3], dtype=np.float32)
    t = np.array([[0, 1, 2], [0, 2, 3]], dtype=np.int64)
    return v, t


def _box(center, size, rot_y=0.0):
    cx, cy, cz = center
    sx, sy, sz = (s * 0.5 for s in size)
    corners = np.array(
        [[-sx, -sy, -sz], [sx, -sy, -sz], [sx, sy, -sz], [-sx, sy, -sz],
         [-sx, -sy, sz], [sx, -sy, sz], [sx, sy, sz], [-sx, sy, sz]], dtype=np.float64)
    c, s = math.cos(rot_y), math.sin(rot_y)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    corners = corners @ R.T + np.array([cx, cy, cz])
    faces = [[0, 3, 2, 1], [4, 5, 6, 7], [0, 1, 5, 4], [3, 7, 6, 2], [0, 4, 7, 3], [1, 2, 6, 5]]
    v, t = [], []
    for f in faces:
        base = len(v)
        v.extend(corners[f])
        t.extend([[base, base + 1, base + 2], [base, base + 2, base + 3]])
    return np.array(v, dtype=np.float32), np.array(t, dtype=np.int64)


def _grid_tris(nu, nv, wrap_u=True):
    """Triangles of a (nu x nv) vertex grid, u optionally wrapping."""
    t = []
    uu = nu if wrap_u else nu - 1
    for j in range(nv - 1):
        for i in range(uu):
            i1 = (i + 1) % nu
            a, b, c, d = j * nu + i, j * nu + i1, (j + 1) * nu + i1, (j + 1) * nu + i
            t.append([a, b, c])
            t.append([a, c, d])
    return np.array(t, dtype=np.int64)


def _ellipsoid(center, radii, nu, nv, exponent=1.0):
    """Superellipsoid-ish body: exponent < 1 makes it boxier."""
    u = np.linspace(0, 2 * math.pi, nu, endpoint=False)
    v = np.linspace(-math.pi / 2, math.pi / 2, nv)
    U, V = np.meshgrid(u, v)

    def sgnpow(x, e):
        return np.sign(x) * np.abs(x) ** e

    x = radii[0] * sgnpow(np.cos(V), exponent) * sgnpow(np.cos(U), exponent)
    y = radii[1] * sgnpow(np.sin(V), exponent)
    z = radii[2] * sgnpow(np.cos(V), exponent) * sgnpow(np.sin(U), exponent)
    verts = np.stack([x, y, z], axis=-1).reshape(-1, 3) + np.asarray(center)
    return verts.astype(np.float32), _grid_tris(nu, nv)


def _torus(center, R, r, nu, nv, axis="z"):
    u = np.linspace(0, 2 * math.pi, nu, endpoint=False)
    v = np.linspace(0, 2 * math.pi, nv, endpoint=False)
    U, V = np.meshgrid(u, v)
    x = (R + r * np.cos(V)) * np.cos(U)
    y = (R + r * np.cos(V)) * np.sin(U)
    z = r * np.sin(V)
    p = np.stack([x, y, z], axis=-1).reshape(-1, 3)
    if axis == "z":
        p = p[:, [0, 1, 2]]
    verts = p + np.asarray(center)
    t = []
    for j in range(nv):
        j1 = (j + 1) % nv
        for i in range(nu):
            i1 = (i + 1) % nu
            a, b, c, d = j * nu + i, j * nu + i1, j1 * nu + i1, j1 * nu + i
            t.append([a, b, c])
            t.append([a, c, d])
    return verts.astype(np.float32), np.array(t, dtype=np.int64)


def _disk(center, radius, n, axis="z"):
    ang = np.linspace(0, 2 * math.pi, n, endpoint=False)
    ring = np.stack([radius * np.cos(ang), radius * np.sin(ang), np.zeros(n)], axis=-1)
    verts = np.concatenate([[[0, 0, 0]], ring]) + np.asarray(center)
    t = np.array([[0, 1 + i, 1 + (i + 1) % n] for i in range(n)], dtype=np.int64)
    return verts.astype(np.float32), t


def cornell_box(width=256, height=256, samples=32) -> sc.Scene:
    """Classic Cornell box (555 units), SURVEY.md §8(d) config CB."""
    white = sc.diffuse((0.73, 0.73, 0.73))
    red = sc.diffuse((0.65, 0.05, 0.05))
    green = sc.diffuse((0.12, 0.45, 0.15))
    light = sc.emission((1.0, 0.85, 0.6), 40.0)
    materials = [white, red, green, light]
    meshes = []
    L = 555.0
    meshes.append(sc.Mesh(*_quad((0, 0, 0), (L, 0, 0), (L, 0, L), (0, 0, L)), shader=0))  # floor
    meshes.append(sc.Mesh(*_quad((0, L, 0), (0, L, L), (L, L, L), (L, L, 0)), shader=0))  # ceiling
    meshes.append(sc.Mesh(*_quad((0, 0, L), (L, 0, L), (L, L, L), (0, L, L)), shader=0))  # back
    meshes.append(sc.Mesh(*_quad((L, 0, 0), (L, L, 0), (L, L, L), (L, 0, L)), shader=1))  # left (red)
    meshes.append(sc.Mesh(*_quad((0, 0, 0), (0, 0, L), (0, L, L), (0, L, 0)), shader=2))  # right (green)
    meshes.append(sc.Mesh(*_box((185.0, 82.5, 169.0), (165, 165, 165), -0.314), shader=0))
    meshes.append(sc.Mesh(*_box((368.0, 165.0, 351.0), (165, 330, 165), 0.3), shader=0))
    meshes.append(sc.Mesh(*_quad((213, L - 1, 227), (343, L - 1, 227), (343, L - 1, 332), (213, L - 1, 332)),
                          shader=3))
    cam = sc.Camera(eye=(278.0, 273.0, -800.0), target=(278.0, 273.0, 0.0), up=(0.0, 1.0, 0.0),
                    fov=math.radians(39.3), nearclip=0.1, farclip=1e5)
    return sc.Scene(width, height, cam, meshes, materials, world_color=(0.0, 0.0, 0.0),
                    world_strength=0.0, samples=samples, name="cornell_box")


def cornell_adaptive(width=64, height=64, samples=64, threshold=0.02) -> sc.Scene:
    """Cornell box with adaptive sampling (Film use_adaptive_sampling): the
    walls converge and stop early, the penumbrae keep sampling."""
    scene = cornell_box(width, height, samples)
    scene.adaptive_sampling = True
    scene.adaptive_threshold = threshold
    scene.name = "cornell_adaptive"
    return scene


def cornell_lamps(width=64, height=64, samples=16) -> sc.Scene:
    """Cornell box lit by every lamp kind the device implements: a sphere point
    lamp, a spot lamp, a rectangular and a round area lamp, a sun, plus the
    emissive ceiling quad (mesh light and lamps share the light distribution)."""
    scene = cornell_box(width, height, samples)
    L = 555.0
    scene.lamps = [
        sc.Lamp("point", co=(140.0, 420.0, 200.0), size=25.0, color=(1.0, 0.6, 0.3), strength=4.0e6),
        sc.Lamp("spot", co=(420.0, 500.0, 120.0), direction=(-0.3, -1.0, 0.4), size=10.0,
                spot_angle=math.radians(50.0), spot_smooth=0.3, color=(0.4, 0.7, 1.0), strength=6.0e6),
        sc.Lamp("area", co=(278.0, L - 2.0, 470.0), direction=(0.0, -1.0, 0.0), axisu=(1.0, 0.0, 0.0),
                axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=160.0, sizev=60.0, color=(1.0, 1.0, 1.0),
                strength=3.0e5),
        sc.Lamp("area", co=(30.0, 300.0, 300.0), direction=(1.0, 0.0, 0.0), axisu=(0.0, 1.0, 0.0),
                axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=80.0, sizev=80.0, round=True, color=(0.9, 1.0, 0.8),
                strength=2.0e5),
        sc.Lamp("sun", direction=(0.2, -1.0, 0.6), angle=math.radians(5.0), color=(1.0, 0.95, 0.9),
                strength=2.0),
    ]
    scene.name = "cornell_lamps"
    return scene


def emission_nodes(width=48, height=48, samples=8) -> sc.Scene:
    """Emitters whose emission comes from shader nodes (direct_emissive_eval's
    non-constant branch, kernel_emission.h:54-88): a ceiling mesh light with a
    checker-textured colour on its generated coordinates, a point lamp (with
    lamp MIS) whose strength is a Light Falloff node's Linear output (it reads
    the sample distance), a spot lamp with a Light Path-dependent strength, and
    a constant sun for contrast."""
    from . import nodes

    scene = cornell_box(width, height, samples)
    ck = nodes.checker(color1=(1.0, 0.85, 0.6), color2=(0.3, 0.3, 0.9), scale=3.0)["Color"]
    scene.materials[3] = sc.emission(ck, 40.0)
    falloff = nodes.light_falloff(strength=1.0, smooth=50.0)["Linear"]
    diffuse_ray = nodes.light_path()["Is Diffuse Ray"]
    spot_strength = nodes.math("add", diffuse_ray, 0.5)
    scene.lamps = [
        sc.Lamp("point", co=(140.0, 420.0, 200.0), size=25.0, color=(1.0, 0.6, 0.3), strength=1.0e4,
                shader=sc.emission((1.0, 1.0, 1.0), falloff)),
        sc.Lamp("spot", co=(420.0, 500.0, 120.0), direction=(-0.3, -1.0, 0.4), size=10.0, use_mis=False,
                spot_angle=math.radians(50.0), spot_smooth=0.3, color=(0.4, 0.7, 1.0), strength=6.0e6,
                shader=sc.emission((1.0, 1.0, 1.0), spot_strength)),
        sc.Lamp("sun", direction=(0.2, -1.0, 0.6), angle=math.radians(5.0), color=(1.0, 0.95, 0.9), strength=2.0),
    ]
    scene.name = "emission_nodes"
    return scene


def ies_lamps(width=48, height=48, samples=8, ies_files=()) -> sc.Scene:
    """Point and spot lamps whose strength is an IES Texture node (svm_ies.h)
    on the texture-coordinate normal (the node's default LINK_TEXTURE_NORMAL
    input): `ies_files` are the texts of two IES photometric files (a one-
    quadrant type C downlight, a half-plane type C file with a TILT block);
    the second file is also used by the spot lamp, so both lamps share its
    __ies slot."""
    from . import nodes

    scene = cornell_box(width, height, samples)
    scene.materials[3] = sc.emission((1.0, 1.0, 1.0), 2.0)
    normal = nodes.tex_coord()["Normal"]
    a = nodes.ies_texture(normal, ies_files[0], strength=1.0)["Fac"]
    b = nodes.ies_texture(normal, ies_files[1], strength=nodes.math("add", nodes.light_path()["Is Diffuse Ray"], 0.5))
    scene.lamps = [
        sc.Lamp("point", co=(180.0, 480.0, 250.0), size=15.0, color=(1.0, 0.8, 0.6), strength=3.0e3,
                shader=sc.emission((1.0, 1.0, 1.0), a)),
        sc.Lamp("point", co=(400.0, 300.0, 150.0), size=10.0, color=(0.6, 0.8, 1.0), strength=2.0e3,
                shader=sc.emission((1.0, 1.0, 1.0), b["Fac"])),
        sc.Lamp("spot", co=(300.0, 500.0, 400.0), direction=(-0.2, -1.0, -0.3), size=10.0,
                spot_angle=math.radians(70.0), spot_smooth=0.2, color=(1.0, 1.0, 1.0), strength=1.0e5,
                shader=sc.emission((1.0, 1.0, 1.0), nodes.ies_texture(normal, ies_files[1], 2.0)["Fac"])),
    ]
    scene.name = "ies_lamps"
    return scene


def shading_spectral(width=40, height=40, samples=8) -> sc.Scene:
    """Wavelength and Blackbody nodes (svm_wavelength.h, svm_blackbody.h): the
    back wall's colour sweeps 350-800 nm over its object X coordinate (both
    ends outside the table, where the node returns black), the floor's
    sweeps the same range through Y; a sphere emits the blackbody colour of
    a temperature rising from 700 K to 13000 K over the sphere (every branch
    of the piecewise fit and both clamps)."""
    from . import nodes

    scene = cornell_box(width, height, samples)
    P = nodes.separate_xyz(nodes.tex_coord()["Object"])
    lam_x = nodes.math("add", nodes.math("multiply", P["X"], 450.0 / 555.0), 350.0)
    lam_z = nodes.math("add", nodes.math("multiply", P["Z"], 450.0 / 555.0), 350.0)
    scene.materials[0] = sc.diffuse(nodes.wavelength(lam_x))
    scene.materials[1] = sc.diffuse(nodes.wavelength(lam_z))
    temp = nodes.math("add", nodes.math("multiply", P["Y"], 12300.0 / 140.0), 700.0 - 130.0 * 12300.0 / 140.0)
    scene.materials.append(sc.emission(nodes.blackbody(temp), 3.0))
    scene.meshes.append(sc.Mesh(*_ellipsoid((278.0, 200.0, 250.0), (70.0, 70.0, 70.0), 20, 12),
                                shader=len(scene.materials) - 1))
    scene.name = "shading_spectral"
    return scene


def cornell_camera(kind: str, width=64, height=64, samples=16) -> sc.Scene:
    """Cornell box through the camera models of kernel_camera.h: "dof"
    (perspective, hexagonal anamorphic aperture), "ortho" (orthographic with a
    disk aperture), and the panoramas "equirect", "fisheye_equidistant",
    "fisheye_equisolid" (with depth of field) and "mirrorball" from inside the
    box."""
    scene = cornell_box(width, height, samples)
    cam = scene.camera
    inside = dict(eye=(278.0, 273.0, 200.0), target=(278.0, 273.0, 555.0), up=(0.0, 1.0, 0.0), nearclip=0.1,
                  farclip=1e5)
    if kind == "dof":
        cam.aperturesize = 25.0
        cam.focaldistance = 950.0
        cam.blades = 6
        cam.bladesrotation = 0.3
        cam.aperture_ratio = 1.5
    elif kind == "ortho":
        cam.type = "orthographic"
        cam.ortho_scale = 300.0
        cam.aperturesize = 8.0
        cam.focaldistance = 1000.0
    else:
        scene.camera = sc.Camera(**inside)
        cam = scene.camera
        cam.type = "panorama"
        if kind == "equirect":
            cam.panorama_type = "equirectangular"
            cam.latitude_min, cam.latitude_max = -1.2, 1.3
            cam.longitude_min, cam.longitude_max = -2.5, 2.8
        elif kind == "fisheye_equidistant":
            cam.panorama_type = "fisheye_equidistant"
            cam.fisheye_fov = 3.0
        elif kind == "fisheye_equisolid":
            cam.panorama_type = "fisheye_equisolid"
            cam.fisheye_lens = 9.0
            cam.fisheye_fov = 3.1
            cam.aperturesize = 3.0
            cam.focaldistance = 300.0
        elif kind == "mirrorball":
            cam.panorama_type = "mirrorball"
        else:
            raise ValueError(kind)
    scene.name = "cornell_camera_" + kind
    return scene


def _tfm(translate=(0.0, 0.0, 0.0), rot_y=0.0, scale=(1.0, 1.0, 1.0), rot_x=0.0) -> np.ndarray:
    """3x4 object-to-world transform: translate * rot_y * rot_x * scale."""
    c, s = math.cos(rot_y), math.sin(rot_y)
    ry = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    c, s = math.cos(rot_x), math.sin(rot_x)
    rx = np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    m = np.zeros((3, 4))
    m[:, :3] = ry @ rx @ np.diag(scale)
    m[:, 3] = translate
    return m


def cornell_instanced(width=64, height=64, samples=16) -> sc.Scene:
    """Cornell box whose props are instances (two-level BVH): one box geometry
    placed three times (rotated, non-uniformly scaled), one emissive quad
    geometry placed twice (instanced mesh lights), and a single-use instance
    whose transform the host applies."""
    scene = cornell_box(width, height, samples)
    scene.meshes = scene.meshes[:5]  # walls only
    glossy = sc.glossy((0.8, 0.75, 0.6), 0.2)
    scene.materials = scene.materials + [glossy]
    box_v, box_t = _box((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
    box = sc.Mesh(box_v, box_t, shader=0)
    scene.instances = [
        sc.Instance(box, _tfm((185.0, 82.5, 169.0), -0.314, (165.0, 165.0, 165.0))),
        sc.Instance(box, _tfm((368.0, 165.0, 351.0), 0.3, (165.0, 330.0, 165.0))),
        sc.Instance(box, _tfm((420.0, 40.0, 120.0), 0.9, (60.0, 80.0, 40.0), rot_x=0.4)),
    ]
    lamp_v, lamp_t = _quad((-0.5, 0.0, -0.5), (-0.5, 0.0, 0.5), (0.5, 0.0, 0.5), (0.5, 0.0, -0.5))
    lamp = sc.Mesh(lamp_v, lamp_t, shader=3)
    scene.instances += [
        sc.Instance(lamp, _tfm((230.0, 554.0, 280.0), 0.0, (90.0, 1.0, 90.0))),
        sc.Instance(lamp, _tfm((340.0, 554.0, 260.0), 0.5, (60.0, 1.0, 110.0))),
    ]
    ev, et = _ellipsoid((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), 24, 12)
    scene.instances.append(sc.Instance(sc.Mesh(ev, et, shader=4, smooth=True), _tfm((150.0, 300.0, 380.0), 0.2,
                                                                                  (60.0, 45.0, 60.0))))
    scene.name = "cornell_instanced"
    return scene


def cornell_displace(width=48, height=48, samples=8) -> sc.Scene:
    """Instanced Cornell box whose materials carry true-displacement programs
    (SHADER_EVAL_DISPLACE, MeshManager::displace): a scalar Displacement node
    in object space on the walls and instanced boxes (instanced ones with
    object-space transforms), a world-space Displacement along a linked normal
    on the red wall, and a Vector Displacement node in world space on the
    smooth glossy ellipsoid."""
    import dataclasses

    from . import nodes as nd

    scene = cornell_instanced(width, height, samples)
    pos = nd.separate_xyz(nd.geometry()["Position"])
    h = nd.math("sine", nd.math("multiply", pos["X"], 0.05))
    h2 = nd.math("sine", nd.math("multiply", pos["Y"], 0.03))
    mats = list(scene.materials)
    mats[0] = dataclasses.replace(mats[0], displacement=nd.displacement(h, 0.5, 3.0, space="object"))
    mats[1] = dataclasses.replace(mats[1], displacement=nd.displacement(
        h2, 0.25, 2.0, normal=nd.geometry()["Normal"], space="world"))
    mats[4] = dataclasses.replace(mats[4], displacement=nd.vector_displacement(
        nd.combine_xyz(h2, 0.25, h), 0.1, 2.0, space="world"))
    scene.materials = mats
    scene.name = "cornell_displace"
    return scene


def bmw27_standin(width=1280, height=720, samples=128, detail=1.0, materials="basic") -> sc.Scene:
    """BMW27-class stand-in (SURVEY.md §8(d) config BMW): ~0.7M triangles at
    detail=1.0, glossy / glass / diffuse materials, two emissive studio panels,
    dim constant world.  materials="production" swaps in the node setups a
    Blender user would give the same objects (the extended shading kernel):
    Principled BSDFs with Blender's default multiscatter GGX (clear-coated
    paint, rough glass, bump-mapped tyres from a noise height, rims with
    noise-driven roughness) and a checker / noise floor."""
    rng = np.random.default_rng(0x5EED + 1)
    if materials == "production":
        from . import nodes as nd

        grain = nd.noise_texture(scale=40.0, detail=3.0)["Fac"]
        paint = sc.principled("multiscatter", base_color=(0.55, 0.06, 0.04), metallic=0.3, specular=0.5, roughness=0.25,
                              clearcoat=0.8, clearcoat_roughness=0.05)
        chrome = sc.principled("multiscatter", base_color=(0.85, 0.85, 0.88), metallic=1.0, specular=0.5, roughness=0.08)
        glass_m = sc.principled("multiscatter", base_color=(0.95, 0.97, 1.0), transmission=1.0, roughness=0.1,
                                ior=1.45)
        tyre = sc.principled("multiscatter", base_color=(0.03, 0.03, 0.03), roughness=0.7, specular=0.5,
                             normal=nd.bump(grain, strength=0.4, distance=0.02))
        rim = sc.principled("multiscatter", base_color=(0.7, 0.7, 0.72), metallic=1.0, specular=0.5,
                            roughness=nd.map_range(grain, 0.0, 1.0, 0.15, 0.45))
        ck = nd.checker(nd.tex_coord()["Object"], (0.5, 0.5, 0.5), (0.35, 0.35, 0.37), 0.5)["Color"]
        floor = sc.principled("multiscatter", base_color=ck, roughness=0.6, specular=0.5)
        panel = sc.emission((1.0, 0.97, 0.92), 6.0)
        plastic = sc.principled("multiscatter", base_color=(0.08, 0.08, 0.09), roughness=0.35, specular=0.5)
    else:
        paint = sc.mix(0.25, sc.diffuse((0.55, 0.06, 0.04)), sc.glossy((0.9, 0.9, 0.9), 0.15))
        chrome = sc.glossy((0.85, 0.85, 0.88), 0.08)
        glass_m = sc.glass((0.95, 0.97, 1.0), 0.0, 1.45)
        tyre = sc.diffuse((0.03, 0.03, 0.03))
        rim = sc.glossy((0.7, 0.7, 0.72), 0.3)
        floor = sc.diffuse((0.45, 0.45, 0.45))
        panel = sc.emission((1.0, 0.97, 0.92), 6.0)
        plastic = sc.mix(0.5, sc.diffuse((0.08, 0.08, 0.09)), sc.glossy((0.5, 0.5, 0.5), 0.35))
    materials = [paint, chrome, glass_m, tyre, rim, floor, panel, plastic]
    d = detail
    meshes = []
    # car body: boxy superellipsoid hull + cabin
    meshes.append(sc.Mesh(*_ellipsoid((0, 0.62, 0), (2.2, 0.45, 0.95), int(768 * d), int(320 * d), 0.55),
                          shader=0, smooth=True))
    meshes.append(sc.Mesh(*_ellipsoid((-0.25, 1.05, 0), (1.15, 0.42, 0.8), int(384 * d), int(160 * d), 0.7),
                          shader=2, smooth=True))
    # wheels: tyre tori + rim disks + spokes
    for wx in (-1.35, 1.35):
        for wz in (-0.92, 0.92):
            v, t = _torus((0, 0, 0), 0.33, 0.13, int(192 * d), int(64 * d))
            v = v.copy()
            v += np.array([wx, 0.42, wz], dtype=np.float32)
            meshes.append(sc.Mesh(v, t, shader=3, smooth=True))
            zs = wz + (0.06 if wz > 0 else -0.06)
            v, t = _disk((wx, 0.42, zs), 0.27, int(96 * d))
            meshes.append(sc.Mesh(v, t, shader=4))
            for k in range(10):
                a = 2 * math.pi * k / 10
                bv, bt = _box((wx + 0.13 * math.cos(a), 0.42 + 0.13 * math.sin(a), zs), (0.2, 0.03, 0.03), 0.0)
                meshes.append(sc.Mesh(bv, bt, shader=1))
    # grille / detail: many small chrome and plastic boxes (instancing-free detail)
    n_detail = int(2500 * d)
    for k in range(n_detail):
        x = -2.35 + 0.02 * rng.standard_normal()
        y = 0.35 + 0.35 * rng.random()
        z = -0.7 + 1.4 * rng.random()
        bv, bt = _box((x, y, z), (0.05, 0.02 + 0.02 * rng.random(), 0.02), float(rng.random()))
        meshes.append(sc.Mesh(bv, bt, shader=1 if k % 3 else 7))
    # mirrors, spoiler, bumpers
    meshes.append(sc.Mesh(*_box((2.15, 0.38, 0), (0.2, 0.18, 1.7)), shader=7))
    meshes.append(sc.Mesh(*_box((-2.15, 0.38, 0), (0.2, 0.18, 1.7)), shader=7))
    meshes.append(sc.Mesh(*_box((1.9, 1.05, 0), (0.12, 0.05, 1.5), 0.0), shader=0))
    for z in (-0.95, 0.95):
        meshes.append(sc.Mesh(*_ellipsoid((0.35, 1.0, z), (0.1, 0.06, 0.05), int(64 * d), int(32 * d)), shader=1,
                              smooth=True))
    # studio floor (tessellated) and two emissive panels
    n = int(64 * d) + 2
    xs = np.linspace(-12, 12, n)
    zs = np.linspace(-12, 12, n)
    X, Z = np.meshgrid(xs, zs)
    fv = np.stack([X, np.zeros_like(X), Z], axis=-1).reshape(-1, 3).astype(np.float32)
    meshes.append(sc.Mesh(fv, _grid_tris(n, n, wrap_u=False)[:, [0, 2, 1]], shader=5))
    meshes.append(sc.Mesh(*_quad((-3, 4.5, -2.5), (3, 4.5, -2.5), (3, 4.5, 2.5), (-3, 4.5, 2.5)), shader=6))
    meshes.append(sc.Mesh(*_quad((5.5, 0.5, -3), (5.5, 4.0, -3), (5.5, 4.0, 3), (5.5, 0.5, 3)), shader=6))
    cam = sc.Camera(eye=(5.2, 2.3, 4.6), target=(0.0, 0.6, 0.0), up=(0.0, 1.0, 0.0),
                    fov=math.radians(38.0), nearclip=0.1, farclip=1000.0)
    return sc.Scene(width, height, cam, meshes, materials, world_color=(0.18, 0.2, 0.24),
                    world_strength=0.6, samples=samples, filter_type="blackman_harris",
                    filter_width=1.5, name="bmw27_standin" if materials == "basic" else "bmw27_production")


def _cylinder(radius, height, n, caps=True):
    """Cylinder along +y from y=0 to y=height (object space)."""
    ang = np.linspace(0, 2 * math.pi, n, endpoint=False)
    ring = np.stack([radius * np.cos(ang), np.zeros(n), radius * np.sin(ang)], axis=-1)
    verts = np.concatenate([ring, ring + np.array([0.0, height, 0.0])])
    t = []
    for i in range(n):
        i1 = (i + 1) % n
        t += [[i, n + i1, i1], [i, n + i, n + i1]]
    if caps:
        base = len(verts)
        verts = np.concatenate([verts, [[0.0, 0.0, 0.0], [0.0, height, 0.0]]])
        for i in range(n):
            i1 = (i + 1) % n
            t += [[base, i, i1], [base + 1, n + i1, n + i]]
    return verts.astype(np.float32), np.array(t, dtype=np.int64)


def _merge(parts, shaders):
    """One mesh from several (verts, tris) parts with a material per part."""
    vs, ts, sh = [], [], []
    base = 0
    for (v, t), s in zip(parts, shaders):
        vs.append(v)
        ts.append(t + base)
        sh.append(np.full(len(t), s, dtype=np.int64))
        base += len(v)
    return np.concatenate(vs).astype(np.float32), np.concatenate(ts), np.concatenate(sh)


def barbershop_standin(width=1920, height=1080, samples=512, detail=1.0) -> sc.Scene:
    """Barbershop-class interior stand-in (SURVEY.md §8(d) config BBS): a room
    furnished with INSTANCED props (barber chairs, bottles on shelves, ceiling
    lamp fittings) lit by point and area lamps plus emissive strips; glossy
    mirrors, glass bottles, chrome, tiled floor.  Generator seed 0x5EED + 3."""
    rng = np.random.default_rng(0x5EED + 3)
    d = detail
    wall = sc.diffuse((0.62, 0.58, 0.5))
    tile_a = sc.mix(0.3, sc.diffuse((0.85, 0.85, 0.82)), sc.glossy((0.9, 0.9, 0.9), 0.1))
    tile_b = sc.mix(0.3, sc.diffuse((0.08, 0.08, 0.09)), sc.glossy((0.9, 0.9, 0.9), 0.1))
    mirror = sc.glossy((0.92, 0.92, 0.92), 0.0)
    chrome = sc.glossy((0.8, 0.8, 0.82), 0.12)
    leather = sc.mix(0.2, sc.diffuse((0.45, 0.06, 0.05)), sc.glossy((0.6, 0.6, 0.6), 0.3))
    wood = sc.mix(0.15, sc.diffuse((0.35, 0.2, 0.1)), sc.glossy((0.5, 0.5, 0.5), 0.25))
    bottle = sc.glass((0.7, 0.9, 0.8), 0.05, 1.5)
    strip = sc.emission((1.0, 0.9, 0.75), 3.0)
    ceiling = sc.diffuse((0.8, 0.8, 0.78))
    materials = [wall, tile_a, tile_b, mirror, chrome, leather, wood, bottle, strip, ceiling]
    W_, H_, D_ = 8.0, 3.2, 6.0
    meshes = []
    # tiled floor: n x n checker of quads (geometry, no textures)
    n = max(4, int(24 * d))
    fv, ft, fs = [], [], []
    for j in range(n):
        for i in range(n):
            x0, x1 = W_ * i / n, W_ * (i + 1) / n
            z0, z1 = D_ * j / n, D_ * (j + 1) / n
            base = len(fv)
            fv += [(x0, 0, z0), (x0, 0, z1), (x1, 0, z1), (x1, 0, z0)]
            ft += [[base, base + 1, base + 2], [base, base + 2, base + 3]]
            fs += [1 + (i + j) % 2] * 2
    meshes.append(sc.Mesh(np.array(fv, np.float32), np.array(ft), shader=np.array(fs)))
    meshes.append(sc.Mesh(*_quad((0, H_, 0), (W_, H_, 0), (W_, H_, D_), (0, H_, D_)), shader=9))  # ceiling
    meshes.append(sc.Mesh(*_quad((0, 0, D_), (W_, 0, D_), (W_, H_, D_), (0, H_, D_)), shader=0))  # back
    meshes.append(sc.Mesh(*_quad((0, 0, 0), (0, 0, D_), (0, H_, D_), (0, H_, 0)), shader=0))  # left
    meshes.append(sc.Mesh(*_quad((W_, 0, 0), (W_, H_, 0), (W_, H_, D_), (W_, 0, D_)), shader=0))  # right
    meshes.append(sc.Mesh(*_quad((0, 0, 0), (W_, 0, 0), (W_, H_, 0), (0, H_, 0)), shader=0))  # front (behind camera)
    # mirrors along the back wall, counter below them, emissive strips above
    for k in range(4):
        x = 1.0 + 1.8 * k
        meshes.append(sc.Mesh(*_quad((x, 1.1, D_ - 0.02), (x + 1.3, 1.1, D_ - 0.02), (x + 1.3, 2.3, D_ - 0.02),
                                     (x, 2.3, D_ - 0.02)), shader=3))
        meshes.append(sc.Mesh(*_quad((x, 2.45, D_ - 0.05), (x + 1.3, 2.45, D_ - 0.05), (x + 1.3, 2.55, D_ - 0.05),
                                     (x, 2.55, D_ - 0.05)), shader=8))
    meshes.append(sc.Mesh(*_box((W_ / 2, 0.45, D_ - 0.35), (W_ - 0.6, 0.9, 0.6)), shader=6))
    # barber chair (one geometry, instanced 4 times): base pole, seat, back, arms, footrest
    m = max(12, int(96 * d))
    cv, ct, cs = _merge([
        _cylinder(0.28, 0.05, m),
        _cylinder(0.06, 0.45, m // 2),
        _ellipsoid((0, 0.55, 0), (0.3, 0.1, 0.28), m, m // 2),
        _box((0, 0.95, -0.27), (0.5, 0.7, 0.1), 0.0),
        _box((-0.3, 0.7, 0.0), (0.08, 0.06, 0.5), 0.0),
        _box((0.3, 0.7, 0.0), (0.08, 0.06, 0.5), 0.0),
        _torus((0, 0, 0), 0.2, 0.025, m, m // 4),
    ], [4, 4, 5, 5, 4, 4, 4])
    # torus lies in xy; move it to a footrest in front of the chair
    chair = sc.Mesh(cv, ct, shader=cs, smooth=False)
    # bottle (instanced on the shelves): body + neck
    bv, bt, bs = _merge([_cylinder(0.04, 0.18, m // 2), _cylinder(0.015, 0.08, m // 4)], [7, 7])
    bv = bv.copy()
    bv[len(_cylinder(0.04, 0.18, m // 2)[0]):, 1] += 0.18
    bottle_mesh = sc.Mesh(bv, bt, shader=bs)
    # lamp fitting (instanced): a chrome shade
    lv, lt = _ellipsoid((0, 0, 0), (0.18, 0.1, 0.18), m, m // 2)
    lamp_mesh = sc.Mesh(lv, lt, shader=4, smooth=True)
    instances = []
    for k in range(4):
        instances.append(sc.Instance(chair, _tfm((1.65 + 1.8 * k, 0.0, D_ - 1.6), math.pi + 0.15 * (k - 1.5))))
    n_bottles = max(8, int(180 * d))
    for k in range(n_bottles):
        shelf = k % 3
        x = 0.6 + (W_ - 1.2) * (k // 3) / max(1, n_bottles // 3) + 0.03 * rng.standard_normal()
        y = 1.0 + 0.0 * shelf if shelf == 0 else (0.9 + 0.0)
        y = 0.9 if shelf == 0 else (2.65 if shelf == 1 else 0.9)
        z = D_ - 0.25 - 0.12 * shelf + 0.02 * rng.standard_normal()
        s = 0.8 + 0.5 * rng.random()
        instances.append(sc.Instance(bottle_mesh, _tfm((x, y, z), float(rng.random() * 6.28), (s, s * (0.8 + 0.6 * rng.random()), s))))
    lamps = []
    for k in range(6):
        x = 1.0 + (W_ - 2.0) * (k % 3) / 2.0
        z = 1.5 + 2.5 * (k // 3)
        instances.append(sc.Instance(lamp_mesh, _tfm((x, H_ - 0.25, z), 0.0)))
        lamps.append(sc.Lamp("point", co=(x, H_ - 0.45, z), size=0.06, color=(1.0, 0.85, 0.65), strength=25.0))
    lamps.append(sc.Lamp("area", co=(W_ / 2, H_ - 0.01, D_ / 2), direction=(0.0, -1.0, 0.0), axisu=(1.0, 0.0, 0.0),
                         axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=2.0, sizev=1.0, color=(0.9, 0.95, 1.0),
                         strength=30.0))
    lamps.append(sc.Lamp("area", co=(0.02, 1.6, 2.0), direction=(1.0, 0.0, 0.0), axisu=(0.0, 1.0, 0.0),
                         axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=1.2, sizev=2.0, color=(1.0, 0.95, 0.85),
                         strength=20.0))
    cam = sc.Camera(eye=(W_ * 0.5, 1.55, 0.35), target=(W_ * 0.55, 1.2, D_), up=(0.0, 1.0, 0.0),
                    fov=math.radians(60.0), nearclip=0.05, farclip=100.0)
    return sc.Scene(width, height, cam, meshes, materials, world_color=(0.0, 0.0, 0.0), world_strength=0.0,
                    samples=samples, filter_type="blackman_harris", filter_width=1.5, lamps=lamps,
                    instances=instances, max_bounce=12, max_diffuse_bounce=4, max_glossy_bounce=12,
                    max_transmission_bounce=12, name="barbershop_standin")


# ---------------------------------------------------------------------------
# Hair (curves): SURVEY.md §8(a8), §8(d) config JNK


def _strands(rng, roots, normals, n_keys, length, radius_root, radius_tip, kink, gravity=0.0):
    """Hair strands growing from `roots` along `normals`: n_keys keys per
    strand, radius tapering root to tip, a random kink per key and an optional
    droop along -y.  Returns (keys, radius, curve_first, curve_nkeys)."""
    n = len(roots)
    t = np.linspace(0.0, 1.0, n_keys)
    keys = np.zeros((n, n_keys, 3), dtype=np.float64)
    tang = normals / np.linalg.norm(normals, axis=1, keepdims=True)
    side = np.cross(tang, rng.standard_normal((n, 3)))
    side /= np.maximum(np.linalg.norm(side, axis=1, keepdims=True), 1e-9)
    for k in range(n_keys):
        wob = kink * np.sin(7.0 * t[k] + rng.random((n, 1)) * 6.28) * t[k]
        droop = np.array([0.0, -gravity * length * t[k] ** 2, 0.0])
        keys[:, k] = roots + tang * (length * t[k]) + side * wob * length + droop
    radius = np.broadcast_to(radius_root + (radius_tip - radius_root) * t, (n, n_keys))
    first = np.arange(n) * n_keys
    return (keys.reshape(-1, 3).astype(np.float32), radius.reshape(-1).astype(np.float32), first,
            np.full(n, n_keys))


def _sphere_fur(rng, center, radius, n, n_keys, length, r_root, r_tip, kink, gravity=0.0):
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    roots = np.asarray(center) + d * radius
    return _strands(rng, roots, d, n_keys, length, r_root, r_tip, kink, gravity)


def hair_ball(width=48, height=48, samples=8, shape="ribbon", strands=300, name=None, fur="plain") -> sc.Scene:
    """A furry ball on a floor (golden parity case for curves): strands with 5
    keys (4 Catmull-Rom segments each) of two hair materials around a diffuse
    core, lit by an area lamp and an emissive panel; unaligned BVH nodes bound
    the curve-only subtrees.  fur="principled": Principled Hair BSDFs (melanin
    with tint and random colour / roughness; a mix of the absorption and
    direct-colour parametrizations with coat); fur="hair_bsdf": the Hair BSDF
    node's reflection and transmission components, also on the core mesh
    (tangent from dPdv there)."""
    rng = np.random.default_rng(0x5EED + 40)
    white = sc.diffuse((0.7, 0.7, 0.7))
    core = sc.diffuse((0.5, 0.3, 0.2))
    fur_a = sc.diffuse((0.8, 0.5, 0.25))
    fur_b = sc.mix(0.3, sc.glossy((0.9, 0.8, 0.7), 0.25), sc.diffuse((0.3, 0.2, 0.1)))
    if fur == "principled":
        fur_a = sc.principled_hair("melanin", melanin=0.65, melanin_redness=0.4, tint=(0.9, 0.75, 0.6),
                                   random=0.3, random_color=0.4, random_roughness=0.3, roughness=0.35,
                                   radial_roughness=0.5)
        fur_b = sc.mix(0.4, sc.principled_hair("absorption", absorption_coefficient=(0.3, 0.6, 1.2), coat=0.4,
                                               roughness=0.08, radial_roughness=0.3),
                       sc.principled_hair("color", color=(0.45, 0.3, 0.2), ior=1.6, offset=0.06))
    elif fur == "hair_bsdf":
        fur_a = sc.mix(0.5, sc.hair((0.9, 0.7, 0.5), "reflection", roughness_u=0.15, roughness_v=0.4, offset=0.05),
                       sc.hair((0.8, 0.5, 0.3), "transmission", roughness_u=0.3, roughness_v=0.6))
        fur_b = sc.hair((0.6, 0.6, 0.65), "reflection", roughness_u=0.05, roughness_v=0.2)
        core = sc.mix(0.5, sc.diffuse((0.5, 0.3, 0.2)), sc.hair((0.8, 0.8, 0.8), "reflection", roughness_u=0.2,
                                                                   roughness_v=0.3, offset=0.1))
    light = sc.emission((1.0, 0.9, 0.8), 6.0)
    materials = [white, core, fur_a, fur_b, light]
    meshes = [sc.Mesh(*_quad((-3, -1, -3), (3, -1, -3), (3, -1, 3), (-3, -1, 3)), shader=0),
              sc.Mesh(*_ellipsoid((0.0, 0.0, 0.0), (0.6, 0.6, 0.6), 24, 14), shader=1, smooth=True),
              sc.Mesh(*_quad((-1.5, 2.5, -1.0), (-0.5, 2.5, -1.0), (-0.5, 2.5, 0.0), (-1.5, 2.5, 0.0)), shader=4)]
    keys, rad, first, nk = _sphere_fur(rng, (0.0, 0.0, 0.0), 0.6, strands, 5, 0.55, 0.02, 0.004, 0.25, 0.3)
    shader = np.where(np.arange(strands) % 3 == 0, 3, 2)
    hairs = [sc.Hair(keys, rad, first, nk, shader=shader)]
    lamps = [sc.Lamp("area", co=(1.5, 2.0, -1.5), direction=(-0.5, -0.7, 0.5), axisu=(1.0, 0.0, 0.0),
                     axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=1.0, sizev=1.0, color=(1.0, 0.95, 0.9), strength=40.0)]
    cam = sc.Camera(eye=(0.0, 0.6, -3.2), target=(0.0, 0.0, 0.0), fov=math.radians(45.0), nearclip=0.01,
                    farclip=100.0)
    return sc.Scene(width, height, cam, meshes, materials, world_color=(0.15, 0.17, 0.2), world_strength=1.0,
                    samples=samples, lamps=lamps, hairs=hairs, hair_shape=shape,
                    name=name or f"hair_ball_{shape}" + ("" if fur == "plain" else "_" + fur))


def junkshop_standin(width=3840, height=2160, samples=1024, detail=1.0, shape="ribbon") -> sc.Scene:
    """Junk Shop-class stand-in (SURVEY.md §8(d) config JNK): a cluttered shop
    interior (shelves of boxes, a counter, barrels) with furry props -- a rug,
    brushes and fur balls, Principled Hair BSDF strands -- about 1.3M curve
    segments at detail 1, lit by
    area lamps and a window panel -- and volumes: a dusty (homogeneous,
    forward-scattering) atmosphere in the world and a smoke volume in the
    window light (a volume-only box with a principled volume)."""
    rng = np.random.default_rng(0x5EED + 4)
    wall = sc.diffuse((0.55, 0.5, 0.45))
    wood = sc.mix(0.2, sc.glossy((0.6, 0.45, 0.3), 0.3), sc.diffuse((0.45, 0.3, 0.18)))
    metal = sc.glossy((0.8, 0.8, 0.85), 0.15)
    cardboard = sc.diffuse((0.6, 0.48, 0.32))
    # fur and rug strands with the Principled Hair BSDF (the node Blender
    # hair uses): melanin-pigmented, direct-coloured with a coat, and a
    # red direct-coloured rug
    fur1 = sc.principled_hair("melanin", melanin=0.55, melanin_redness=0.6, tint=(1.0, 0.9, 0.8), roughness=0.3,
                              radial_roughness=0.4)
    fur2 = sc.principled_hair("color", color=(0.22, 0.16, 0.1), coat=0.3, roughness=0.25, radial_roughness=0.35)
    rug = sc.principled_hair("color", color=(0.5, 0.12, 0.1), roughness=0.5, radial_roughness=0.6)
    window = sc.emission((1.0, 0.97, 0.9), 8.0)
    smoke = sc.material(volume=sc.principled_volume((0.7, 0.7, 0.72), density=0.35, anisotropy=0.3,
                                                    absorption_color=(0.4, 0.4, 0.45)))
    materials = [wall, wood, metal, cardboard, fur1, fur2, rug, window, smoke]
    meshes = []
    W, D, H = 10.0, 8.0, 4.0
    meshes.append(sc.Mesh(*_quad((-W, 0, -D), (W, 0, -D), (W, 0, D), (-W, 0, D)), shader=1))
    meshes.append(sc.Mesh(*_quad((-W, H, -D), (-W, H, D), (W, H, D), (W, H, -D)), shader=0))
    meshes.append(sc.Mesh(*_quad((-W, 0, D), (W, 0, D), (W, H, D), (-W, H, D)), shader=0))
    meshes.append(sc.Mesh(*_quad((-W, 0, -D), (-W, 0, D), (-W, H, D), (-W, H, -D)), shader=0))
    meshes.append(sc.Mesh(*_quad((W, 0, -D), (W, H, -D), (W, H, D), (W, 0, D)), shader=0))
    meshes.append(sc.Mesh(*_quad((-3, 1.2, D - 0.01), (3, 1.2, D - 0.01), (3, 3.5, D - 0.01),
                                 (-3, 3.5, D - 0.01)), shader=7))
    # shelves with boxes along the walls
    for side in (-1, 1):
        x = side * (W - 0.6)
        for level in range(4):
            y = 0.5 + level * 0.9
            meshes.append(sc.Mesh(*_box((x, y, 0.0), (1.0, 0.06, 12.0)), shader=1))
            nb = int(10 * detail) + 4
            for b in range(nb):
                sz = 0.25 + 0.3 * rng.random()
                meshes.append(sc.Mesh(*_box((x, y + sz / 2 + 0.03, -5.5 + 11.0 * (b + rng.random() * 0.5) / nb),
                                            (sz, sz, sz), rng.random() * 3.0), shader=3))
    # counter and barrels
    meshes.append(sc.Mesh(*_box((0.0, 0.55, 2.5), (5.0, 1.1, 1.0)), shader=1))
    for k in range(6):
        cx, cz = -4.0 + 1.6 * k, -4.5 + (k % 2)
        v, t = _cylinder(0.45, 1.1, 32)
        meshes.append(sc.Mesh(v + np.array([cx, 0.0, cz], dtype=np.float32), t, shader=2))
    # fur: a rug, fur balls on the counter, brushes
    n_rug = int(220000 * detail)
    roots = np.stack([rng.uniform(-2.5, 2.5, n_rug), np.full(n_rug, 0.0), rng.uniform(-2.0, 1.5, n_rug)], axis=1)
    normals = np.tile([0.0, 1.0, 0.0], (n_rug, 1)) + 0.25 * rng.standard_normal((n_rug, 3))
    k1, r1, f1, n1 = _strands(rng, roots, normals, 4, 0.09, 0.004, 0.001, 0.3)
    hairs = [sc.Hair(k1, r1, f1, n1, shader=6)]
    for b in range(5):
        c = (-1.8 + 0.9 * b, 1.1 + 0.35, 2.5)
        meshes.append(sc.Mesh(*_ellipsoid(c, (0.3, 0.3, 0.3), 20, 12), shader=4))
        kb, rb, fb, nb_ = _sphere_fur(rng, c, 0.3, int(40000 * detail), 5, 0.25, 0.006, 0.001, 0.3, 0.4)
        hairs.append(sc.Hair(kb, rb, fb, nb_, shader=4 + (b % 2)))
    for b in range(3):
        x = 6.0 - 1.2 * b
        roots = np.stack([x + rng.uniform(-0.3, 0.3, int(20000 * detail)), np.full(int(20000 * detail), 0.9),
                          -2.0 + rng.uniform(-0.1, 0.1, int(20000 * detail))], axis=1)
        meshes.append(sc.Mesh(*_box((x, 0.45, -2.0), (0.7, 0.9, 0.25)), shader=1))
        kk, rr, ff, nn = _strands(rng, roots, np.tile([0.0, 1.0, 0.0], (len(roots), 1)), 4, 0.4, 0.003, 0.002, 0.1)
        hairs.append(sc.Hair(kk, rr, ff, nn, shader=5))
    meshes.append(sc.Mesh(*_box((0.0, 2.3, D - 1.2), (5.0, 2.4, 1.6)), shader=8))
    lamps = [sc.Lamp("area", co=(0.0, H - 0.05, 0.0), direction=(0.0, -1.0, 0.0), axisu=(1.0, 0.0, 0.0),
                     axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=3.0, sizev=2.0, color=(1.0, 0.9, 0.75), strength=600.0),
             sc.Lamp("area", co=(-6.0, H - 0.05, -4.0), direction=(0.0, -1.0, 0.0), axisu=(1.0, 0.0, 0.0),
                     axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=1.5, sizev=1.5, color=(0.9, 0.95, 1.0), strength=200.0)]
    cam = sc.Camera(eye=(0.0, 2.2, -7.2), target=(0.0, 0.9, 2.0), fov=math.radians(55.0), nearclip=0.05,
                    farclip=100.0)
    return sc.Scene(width, height, cam, meshes, materials, world_color=(0.0, 0.0, 0.0), world_strength=0.0,
                    samples=samples, filter_type="blackman_harris", filter_width=1.5, lamps=lamps, hairs=hairs,
                    hair_shape=shape, max_bounce=8, name="junkshop_standin",
                    world_volume=sc.volume_scatter((0.9, 0.88, 0.85), density=0.012, anisotropy=0.5))


# ---------------------------------------------------------------------------
# Subsurface scattering: SURVEY.md §8(a18), §8(d) config CLS


def sss_cornell(width=48, height=48, samples=8, instanced=False, blur=False) -> sc.Scene:
    """Cornell box with random-walk subsurface scattering (golden parity case):
    a Subsurface Scattering node sphere, a principled random-walk sphere
    mixing subsurface with specular and sheen, a node mixing SSS with a
    glossy layer, and (instanced=True) the same materials on instanced
    geometry (local intersections through bvh_instance_push).  blur=True
    gives the node sphere a checker colour with the node's default texture
    blur and the principled sphere a bumped normal (the exit point's shader
    evaluated again, kernel_subsurface.h:132-158)."""
    from . import nodes

    s = cornell_box(width, height, samples)
    base = len(s.materials)
    if blur:
        checker = nodes.checker(None, (0.9, 0.6, 0.5), (0.4, 0.7, 0.9), scale=3.0)["Color"]
        skin = sc.subsurface(checker, scale=60.0, radius=(1.0, 0.4, 0.2), falloff="random_walk")
    else:
        skin = sc.subsurface((0.9, 0.6, 0.5), scale=60.0, radius=(1.0, 0.4, 0.2), falloff="random_walk",
                              texture_blur=0.0)
    wax = sc.principled(subsurface_method="random_walk", base_color=(0.9, 0.85, 0.7), subsurface=0.6,
                        subsurface_color=(0.9, 0.7, 0.4), subsurface_radius=(40.0, 25.0, 15.0), specular=0.4,
                        roughness=0.35, sheen=0.3,
                        **({"normal": nodes.vector_math("normalize", nodes.vector_math(
                            "add", nodes.geometry()["Normal"], (0.2, 0.0, 0.1))["Vector"])["Vector"]}
                           if blur else {}))
    jade = sc.mix(0.25, sc.glossy((0.9, 0.9, 0.9), 0.15),
                  sc.subsurface((0.3, 0.8, 0.5), scale=35.0, radius=(0.5, 1.0, 0.6), falloff="random_walk",
                                texture_blur=0.0))
    thin = sc.subsurface((0.8, 0.8, 0.9), scale=1e-9, radius=(1.0, 1.0, 1.0), falloff="random_walk",
                          texture_blur=0.0)  # radii below BSSRDF_MIN_RADIUS: diffuse
    s.materials.extend([skin, wax, jade, thin])
    centers = [(140.0, 120.0, 220.0), (300.0, 120.0, 260.0), (430.0, 300.0, 300.0), (200.0, 380.0, 380.0)]
    if instanced:
        ev, et = _ellipsoid((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), 20, 12)
        for i, c in enumerate(centers):
            geo = sc.Mesh(ev, et, shader=base + i, smooth=True)
            s.instances.append(sc.Instance(geo, _tfm(c, 0.3 * i, (70.0, 60.0 + 5 * i, 70.0))))
            s.instances.append(sc.Instance(geo, _tfm((c[0] * 0.7 + 60.0, 40.0, 120.0 + 50 * i), 0.0,
                                                     (30.0, 30.0, 30.0))))
    else:
        for i, c in enumerate(centers):
            s.meshes.append(sc.Mesh(*_ellipsoid(c, (70.0, 65.0, 70.0), 20, 12), shader=base + i, smooth=i % 2 == 0))
    s.lamps = [sc.Lamp("point", co=(140.0, 480.0, 40.0), size=20.0, color=(1.0, 0.8, 0.6), strength=3.0e6)]
    s.name = ("sss_instanced" if instanced else "sss_cornell") + ("_blur" if blur else "")
    return s


def bump_cornell(width=48, height=48, samples=8, camera="perspective") -> sc.Scene:
    """Cornell box with Bump nodes (golden parity case for ray differentials):
    a diffuse sphere bumped by a noise texture over generated coordinates, a
    glossy sphere bumped by a checker, an object-space bump from a position
    ramp on the back wall, a Principled sphere with a bumped normal, a mirror
    and a glass sphere (bounces whose reflected / refracted differentials
    reach the bumped surfaces).  camera: "perspective", "ortho" (dP
    differentials) or "equirect" (panorama differentials from inside)."""
    from . import nodes

    s = cornell_box(width, height, samples)
    if camera == "ortho":
        s.camera.type = "orthographic"
        s.camera.ortho_scale = 560.0
    elif camera == "equirect":
        s.camera = sc.Camera(eye=(278.0, 273.0, 200.0), target=(278.0, 273.0, 555.0), up=(0.0, 1.0, 0.0),
                             nearclip=0.1, farclip=1e5)
        s.camera.type = "panorama"
        s.camera.panorama_type = "equirectangular"
        s.camera.latitude_min, s.camera.latitude_max = -1.2, 1.3
        s.camera.longitude_min, s.camera.longitude_max = -2.5, 2.8
    base = len(s.materials)
    noise = nodes.noise_texture(None, scale=0.05, detail=2.0)["Fac"]
    checker = nodes.checker(None, (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), scale=4.0)["Fac"]
    ramp = nodes.math("sine", nodes.math("multiply", nodes.separate_xyz(nodes.geometry()["Position"])["X"], 0.05))
    bumpy = sc.diffuse((0.8, 0.6, 0.4), normal=nodes.bump(noise, strength=1.0, distance=2.0))
    tiles = sc.glossy((0.8, 0.8, 0.9), 0.3, normal=nodes.bump(checker, strength=0.6, distance=0.5, invert=True))
    wall = sc.diffuse((0.7, 0.7, 0.7), normal=nodes.bump(ramp, strength=0.8, distance=1.0, object_space=True))
    plastic = sc.principled(base_color=(0.2, 0.4, 0.8), roughness=0.3, specular=0.5,
                            normal=nodes.bump(noise, strength=0.5, distance=3.0))
    mirror = sc.glossy((0.9, 0.9, 0.9), 0.0)
    glass = sc.glass((0.95, 0.97, 1.0), 0.0, ior=1.45)
    s.materials.extend([bumpy, tiles, wall, plastic, mirror, glass])
    centers = [(140.0, 110.0, 220.0), (300.0, 110.0, 260.0), None, (430.0, 300.0, 300.0), (200.0, 380.0, 380.0),
               (420.0, 100.0, 120.0)]
    for i, c in enumerate(centers):
        if c is None:
            s.meshes.append(sc.Mesh(*_quad((40.0, 20.0, 540.0), (520.0, 20.0, 540.0), (520.0, 520.0, 540.0),
                                           (40.0, 520.0, 540.0)), shader=base + i))
        else:
            s.meshes.append(sc.Mesh(*_ellipsoid(c, (70.0, 65.0, 70.0), 20, 12), shader=base + i, smooth=True))
    s.name = "bump_cornell_" + camera
    return s


def bump_paths(width=40, height=40, samples=8) -> sc.Scene:
    """Bump nodes on the other branches of a path (golden parity case for the
    differentials each one carries): a burley BSSRDF with a bumped normal (its
    exit points' indirect rays keep the entry's dP in the slot records), a
    pane whose transparency follows the Layer Weight of a bumped normal (shadow
    rays evaluate it with the shading point's dP), a rough multiscatter glass,
    a translucent and a velvet sphere, a Beckmann glossy sphere bumped by a UV
    checker, one bumped by its vertex colours and one through the Object /
    Camera / Window texture coordinates."""
    from . import nodes

    s = cornell_box(width, height, samples)
    base = len(s.materials)
    tc = nodes.tex_coord()
    noise = nodes.noise_texture(None, scale=0.05, detail=2.0)["Fac"]
    uv_checker = nodes.checker(tc["UV"], (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), scale=6.0)["Fac"]
    vcol = nodes.separate_xyz(nodes.vertex_color("Col")["Color"])["Y"]
    coords = nodes.math("add", nodes.separate_xyz(tc["Object"])["X"],
                        nodes.math("add", nodes.separate_xyz(tc["Camera"])["Y"],
                                   nodes.separate_xyz(tc["Window"])["X"]))
    wave = nodes.math("sine", nodes.math("multiply", coords, 0.4))
    pane_bump = nodes.bump(nodes.checker(tc["Object"], (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), scale=0.05)["Fac"],
                           strength=1.0, distance=4.0)
    mats = [
        sc.subsurface((0.8, 0.5, 0.4), scale=40.0, radius=(1.0, 0.5, 0.25),
                      normal=nodes.bump(noise, strength=1.0, distance=3.0)),
        sc.glass((0.95, 0.95, 1.0), 0.25, ior=1.4, distribution="multi_ggx",
                 normal=nodes.bump(noise, strength=0.7, distance=2.0)),
        sc.translucent((0.7, 0.8, 0.5), normal=nodes.bump(noise, strength=0.8, distance=2.0, invert=True)),
        sc.velvet((0.8, 0.3, 0.5), sigma=0.6, normal=nodes.bump(vcol, strength=1.0, distance=0.5)),
        sc.glossy((0.8, 0.8, 0.6), 0.25, distribution="beckmann",
                  normal=nodes.bump(uv_checker, strength=0.8, distance=0.3)),
        sc.diffuse((0.6, 0.7, 0.9), normal=nodes.bump(wave, strength=1.0, distance=1.5)),
    ]
    s.materials.extend(mats)
    centers = [(130.0, 110.0, 230.0), (290.0, 100.0, 160.0), (440.0, 110.0, 280.0), (130.0, 330.0, 380.0),
               (290.0, 320.0, 420.0), (440.0, 330.0, 380.0)]
    rng = np.random.default_rng(91)
    for i, c in enumerate(centers):
        m = sc.Mesh(*_ellipsoid(c, (68.0, 64.0, 68.0), 20, 12), shader=base + i, smooth=i % 2 == 0)
        nt = len(m.tris)
        m.uv = rng.uniform(0.0, 1.0, (nt, 3, 2)).astype(np.float32)
        m.vertex_colors = {"Col": rng.uniform(0.0, 1.0, (nt, 3, 4))}
        s.meshes.append(m)
    facing = nodes.layer_weight(0.4, normal=pane_bump)["Facing"]
    s.materials.append(sc.mix(facing, sc.transparent((1.0, 1.0, 1.0)), sc.diffuse((0.7, 0.7, 0.75))))
    s.meshes.append(sc.Mesh(*_quad((60.0, 420.0, 100.0), (500.0, 420.0, 100.0), (500.0, 420.0, 500.0),
                                   (60.0, 420.0, 500.0)), shader=len(s.materials) - 1))
    s.lamps = [sc.Lamp("point", co=(278.0, 500.0, 280.0), size=20.0, color=(1.0, 0.9, 0.8), strength=2.0e6)]
    s.name = "bump_paths"
    return s


def bump_displace(width=40, height=40, samples=8) -> sc.Scene:
    """Displacement method "bump" (Blender's default; golden parity case):
    graph.cpp bump_from_displacement turns the material's Displacement output
    into a bump program ahead of the surface program (svm.cpp:864-880) that
    sets the shading normal — a scalar Displacement of a noise height in
    object space on a diffuse sphere and on the instanced boxes, a Vector
    Displacement in world space on a glossy sphere, a world-space Displacement
    on a Principled BSDF with subsurface (burley: SD_HAS_BSSRDF_BUMP, the exit
    points re-run the bump program) and a Mix of glass and diffuse."""
    import dataclasses

    from . import nodes as nd

    s = cornell_instanced(width, height, samples)
    pos = nd.separate_xyz(nd.geometry()["Position"])
    noise = nd.noise_texture(None, scale=0.04, detail=2.0)["Fac"]
    wave = nd.math("sine", nd.math("multiply", pos["X"], 0.09))
    mats = list(s.materials)
    # the walls' and instanced boxes' material (object-space transforms in the
    # bump program) and the host-transformed glossy ellipsoid's
    mats[0] = dataclasses.replace(mats[0], displacement=nd.displacement(noise, 0.5, 12.0, space="object"),
                                  displacement_method="bump")
    mats[-1] = dataclasses.replace(mats[-1], displacement=nd.displacement(wave, 0.5, 5.0, space="object"),
                                   displacement_method="bump")
    base = len(mats)
    mats.extend([
        dataclasses.replace(sc.diffuse((0.7, 0.6, 0.5)), displacement=nd.displacement(noise, 0.5, 10.0),
                            displacement_method="bump"),
        dataclasses.replace(sc.glossy((0.8, 0.8, 0.9), 0.2), displacement=nd.vector_displacement(
            nd.combine_xyz(wave, nd.math("multiply", noise, 2.0), 0.0), 0.0, 6.0, space="world"),
            displacement_method="bump"),
        dataclasses.replace(sc.principled(base_color=(0.85, 0.6, 0.5), subsurface=0.6,
                                          subsurface_color=(0.9, 0.5, 0.4), subsurface_radius=(20.0, 8.0, 5.0),
                                          roughness=0.4),
                            displacement=nd.displacement(wave, 0.5, 6.0, space="world"), displacement_method="bump"),
        dataclasses.replace(sc.mix(0.4, sc.glass((0.95, 0.95, 1.0), 0.1, ior=1.4), sc.diffuse((0.3, 0.5, 0.8))),
                            displacement=nd.displacement(noise, 0.3, 8.0), displacement_method="bump"),
    ])
    s.materials = mats
    centers = [(90.0, 70.0, 330.0), (470.0, 70.0, 250.0), (280.0, 430.0, 300.0), (450.0, 400.0, 420.0)]
    for i, c in enumerate(centers):
        s.meshes.append(sc.Mesh(*_ellipsoid(c, (62.0, 60.0, 62.0), 20, 12), shader=base + i, smooth=i % 2 == 0))
    s.name = "bump_displace"
    return s


def bump_both(width=40, height=40, samples=8) -> sc.Scene:
    """Displacement method "both" (golden parity case): true displacement moved
    the meshes' vertices (stand-in for MeshManager::displace: each vertex pushed
    along its direction from the body's centre by a wave of its position) and
    kept their undisplaced positions (Mesh::add_undisplaced,
    ATTR_STD_POSITION_UNDISPLACED); the bump program from the same Displacement
    output then runs at the undisplaced position (svm.cpp:744-750,
    NODE_ENTER_BUMP_EVAL / NODE_LEAVE_BUMP_EVAL, the Bump node in object space).
    Two world-space meshes (one smooth), a geometry instanced twice (undisplaced
    positions in object space, moved to world space by the instance transform)
    and a mesh whose material has method "both" but was not displaced (its
    undisplaced positions are its verts)."""
    import dataclasses

    from . import nodes as nd

    s = cornell_instanced(width, height, samples)
    pos = nd.separate_xyz(nd.geometry()["Position"])
    noise = nd.noise_texture(None, scale=0.05, detail=2.0)["Fac"]
    wave = nd.math("sine", nd.math("multiply", pos["Y"], 0.11))
    base = len(s.materials)
    s.materials = list(s.materials) + [
        dataclasses.replace(sc.diffuse((0.7, 0.6, 0.5)), displacement=nd.displacement(noise, 0.5, 10.0, space="object"),
                            displacement_method="both"),
        dataclasses.replace(sc.glossy((0.8, 0.8, 0.9), 0.25), displacement=nd.displacement(wave, 0.5, 6.0,
                                                                                            space="world"),
                            displacement_method="both"),
        dataclasses.replace(sc.mix(0.3, sc.glass((0.95, 0.95, 1.0), 0.1, ior=1.4), sc.diffuse((0.3, 0.5, 0.8))),
                            displacement=nd.vector_displacement(nd.combine_xyz(wave, noise, 0.0), 0.0, 4.0,
                                                                space="world"),
                            displacement_method="both"),
    ]

    def displaced(center, radii, nu, nv, shader, amp, smooth, tfm_space=False):
        v, t = _ellipsoid(center, radii, nu, nv)
        v = np.asarray(v, dtype=np.float32)
        d = v - np.asarray(center, dtype=np.float32)
        d = d / np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-6)
        h = (amp * np.sin(v[:, 0] * (0.35 if tfm_space else 0.08)) * np.cos(v[:, 2] * (0.3 if tfm_space else 0.07)))
        dv = (v + d * h[:, None].astype(np.float32)).astype(np.float32)
        return sc.Mesh(dv, t, shader=shader, smooth=smooth, undisplaced=v)

    s.meshes = list(s.meshes) + [
        displaced((120.0, 80.0, 300.0), (60.0, 58.0, 60.0), 20, 12, base, 6.0, False),
        displaced((440.0, 380.0, 400.0), (62.0, 60.0, 62.0), 22, 12, base + 1, 5.0, True),
        sc.Mesh(*_ellipsoid((300.0, 120.0, 160.0), (55.0, 50.0, 55.0), 18, 10), shader=base + 2, smooth=True),
    ]
    inst = displaced((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), 16, 10, base, 0.12, True, tfm_space=True)
    s.instances = list(s.instances) + [
        sc.Instance(inst, _tfm((260.0, 300.0, 420.0), 0.4, (50.0, 40.0, 50.0))),
        sc.Instance(inst, _tfm((470.0, 120.0, 330.0), -0.7, (40.0, 55.0, 40.0))),
    ]
    s.name = "bump_both"
    return s


def shading_holdout(width=48, height=48, samples=8) -> sc.Scene:
    """Holdouts with a transparent film (kernel_path.h:285-296 with
    shader_holdout_apply, kernel_shader.h:1020-1050): a Holdout closure mixed
    at 0.5 into a diffuse sphere (the path goes on at half the alpha), a pure
    Holdout quad (weight 1: the path ends), an object holdout (use_holdout)
    and an object holdout whose material is part transparent (only the
    transparent closures stay, weight 1 - transparency), a glass sphere in
    front of a holdout (refracted camera rays have lost
    PATH_RAY_TRANSPARENT_BACKGROUND: no holdout there), all over a floor that
    catches their shadows; the world seen directly is transparent too."""
    white = sc.diffuse((0.7, 0.7, 0.7))
    half = sc.mix(0.5, sc.diffuse((0.8, 0.3, 0.2)), sc.holdout())
    pure = sc.holdout()
    blue = sc.diffuse((0.2, 0.3, 0.8))
    seethrough = sc.mix(0.4, sc.diffuse((0.3, 0.8, 0.3)), sc.transparent((0.9, 0.9, 0.9)))
    glass = sc.Closure("glass", (1.0, 1.0, 1.0), roughness=0.0, ior=1.45)
    light = sc.emission((1.0, 0.95, 0.9), 8.0)
    materials = [white, half, pure, blue, seethrough, glass, light]
    meshes = [
        sc.Mesh(*_quad((-3, -1, -3), (3, -1, -3), (3, -1, 3), (-3, -1, 3)), shader=0),
        sc.Mesh(*_ellipsoid((-0.9, -0.45, 0.3), (0.5, 0.5, 0.5), 20, 12), shader=1, smooth=True),
        sc.Mesh(*_quad((0.2, -1.0, 0.9), (1.2, -1.0, 0.9), (1.2, 0.2, 0.9), (0.2, 0.2, 0.9)), shader=2),
        sc.Mesh(*_box((0.9, -0.6, -0.2), (0.6, 0.8, 0.6), 0.4), shader=3, holdout=True),
        sc.Mesh(*_box((-0.2, -0.7, -0.9), (0.5, 0.6, 0.5), -0.3), shader=4, holdout=True),
        sc.Mesh(*_ellipsoid((0.3, -0.6, -1.6), (0.35, 0.35, 0.35), 20, 12), shader=5, smooth=True),
        sc.Mesh(*_quad((-1.5, 2.5, -1.0), (-0.5, 2.5, -1.0), (-0.5, 2.5, 0.0), (-1.5, 2.5, 0.0)), shader=6),
    ]
    lamps = [sc.Lamp("point", co=(1.5, 2.0, -1.5), size=0.2, color=(1.0, 0.9, 0.8), strength=60.0)]
    cam = sc.Camera(eye=(0.0, 0.8, -3.6), target=(0.0, -0.3, 0.0), fov=math.radians(45.0), nearclip=0.01,
                    farclip=100.0)
    s = sc.Scene(width, height, cam, meshes, materials, world_color=(0.3, 0.35, 0.45), world_strength=1.0,
                 samples=samples, lamps=lamps, name="shading_holdout")
    s.film_transparent = True
    s.transparent_max_bounce = 8
    return s


def shadow_catcher(width=48, height=48, samples=8, transparent_film=False) -> sc.Scene:
    """Shadow catcher (golden parity case; kernel_path.h:265-281,
    kernel_accumulate.h:526-620): a floor that is a shadow catcher under a
    diffuse sphere, a glossy box, a half-transparent pane (its shadow through
    the transparent-shadow evaluation, seen by the catcher) and a second,
    smaller catcher quad lifted off the floor (catchers are hidden from the
    shadow rays of paths behind a catcher); a point lamp with two samples, an
    area lamp and a mesh light (the all-lights connection behind a catcher,
    lamps' and mesh lights' sample streams), a coloured world.
    transparent_film=True: the catcher's shadow lowers the alpha instead of
    darkening the background seen through it."""
    white = sc.diffuse((0.7, 0.7, 0.7))
    red = sc.diffuse((0.8, 0.25, 0.2))
    gloss = sc.glossy((0.8, 0.8, 0.9), 0.25)
    pane = sc.mix(0.5, sc.transparent((0.9, 0.9, 0.9)), sc.diffuse((0.2, 0.6, 0.3)))
    light = sc.emission((1.0, 0.9, 0.8), 6.0)
    materials = [white, red, gloss, pane, light]
    meshes = [
        sc.Mesh(*_quad((-3, -1, -3), (3, -1, -3), (3, -1, 3), (-3, -1, 3)), shader=0, shadow_catcher=True),
        sc.Mesh(*_ellipsoid((-0.8, -0.45, 0.2), (0.5, 0.5, 0.5), 20, 12), shader=1, smooth=True),
        sc.Mesh(*_box((0.8, -0.55, -0.1), (0.6, 0.9, 0.6), 0.4), shader=2),
        sc.Mesh(*_quad((-0.4, -0.2, -1.2), (0.6, -0.2, -1.2), (0.6, 0.7, -1.2), (-0.4, 0.7, -1.2)), shader=3),
        sc.Mesh(*_quad((0.9, -0.7, -1.8), (1.7, -0.7, -1.8), (1.7, -0.7, -1.0), (0.9, -0.7, -1.0)), shader=0,
                shadow_catcher=True),
        sc.Mesh(*_quad((-1.6, 2.2, -1.2), (-0.8, 2.2, -1.2), (-0.8, 2.2, -0.4), (-1.6, 2.2, -0.4)), shader=4),
    ]
    lamps = [sc.Lamp("point", co=(1.5, 2.0, -1.5), size=0.2, color=(1.0, 0.9, 0.8), strength=60.0, samples=2),
             sc.Lamp("area", co=(-1.8, 1.8, 1.0), direction=(0.0, -1.0, 0.0), axisv=(0.0, 0.0, 1.0), size=0.8,
                     color=(0.7, 0.8, 1.0), strength=40.0)]
    cam = sc.Camera(eye=(0.0, 0.8, -3.6), target=(0.0, -0.3, 0.0), fov=math.radians(45.0), nearclip=0.01,
                    farclip=100.0)
    s = sc.Scene(width, height, cam, meshes, materials, world_color=(0.3, 0.35, 0.45), world_strength=1.0,
                 samples=samples, lamps=lamps, name="shadow_catcher" + ("_film" if transparent_film else ""))
    s.film_transparent = transparent_film
    s.transparent_max_bounce = 8
    return s


def branched_cornell(width=40, height=40, samples=4, sample_all=True) -> sc.Scene:
    """Branched path tracing (golden parity case; kernel_path_branched.h):
    at each camera hit (and through the transparent pane in front) every BSDF
    closure spawns its own indirect paths (2 diffuse, 2 glossy, 1 transmission
    samples), with direct light from every lamp's samples (a point lamp with
    two samples, an area lamp) and the mesh light; indirect paths sample all
    lights too.  Closures: diffuse walls, a diffuse + glossy mix (two closures
    sampled separately), a glass sphere (reflection and refraction closures)
    and a half-transparent pane (the camera segment carries on through it).
    sample_all=False: one light sample per hit, direct and indirect."""
    s = cornell_box(width, height, samples)
    base = len(s.materials)
    s.materials.extend([
        sc.mix(0.5, sc.glossy((0.9, 0.85, 0.8), 0.2), sc.diffuse((0.3, 0.5, 0.8))),
        sc.Closure("glass", (1.0, 1.0, 1.0), roughness=0.0, ior=1.45),
        sc.mix(0.5, sc.transparent((0.9, 0.9, 0.9)), sc.diffuse((0.8, 0.7, 0.3))),
    ])
    s.meshes.append(sc.Mesh(*_ellipsoid((140.0, 90.0, 200.0), (80.0, 80.0, 80.0), 20, 12), shader=base, smooth=True))
    s.meshes.append(sc.Mesh(*_ellipsoid((400.0, 90.0, 150.0), (80.0, 80.0, 80.0), 20, 12), shader=base + 1,
                            smooth=True))
    s.meshes.append(sc.Mesh(*_quad((180.0, 150.0, -60.0), (380.0, 150.0, -60.0), (380.0, 350.0, -60.0),
                                   (180.0, 350.0, -60.0)), shader=base + 2))
    s.lamps = [sc.Lamp("point", co=(140.0, 480.0, 40.0), size=20.0, color=(1.0, 0.8, 0.6), strength=2.0e6, samples=2),
               sc.Lamp("area", co=(420.0, 540.0, 380.0), direction=(0.0, -1.0, 0.0), axisv=(0.0, 0.0, 1.0),
                       size=60.0, color=(0.6, 0.8, 1.0), strength=4.0e4)]
    s.integrator = "branched_path"
    s.diffuse_samples, s.glossy_samples, s.transmission_samples = 2, 2, 1
    s.sample_all_lights_direct = s.sample_all_lights_indirect = sample_all
    s.max_bounce = 4
    s.name = "branched_cornell" + ("" if sample_all else "_one_light")
    return s


def data_passes(width=40, height=40, samples=8) -> sc.Scene:
    """Data passes (golden parity case; kernel_passes.h:173-225
    kernel_write_data_passes): depth, normal, UV, object and material index
    written at each camera path's first hit that is opaque enough (a
    half-transparent pane in front is passed through below the alpha
    threshold), next to the combined pass.  Objects and materials carry pass
    indices; the floor and the sphere have UV maps, the box has none (its UV
    pass reads 0); a glossy-diffuse mix gives the normal pass a weighted
    average."""
    import dataclasses

    rng = np.random.default_rng(3)
    white = dataclasses.replace(sc.diffuse((0.7, 0.7, 0.7)), pass_index=3)
    red = dataclasses.replace(sc.diffuse((0.8, 0.25, 0.2)), pass_index=7)
    mixed = dataclasses.replace(sc.mix(0.4, sc.glossy((0.8, 0.8, 0.9), 0.3), sc.diffuse((0.2, 0.4, 0.8))),
                                pass_index=11)
    pane = dataclasses.replace(sc.mix(0.7, sc.transparent((0.9, 0.9, 0.9)), sc.diffuse((0.2, 0.6, 0.3))),
                               pass_index=5)
    light = sc.emission((1.0, 0.9, 0.8), 6.0)
    materials = [white, red, mixed, pane, light]
    floor = sc.Mesh(*_quad((-3, -1, -3), (3, -1, -3), (3, -1, 3), (-3, -1, 3)), shader=0, pass_index=1)
    floor.uv = rng.uniform(0.0, 1.0, (len(floor.tris), 3, 2)).astype(np.float32)
    ball = sc.Mesh(*_ellipsoid((-0.8, -0.45, 0.2), (0.5, 0.5, 0.5), 20, 12), shader=1, smooth=True, pass_index=2)
    ball.uv = rng.uniform(0.0, 1.0, (len(ball.tris), 3, 2)).astype(np.float32)
    meshes = [
        floor, ball,
        sc.Mesh(*_box((0.8, -0.55, -0.1), (0.6, 0.9, 0.6), 0.4), shader=2, pass_index=4),
        sc.Mesh(*_quad((-0.4, -0.2, -1.2), (0.6, -0.2, -1.2), (0.6, 0.7, -1.2), (-0.4, 0.7, -1.2)), shader=3,
                pass_index=6),
        sc.Mesh(*_quad((-1.6, 2.2, -1.2), (-0.8, 2.2, -1.2), (-0.8, 2.2, -0.4), (-1.6, 2.2, -0.4)), shader=4),
    ]
    lamps = [sc.Lamp("point", co=(1.5, 2.0, -1.5), size=0.2, color=(1.0, 0.9, 0.8), strength=60.0)]
    cam = sc.Camera(eye=(0.0, 0.8, -3.6), target=(0.0, -0.3, 0.0), fov=math.radians(45.0), nearclip=0.01,
                    farclip=100.0)
    s = sc.Scene(width, height, cam, meshes, materials, world_color=(0.3, 0.35, 0.45), world_strength=1.0,
                 samples=samples, lamps=lamps, name="data_passes")
    s.passes = ["depth", "normal", "uv", "object_id", "material_id"]
    return s


def light_passes(width=40, height=40, samples=8, mist_falloff=2.0, film_transparent=False) -> sc.Scene:
    """Light passes (golden parity case; kernel_passes.h:251-337, the
    PathRadiance components of kernel_accumulate.h): mist, emission,
    background, shadow and the diffuse / glossy / transmission direct,
    indirect and colour passes beside the combined pass, which is then the
    sum of the components (path_radiance_clamp_and_sum).  A diffuse floor, a
    glossy-diffuse box, a glass ball, a half-transparent pane (mist and colour
    passes see through it), an emitting quad and a lamp with MIS; the world
    is seen by camera rays (the background pass)."""
    white = sc.diffuse((0.7, 0.7, 0.7))
    mixed = sc.mix(0.4, sc.glossy((0.8, 0.8, 0.9), 0.3), sc.diffuse((0.2, 0.4, 0.8)))
    glass = sc.glass((0.95, 0.9, 0.85), 0.1, ior=1.45)
    pane = sc.mix(0.6, sc.transparent((0.9, 0.9, 0.9)), sc.diffuse((0.2, 0.6, 0.3)))
    light = sc.emission((1.0, 0.9, 0.8), 6.0)
    materials = [white, mixed, glass, pane, light]
    meshes = [
        sc.Mesh(*_quad((-3, -1, -3), (3, -1, -3), (3, -1, 3), (-3, -1, 3)), shader=0),
        sc.Mesh(*_box((0.8, -0.55, -0.1), (0.6, 0.9, 0.6), 0.4), shader=1),
        sc.Mesh(*_ellipsoid((-0.8, -0.45, 0.2), (0.5, 0.5, 0.5), 20, 12), shader=2, smooth=True),
        sc.Mesh(*_quad((-0.4, -0.2, -1.2), (0.6, -0.2, -1.2), (0.6, 0.7, -1.2), (-0.4, 0.7, -1.2)), shader=3),
        sc.Mesh(*_quad((-1.6, 2.2, -1.2), (-0.8, 2.2, -1.2), (-0.8, 2.2, -0.4), (-1.6, 2.2, -0.4)), shader=4),
    ]
    lamps = [sc.Lamp("point", co=(1.5, 2.0, -1.5), size=0.2, color=(1.0, 0.9, 0.8), strength=60.0)]
    cam = sc.Camera(eye=(0.0, 0.8, -3.6), target=(0.0, -0.3, 0.0), fov=math.radians(45.0), nearclip=0.01,
                    farclip=100.0)
    s = sc.Scene(width, height, cam, meshes, materials, world_color=(0.3, 0.35, 0.45), world_strength=1.0,
                 samples=samples, lamps=lamps, name="light_passes")
    s.passes = ["mist", "emission", "background", "shadow", "diffuse_direct", "diffuse_indirect", "diffuse_color",
                "glossy_direct", "glossy_indirect", "glossy_color", "transmission_direct", "transmission_indirect",
                "transmission_color", "volume_direct", "volume_indirect"]
    s.mist_start, s.mist_depth, s.mist_falloff = 1.0, 6.0, mist_falloff
    s.film_transparent = film_transparent
    return s


def shading_info(width=48, height=48, samples=8) -> sc.Scene:
    """Particle Info and texture mapping: boxes instanced with a particle each
    (index, age, lifetime, size, location, velocity, angular velocity driving
    colours; Random hashes the index) beside quads whose colours run through a
    TextureMapping matrix (svm_node_texture_mapping) with and without the
    min/max clamp (svm_node_min_max) and the normalize of type NORMAL."""
    from . import nodes as nd

    pi = nd.particle_info()
    col_a = nd.combine_xyz(nd.math("multiply", pi["Index"], 0.15), nd.math("divide", pi["Age"], pi["Lifetime"]),
                           nd.math("multiply", pi["Size"], 2.0))
    col_b = nd.mix_rgb("mix", pi["Random"], nd.vector_math("absolute", pi["Velocity"])["Vector"],
                       nd.mapping(pi["Location"], scale=(0.3, 0.3, 0.3), location=(0.5, 0.5, 0.5)))
    col_c = nd.vector_math("fraction", pi["Angular Velocity"])["Vector"]
    P = nd.tex_coord()["Object"]
    rot = [[0.8, -0.3, 0.1, 0.2], [0.25, 0.9, -0.2, -0.1], [0.0, 0.35, 1.1, 0.3]]
    tm = nd.texture_mapping(P, rot)
    tm_clamped = nd.texture_mapping(P, rot, (-0.2, 0.1, -0.3), (0.6, 0.7, 0.4))
    tm_normal = nd.texture_mapping(nd.geometry()["Normal"], [[1.0, 0.2, 0.0, 0.0], [-0.3, 1.0, 0.1, 0.0],
                                                             [0.0, 0.4, 0.7, 0.0]], normalize=True)
    materials = [sc.diffuse((0.6, 0.6, 0.6)), sc.diffuse(col_a), sc.mix(0.3, sc.diffuse(col_b), sc.glossy(col_b, 0.3)),
                 sc.diffuse(col_c),
                 sc.diffuse(nd.checker(tm, (0.9, 0.3, 0.1), (0.1, 0.3, 0.9), 2.0)["Color"]),
                 sc.diffuse(nd.mapping(tm_clamped, location=(0.4, 0.4, 0.4))),
                 sc.diffuse(nd.mapping(tm_normal, scale=(0.5, 0.5, 0.5), location=(0.5, 0.5, 0.5))),
                 sc.emission((1.0, 0.95, 0.9), 6.0)]
    box = sc.Mesh(*_box((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)), shader=1)
    box2 = sc.Mesh(*_box((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)), shader=2)
    box3 = sc.Mesh(*_box((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)), shader=3)
    rng = np.random.default_rng(0x5EED + 77)
    instances = []
    for k in range(9):
        part = {"index": 3 + 5 * k, "age": float(rng.uniform(0, 40)), "lifetime": float(rng.uniform(40, 90)),
                "size": float(rng.uniform(0.05, 0.4)), "rotation": tuple(float(x) for x in rng.normal(size=4)),
                "location": tuple(float(x) for x in rng.uniform(-2, 2, 3)),
                "velocity": tuple(float(x) for x in rng.normal(0, 0.8, 3)),
                "angular_velocity": tuple(float(x) for x in rng.normal(0, 2.0, 3))}
        x, z = -1.6 + 0.8 * (k % 3), -0.6 + 0.8 * (k // 3)
        mesh = (box, box2, box3)[k % 3]
        instances.append(sc.Instance(mesh, _tfm((x, -0.75, z), 0.3 * k, (0.45, 0.45, 0.45)), particle=part))
    meshes = [sc.Mesh(*_quad((-3, -1, -3), (3, -1, -3), (3, -1, 3), (-3, -1, 3)), shader=0)]
    for i in range(3):
        x0 = 0.5 + 0.75 * i
        meshes.append(sc.Mesh(*_quad((x0, -1.0, -0.5), (x0 + 0.65, -1.0, -0.5), (x0 + 0.65, 0.4, -0.5),
                                     (x0, 0.4, -0.5)), shader=4 + i))
    meshes.append(sc.Mesh(*_quad((-1.5, 2.5, -1.0), (-0.5, 2.5, -1.0), (-0.5, 2.5, 0.0), (-1.5, 2.5, 0.0)), shader=7))
    lamps = [sc.Lamp("point", co=(1.5, 2.0, -1.5), size=0.2, color=(1.0, 0.9, 0.8), strength=60.0)]
    cam = sc.Camera(eye=(0.0, 1.2, -4.0), target=(0.0, -0.4, 0.2), fov=math.radians(45.0), nearclip=0.01,
                    farclip=100.0)
    return sc.Scene(width, height, cam, meshes, materials, world_color=(0.2, 0.22, 0.25), world_strength=1.0,
                    samples=samples, lamps=lamps, instances=instances, name="shading_info")


def hair_info(width=48, height=48, samples=8, shape="ribbon") -> sc.Scene:
    """Hair Info on curves (svm_node_hair_info, curve_thickness,
    curve_tangent_normal; Intercept / Random through the curves'
    ATTR_STD_CURVE_INTERCEPT key and ATTR_STD_CURVE_RANDOM curve attributes,
    curve_attribute_float): the fur of hair_ball coloured by them, Is Strand
    on the mesh core (0) and on the strands (1)."""
    from . import nodes as nd

    s = hair_ball(width, height, samples, shape=shape, name=f"hair_info_{shape}")
    hi = nd.hair_info()
    fur_a = sc.diffuse(nd.combine_xyz(hi["Intercept"], hi["Random"], nd.math("multiply", hi["Thickness"], 20.0)))
    fur_b = sc.mix(0.3, sc.diffuse(nd.mapping(hi["Tangent Normal"], scale=(0.5, 0.5, 0.5), location=(0.5, 0.5, 0.5))),
                   sc.glossy(nd.combine_xyz(hi["Is Strand"], 0.4, hi["Intercept"]), 0.3))
    core = sc.diffuse(nd.combine_xyz(hi["Is Strand"], 0.3, nd.math("add", hi["Thickness"], 0.5)))
    s.materials[1], s.materials[2], s.materials[3] = core, fur_a, fur_b
    hr = s.hairs[0]
    nk = np.asarray(hr.curve_nkeys)
    intercept = np.concatenate([np.linspace(0.0, 1.0, int(n)) for n in nk]).astype(np.float32)
    rng = np.random.default_rng(0x5EED + 78)
    hr.attributes = {sc.ATTR_STD_CURVE_INTERCEPT: ("curve_key", intercept),
                     sc.ATTR_STD_CURVE_RANDOM: ("curve", rng.uniform(0.0, 1.0, len(nk)).astype(np.float32))}
    return s


def shading_raytrace(width=40, height=40, samples=8) -> sc.Scene:
    """Shader ray tracing (golden parity case, svm_ao.h / svm_bevel.h): Bevel
    normals on a glossy box (host-applied transform) and an instanced rotated
    box (object-space normal transforms, 4 local probe hits at most), Bevel
    feeding a Principled BSDF on a smooth superellipsoid, an Ambient Occlusion
    colour (8 rays of 200 units) on a diffuse sphere, AO from inside the same
    object only (only_local + inside) driving a mix, AO with the world's
    distance (Distance 0) on the back wall's stand-in quad, and the Wireframe
    node in pixel size (ray differentials) and as a bump height (its
    *_BUMP_DX / _DY one-sided differences)."""
    from . import nodes as nd

    s = cornell_box(width, height, samples)
    base = len(s.materials)
    ao = nd.ambient_occlusion((0.85, 0.7, 0.5), distance=200.0, samples=8)
    ao_local = nd.ambient_occlusion((1.0, 1.0, 1.0), distance=90.0, samples=6, inside=True, only_local=True)
    ao_world = nd.ambient_occlusion((0.6, 0.8, 0.6), distance=0.0, samples=4)
    s.materials.extend([
        sc.glossy((0.8, 0.8, 0.85), 0.25, normal=nd.bevel(8.0, samples=4)),
        sc.principled(base_color=(0.3, 0.5, 0.8), roughness=0.35, normal=nd.bevel(12.0, samples=6)),
        sc.diffuse(ao["Color"]),
        sc.mix(ao_local["AO"], sc.diffuse((0.9, 0.3, 0.2)), sc.glossy((0.9, 0.9, 0.9), 0.1)),
        sc.diffuse(ao_world["Color"]),
        sc.mix(nd.wireframe(2.0, use_pixel_size=True), sc.diffuse((0.2, 0.3, 0.7)), sc.diffuse((0.9, 0.9, 0.9))),
        sc.glossy((0.8, 0.6, 0.3), 0.3, normal=nd.bump(nd.wireframe(6.0), strength=1.0, distance=2.0)),
    ])
    s.meshes.append(sc.Mesh(*_box((150.0, 80.0, 200.0), (120.0, 160.0, 120.0), 0.4), shader=base))
    bv, bt = _box((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
    s.instances.append(sc.Instance(sc.Mesh(bv, bt, shader=base), _tfm((400.0, 70.0, 300.0), 0.7, (110.0, 140.0, 90.0),
                                                                      rot_x=0.3)))
    s.meshes.append(sc.Mesh(*_ellipsoid((420.0, 330.0, 200.0), (70.0, 60.0, 70.0), 20, 12, exponent=0.5),
                            shader=base + 1, smooth=True))
    s.meshes.append(sc.Mesh(*_ellipsoid((160.0, 350.0, 380.0), (65.0, 65.0, 65.0), 20, 12), shader=base + 2,
                            smooth=True))
    s.meshes.append(sc.Mesh(*_ellipsoid((280.0, 200.0, 420.0), (60.0, 60.0, 60.0), 16, 10), shader=base + 3))
    s.meshes.append(sc.Mesh(*_quad((60.0, 430.0, 520.0), (500.0, 430.0, 520.0), (500.0, 540.0, 520.0),
                                   (60.0, 540.0, 520.0)), shader=base + 4))
    s.meshes.append(sc.Mesh(*_ellipsoid((300.0, 70.0, 150.0), (55.0, 55.0, 55.0), 12, 8), shader=base + 5))
    s.meshes.append(sc.Mesh(*_ellipsoid((80.0, 230.0, 280.0), (50.0, 50.0, 50.0), 12, 8), shader=base + 6,
                            smooth=True))
    s.name = "shading_raytrace"
    return s


def sss_disk_cornell(width=48, height=48, samples=8, instanced=False, transparent=False) -> sc.Scene:
    """Cornell box with disk BSSRDFs (golden parity case): Subsurface
    Scattering nodes with the cubic (sharpness 0.5, blurred checker colour),
    gaussian (bumped normal: SD_HAS_BSSRDF_BUMP) and default burley (texture
    blur 1 over a noise colour) profiles, the cubic profile at sharpness 1
    with one radius channel below BSSRDF_MIN_RADIUS, and the Principled BSDF's
    default subsurface method; instanced=True puts them on instanced geometry,
    transparent=True adds a half-transparent pane so the exit points' light
    samples take the transparent-shadow evaluation."""
    from . import nodes

    s = cornell_box(width, height, samples)
    base = len(s.materials)
    checker = nodes.checker(None, (0.9, 0.55, 0.45), (0.5, 0.8, 0.6), scale=3.0)["Color"]
    noise = nodes.noise_texture(None, scale=0.02, detail=1.0)["Color"]
    bumped = nodes.vector_math("normalize", nodes.vector_math("add", nodes.geometry()["Normal"],
                                                              nodes.vector_math("scale", noise, scale=0.4)["Vector"])
                               ["Vector"])["Vector"]
    cubic = sc.subsurface(checker, scale=40.0, radius=(1.0, 0.5, 0.25), falloff="cubic", sharpness=0.5,
                          texture_blur=0.5)
    gauss = sc.subsurface((0.3, 0.8, 0.5), scale=30.0, radius=(0.5, 1.0, 0.6), falloff="gaussian", texture_blur=0.0,
                          normal=bumped)
    burley = sc.subsurface(noise, scale=50.0, radius=(1.0, 0.4, 0.2))
    skin = sc.principled(base_color=(0.85, 0.62, 0.52), subsurface=0.7, subsurface_color=(0.9, 0.5, 0.4),
                         subsurface_radius=(30.0, 12.0, 8.0), roughness=0.45, specular=0.35)
    sharp = sc.mix(0.3, sc.glossy((0.9, 0.9, 0.9), 0.2),
                   sc.subsurface((0.8, 0.7, 0.9), scale=45.0, radius=(1.0, 0.0, 0.3), falloff="cubic",
                                 sharpness=1.0, texture_blur=0.0))
    s.materials.extend([cubic, gauss, burley, skin, sharp])
    centers = [(140.0, 120.0, 220.0), (300.0, 120.0, 260.0), (430.0, 300.0, 300.0), (200.0, 380.0, 380.0),
               (420.0, 110.0, 120.0)]
    if instanced:
        ev, et = _ellipsoid((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), 20, 12)
        for i, c in enumerate(centers):
            geo = sc.Mesh(ev, et, shader=base + i, smooth=True)
            s.instances.append(sc.Instance(geo, _tfm(c, 0.3 * i, (70.0, 60.0 + 5 * i, 70.0))))
    else:
        for i, c in enumerate(centers):
            s.meshes.append(sc.Mesh(*_ellipsoid(c, (70.0, 65.0, 70.0), 20, 12), shader=base + i, smooth=i % 2 == 0))
    if transparent:
        s.materials.append(sc.mix(0.5, sc.transparent((1.0, 1.0, 1.0)), sc.diffuse((0.7, 0.7, 0.75))))
        s.meshes.append(sc.Mesh(*_quad((60.0, 300.0, 100.0), (260.0, 300.0, 100.0), (260.0, 300.0, 300.0),
                                       (60.0, 300.0, 300.0)), shader=len(s.materials) - 1))
    s.lamps = [sc.Lamp("point", co=(140.0, 480.0, 40.0), size=20.0, color=(1.0, 0.8, 0.6), strength=3.0e6)]
    s.name = "sss_disk" + ("_instanced" if instanced else "") + ("_transparent" if transparent else "")
    return s


def volume_cornell(width=48, height=48, samples=8, heterogeneous=False) -> sc.Scene:
    """Cornell box with volumes (golden parity case): homogeneous fog in the
    world (Henyey-Greenstein, forward scattering), a volume-only box with a
    principled volume, a glass sphere filled with an absorbing medium, a
    glowing principled-volume box and a point lamp whose MIS hits are
    attenuated by the fog.  heterogeneous=True drives the density of a
    scattering box and the world fog by textures of the position (ray
    marching with the jittered step of kernel_volume_step_init)."""
    s = cornell_box(width, height, samples)
    base = len(s.materials)
    smoke = sc.material(volume=sc.principled_volume((0.8, 0.5, 0.35), density=0.012, anisotropy=-0.3,
                                                    absorption_color=(0.3, 0.6, 0.2)))
    tinted_glass = sc.material(sc.glass((1.0, 1.0, 1.0), 0.0, ior=1.33),
                               volume=sc.volume_absorption((0.1, 0.5, 0.9), density=0.02))
    glow = sc.material(volume=sc.principled_volume((0.6, 0.6, 0.6), density=0.004,
                                                   emission_strength=0.02, emission_color=(1.0, 0.5, 0.2)))
    mats = [smoke, tinted_glass, glow]
    fog = sc.volume_scatter((0.9, 0.9, 0.95), density=0.0006, anisotropy=0.4)
    if heterogeneous:
        from . import nodes

        co = nodes.tex_coord()["Object"]
        dens = nodes.math("multiply", nodes.checker(co, (1.0, 1.0, 1.0), (0.1, 0.1, 0.1), scale=0.02)["Fac"],
                          0.03)
        mats.append(sc.material(volume=sc.mix(0.3, sc.volume_scatter((0.7, 0.8, 0.9), density=dens, anisotropy=0.2),
                                              sc.volume_absorption((0.5, 0.2, 0.2), density=dens))))
        px = nodes.separate_xyz(nodes.tex_coord()["Object"])["X"]
        fog = sc.volume_scatter((0.9, 0.9, 0.95), density=nodes.math("multiply", px, 0.000002), anisotropy=0.0)
    s.materials.extend(mats)
    s.meshes.append(sc.Mesh(*_box((150.0, 300.0, 300.0), (140, 160, 140), 0.4), shader=base))
    s.meshes.append(sc.Mesh(*_ellipsoid((400.0, 110.0, 140.0), (90.0, 90.0, 90.0), 24, 14), shader=base + 1,
                            smooth=True))
    s.meshes.append(sc.Mesh(*_box((420.0, 420.0, 380.0), (110, 90, 110), -0.2), shader=base + 2))
    if heterogeneous:
        s.meshes.append(sc.Mesh(*_box((260.0, 120.0, 330.0), (160, 200, 160), 0.2), shader=base + 3))
    s.world_volume = fog
    s.lamps = [sc.Lamp("point", co=(100.0, 450.0, 100.0), size=25.0, color=(1.0, 0.9, 0.8), strength=2.0e6)]
    s.name = "volume_hetero" if heterogeneous else "volume_cornell"
    return s


def sss_fog(width=48, height=48, samples=8, method="disk", box=False) -> sc.Scene:
    """Subsurface scattering in a volume scene (golden parity cases): the
    disk-BSSRDF (method="disk", sss_disk_cornell) or random-walk (sss_cornell)
    spheres in world fog, so the exit points' light samples are attenuated by
    the fog and every indirect ray carries its own volume stack
    (kernel_path_subsurface.h:26-110).  box=True adds a smoke box overlapping
    two of the spheres: their objects intersect a volume
    (SD_OBJECT_INTERSECTS_VOLUME), so each exit ray's stack is updated by the
    volume surfaces between the path's previous point and the exit point
    (kernel_volume_stack_update_for_subsurface)."""
    s = sss_disk_cornell(width, height, samples) if method == "disk" else sss_cornell(width, height, samples)
    s.world_volume = sc.volume_scatter((0.9, 0.9, 0.95), density=0.0008, anisotropy=0.3)
    if box:
        s.materials.append(sc.material(volume=sc.principled_volume((0.7, 0.6, 0.5), density=0.01, anisotropy=0.2)))
        s.meshes.append(sc.Mesh(*_box((250.0, 120.0, 240.0), (200, 160, 180), 0.3), shader=len(s.materials) - 1))
    s.name = "sss_%s_fog%s" % ("disk" if method == "disk" else "walk", "_box" if box else "")
    return s


def volume_camera_inside(width=48, height=48, samples=8) -> sc.Scene:
    """volume_cornell with the camera inside a volume object (golden parity
    case): a thin smoke box around the eye reaching into the room, so
    KernelCamera.is_inside_volume is set and every camera ray's volume stack is
    found by the record-all volume query (kernel_volume_stack_init,
    kernel_volume.h:1165-1306) -- the box the ray leaves without having
    entered it."""
    s = volume_cornell(width, height, samples)
    s.materials.append(sc.material(volume=sc.volume_scatter((0.8, 0.85, 0.9), density=0.0015, anisotropy=0.1)))
    s.meshes.append(sc.Mesh(*_box((278.0, 273.0, -350.0), (700, 700, 1100), 0.0), shader=len(s.materials) - 1))
    s.name = "volume_camera_inside"
    return s


def volume_decoupled(width=48, height=48, samples=8, heterogeneous=False, sampling="distance") -> sc.Scene:
    """volume_cornell as the reference's CPU device integrates it: decoupled
    ray marching (KernelIntegrator.volume_decoupled, kernel_volume.h:754-1128)
    with direct light from every lamp at each scatter segment
    (kernel_branched_path_volume_connect_light).  sampling: the smoke box's
    and the tinted glass's volume sampling method ("multiple_importance" also
    gives the point lamp two samples and adds a second, area lamp, so
    equiangular / distance MIS and the per-lamp branched sample streams are
    exercised)."""
    import dataclasses

    s = volume_cornell(width, height, samples, heterogeneous=heterogeneous)
    s.volume_decoupled = True
    if sampling != "distance":
        mats = list(s.materials)
        base = len(mats) - (4 if heterogeneous else 3)
        mats[base] = dataclasses.replace(mats[base], volume_sampling=sampling)
        mats[base + 1] = dataclasses.replace(mats[base + 1], volume_sampling="equiangular")
        s.materials = mats
        s.lamps = [dataclasses.replace(s.lamps[0], samples=2),
                   sc.Lamp("area", co=(420.0, 300.0, 80.0), direction=(0.0, 0.0, 1.0), size=60.0,
                           color=(0.6, 0.8, 1.0), strength=4.0e4)]
    s.name = "volume_decoupled" + ("_hetero" if heterogeneous else "") + ("" if sampling == "distance" else "_mis")
    return s


def voxel_cornell(width=40, height=40, samples=8) -> sc.Scene:
    """Point Density textures (golden parity case; NODE_TEX_VOXEL, svm_voxel.h,
    3D textures through kernel_tex_image_interp_3d): a volume box whose
    scattering density and colour come from a 12x10x8 float4 voxel grid in
    world space (the node's transform maps the box to the unit cube; linear,
    clip extension), a diffuse ellipsoid coloured by another grid in object
    space (instanced twice, its mesh with a generated-texture transform:
    volume_normalized_position; tricubic, repeat), and a glossy box coloured
    by a closest-interpolated grid (extend) whose TextureInfo carries a 3D
    transform (use_transform_3d)."""
    from . import nodes as nd

    rng = np.random.default_rng(0x5EED + 87)
    s = cornell_box(width, height, samples)
    base = len(s.materials)

    def grid(d, h, w):
        g = rng.random((d, h, w, 4), dtype=np.float64).astype(np.float32)
        g[..., 3] *= 0.02  # density (alpha)
        return g

    g1 = nd.Image(pixels=grid(8, 10, 12), data_type="float4", interpolation="linear", extension="clip", depth=8)
    lo, size = np.array([80.0, 180.0, 220.0]), np.array([200.0, 220.0, 180.0])
    tfm = np.zeros((3, 4))
    tfm[:, :3] = np.diag(1.0 / size)
    tfm[:, 3] = -lo / size
    pd1 = nd.point_density(g1, space="world", tfm=tfm)
    smoke = sc.material(volume=sc.volume_scatter(pd1["Color"], density=pd1["Density"], anisotropy=0.3))
    g2 = nd.Image(pixels=grid(6, 7, 9), data_type="float4", interpolation="cubic", extension="repeat", depth=6)
    pd2 = nd.point_density(g2, space="object")
    tinted = sc.diffuse(pd2["Color"])
    g3 = nd.Image(pixels=grid(5, 4, 6), data_type="float4", interpolation="closest", extension="extend", depth=5,
                  transform_3d=np.array([[0.004, 0.0, 0.0, -0.8], [0.0, 0.005, 0.0, -0.2], [0.0, 0.0, 0.003, -0.6]]))
    pd3 = nd.point_density(g3, space="world")
    shiny = sc.glossy(pd3["Color"], 0.3)
    s.materials.extend([smoke, tinted, shiny])
    s.meshes.append(sc.Mesh(*_box(tuple(lo + size / 2), tuple(size), 0.0), shader=base))
    s.meshes.append(sc.Mesh(*_box((410.0, 100.0, 150.0), (110, 200, 110), 0.4), shader=base + 2))
    ev, et = _ellipsoid((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), 20, 12)
    ell = sc.Mesh(ev, et, shader=base + 1, smooth=True,
                  generated_transform=np.array([[0.5, 0.0, 0.0, 0.5], [0.0, 0.5, 0.0, 0.5], [0.0, 0.0, 0.5, 0.5]]))
    s.instances = [sc.Instance(ell, _tfm((380.0, 380.0, 420.0), 0.3, (70.0, 55.0, 70.0))),
                   sc.Instance(ell, _tfm((170.0, 90.0, 420.0), -0.5, (60.0, 60.0, 45.0)))]
    s.name = "voxel_cornell"
    return s


def classroom_standin(width=1920, height=1080, samples=256, detail=1.0) -> sc.Scene:
    """Classroom-class stand-in (SURVEY.md §8(d) config CLS): a classroom with
    rows of desks and chairs, a blackboard, windows, 60 area lights in the
    ceiling grid and subsurface objects (disk BSSRDFs) -- skin-like busts,
    wax candles and a jade vase on the desks -- at 1920x1080, 256 spp."""
    rng = np.random.default_rng(0x5EED + 2)
    wall = sc.diffuse((0.7, 0.68, 0.62))
    floor = sc.mix(0.15, sc.glossy((0.7, 0.6, 0.5), 0.2), sc.diffuse((0.45, 0.3, 0.2)))
    wood = sc.principled(base_color=(0.5, 0.33, 0.2), roughness=0.45, specular=0.4)
    metal = sc.glossy((0.75, 0.75, 0.78), 0.25)
    board = sc.diffuse((0.08, 0.15, 0.1))
    glass = sc.glass((0.95, 0.97, 1.0), 0.0, ior=1.45)
    # subsurface with the defaults of Blender's nodes: the Principled BSDF's
    # "Christensen-Burley" method and the Subsurface Scattering node's burley
    # falloff with texture blur 1 (disk BSSRDFs, up to four exit points)
    skin = sc.principled(base_color=(0.85, 0.62, 0.52), subsurface=0.8, subsurface_color=(0.9, 0.5, 0.4),
                         subsurface_radius=(0.12, 0.05, 0.03), roughness=0.45, specular=0.35)
    wax = sc.subsurface((0.95, 0.9, 0.75), scale=0.05, radius=(1.0, 0.8, 0.5))
    jade = sc.mix(0.2, sc.glossy((0.9, 0.9, 0.9), 0.1), sc.subsurface((0.3, 0.75, 0.5), scale=0.04,
                                                                       radius=(0.4, 1.0, 0.6)))
    window = sc.emission((1.0, 0.98, 0.92), 1.5)
    materials = [wall, floor, wood, metal, board, glass, skin, wax, jade, window]
    meshes = []
    W, D, H = 6.0, 8.0, 3.2
    meshes.append(sc.Mesh(*_quad((-W, 0, -D), (W, 0, -D), (W, 0, D), (-W, 0, D)), shader=1))
    meshes.append(sc.Mesh(*_quad((-W, H, -D), (-W, H, D), (W, H, D), (W, H, -D)), shader=0))
    meshes.append(sc.Mesh(*_quad((-W, 0, D), (W, 0, D), (W, H, D), (-W, H, D)), shader=0))
    meshes.append(sc.Mesh(*_quad((-W, 0, -D), (-W, H, -D), (W, H, -D), (W, 0, -D)), shader=0))
    meshes.append(sc.Mesh(*_quad((W, 0, -D), (W, H, -D), (W, H, D), (W, 0, D)), shader=0))
    # window wall: panes of emissive sky behind glass
    meshes.append(sc.Mesh(*_quad((-W, 0, -D), (-W, 0, D), (-W, H, D), (-W, H, -D)), shader=0))
    for k in range(4):
        z0 = -6.0 + 3.2 * k
        meshes.append(sc.Mesh(*_quad((-W + 0.01, 1.0, z0), (-W + 0.01, 1.0, z0 + 2.2), (-W + 0.01, 2.6, z0 + 2.2),
                                     (-W + 0.01, 2.6, z0)), shader=9))
        meshes.append(sc.Mesh(*_box((-W + 0.15, 1.8, z0 + 1.1), (0.02, 1.6, 2.2)), shader=5))
    meshes.append(sc.Mesh(*_quad((-3.0, 0.9, D - 0.02), (3.0, 0.9, D - 0.02), (3.0, 2.4, D - 0.02),
                                 (-3.0, 2.4, D - 0.02)), shader=4))
    # desks and chairs
    ncols, nrows = 4, int(5 * detail) + 1
    for r in range(nrows):
        for c in range(ncols):
            x = -4.2 + c * 2.8
            z = -5.5 + r * 2.0
            meshes.append(sc.Mesh(*_box((x, 0.75, z), (1.4, 0.05, 0.7)), shader=2))
            for lx in (-0.65, 0.65):
                for lz in (-0.3, 0.3):
                    v, t = _cylinder(0.025, 0.75, 10, caps=False)
                    meshes.append(sc.Mesh(v + np.array([x + lx, 0.0, z + lz], dtype=np.float32), t, shader=3))
            meshes.append(sc.Mesh(*_box((x, 0.45, z - 0.65), (0.45, 0.04, 0.45)), shader=2))
            meshes.append(sc.Mesh(*_box((x, 0.75, z - 0.88), (0.45, 0.6, 0.04)), shader=2))
            # subsurface props on every desk
            kind = (r + c) % 3
            nu, nv = int(40 * detail) + 8, int(28 * detail) + 6
            if kind == 0:
                meshes.append(sc.Mesh(*_ellipsoid((x - 0.3, 0.93, z), (0.09, 0.13, 0.09), nu, nv), shader=6,
                                      smooth=True))
            elif kind == 1:
                v, t = _cylinder(0.04, 0.22 + 0.1 * rng.random(), nu)
                meshes.append(sc.Mesh(v + np.array([x + 0.3, 0.775, z + 0.1], dtype=np.float32), t, shader=7,
                                      smooth=True))
            else:
                meshes.append(sc.Mesh(*_ellipsoid((x, 0.9, z + 0.15), (0.08, 0.14, 0.08), nu, nv, exponent=0.8),
                                      shader=8, smooth=True))
    # bookshelves along the back wall
    for shelf in range(5):
        y = 0.3 + 0.45 * shelf
        meshes.append(sc.Mesh(*_box((3.5, y, D - 0.25), (4.0, 0.03, 0.4)), shader=2))
        nbooks = int(70 * detail) + 10
        for b in range(nbooks):
            bw = 0.03 + 0.03 * rng.random()
            bh = 0.25 + 0.15 * rng.random()
            meshes.append(sc.Mesh(*_box((1.6 + 3.8 * (b + 0.5) / nbooks, y + 0.015 + bh / 2, D - 0.25),
                                        (bw, bh, 0.28), 0.05 * rng.standard_normal()), shader=2 + (b % 3 == 0) * 2))
    # 60 ceiling area lights (6 x 10 grid)
    lamps = []
    for i in range(6):
        for j in range(10):
            lamps.append(sc.Lamp("area", co=(-5.0 + 2.0 * i, H - 0.02, -7.2 + 1.6 * j), direction=(0.0, -1.0, 0.0),
                                 axisu=(1.0, 0.0, 0.0), axisv=(0.0, 0.0, 1.0), size=1.0, sizeu=0.6, sizev=0.3,
                                 color=(1.0, 0.95, 0.88), strength=5.0))
    cam = sc.Camera(eye=(4.5, 1.7, -7.4), target=(-1.0, 0.8, 2.0), fov=math.radians(62.0), nearclip=0.05,
                    farclip=100.0)
    return sc.Scene(width, height, cam, meshes, materials, world_color=(0.0, 0.0, 0.0), world_strength=0.0,
                    samples=samples, filter_type="blackman_harris", filter_width=1.5, lamps=lamps, max_bounce=8,
                    name="classroom_standin")


CONFIGS = {
    "cornell_lamps": cornell_lamps,
    "cornell_instanced": cornell_instanced,
    "cornell_box": cornell_box,
    "bmw27_standin": bmw27_standin,
    # the bench frame with production node setups (Principled, bump, textures)
    "bmw27_production": lambda **kw: bmw27_standin(materials="production", **kw),
    "barbershop_standin": barbershop_standin,
    "junkshop_standin": junkshop_standin,
    "classroom_standin": classroom_standin,
}


# ---------------------------------------------------------------------------
# Shader-node coverage scenes (SVM texture / converter / input nodes)


def _node_world():
    """Direction-dependent world: a sky ramp over the ray direction's height
    for camera rays, a warm gradient for every other ray (light path node)."""
    from . import nodes as nd

    D = nd.geometry()["Position"]  # background: P = ray direction
    up = nd.separate_xyz(D)["Y"]
    sky = nd.color_ramp(nd.map_range(up, -1.0, 1.0, 0.0, 1.0),
                        [(0.0, (0.15, 0.12, 0.1, 1.0)), (0.45, (0.6, 0.65, 0.7, 1.0)),
                         (1.0, (0.25, 0.45, 0.95, 1.0))])["Color"]
    radial = nd.gradient(D, "radial")["Fac"]
    warm = nd.mix_rgb("multiply", radial, (1.0, 0.8, 0.5), (0.9, 0.9, 0.9))
    col = nd.mix_rgb("mix", nd.light_path()["Is Camera Ray"], warm, sky)
    return col


def _grid_scene(colors, width, height, samples, name, glossy_every=0):
    """One camera-facing quad per entry of `colors` (a color socket or
    constant), on a square grid in z = 0, lit by the node world only."""
    n = len(colors)
    cols = int(math.ceil(math.sqrt(n)))
    rows = int(math.ceil(n / cols))
    meshes, materials = [], []
    for i, c in enumerate(colors):
        r, q = divmod(i, cols)
        x0, y0 = q - cols / 2.0, (rows - 1 - r) - rows / 2.0
        # split the quad along a diagonal: barycentrics differ per half
        meshes.append(sc.Mesh(*_quad((x0 + 0.9, y0, 0.0), (x0, y0, 0.0), (x0, y0 + 0.9, 0.0),
                                     (x0 + 0.9, y0 + 0.9, 0.0)), shader=i))
        if glossy_every and i % glossy_every == glossy_every - 1:
            materials.append(sc.mix(0.3, sc.diffuse(c), sc.glossy(c, 0.3)))
        else:
            materials.append(sc.diffuse(c))
    # a back plane catching light bounced off the quads
    meshes.append(sc.Mesh(*_quad((cols, -rows, 1.5), (-cols, -rows, 1.5), (-cols, rows, 1.5), (cols, rows, 1.5)),
                          shader=n))
    materials.append(sc.diffuse((0.5, 0.5, 0.5)))
    ext = max(cols, rows)
    cam = sc.Camera(eye=(-0.05, 0.0, -2.2 * ext), target=(-0.05, 0.0, 0.0), up=(0.0, 1.0, 0.0),
                    fov=math.radians(30.0), nearclip=0.01, farclip=1e4)
    s = sc.Scene(width, height, cam, meshes, materials, samples=samples, name=name)
    s.world_color = _node_world()
    s.world_strength = 1.0
    s.world_map_resolution = 64  # world importance map (the spatially varying world is a light)
    return s


def _uv_inputs(lo_a, hi_a, lo_b, hi_b):
    """Two float sockets varying across each triangle (barycentric u, v)."""
    from . import nodes as nd

    uv = nd.separate_xyz(nd.geometry()["Parametric"])
    return nd.map_range(uv["X"], 0.0, 1.0, lo_a, hi_a), nd.map_range(uv["Y"], 0.0, 1.0, lo_b, hi_b)


def shading_math(width=64, height=64, samples=8) -> sc.Scene:
    """Every restated Math operation (svm_math_util.h svm_math), one quad
    each: result clamped to [0, 1] in red, the two operands in green / blue."""
    from . import nodes as nd

    colors = []
    for op in nd.MATH_OPS_GRID:
        a, b = _uv_inputs(-2.5, 2.5, -1.5, 2.5)
        r = nd.math(op, a, b, 0.3, clamp=True)
        colors.append(nd.combine_xyz(r, nd.math("multiply", a, 0.2, clamp=True),
                                     nd.math("multiply", b, 0.2, clamp=True)))
    return _grid_scene(colors, width, height, samples, "shading_math", glossy_every=5)


def shading_math_libm(width=32, height=32, samples=8) -> sc.Scene:
    """The Math operations backed by libm functions the kernel restates from
    glibc (tan, sinh, cosh, tanh; cy_math.h) and Vector Math tangent, over
    arguments that cross the reduction and branch boundaries."""
    from . import nodes as nd

    colors = []
    for op in ("tangent", "sinh", "cosh", "tanh"):
        a, b = _uv_inputs(-4.0, 4.0, -1.5, 2.5)
        r = nd.math(op, a, b, 0.3)
        colors.append(nd.combine_xyz(nd.math("multiply", r, 0.1), nd.math("multiply", a, 0.2, clamp=True),
                                     nd.math("multiply", b, 0.2, clamp=True)))
    a, b = _uv_inputs(-6.0, 6.0, -1.5, 1.5)
    colors.append(nd.vector_math("tangent", nd.combine_xyz(a, b, 1.2))["Vector"])
    return _grid_scene(colors, width, height, samples, "shading_math_libm")


def shading_vector(width=64, height=64, samples=8) -> sc.Scene:
    """Vector Math operations, the four Mapping types, separate / combine XYZ."""
    from . import nodes as nd

    colors = []

    def vecs():
        a, b = _uv_inputs(-2.0, 2.0, -1.0, 3.0)
        va = nd.combine_xyz(a, b, 0.7)
        vb = nd.combine_xyz(nd.math("subtract", 1.3, a), b, nd.math("subtract", a, b))
        return va, vb

    for op in nd.VECTOR_MATH_OPS:
        if op == "tangent":
            continue
        va, vb = vecs()
        vc = nd.combine_xyz(2.0, -0.5, 1.25)
        node = nd.vector_math(op, va, vb, vc, scale=0.35)
        out = node["Value"] if op in nd.VECTOR_MATH_VALUE_OPS else node["Vector"]
        colors.append(nd.mix_rgb("mix", 1.0, (0.0, 0.0, 0.0), out, clamp=True))
    for kind in nd.MAPPING_TYPES:
        va, _ = vecs()
        m = nd.mapping(va, location=(0.2, -0.3, 0.1), rotation=(0.4, -1.1, 2.3), scale=(1.5, 0.5, -2.0),
                       kind=kind)
        colors.append(nd.mix_rgb("mix", 1.0, (0.0, 0.0, 0.0), m, clamp=True))
    return _grid_scene(colors, width, height, samples, "shading_vector", glossy_every=4)


def shading_color(width=64, height=64, samples=8) -> sc.Scene:
    """MixRGB blend types, HSV, gamma, bright/contrast, invert, separate and
    combine HSV, color ramps, clamp and map-range types."""
    from . import nodes as nd

    colors = []
    for blend in nd.MIX_TYPES:
        a, b = _uv_inputs(0.0, 1.0, 0.0, 1.0)
        c1 = nd.combine_xyz(a, 0.35, b)
        c2 = nd.combine_hsv(b, 0.8, nd.math("add", a, 0.2))
        colors.append(nd.mix_rgb(blend, nd.math("multiply", a, 1.2), c1, c2, clamp=(blend == "linear_light")))
    a, b = _uv_inputs(0.0, 1.0, 0.0, 1.0)
    base = nd.combine_xyz(a, b, 0.4)
    colors.append(nd.hsv(base, hue=0.3, saturation=1.4, value_=0.9, fac=0.8))
    colors.append(nd.gamma(base, 2.2))
    colors.append(nd.gamma(base, nd.math("add", a, 0.5)))
    colors.append(nd.bright_contrast(base, 0.1, 0.6))
    colors.append(nd.invert(base, 0.7))
    sh = nd.separate_hsv(base)
    colors.append(nd.combine_hsv(sh["S"], sh["V"], sh["H"]))
    colors.append(nd.color_ramp(a, [(0.1, (1.0, 0.0, 0.0, 1.0)), (0.5, (0.0, 1.0, 0.2, 0.5)),
                                    (0.9, (0.1, 0.2, 1.0, 0.0))])["Color"])
    ramp_c = nd.color_ramp(b, [(0.0, (0.9, 0.9, 0.1, 1.0)), (0.3, (0.1, 0.5, 0.9, 0.25)),
                               (0.7, (0.8, 0.2, 0.4, 0.75))], interpolation="constant")
    colors.append(nd.combine_xyz(ramp_c["Alpha"], a, 0.3))
    for kind in nd.CLAMP_TYPES:
        v = nd.clamp(nd.math("multiply", a, 1.4), 0.8, nd.math("multiply", b, 0.6), kind=kind)
        colors.append(nd.combine_xyz(v, 0.2, b))
    for kind in nd.MAP_RANGE_TYPES:
        v = nd.map_range(a, 0.8, 0.2, 0.1, 0.9, steps=nd.math("multiply", b, 6.0), kind=kind)
        colors.append(nd.combine_xyz(v, b, 0.5))
    # color -> float conversion (film rgb_to_y) and float -> color
    colors.append(nd.math("power", base, 0.5))
    return _grid_scene(colors, width, height, samples, "shading_color", glossy_every=6)


def shading_noise(width=64, height=64, samples=8) -> sc.Scene:
    """The procedural noise textures (svm_noise.h and its users): Noise in
    1-4 D with and without distortion, every Musgrave type in 3 D plus 1/2/4 D
    fBm, Wave bands / rings with each profile and direction, Magic at three
    depths, Brick with offset / squash, White Noise in 1-4 D."""
    from . import nodes as nd

    tc = nd.tex_coord()
    P = nd.mapping(tc["Object"], scale=(1.7, 1.7, 1.7), location=(0.3, -0.2, 0.1))
    W = nd.separate_xyz(tc["Object"])["Y"]
    colors = []
    for dims in (1, 2, 3, 4):
        colors.append(nd.noise_texture(P, w=W, scale=2.5, detail=3.5, roughness=0.6, dimensions=dims)["Color"])
    colors.append(nd.noise_texture(P, w=W, scale=4.0, detail=1.0, distortion=2.5, dimensions=3)["Color"])
    colors.append(nd.noise_texture(P, w=W, scale=3.0, detail=0.0, distortion=1.0, dimensions=2)["Color"])
    colors.append(nd.noise_texture(P, w=W, scale=1.5, detail=6.7, roughness=0.45, distortion=0.7,
                                   dimensions=4)["Color"])
    for kind in nd.MUSGRAVE_TYPES:
        fac = nd.musgrave_texture(P, kind, scale=2.0, detail=4.3, dimension=1.2, lacunarity=2.1, offset=0.8,
                                  gain=1.3)["Fac"]
        colors.append(nd.mix_rgb("mix", nd.math("multiply", fac, 0.4), (0.1, 0.1, 0.3), (1.0, 0.8, 0.2),
                                 clamp=True))
    for dims in (1, 2, 4):
        fac = nd.musgrave_texture(P, "fBm", w=W, scale=3.0, detail=2.5, dimensions=dims)["Fac"]
        colors.append(nd.mix_rgb("mix", nd.math("add", nd.math("multiply", fac, 0.5), 0.5), (0.0, 0.2, 0.1),
                                 (0.9, 0.9, 0.6), clamp=True))
    for kind, direction, profile in (("bands", "x", "sin"), ("bands", "diagonal", "saw"), ("rings", "spherical",
                                     "tri"), ("rings", "z", "sin"), ("bands", "y", "tri")):
        colors.append(nd.wave_texture(P, kind, direction, profile, scale=1.5, distortion=3.0 if profile == "sin"
                                      else 0.0, detail=2.0, detail_scale=1.5, phase=0.7)["Color"])
    for depth in (0, 2, 7):
        colors.append(nd.magic_texture(P, depth=depth, scale=1.2, distortion=1.4 if depth else 0.0)["Color"])
    colors.append(nd.brick_texture(P, (0.7, 0.2, 0.1), (0.5, 0.4, 0.3), (0.9, 0.9, 0.85), scale=2.0,
                                   mortar_size=0.03, mortar_smooth=0.4, bias=0.1, brick_width=0.45, row_height=0.2,
                                   offset=0.4, squash=0.8)["Color"])
    for dims in (1, 2, 3, 4):
        colors.append(nd.white_noise_texture(nd.mapping(tc["Object"], scale=(9.0, 9.0, 9.0)), w=W,
                                             dimensions=dims)["Color"])
    return _grid_scene(colors, width, height, samples, "shading_noise")


def shading_voronoi(width=64, height=64, samples=8) -> sc.Scene:
    """Voronoi Texture (svm_voronoi.h): every feature in 1-4 D with the four
    distance metrics, its Distance / Color / Position / W / Radius outputs."""
    from . import nodes as nd

    tc = nd.tex_coord()
    P = nd.mapping(tc["Object"], scale=(1.3, 1.3, 1.3), location=(0.2, 0.1, -0.3))
    W = nd.math("multiply", nd.separate_xyz(tc["Object"])["X"], 0.7)
    colors = []

    def shade(v, lo=(0.05, 0.1, 0.3), hi=(1.0, 0.9, 0.6)):
        return nd.mix_rgb("mix", v, lo, hi, clamp=True)

    metrics = ("euclidean", "manhattan", "chebychev", "minkowski")
    for dims in (1, 2, 3, 4):
        for feature in ("f1", "f2", "smooth_f1"):
            m = metrics[(dims + len(feature)) % 4]
            v = nd.voronoi_texture(P, feature, m, w=W, scale=3.0, smoothness=0.6, exponent=0.7, randomness=0.9,
                                   dimensions=dims)
            colors.append(nd.mix_rgb("mix", 0.5, v["Color"], shade(v["Distance"]), clamp=True))
            if feature == "f1":
                pos = v["W"] if dims == 1 else v["Position"]
                colors.append(nd.vector_math("fraction", pos)["Vector"] if dims > 1 else shade(
                    nd.math("fraction", pos)))
        e = nd.voronoi_texture(P, "distance_to_edge", w=W, scale=2.5, randomness=0.8, dimensions=dims)
        colors.append(shade(nd.math("multiply", e["Distance"], 4.0)))
        r = nd.voronoi_texture(P, "n_sphere_radius", w=W, scale=2.5, randomness=1.0, dimensions=dims)
        colors.append(shade(nd.math("multiply", r["Radius"], 2.0), (0.3, 0.05, 0.05), (0.9, 1.0, 0.8)))
    return _grid_scene(colors, width, height, samples, "shading_voronoi")


def shading_coords(width=64, height=64, samples=8) -> sc.Scene:
    """Texture coordinate and geometry outputs, checker and gradient
    textures, light path and light falloff outputs."""
    from . import nodes as nd

    colors = []

    def show(v):
        return nd.mix_rgb("mix", 1.0, (0.0, 0.0, 0.0), nd.mapping(v, scale=(0.25, 0.25, 0.25),
                                                                    location=(0.5, 0.5, 0.5)), clamp=True)

    tc = nd.tex_coord()
    for name in nd.TEXCO_OUTPUTS:
        colors.append(show(tc[name]))
    g = nd.geometry()
    for name in ("Position", "Normal", "Incoming", "True Normal", "Parametric"):
        colors.append(show(g[name]))
    P = tc["Object"]
    colors.append(nd.checker(P, (0.9, 0.2, 0.1), (0.1, 0.3, 0.9), 3.0)["Color"])
    colors.append(nd.checker(nd.mapping(P, rotation=(0.3, 0.2, 0.7)), (0.9, 0.9, 0.9), (0.05, 0.05, 0.05),
                             nd.math("add", nd.separate_xyz(g["Parametric"])["X"], 2.0))["Color"])
    for kind in nd.GRADIENT_TYPES:
        local = nd.vector_math("fraction", nd.mapping(P, scale=(1.1, 1.1, 1.1)))["Vector"]
        centred = nd.mapping(local, location=(-0.5, -0.5, 0.0), scale=(2.0, 2.0, 2.0))
        colors.append(nd.gradient(centred, kind)["Color"])
    lp = nd.light_path()
    for name in nd.LIGHT_PATH_OUTPUTS:
        if name in ("Is Shadow Ray", "Is Volume Scatter Ray", "Is Transmission Ray", "Transmission Depth"):
            continue  # zero on every path of this scene
        v = lp[name]
        if name == "Ray Length":
            v = nd.math("multiply", v, 0.05)
        elif name.endswith("Depth"):
            v = nd.math("multiply", v, 0.3)
        colors.append(nd.combine_xyz(v, 0.3, nd.math("subtract", 1.0, v)))
    lf = nd.light_falloff(2.0, 0.5)
    for name in nd.LIGHT_FALLOFF_OUTPUTS:
        colors.append(nd.combine_xyz(nd.math("multiply", lf[name], 0.01, clamp=True), 0.5, 0.2))
    return _grid_scene(colors, width, height, samples, "shading_coords", glossy_every=3)


def world_lit(width=64, height=64, samples=8, map_resolution=128, with_lamp=False) -> sc.Scene:
    """Objects lit mainly by a world shader with a bright direction (a sun-like
    spot over a sky gradient): the background light (world importance
    sampling, kernel_light_background.h) carries the direct light, and escaping
    BSDF rays are MIS-weighted against it."""
    from . import nodes as nd

    D = nd.geometry()["Position"]
    sun_dir = (0.45, 0.8, -0.4)
    n = math.sqrt(sum(c * c for c in sun_dir))
    sun_dir = tuple(c / n for c in sun_dir)
    cosang = nd.vector_math("dot_product", D, sun_dir)["Value"]
    spot = nd.map_range(cosang, 0.97, 1.0, 0.0, 40.0, kind="smoothstep")
    up = nd.separate_xyz(D)["Y"]
    sky = nd.mix_rgb("mix", nd.map_range(up, -0.2, 1.0, 0.0, 1.0), (0.25, 0.2, 0.15), (0.3, 0.5, 0.9))
    world = nd.mix_rgb("add", 1.0, sky, nd.combine_xyz(spot, nd.math("multiply", spot, 0.85),
                                                       nd.math("multiply", spot, 0.6)))
    meshes, materials = [], []
    materials.append(sc.diffuse((0.6, 0.6, 0.6)))
    meshes.append(sc.Mesh(*_quad((-6, 0, -6), (-6, 0, 6), (6, 0, 6), (6, 0, -6)), shader=0))
    materials.append(sc.diffuse((0.7, 0.2, 0.15)))
    meshes.append(sc.Mesh(*_box((-1.6, 0.75, 0.5), (1.5, 1.5, 1.5), 0.4), shader=1))
    materials.append(sc.glossy((0.9, 0.9, 0.9), 0.25))
    meshes.append(sc.Mesh(*_ellipsoid((1.2, 0.9, 0.0), (0.9, 0.9, 0.9), 24, 12), shader=2))
    materials.append(sc.mix(0.4, sc.diffuse((0.1, 0.4, 0.8)), sc.glossy((0.8, 0.8, 0.8), 0.05)))
    meshes.append(sc.Mesh(*_box((0.0, 0.4, -1.8), (2.5, 0.8, 0.8), -0.2), shader=3))
    cam = sc.Camera(eye=(0.5, 3.0, -7.5), target=(0.0, 0.6, 0.0), up=(0.0, 1.0, 0.0), fov=math.radians(45.0),
                    nearclip=0.01, farclip=1e4)
    lamps = []
    if with_lamp:
        lamps.append(sc.Lamp(kind="point", co=(-2.0, 3.0, -2.0), color=(1.0, 0.9, 0.8), strength=30.0, size=0.3))
    s = sc.Scene(width, height, cam, meshes, materials, samples=samples, name="world_lit", lamps=lamps)
    s.world_color = world
    s.world_strength = 1.0
    s.world_map_resolution = map_resolution
    return s


def sky_lit(width=32, height=32, samples=4, kind="preetham", model=None, map_resolution=64) -> sc.Scene:
    """Objects on a ground plane under a Sky Texture world (svm_sky.h), Z up as
    the sky models assume: the camera sees the horizon and the sky, the world
    importance map (background light, kernel_light_background.h) samples it.
    `model` is the host-precomputed data of the Hosek-Wilkie / Nishita models
    (nodes.sky_texture)."""
    from . import nodes as nd

    D = nd.geometry()["Position"]
    sun = (0.3, 0.55, 0.78)
    if kind == "nishita_improved":
        sky = nd.sky_texture(D, kind, sun_disc=True, sun_size=0.05, sun_intensity=0.002,
                             sun_elevation=math.radians(12.0), sun_rotation=math.radians(-30.0), model=model)
    else:
        sky = nd.sky_texture(D, kind, sun_direction=sun, turbidity=3.0, ground_albedo=0.4, model=model)
    meshes, materials = [], []
    materials.append(sc.diffuse((0.5, 0.5, 0.45)))
    meshes.append(sc.Mesh(*_quad((-8, -8, 0), (8, -8, 0), (8, 8, 0), (-8, 8, 0)), shader=0))
    materials.append(sc.diffuse((0.7, 0.25, 0.15)))
    meshes.append(sc.Mesh(*_box((-1.4, 0.6, 0.75), (1.5, 1.5, 1.5), 0.3), shader=1))
    materials.append(sc.glossy((0.9, 0.9, 0.9), 0.2))
    meshes.append(sc.Mesh(*_ellipsoid((1.1, -0.2, 0.9), (0.9, 0.9, 0.9), 24, 12), shader=2))
    cam = sc.Camera(eye=(0.0, -7.0, 1.6), target=(0.0, 0.0, 1.4), up=(0.0, 0.0, 1.0), fov=math.radians(60.0),
                    nearclip=0.01, farclip=1e4)
    s = sc.Scene(width, height, cam, meshes, materials, samples=samples, name=f"sky_{kind}")
    s.world_color = sky["Color"]
    s.world_strength = 1.0
    s.world_map_resolution = map_resolution
    return s


def transparent_shadows(width=48, height=48, samples=8) -> sc.Scene:
    """Transparent BSDFs seen directly and casting tinted shadows: a stack of
    three tinted transparent panes, a half-transparent leaf whose transparency
    follows a checker texture (texture nodes evaluated for shadow rays), and a
    point lamp plus the ceiling light (kernel_shadow.h record-all path)."""
    from . import nodes as nd

    s = cornell_box(width, height, samples)
    mats = s.materials
    base = len(mats)
    mats.append(sc.transparent((0.9, 0.5, 0.3)))
    mats.append(sc.mix(0.35, sc.transparent((0.3, 0.8, 0.9)), sc.diffuse((0.2, 0.6, 0.3))))
    P = nd.tex_coord()["Object"]
    fac = nd.checker(nd.mapping(P, scale=(0.02, 0.02, 0.02)), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), 1.0)["Fac"]
    mats.append(sc.mix(fac, sc.diffuse((0.8, 0.8, 0.2)), sc.transparent((0.95, 0.95, 0.95))))
    for k, z in enumerate((150.0, 200.0, 250.0)):
        s.meshes.append(sc.Mesh(*_quad((120, 300, z), (320, 300, z), (320, 470, z + 40), (120, 470, z + 40)),
                                shader=base))
    s.meshes.append(sc.Mesh(*_quad((300, 400, 120), (480, 400, 120), (480, 400, 420), (300, 400, 420)),
                            shader=base + 1))
    s.meshes.append(sc.Mesh(*_quad((80, 20, 80), (250, 20, 80), (250, 250, 160), (80, 250, 160)), shader=base + 2))
    s.lamps = [sc.Lamp(kind="point", co=(400.0, 500.0, 250.0), color=(1.0, 0.95, 0.9), strength=2.0e5, size=10.0)]
    s.name = "transparent_shadows"
    return s


def shading_aov(width=40, height=40, samples=8) -> sc.Scene:
    """AOV outputs (golden parity case; NODE_AOV_START / _COLOR / _VALUE,
    svm_aov.h, film AOV passes after the combined pass): colour and value AOVs
    from constants, a noise texture and a Fresnel node on the Cornell box's
    materials; a pane 30 % transparent (alpha 0.7 >= the film's alpha
    threshold: the first hit ends the AOV writes) and one 80 % transparent
    (alpha 0.2: the surface behind writes its AOVs too, PATH_RAY_SINGLE_PASS_DONE
    unset); a glass sphere (refracted rays are no camera rays); an AOV output
    without a pass (dropped) and a pass no material writes (zero)."""
    import dataclasses

    from . import nodes as nd

    s = cornell_box(width, height, samples)
    noise = nd.noise_texture(None, scale=0.03, detail=2.0)
    fres = nd.fresnel(1.5)
    mats = list(s.materials)
    for i, m in enumerate(mats):
        col = m.color if isinstance(m.color, tuple) else (0.5, 0.5, 0.5)
        mats[i] = dataclasses.replace(m, aovs={"albedo": col, "mask": float(i) * 0.25, "unused": (1.0, 0.0, 0.0)})
    base = len(mats)
    mats.append(dataclasses.replace(sc.diffuse(noise["Color"]),
                                    aovs={"albedo": noise["Color"], "mask": fres, "fac": noise["Fac"]}))
    mats.append(dataclasses.replace(sc.mix(0.3, sc.diffuse((0.2, 0.6, 0.3)), sc.transparent((0.9, 0.9, 0.9))),
                                    aovs={"albedo": (0.2, 0.6, 0.3), "mask": 2.0}))
    mats.append(dataclasses.replace(sc.mix(0.8, sc.diffuse((0.7, 0.2, 0.2)), sc.transparent((0.9, 0.9, 0.9))),
                                    aovs={"albedo": (0.7, 0.2, 0.2), "mask": 3.0, "fac": fres}))
    mats.append(dataclasses.replace(sc.glass((1.0, 1.0, 1.0), 0.0, ior=1.45), aovs={"mask": 4.0}))
    s.materials = mats
    s.meshes.append(sc.Mesh(*_ellipsoid((150.0, 100.0, 300.0), (80.0, 80.0, 80.0), 20, 12), shader=base,
                            smooth=True))
    s.meshes.append(sc.Mesh(*_quad((300, 60, 200), (480, 60, 200), (480, 260, 240), (300, 260, 240)), shader=base + 1))
    s.meshes.append(sc.Mesh(*_quad((120, 280, 180), (320, 280, 180), (320, 470, 220), (120, 470, 220)),
                            shader=base + 2))
    s.meshes.append(sc.Mesh(*_ellipsoid((420.0, 380.0, 380.0), (70.0, 70.0, 70.0), 20, 12), shader=base + 3,
                            smooth=True))
    s.aovs = [("albedo", "color"), ("mask", "value"), ("fac", "value"), ("spare", "color")]
    s.name = "shading_aov"
    return s


def _closure_gallery(width, height, samples, name, materials, with_lamp=True):
    """A Cornell box with a 3 x 2 grid of spheres, one per material, lit by
    the ceiling light, a sphere point lamp and an area lamp behind the
    spheres (transmission through translucent / refractive surfaces)."""
    s = cornell_box(width, height, samples)
    base = len(s.materials)
    s.materials.extend(materials)
    centers = [(120.0, 330.0, 200.0), (278.0, 330.0, 200.0), (436.0, 330.0, 200.0),
               (120.0, 140.0, 200.0), (278.0, 140.0, 200.0), (436.0, 140.0, 200.0)]
    for i in range(len(materials)):
        c = centers[i % len(centers)]
        s.meshes.append(sc.Mesh(*_ellipsoid(c, (70.0, 70.0, 70.0), 20, 12), shader=base + i))
    if with_lamp:
        s.lamps = [
            sc.Lamp("point", co=(140.0, 480.0, 40.0), size=20.0, color=(1.0, 0.8, 0.6), strength=3.0e6),
            sc.Lamp("area", co=(278.0, 240.0, 420.0), direction=(0.0, 0.0, -1.0), axisu=(1.0, 0.0, 0.0),
                    axisv=(0.0, 1.0, 0.0), size=1.0, sizeu=300.0, sizev=200.0, color=(0.7, 0.9, 1.0),
                    strength=2.0e5),
        ]
    s.name = name
    return s


def closures_diffuse(width=48, height=48, samples=8) -> sc.Scene:
    """Diffuse-family closures (closure/bsdf_oren_nayar.h, bsdf_diffuse.h
    translucent, bsdf_ashikhmin_velvet.h, bsdf_toon.h), each mixed or bare."""
    mats = [
        sc.diffuse((0.8, 0.5, 0.3), roughness=0.6),  # Oren-Nayar
        sc.mix(0.5, sc.translucent((0.3, 0.8, 0.4)), sc.diffuse((0.7, 0.7, 0.7), roughness=1.0)),
        sc.velvet((0.9, 0.3, 0.5), sigma=0.4),
        sc.toon((0.4, 0.6, 0.9), size=0.45, smooth=0.1),
        sc.toon((0.9, 0.9, 0.6), size=0.2, smooth=0.05, glossy=True),
        sc.mix(0.4, sc.toon((0.2, 0.8, 0.8), size=0.7, smooth=0.0), sc.velvet((0.8, 0.8, 0.2), sigma=1.0)),
    ]
    return _closure_gallery(width, height, samples, "closures_diffuse", mats)


def closures_microfacet(width=48, height=48, samples=8) -> sc.Scene:
    """Microfacet closures (closure/bsdf_microfacet.h, bsdf_ashikhmin_shirley.h):
    Beckmann reflection / refraction / glass (table-sampled slopes), isotropic
    Ashikhmin-Shirley, anisotropic GGX and Beckmann with a tangent and a
    rotation from nodes, GGX refraction."""
    from . import nodes as nd

    g = nd.geometry()
    tangent = nd.vector_math("cross_product", g["Normal"], (0.0, 1.0, 0.0))["Vector"]
    rot = nd.math("multiply", nd.separate_xyz(g["Parametric"])["X"], 0.25)
    mats = [
        sc.mix(0.3, sc.diffuse((0.6, 0.2, 0.2)), sc.glossy((0.9, 0.8, 0.7), 0.35, distribution="beckmann")),
        sc.glass((0.95, 0.95, 1.0), 0.2, ior=1.5, distribution="beckmann"),
        sc.mix(0.5, sc.refraction((0.9, 1.0, 0.9), 0.3, ior=1.33, distribution="beckmann"),
               sc.refraction((1.0, 0.9, 0.9), 0.25, ior=1.45, distribution="ggx")),
        sc.mix(0.5, sc.glossy((0.8, 0.8, 0.9), 0.4, distribution="ashikhmin_shirley"),
               sc.diffuse((0.2, 0.3, 0.6))),
        sc.anisotropic((0.9, 0.7, 0.4), 0.4, 0.7, rot, tangent, distribution="ggx"),
        sc.anisotropic((0.7, 0.8, 0.9), 0.3, -0.5, 0.1, tangent, distribution="beckmann"),
    ]
    return _closure_gallery(width, height, samples, "closures_microfacet", mats)


def closures_principled(width=48, height=48, samples=8) -> sc.Scene:
    """Principled BSDF (svm_closure.h:100-463, GGX distribution): dielectric
    with specular, anisotropic metal, rough glass (transmission), sheen,
    clearcoat over half-metal, node-driven base colour and roughness."""
    from . import nodes as nd

    g = nd.geometry()
    tangent = nd.vector_math("cross_product", g["Normal"], (0.0, 1.0, 0.0))["Vector"]
    u = nd.separate_xyz(g["Parametric"])["X"]
    checker = nd.checker(nd.tex_coord()["Object"], (0.9, 0.3, 0.1), (0.1, 0.4, 0.8), 0.02)["Color"]
    mats = [
        sc.principled(base_color=(0.8, 0.2, 0.1), roughness=0.4, specular=0.5),
        sc.principled(base_color=(0.9, 0.7, 0.3), metallic=1.0, roughness=0.3, anisotropic=0.6,
                      anisotropic_rotation=0.1, tangent=tangent, specular=0.5),
        sc.principled(base_color=(0.9, 0.95, 1.0), transmission=1.0, roughness=0.1, ior=1.45, specular=0.5,
                      transmission_roughness=0.2),
        sc.principled(base_color=(0.3, 0.5, 0.8), sheen=1.0, sheen_tint=0.5, roughness=0.8, specular=0.3),
        sc.principled(base_color=(0.1, 0.1, 0.1), clearcoat=1.0, clearcoat_roughness=0.1, roughness=0.5,
                      specular=0.5, metallic=0.5),
        sc.principled(base_color=checker, roughness=nd.math("multiply", u, 0.8), specular=0.5, specular_tint=0.5,
                      ior=1.5, transmission=0.3),
    ]
    return _closure_gallery(width, height, samples, "closures_principled", mats)


def _test_image(seed, h, w, data_type, **kw):
    """A deterministic synthetic image (no image files are available): smooth
    gradients plus noise, in the texel type's range."""
    from . import nodes as nd

    rng = np.random.default_rng(seed)
    ch = 4 if data_type.endswith("4") else 1
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    base = np.stack([(xx / max(w - 1, 1)), (yy / max(h - 1, 1)), 0.5 + 0.5 * np.sin(xx * 0.7 + yy * 0.4),
                     0.2 + 0.8 * rng.random((h, w))], axis=2)[:, :, :ch]
    base = np.clip(base + 0.15 * rng.standard_normal(base.shape), 0.0, 1.0)
    if data_type in ("byte4", "byte"):
        px = np.round(base * 255).astype(np.uint8)
    elif data_type in ("ushort4", "ushort"):
        px = np.round(base * 65535).astype(np.uint16)
    elif data_type in ("half4", "half"):
        px = (base * 2.5).astype(np.float16).view(np.uint16)
    else:
        px = (base * np.array([3.0, 1.5, 0.8, 1.0])[:ch]).astype(np.float32)
    return nd.Image(px, data_type, **kw)


def shading_image(width=48, height=48, samples=8) -> sc.Scene:
    """Image and environment texture nodes (kernel_cpu_image.h, svm_image.h):
    every ImageDataType, closest / linear / cubic / smart interpolation,
    repeat / extend / clip, flat / sphere / tube projections, UDIM tiles,
    sRGB-compressed bytes, alpha unassociation, a mirror-ball environment
    lookup on a surface and an equirectangular HDR world (also the world
    light's importance map)."""
    from . import nodes as nd

    g = nd.geometry()
    uv = nd.separate_xyz(g["Parametric"])

    def uvw(su=1.0, sv=1.0, ou=0.0, ov=0.0):
        return nd.mapping(nd.combine_xyz(uv["X"], uv["Y"], 0.0), location=(ou, ov, 0.0), scale=(su, sv, 1.0))

    colors = []
    im = _test_image(1, 23, 37, "byte4", interpolation="linear", extension="repeat", compress_as_srgb=True)
    colors.append(nd.image_texture(im, uvw(2.3, 1.7, -0.4, -0.3))["Color"])
    im = _test_image(2, 16, 16, "float4", interpolation="cubic", extension="extend")
    colors.append(nd.image_texture(im, uvw(1.4, 1.4, -0.2, -0.2))["Color"])
    im = _test_image(3, 12, 20, "byte", interpolation="closest", extension="clip")
    colors.append(nd.image_texture(im, uvw(1.3, 1.2, -0.1, -0.1))["Color"])
    im = _test_image(4, 9, 13, "half4", interpolation="linear", extension="repeat")
    tex = nd.image_texture(im, uvw(1.9, 1.1), alpha_unassociate=True)
    colors.append(nd.mix_rgb("mix", tex["Alpha"], (0.1, 0.1, 0.1), tex["Color"]))
    im = _test_image(5, 7, 9, "float", interpolation="smart", extension="repeat")
    colors.append(nd.image_texture(im, nd.combine_xyz(uv["X"], uv["Y"], nd.math("multiply", uv["X"], 0.7)),
                                   projection="tube")["Color"])
    im = _test_image(6, 8, 8, "ushort4", interpolation="closest", extension="extend")
    colors.append(nd.image_texture(im, nd.combine_xyz(uv["X"], uv["Y"], 0.3), projection="sphere")["Color"])
    im = _test_image(7, 6, 6, "ushort", interpolation="linear", extension="clip")
    colors.append(nd.image_texture(im, uvw(1.2, 1.2, -0.1, -0.1))["Color"])
    im = _test_image(8, 10, 10, "half", interpolation="cubic", extension="clip")
    colors.append(nd.image_texture(im, uvw(1.3, 1.3, -0.15, -0.15))["Color"])
    udim = nd.Image(tiles={1001: _test_image(9, 8, 8, "byte4", interpolation="closest"),
                           1002: _test_image(10, 8, 8, "float4", interpolation="linear"),
                           1011: _test_image(11, 8, 8, "byte4", interpolation="linear")})
    colors.append(nd.image_texture(udim, uvw(2.0, 1.6))["Color"])
    env_small = _test_image(12, 8, 16, "float4", interpolation="linear")
    colors.append(nd.environment_texture(env_small, g["Normal"], projection="mirror_ball")["Color"])
    s = _grid_scene(colors, width, height, samples, "shading_image", glossy_every=4)
    hdr = _test_image(13, 16, 32, "float4", interpolation="linear")
    s.world_color = nd.environment_texture(hdr, g["Position"])["Color"]
    s.world_strength = 1.0
    s.world_map_resolution = 32
    return s


def shading_attributes(width=48, height=48, samples=8) -> sc.Scene:
    """Geometry attributes (geom_attribute.h, geom_triangle.h:114-356,
    svm_attribute.h, svm_vertex_color.h): the UV map through an image
    texture's default vector and the Texture Coordinate node, generated
    coordinates (a checker and a noise texture with default vectors), byte
    vertex colours (active and named layers, colour and alpha), named float /
    float2 / float3 attributes per vertex, face and corner read as Color,
    Vector and Fac, a missing attribute (zero), and a shared (instanced) mesh
    whose attributes are indexed through corrected offsets; the world reads
    Generated (the ray direction in a background shader)."""
    from . import nodes as nd

    im = _test_image(21, 13, 17, "byte4", interpolation="linear", extension="repeat")
    tc = nd.tex_coord()
    wear = nd.attribute("wear")
    colors = [
        nd.image_texture(im)["Color"],
        tc["UV"],
        tc["Generated"],
        nd.checker(scale=3.0)["Color"],
        nd.noise_texture(scale=4.0, detail=1.0)["Color"],
        nd.vertex_color()["Color"],
        nd.mix_rgb("mix", nd.vertex_color("Tint")["Alpha"], (0.1, 0.3, 0.1), nd.vertex_color("Tint")["Color"]),
        nd.color_ramp(wear["Fac"], [(0.0, (0.9, 0.2, 0.1, 1.0)), (1.0, (0.1, 0.3, 0.9, 1.0))])["Color"],
        nd.attribute("facecol")["Color"],
        nd.attribute("cornerf2")["Vector"],
        nd.mix_rgb("add", 0.5, nd.attribute("missing")["Color"], (0.2, 0.2, 0.6)),
        nd.mix_rgb("mix", nd.attribute("Col")["Fac"], nd.attribute("Col")["Color"], (0.9, 0.9, 0.2)),
        nd.combine_xyz(nd.attribute("uv")["Fac"], 0.3, 0.5),
        wear["Vector"],
    ]
    s = _grid_scene(colors, width, height, samples, "shading_attributes", glossy_every=5)
    rng = np.random.default_rng(77)
    for i, m in enumerate(s.meshes[:len(colors)]):
        nv, nt = len(m.verts), len(m.tris)
        m.uv = rng.uniform(-0.2, 1.3, (nt, 3, 2)).astype(np.float32)
        m.vertex_colors = {"Col": rng.uniform(0.0, 1.0, (nt, 3, 4)), "Tint": rng.uniform(0.0, 1.0, (nt, 3, 4))}
        m.attributes = {"wear": ("vertex", rng.uniform(0.0, 1.0, nv).astype(np.float32)),
                        "facecol": ("face", rng.uniform(0.0, 1.0, (nt, 3)).astype(np.float32)),
                        "cornerf2": ("corner", rng.uniform(0.0, 1.0, (3 * nt, 2)).astype(np.float32))}
    # a box shared by two objects (instanced: object-space vertices, own BVH)
    # whose generated coordinates and per-vertex attribute colour it
    bv, bt = _box((0.0, 0.0, 0.0), (0.5, 0.5, 0.5))
    n = len(s.materials)
    s.materials.append(sc.diffuse(nd.mix_rgb("mix", nd.attribute("wear")["Fac"], tc["Generated"], (0.8, 0.1, 0.1))))
    box = sc.Mesh(bv, bt, shader=n)
    box.attributes = {"wear": ("vertex", rng.uniform(0.0, 1.0, len(bv)).astype(np.float32))}
    box.uv = rng.uniform(0.0, 1.0, (len(bt), 3, 2)).astype(np.float32)
    s.instances = [sc.Instance(box, _tfm((-1.6, -1.2, -0.6), rot_y=0.5)),
                   sc.Instance(box, _tfm((1.5, 1.1, -0.5), rot_y=-0.3, scale=(0.8, 1.2, 0.8)))]
    gen = nd.separate_xyz(nd.tex_coord()["Generated"])
    s.world_color = nd.combine_xyz(nd.map_range(gen["Y"], -1.0, 1.0, 0.1, 0.6), 0.35,
                                   nd.map_range(gen["X"], -1.0, 1.0, 0.2, 0.7))
    return s


def closures_multiscatter(width=48, height=48, samples=8, filter_glossy=0.0) -> sc.Scene:
    """Multiple-scattering GGX (closure/bsdf_microfacet_multi.h, the
    MF_MULTI_GLOSSY walk of bsdf_microfacet_multi_impl.h): the Glossy BSDF's
    Multiscatter GGX distribution with a node-driven colour, the anisotropic
    variant with a tangent frame, and Principled BSDFs with the multiscatter
    distribution (Blender's default) as dielectric, tinted metal, anisotropic
    metal and clearcoat over a rough base; the walk steps each shading point's
    LCG.  filter_glossy > 0 also blurs the closures (bsdf_blur)."""
    from . import nodes as nd

    g = nd.geometry()
    tangent = nd.vector_math("cross_product", g["Normal"], (0.0, 1.0, 0.0))["Vector"]
    u = nd.separate_xyz(g["Parametric"])["X"]
    tint = nd.mix_rgb("mix", u, (0.9, 0.5, 0.2), (0.3, 0.7, 0.9))
    mats = [
        sc.mix(0.3, sc.diffuse((0.2, 0.5, 0.2)), sc.glossy(tint, 0.45, distribution="multi_ggx")),
        sc.anisotropic((0.9, 0.8, 0.6), 0.5, 0.6, 0.1, tangent, distribution="multi_ggx"),
        sc.principled("multiscatter", base_color=(0.8, 0.25, 0.1), roughness=0.5, specular=0.5),
        sc.principled("multiscatter", base_color=(0.95, 0.7, 0.35), metallic=1.0, roughness=0.35,
                      specular_tint=0.4),
        sc.principled("multiscatter", base_color=(0.7, 0.75, 0.8), metallic=1.0, roughness=0.6, anisotropic=0.5,
                      anisotropic_rotation=0.2, tangent=tangent),
        sc.principled("multiscatter", base_color=(0.1, 0.2, 0.6), roughness=0.9, clearcoat=0.8,
                      clearcoat_roughness=0.2, specular=0.6, metallic=0.3),
    ]
    s = _closure_gallery(width, height, samples, "closures_multiscatter", mats)
    s.filter_glossy = filter_glossy
    return s


def closures_multiscatter_glass(width=48, height=48, samples=8) -> sc.Scene:
    """Multiple-scattering GGX glass (the MF_MULTI_GLASS walk of
    bsdf_microfacet_multi_impl.h, beta() through glibc's lgammaf): Glass BSDFs
    with the Multiscatter GGX distribution (node-driven colour, rough and
    nearly smooth), and default Principled BSDFs (multiscatter distribution)
    with rough transmission -- a clear and a tinted glass, and a partly
    transmissive dielectric."""
    from . import nodes as nd

    g = nd.geometry()
    u = nd.separate_xyz(g["Parametric"])["X"]
    tint = nd.mix_rgb("mix", u, (0.95, 0.85, 0.6), (0.6, 0.9, 0.95))
    mats = [
        sc.glass(tint, 0.35, 1.45, distribution="multi_ggx"),
        sc.glass((0.9, 0.95, 0.9), 0.08, 1.33, distribution="multi_ggx"),
        sc.principled("multiscatter", base_color=(0.95, 0.95, 0.95), transmission=1.0, roughness=0.3, ior=1.45),
        sc.principled("multiscatter", base_color=(0.5, 0.8, 0.6), transmission=1.0, roughness=0.6, ior=1.5,
                      specular_tint=0.5),
        sc.principled("multiscatter", base_color=(0.8, 0.4, 0.2), transmission=0.5, roughness=0.45, metallic=0.2),
        sc.mix(0.5, sc.glass((0.9, 0.9, 0.9), 0.5, 1.6, distribution="multi_ggx"), sc.diffuse((0.3, 0.3, 0.7))),
    ]
    return _closure_gallery(width, height, samples, "closures_multiscatter_glass", mats)


def closures_layered(width=48, height=48, samples=8, triple=False) -> sc.Scene:
    """Materials needing more than 8 closures (the device's 16- and 64-closure
    shading variants): two Principled BSDFs mixed by a node-driven factor
    (16), a Principled BSDF over a multiscatter glossy and a translucent
    layer (11), and a deep mix tree of nine lobes; `triple` adds a mix of
    three Principled BSDFs (24: the 64-closure variant)."""
    from . import nodes as nd

    g = nd.geometry()
    u = nd.separate_xyz(g["Parametric"])["X"]
    p1 = sc.principled(base_color=(0.8, 0.3, 0.2), roughness=0.4, specular=0.5, clearcoat=0.5, sheen=0.3)
    p2 = sc.principled("multiscatter", base_color=(0.3, 0.6, 0.8), metallic=0.7, roughness=0.5, specular=0.4)
    deep = sc.diffuse((0.5, 0.5, 0.5))
    for i, c in enumerate([(0.9, 0.2, 0.2), (0.2, 0.9, 0.2), (0.2, 0.2, 0.9), (0.9, 0.9, 0.2)]):
        deep = sc.mix(0.5, deep, sc.mix(0.4, sc.glossy(c, 0.2 + 0.15 * i), sc.diffuse(c, roughness=0.3 * i)))
    mats = [
        sc.mix(u, p1, p2),
        sc.mix(0.5, sc.principled(base_color=(0.9, 0.8, 0.4), roughness=0.3, specular=0.5, clearcoat=1.0),
               sc.mix(0.5, sc.glossy((0.8, 0.8, 0.8), 0.5, distribution="multi_ggx"),
                      sc.translucent((0.4, 0.8, 0.4)))),
        deep,
        sc.mix(0.3, p1, sc.mix(0.5, p2, sc.principled(base_color=(0.4, 0.9, 0.4), roughness=0.2, specular=0.5)))
        if triple else sc.diffuse((0.6, 0.6, 0.6)),
        sc.mix(0.5, p2, sc.glossy((0.9, 0.6, 0.3), 0.3)),
        sc.principled(base_color=(0.2, 0.2, 0.2), roughness=0.6, specular=0.5),
    ]
    return _closure_gallery(width, height, samples, "closures_layered_triple" if triple else "closures_layered",
                            mats)


def shading_normals(width=48, height=48, samples=8) -> sc.Scene:
    """Normal perturbation and object data (svm_tex_coord.h:255-390,
    kernel_montecarlo.h ensure_valid_reflection, svm_geometry.h): tangent-space
    normal maps (UV tangents, their sign and the vertex normals, smooth and
    flat shading, strength above and below one), object / world / Blender
    object-space maps, the Tangent node (radial about each axis, UV map) and
    the Geometry node's Tangent feeding anisotropic BSDFs, Object Info (location,
    colour, pass index, random, material index) and an instanced, rotated mesh
    whose maps go through its object transform."""
    from . import nodes as nd

    def bumpy(seed):
        n = nd.noise_texture(scale=3.0 + seed, detail=1.0)["Color"]
        return nd.mix_rgb("mix", 0.6, (0.5, 0.5, 1.0), n)

    oi = nd.object_info()
    mats = [
        sc.diffuse((0.7, 0.6, 0.5), normal=nd.normal_map(bumpy(0))),
        sc.glossy((0.8, 0.8, 0.8), 0.3, normal=nd.normal_map(bumpy(1), strength=0.5)),
        sc.diffuse((0.5, 0.7, 0.6), normal=nd.normal_map(bumpy(2), strength=2.5)),
        sc.diffuse((0.6, 0.5, 0.7), normal=nd.normal_map(bumpy(3), space="object")),
        sc.glossy((0.7, 0.7, 0.6), 0.2, normal=nd.normal_map(bumpy(4), space="world")),
        sc.diffuse((0.6, 0.6, 0.6), normal=nd.normal_map(bumpy(5), space="blender_object", strength=0.8)),
        sc.anisotropic((0.9, 0.7, 0.5), 0.4, 0.7, 0.0, nd.tangent("radial", "x")),
        sc.anisotropic((0.5, 0.7, 0.9), 0.4, -0.6, 0.1, nd.tangent("radial", "y")),
        sc.anisotropic((0.7, 0.9, 0.5), 0.3, 0.5, 0.0, nd.tangent("uv_map")),
        sc.anisotropic((0.8, 0.8, 0.5), 0.35, 0.8, 0.0),  # default: geometry Tangent (radial z)
        sc.principled(base_color=(0.9, 0.6, 0.3), metallic=1.0, roughness=0.4, anisotropic=0.7),
        sc.diffuse(nd.combine_xyz(oi["Random"], nd.math("multiply", oi["Object Index"], 0.1),
                                  nd.math("multiply", oi["Material Index"], 0.2))),
        sc.diffuse(nd.mix_rgb("mix", 0.5, oi["Color"], nd.vector_math("fraction", oi["Location"])["Vector"])),
        # Fresnel / Layer Weight (svm_fresnel.h), facing bent through powf
        sc.mix(nd.layer_weight(0.3)["Facing"], sc.diffuse((0.2, 0.3, 0.8)), sc.glossy((0.9, 0.9, 0.9), 0.2)),
        sc.mix(nd.layer_weight(0.85, normal=nd.normal_map(bumpy(8)))["Facing"], sc.diffuse((0.8, 0.3, 0.2)),
               sc.glossy((0.9, 0.9, 0.9), 0.3)),
        sc.mix(nd.fresnel(nd.math("add", 1.2, nd.separate_xyz(nd.geometry()["Parametric"])["X"])),
               sc.diffuse((0.3, 0.7, 0.3)), sc.glossy((0.9, 0.9, 0.9), 0.1)),
        sc.mix(nd.layer_weight(0.4)["Fresnel"], sc.diffuse((0.6, 0.6, 0.2)), sc.glossy((0.8, 0.8, 0.9), 0.25)),
    ]
    s = _grid_scene([(0.5, 0.5, 0.5)] * len(mats), width, height, samples, "shading_normals")
    rng = np.random.default_rng(5)
    for i, m in enumerate(mats):
        s.materials[i] = m
        mesh = s.meshes[i]
        nt = len(mesh.tris)
        mesh.uv = rng.uniform(-0.3, 1.4, (nt, 3, 2)).astype(np.float32)
        mesh.smooth = (i % 2 == 0)
        mesh.object_color = tuple(float(x) for x in rng.uniform(0.0, 1.0, 3))
        mesh.pass_index = i
        mesh.object_random = float(np.float32(rng.uniform(0.0, 1.0)))
    s.materials[11].pass_index = 3
    s.materials[12].pass_index = 5
    # a sphere shared by two rotated objects: object-space maps and tangents
    # go through each object's transform
    sv, st = _ellipsoid((0.0, 0.0, 0.0), (0.45, 0.45, 0.45), 16, 10)
    n = len(s.materials)
    s.materials.append(sc.glossy((0.8, 0.7, 0.6), 0.35, normal=nd.normal_map(bumpy(6), strength=1.5)))
    s.materials.append(sc.diffuse((0.6, 0.7, 0.8), normal=nd.normal_map(bumpy(7), space="object")))
    ball = sc.Mesh(sv, st, shader=np.array([n + (k % 2) for k in range(len(st))]), smooth=True)
    ball.uv = rng.uniform(0.0, 1.0, (len(st), 3, 2)).astype(np.float32)
    ball.object_color = (0.9, 0.2, 0.3)
    s.instances = [sc.Instance(ball, _tfm((-1.5, 1.2, -0.7), rot_y=0.7, rot_x=0.4), pass_index=7, object_random=0.3),
                   sc.Instance(ball, _tfm((1.4, -1.1, -0.6), rot_y=-1.1, scale=(1.2, 0.8, 1.0)))]
    return s


def shading_converters(width=48, height=48, samples=8) -> sc.Scene:
    """Input / vector / converter nodes (svm_camera.h, svm_normal.h,
    svm_ramp.h curves, svm_vector_rotate.h, svm_vector_transform.h): Camera
    Data outputs, the Normal node's dot product, RGB and Vector Curves with
    values beyond the curve range (linear extrapolation), Vector Rotate about an
    axis / X / Y / Z / Euler (inverted too) and Vector Transform between world,
    object and camera spaces on a rotated, scaled instance."""
    from . import nodes as nd

    g = nd.geometry()
    P, N = g["Position"], g["Normal"]
    cam = nd.camera_data()

    def show(v, s=0.25):
        return nd.mix_rgb("mix", 1.0, (0.0, 0.0, 0.0), nd.mapping(v, scale=(s, s, s), location=(0.5, 0.5, 0.5)),
                          clamp=True)

    wave = nd.noise_texture(scale=2.0, detail=1.0)["Color"]
    wide = nd.mapping(wave, scale=(2.0, 2.0, 2.0), location=(-0.5, -0.5, -0.5))  # reaches below 0 and above 1
    colors = [
        show(cam["View Vector"], 0.5),
        nd.combine_xyz(nd.math("multiply", cam["View Z Depth"], 0.05), nd.math("multiply", cam["View Distance"], 0.04),
                       0.3),
        nd.combine_xyz(nd.normal((0.3, 0.5, -0.8), N)["Dot"], 0.4, nd.normal((0.0, 1.0, 0.0), N)["Dot"]),
        nd.rgb_curves(wide, r=((0.0, 0.1), (0.4, 0.7), (1.0, 0.9)), g=((0.0, 0.0), (1.0, 1.0)),
                      b=((0.0, 1.0), (0.5, 0.2), (1.0, 0.5))),
        nd.rgb_curves(wave, r=((0.0, 0.0), (1.0, 1.0)), g=((0.0, 0.3), (1.0, 0.6)), fac=0.6),
        show(nd.vector_curves(nd.mapping(P, scale=(0.7, 0.7, 0.7)), x=((-1, 0.5), (1, -0.5)),
                              y=((-1, -1), (0, 0.3), (1, 1)))),
        show(nd.vector_rotate(P, "axis", center=(0.2, 0.1, 0.0), axis=(0.3, 1.0, 0.2), angle=0.9)),
        show(nd.vector_rotate(P, "x", angle=1.2, invert=True)),
        show(nd.vector_rotate(P, "y", angle=-0.7)),
        show(nd.vector_rotate(P, "z", center=(0.5, 0.5, 0.0), angle=2.0)),
        show(nd.vector_rotate(P, "euler_xyz", rotation=(0.3, 0.6, 0.9))),
        show(nd.vector_rotate(P, "euler_xyz", rotation=(0.3, -0.4, 1.1), invert=True)),
        show(nd.vector_transform(P, "point", "world", "camera"), 0.1),
        show(nd.vector_transform(N, "normal", "world", "camera"), 0.5),
        show(nd.vector_transform(nd.geometry()["Incoming"], "vector", "camera", "world"), 0.5),
    ]
    s = _grid_scene(colors, width, height, samples, "shading_converters", glossy_every=4)
    # object-space transforms on a rotated, scaled instance shared by two objects
    bv, bt = _box((0.0, 0.0, 0.0), (0.6, 0.6, 0.6))
    n = len(s.materials)
    s.materials.append(sc.diffuse(show(nd.vector_transform(P, "point", "world", "object"), 0.8)))
    s.materials.append(sc.diffuse(show(nd.vector_transform(N, "normal", "object", "world"), 0.5)))
    s.materials.append(sc.diffuse(show(nd.vector_transform(P, "point", "camera", "object"), 0.2)))
    box = sc.Mesh(bv, bt, shader=np.array([n + (k % 3) for k in range(len(bt))]))
    s.instances = [sc.Instance(box, _tfm((-1.7, 1.3, -0.7), rot_y=0.6, rot_x=0.3, scale=(1.0, 0.7, 1.2))),
                   sc.Instance(box, _tfm((1.6, -1.2, -0.6), rot_y=-0.8))]
    return s
