"""Cycles XML scene ingestion: the standalone host's reader
(`blender/intern/cycles/app/cycles_xml.cpp`) restated over this repository's
host scene model (scene.py), so a scene written for `cycles --xml` reaches the
HIP device the way a Blender-synced one does.

    scene = read_file("cornell.xml", samples=16)
    ds = scene_mod.compile_scene(scene)

Semantics follow the reference reader element by element:
  * `<transform matrix|translate|rotate|scale>` composes onto the state's
    transform in that order (xml_read_transform, cycles_xml.cpp:550-579; the
    16-value matrix is transposed, rotate is degrees + axis);
  * `<state shader interpolation>` selects the shader of the meshes and lights
    that follow and their smooth / flat shading (xml_read_state, :581-610);
  * `<mesh P verts nverts UV>` adds one object per mesh with the state's
    transform, polygons fanned into triangles from their first corner and the
    optional per-corner UV map "UVMap" (xml_read_mesh, :394-536); subdivision
    surfaces are refused;
  * `<light>` reads the Light node sockets (type point | distant | area | spot |
    background (world importance sampling with its map_resolution),
    strength, co, dir, size, axisu/v, sizeu/v, round, spot_angle, spot_smooth,
    angle, use_mis default false, cast_shadow, max_bounces) with the state's
    shader; the transform does not apply (xml_read_light, :538-546);
  * `<camera>` (width, height, Camera sockets) takes the state's transform as
    its matrix (xml_read_camera, :189-202);
  * `<film>` (exposure, filter_type, filter_width) and `<integrator>` (bounce
    limits, seed, filter_glossy, caustics, light_sampling_threshold) read their
    node sockets; `<background>` holds the world shader graph;
  * `<shader name>` children are shader nodes (NodeType names of
    render/nodes.cpp, sockets by identifier, enums by name) and
    `<connect from="node socket" to="node socket">` links (case-insensitive
    socket names, xml_read_shader_graph :209-356); the graph's `output` node
    takes surface / volume;
  * `<include src>` reads another file relative to the current one.

Shader graphs are translated to the node / closure builders of nodes.py and
scene.py; node types or sockets outside that set raise ValueError naming
them (never silently dropped).  The reference host's default shaders
(shader.cpp:621-687): a mesh without a state shader gets default_surface
(diffuse 0.8), a light without one default_light (emission 0.8 x 0), the
world without a `<background>` graph is black.
"""
from __future__ import annotations

import math
import os
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from . import nodes
from . import scene as sc

f32 = np.float32

# --------------------------------------------------------------------------
# attribute parsing (graph/node_xml.cpp: whitespace-separated values, booleans
# "true" case-insensitive, enums by their registered names)


def _floats(s: str) -> list:
    return [float(t) for t in re.split(r"[\s,]+", s.strip()) if t]


def _ints(s: str) -> list:
    return [int(t) for t in re.split(r"[\s,]+", s.strip()) if t]


def _bool(s: str) -> bool:
    return s.strip().lower() == "true"


def _attr(el, name):
    """Attribute lookup by socket identifier (pugixml is case-sensitive; the
    reader matches sockets by their identifier)."""
    return el.attrib.get(name)


# --------------------------------------------------------------------------
# transforms (util_transform.h; Transform = 3x4 float rows, composed in float)


def _translate(t) -> np.ndarray:
    m = np.eye(4, dtype=f32)
    m[:3, 3] = f32(t)
    return m


def _scale(s) -> np.ndarray:
    return np.diag([f32(s[0]), f32(s[1]), f32(s[2]), f32(1.0)]).astype(f32)


def _rotate(angle: float, axis) -> np.ndarray:
    """transform_rotate (util_transform.h:196-218): axis normalised, Rodrigues."""
    angle = f32(angle)
    s, c = f32(math.sin(angle)), f32(math.cos(angle))
    t = f32(1.0) - c
    a = np.asarray(axis, dtype=f32)
    ln = f32(np.sqrt(f32(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])))
    x, y, z = (a / ln).astype(f32) if ln != 0 else a
    m = np.eye(4, dtype=f32)
    m[0, :3] = [x * x * t + c, x * y * t - s * z, x * z * t + s * y]
    m[1, :3] = [y * x * t + s * z, y * y * t + c, y * z * t - s * x]
    m[2, :3] = [z * x * t - s * y, z * y * t + s * x, z * z * t + c]
    return m


def _compose(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return (a.astype(f32) @ b.astype(f32)).astype(f32)


def read_transform(el, tfm: np.ndarray) -> np.ndarray:
    """xml_read_transform (cycles_xml.cpp:550-579)."""
    if _attr(el, "matrix") is not None:
        m = _floats(_attr(el, "matrix"))
        if len(m) == 16:
            # ProjectionTransform of the 16 values, transposed
            tfm = _compose(tfm, np.asarray(m, dtype=f32).reshape(4, 4).T)
    if _attr(el, "translate") is not None:
        v = _floats(_attr(el, "translate"))
        if len(v) == 3:
            tfm = _compose(tfm, _translate(v))
    if _attr(el, "rotate") is not None:
        v = _floats(_attr(el, "rotate"))
        if len(v) == 4:
            tfm = _compose(tfm, _rotate(math.radians(v[0]), v[1:]))
    if _attr(el, "scale") is not None:
        v = _floats(_attr(el, "scale"))
        if len(v) == 3:
            tfm = _compose(tfm, _scale(v))
    return tfm


# --------------------------------------------------------------------------
# shader graphs (xml_read_shader_graph) -> nodes.py / scene.py builders

MATH_NAMES = {"inversesqrt": "inv_sqrt", "smoothmin": "smooth_min", "smoothmax": "smooth_max"}
DISTRIBUTIONS = {"sharp": "sharp", "beckmann": "beckmann", "GGX": "ggx", "ashikhmin_shirley": "ashikhmin_shirley",
                 "Multiscatter GGX": "multi_ggx"}
GRADIENT_NAMES = {n: n for n in nodes.GRADIENT_TYPES}

# node type -> {socket identifier: (kind, default)}; kind f (float), c (colour /
# vector / point), e (enum name), b (boolean), i (int), n (vector input that
# defaults to unlinked: None)
_C08 = (0.8, 0.8, 0.8)
_Z3 = (0.0, 0.0, 0.0)
NODE_SOCKETS = {
    "diffuse_bsdf": {"color": ("c", _C08), "normal": ("n", None), "roughness": ("f", 0.0)},
    "glossy_bsdf": {"color": ("c", _C08), "normal": ("n", None), "distribution": ("e", "GGX"),
                    "roughness": ("f", 0.5)},
    "glass_bsdf": {"color": ("c", _C08), "normal": ("n", None), "distribution": ("e", "GGX"),
                   "roughness": ("f", 0.0), "IOR": ("f", 0.3)},
    "refraction_bsdf": {"color": ("c", _C08), "normal": ("n", None), "distribution": ("e", "GGX"),
                        "roughness": ("f", 0.0), "IOR": ("f", 0.3)},
    "translucent_bsdf": {"color": ("c", _C08), "normal": ("n", None)},
    "transparent_bsdf": {"color": ("c", (1.0, 1.0, 1.0))},
    "velvet_bsdf": {"color": ("c", _C08), "normal": ("n", None), "sigma": ("f", 1.0)},
    "emission": {"color": ("c", _C08), "strength": ("f", 10.0)},
    "background_shader": {"color": ("c", _C08), "strength": ("f", 1.0)},
    "mix_closure": {"fac": ("f", 0.5), "closure1": ("x", None), "closure2": ("x", None)},
    "absorption_volume": {"color": ("c", _C08), "density": ("f", 1.0)},
    "scatter_volume": {"color": ("c", _C08), "density": ("f", 1.0), "anisotropy": ("f", 0.0)},
    "value": {"value": ("f", 0.0)},
    "color": {"value": ("c", _Z3)},
    "texture_coordinate": {},
    "geometry": {},
    "light_path": {},
    "fresnel": {"normal": ("n", None), "IOR": ("f", 1.45)},
    "layer_weight": {"normal": ("n", None), "blend": ("f", 0.5)},
    "math": {"type": ("e", "add"), "use_clamp": ("b", False), "value1": ("f", 0.5), "value2": ("f", 0.5),
             "value3": ("f", 0.0)},
    "vector_math": {"type": ("e", "add"), "vector1": ("c", _Z3), "vector2": ("c", _Z3), "vector3": ("c", _Z3),
                    "scale": ("f", 1.0)},
    "mix": {"type": ("e", "mix"), "use_clamp": ("b", False), "fac": ("f", 0.5), "color1": ("c", _Z3),
            "color2": ("c", _Z3)},
    "invert": {"fac": ("f", 1.0), "color": ("c", _Z3)},
    "gamma": {"color": ("c", _Z3), "gamma": ("f", 1.0)},
    "hsv": {"hue": ("f", 0.5), "saturation": ("f", 1.0), "value": ("f", 1.0), "fac": ("f", 1.0),
            "color": ("c", _Z3)},
    "brightness_contrast": {"color": ("c", _Z3), "bright": ("f", 0.0), "contrast": ("f", 0.0)},
    "separate_xyz": {"vector": ("c", _Z3)},
    "combine_xyz": {"x": ("f", 0.0), "y": ("f", 0.0), "z": ("f", 0.0)},
    "checker_texture": {"vector": ("n", None), "color1": ("c", _Z3), "color2": ("c", _Z3), "scale": ("f", 1.0)},
    "gradient_texture": {"type": ("e", "linear"), "vector": ("n", None)},
    "noise_texture": {"dimensions": ("e", "3D"), "vector": ("n", None), "w": ("f", 0.0), "scale": ("f", 1.0),
                      "detail": ("f", 2.0), "roughness": ("f", 0.5), "distortion": ("f", 0.0)},
    "principled_bsdf": {"distribution": ("e", "Multiscatter GGX"), "subsurface_method": ("e", "burley"),
                        "base_color": ("c", _C08), "subsurface_color": ("c", _C08), "metallic": ("f", 0.0),
                        "subsurface": ("f", 0.0), "subsurface_radius": ("c", (0.1, 0.1, 0.1)),
                        "specular": ("f", 0.0), "roughness": ("f", 0.5), "specular_tint": ("f", 0.0),
                        "anisotropic": ("f", 0.0), "sheen": ("f", 0.0), "sheen_tint": ("f", 0.0),
                        "clearcoat": ("f", 0.0), "clearcoat_roughness": ("f", 0.03), "ior": ("f", 0.0),
                        "transmission": ("f", 0.0), "transmission_roughness": ("f", 0.0),
                        "anisotropic_rotation": ("f", 0.0), "emission": ("c", _Z3), "alpha": ("f", 1.0),
                        "normal": ("n", None), "clearcoat_normal": ("n", None), "tangent": ("n", None)},
    "subsurface_scattering": {"color": ("c", _C08), "normal": ("n", None), "falloff": ("e", "burley"),
                              "scale": ("f", 0.01), "radius": ("c", (0.1, 0.1, 0.1)), "sharpness": ("f", 0.0),
                              "texture_blur": ("f", 1.0)},
    "wavelength": {"wavelength": ("f", 500.0)},
    "blackbody": {"temperature": ("f", 1200.0)},
    "sky_texture": {"type": ("e", "nishita_improved"), "vector": ("n", None), "sun_direction": ("c", (0.0, 0.0, 1.0)),
                    "turbidity": ("f", 2.2), "ground_albedo": ("f", 0.3)},
    "ies_light": {"ies": ("s", None), "filename": ("s", None), "strength": ("f", 1.0), "vector": ("n", None)},
    "bump": {"invert": ("b", False), "use_object_space": ("b", False), "height": ("f", 1.0),
             "normal": ("n", None), "strength": ("f", 1.0), "distance": ("f", 0.1)},
    "ambient_occlusion": {"samples": ("i", 16), "color": ("c", (1.0, 1.0, 1.0)), "distance": ("f", 1.0),
                          "normal": ("n", None), "inside": ("b", False), "only_local": ("b", False)},
    "bevel": {"samples": ("i", 4), "radius": ("f", 0.05), "normal": ("n", None)},
    "wireframe": {"use_pixel_size": ("b", False), "size": ("f", 0.01)},
    "clamp": {"type": ("e", "minmax"), "value": ("f", 1.0), "min": ("f", 0.0), "max": ("f", 1.0)},
    "map_range": {"type": ("e", "linear"), "value": ("f", 1.0), "from_min": ("f", 0.0), "from_max": ("f", 1.0),
                  "to_min": ("f", 0.0), "to_max": ("f", 1.0), "steps": ("f", 4.0)},
    "light_falloff": {"strength": ("f", 100.0), "smooth": ("f", 0.0)},
    "white_noise_texture": {"dimensions": ("e", "3D"), "vector": ("n", None), "w": ("f", 0.0)},
    "object_info": {},
    "output": {"surface": ("x", None), "volume": ("x", None)},
}
# output socket identifier (lower case) -> builder key per node type
NODE_OUTPUTS = {
    "diffuse_bsdf": ("bsdf",), "glossy_bsdf": ("bsdf",), "glass_bsdf": ("bsdf",), "refraction_bsdf": ("bsdf",),
    "translucent_bsdf": ("bsdf",), "transparent_bsdf": ("bsdf",), "velvet_bsdf": ("bsdf",),
    "emission": ("emission",), "background_shader": ("background",), "mix_closure": ("closure",),
    "absorption_volume": ("volume",), "scatter_volume": ("volume",),
    "value": ("value",), "color": ("color",),
    "texture_coordinate": ("generated", "normal", "uv", "object", "camera", "window", "reflection"),
    "geometry": tuple(n.lower().replace(" ", "_") for n in nodes.GEOMETRY_OUTPUTS),
    "light_path": tuple(n.lower().replace(" ", "_") for n in nodes.LIGHT_PATH_OUTPUTS),
    "fresnel": ("fac",), "layer_weight": ("fresnel", "facing"), "math": ("value",), "vector_math": ("vector", "value"),
    "mix": ("color",), "invert": ("color",), "gamma": ("color",), "hsv": ("color",), "brightness_contrast": ("color",),
    "separate_xyz": ("x", "y", "z"), "combine_xyz": ("vector",),
    "checker_texture": ("color", "fac"), "gradient_texture": ("color", "fac"), "noise_texture": ("fac", "color"),
    "principled_bsdf": ("bsdf",), "subsurface_scattering": ("bssrdf",), "wavelength": ("color",),
    "blackbody": ("color",), "sky_texture": ("color",), "ies_light": ("fac",), "bump": ("normal",),
    "ambient_occlusion": ("color", "ao"), "bevel": ("normal",), "wireframe": ("fac",), "clamp": ("result",),
    "map_range": ("result",), "light_falloff": ("quadratic", "linear", "constant"),
    "white_noise_texture": ("value", "color"),
    "object_info": ("location", "color", "object_index", "material_index", "random"),
}


@dataclass
class _GraphNode:
    kind: str
    attrib: dict
    links: dict = field(default_factory=dict)  # input identifier -> (node name, output identifier)


class ShaderGraph:
    """One `<shader>` / `<background>` element's nodes and links."""

    def __init__(self, el, where: str, base: str = "."):
        self.where = where
        self.base = base  # directory of the XML file (ies_light filename)
        self.nodes = {"output": _GraphNode("output", {})}
        self._cache = {}
        for child in el:
            tag = child.tag
            if tag == "connect":
                fr = (child.attrib.get("from") or "").split()
                to = (child.attrib.get("to") or "").split()
                if len(fr) != 2 or len(to) != 2:
                    raise ValueError(f"{where}: invalid from or to value for connect node")
                self._connect(fr, to)
                continue
            kind = "background_shader" if tag == "background" else tag  # name collision (cycles_xml.cpp:327)
            if kind not in NODE_SOCKETS or kind == "output":
                raise ValueError(f"{where}: shader node type {tag!r} is not supported by the XML reader")
            name = child.attrib.get("name")
            if not name:
                raise ValueError(f"{where}: {tag} node without a name")
            known = set(NODE_SOCKETS[kind]) | {"name"}
            extra = [a for a in child.attrib if a not in known]
            if extra:
                raise ValueError(f"{where}: {tag} {name!r}: unsupported sockets {extra}")
            self.nodes[name] = _GraphNode(kind, dict(child.attrib))

    def _connect(self, fr, to):
        """Links are resolved against nodes declared before the connect, as the
        reference's node_map is filled in document order."""
        src, dst = self.nodes.get(fr[0]), self.nodes.get(to[0])
        if src is None or dst is None:
            raise ValueError(f"{self.where}: unknown shader node name {(fr[0] if src is None else to[0])!r}")
        outs = NODE_OUTPUTS.get(src.kind, ())
        out = next((o for o in outs if o == fr[1].lower()), None)
        if out is None:
            raise ValueError(f"{self.where}: unknown output socket {fr[1]!r} on {fr[0]!r}")
        inp = next((i for i in NODE_SOCKETS[dst.kind] if i.lower() == to[1].lower()), None)
        if inp is None:
            raise ValueError(f"{self.where}: unknown input socket {to[1]!r} on {to[0]!r}")
        dst.links[inp] = (fr[0], out)

    # -- evaluation ------------------------------------------------------------
    def _input(self, node: _GraphNode, ident: str):
        kind, default = NODE_SOCKETS[node.kind][ident]
        if ident in node.links:
            return self.output(*node.links[ident])
        raw = node.attrib.get(ident)
        if raw is None:
            return default
        if kind == "f":
            return float(_floats(raw)[0])
        if kind in ("c", "n"):
            v = _floats(raw)
            if len(v) != 3:
                raise ValueError(f"{self.where}: {node.kind}.{ident} needs 3 values")
            return tuple(v)
        if kind == "b":
            return _bool(raw)
        if kind == "i":
            return int(raw)
        if kind in ("e", "s"):
            return raw
        raise ValueError(f"{self.where}: {node.kind}.{ident} cannot be set by value")

    def output(self, name: str, out: str):
        key = (name, out)
        if key not in self._cache:
            self._cache[key] = self._build(self.nodes[name], out)
        return self._cache[key]

    def _build(self, n: _GraphNode, out: str):
        g = lambda ident: self._input(n, ident)  # noqa: E731
        k = n.kind
        if k == "diffuse_bsdf":
            return sc.diffuse(g("color"), roughness=g("roughness"), normal=g("normal"))
        if k in ("glossy_bsdf", "glass_bsdf", "refraction_bsdf"):
            dist = g("distribution")
            if dist not in DISTRIBUTIONS:
                raise ValueError(f"{self.where}: {k} distribution {dist!r}")
            d = DISTRIBUTIONS[dist]
            if k == "glossy_bsdf":
                return sc.glossy(g("color"), g("roughness"), normal=g("normal"), distribution=d)
            if d in ("ashikhmin_shirley", "multi_ggx"):
                raise ValueError(f"{self.where}: {k} distribution {dist!r} is not supported")
            build = sc.glass if k == "glass_bsdf" else sc.refraction
            return build(g("color"), g("roughness"), ior=g("IOR"), normal=g("normal"), distribution=d)
        if k == "translucent_bsdf":
            return sc.translucent(g("color"), normal=g("normal"))
        if k == "transparent_bsdf":
            return sc.transparent(g("color"))
        if k == "velvet_bsdf":
            return sc.velvet(g("color"), sigma=g("sigma"), normal=g("normal"))
        if k == "emission":
            return sc.emission(g("color"), g("strength"))
        if k == "background_shader":
            return sc.background(g("color"), g("strength"))
        if k == "mix_closure":
            a, b = g("closure1"), g("closure2")
            if a is None or b is None:
                raise ValueError(f"{self.where}: mix_closure with an unlinked closure input")
            return sc.mix(g("fac"), a, b)
        if k == "absorption_volume":
            return sc.volume_absorption(g("color"), g("density"))
        if k == "scatter_volume":
            return sc.volume_scatter(g("color"), g("density"), g("anisotropy"))
        if k in ("value", "color"):
            # constant nodes fold into the inputs they feed
            # (ValueNode / ColorNode::constant_fold, nodes.cpp)
            return g("value")
        if k == "texture_coordinate":
            node = nodes.tex_coord()
            return node["UV" if out == "uv" else out.capitalize()]
        if k == "geometry":
            return nodes.geometry()[next(o for o in nodes.GEOMETRY_OUTPUTS if o.lower().replace(" ", "_") == out)]
        if k == "light_path":
            return nodes.light_path()[next(o for o in nodes.LIGHT_PATH_OUTPUTS if o.lower().replace(" ", "_") == out)]
        if k == "fresnel":
            return nodes.fresnel(g("IOR"), normal=g("normal"))
        if k == "layer_weight":
            return nodes.layer_weight(g("blend"), normal=g("normal"))[out.capitalize()]
        if k == "math":
            op = MATH_NAMES.get(g("type"), g("type"))
            return nodes.math(op, g("value1"), g("value2"), g("value3"), clamp=g("use_clamp"))
        if k == "vector_math":
            node = nodes.vector_math(g("type"), g("vector1"), g("vector2"), g("vector3"), scale=g("scale"))
            return node["Vector" if out == "vector" else "Value"]
        if k == "mix":
            return nodes.mix_rgb(g("type"), g("fac"), g("color1"), g("color2"), clamp=g("use_clamp"))
        if k == "invert":
            return nodes.invert(g("color"), fac=g("fac"))
        if k == "gamma":
            return nodes.gamma(g("color"), g("gamma"))
        if k == "hsv":
            return nodes.hsv(g("color"), hue=g("hue"), saturation=g("saturation"), value_=g("value"), fac=g("fac"))
        if k == "brightness_contrast":
            return nodes.bright_contrast(g("color"), bright=g("bright"), contrast=g("contrast"))
        if k == "separate_xyz":
            return nodes.separate_xyz(g("vector"))[out.upper()]
        if k == "combine_xyz":
            return nodes.combine_xyz(g("x"), g("y"), g("z"))
        if k == "checker_texture":
            node = nodes.checker(g("vector"), g("color1"), g("color2"), scale=g("scale"))
            return node[out.capitalize()]
        if k == "gradient_texture":
            return nodes.gradient(g("vector"), kind=g("type"))[out.capitalize()]
        if k == "noise_texture":
            dims = {"1D": 1, "2D": 2, "3D": 3, "4D": 4}.get(g("dimensions"))
            if dims is None:
                raise ValueError(f"{self.where}: noise_texture dimensions {g('dimensions')!r}")
            node = nodes.noise_texture(g("vector"), w=g("w"), scale=g("scale"), detail=g("detail"),
                                       roughness=g("roughness"), distortion=g("distortion"), dimensions=dims)
            return node[out.capitalize()]
        if k == "principled_bsdf":
            return self._principled(g)
        if k == "subsurface_scattering":
            if g("falloff") not in sc.SUBSURFACE_FALLOFFS:
                raise ValueError(f"{self.where}: subsurface_scattering falloff {g('falloff')!r}")
            return sc.subsurface(g("color"), scale=g("scale"), radius=g("radius"), falloff=g("falloff"),
                                 texture_blur=g("texture_blur"), sharpness=g("sharpness"), normal=g("normal"))
        if k == "wavelength":
            return nodes.wavelength(g("wavelength"))
        if k == "blackbody":
            return nodes.blackbody(g("temperature"))
        if k == "sky_texture":
            # the Hosek-Wilkie and Nishita models need intern/sky's precomputation on the host
            if g("type") != "preetham":
                raise ValueError(f"{self.where}: sky_texture type {g('type')!r}: only preetham is computed by the "
                                 "XML reader's host")
            return nodes.sky_texture(self._vector(g, "generated"), "preetham", sun_direction=g("sun_direction"),
                                     turbidity=g("turbidity"))["Color"]
        if k == "ies_light":
            text = g("ies")
            if text is None:
                fn = g("filename")
                if fn is None:
                    raise ValueError(f"{self.where}: ies_light without ies or filename")
                with open(os.path.join(self.base, fn)) as f:
                    text = f.read()
            return nodes.ies_texture(self._vector(g, "normal"), text, strength=g("strength"))["Fac"]
        if k == "bump":
            return nodes.bump(g("height"), strength=g("strength"), distance=g("distance"), invert=g("invert"),
                              normal=g("normal"), object_space=g("use_object_space"))
        if k == "ambient_occlusion":
            node = nodes.ambient_occlusion(g("color"), g("distance"), normal=g("normal"), samples=g("samples"),
                                           inside=g("inside"), only_local=g("only_local"))
            return node["AO" if out == "ao" else "Color"]
        if k == "bevel":
            return nodes.bevel(g("radius"), normal=g("normal"), samples=g("samples"))
        if k == "wireframe":
            return nodes.wireframe(g("size"), use_pixel_size=g("use_pixel_size"))
        if k == "clamp":
            return nodes.clamp(g("value"), g("min"), g("max"), kind=g("type"))
        if k == "map_range":
            return nodes.map_range(g("value"), g("from_min"), g("from_max"), g("to_min"), g("to_max"),
                                   g("steps"), kind=g("type"))
        if k == "light_falloff":
            return nodes.light_falloff(g("strength"), g("smooth"))[out.capitalize()]
        if k == "white_noise_texture":
            dims = {"1D": 1, "2D": 2, "3D": 3, "4D": 4}.get(g("dimensions"))
            if dims is None:
                raise ValueError(f"{self.where}: white_noise_texture dimensions {g('dimensions')!r}")
            return nodes.white_noise_texture(g("vector"), w=g("w"), dimensions=dims)[out.capitalize()]
        if k == "object_info":
            name = {"location": "Location", "color": "Color", "object_index": "Object Index",
                    "material_index": "Material Index", "random": "Random"}[out]
            return nodes.object_info()[name]
        raise ValueError(f"{self.where}: node type {k!r} has no builder")

    @staticmethod
    def _vector(g, link):
        """A texture vector input's default link (graph.cpp default_inputs:
        LINK_TEXTURE_GENERATED / LINK_TEXTURE_NORMAL)."""
        v = g("vector")
        if v is not None:
            return v
        return nodes.tex_coord()["Generated" if link == "generated" else "Normal"]

    def _principled(self, g):
        """PrincipledBsdfNode (nodes.cpp:2665-2850) with its expand(): Alpha
        below 1 (or linked) becomes a mix with a transparent BSDF; Emission
        would become an add closure, which the scene model does not have."""
        dist = {"GGX": "ggx", "Multiscatter GGX": "multiscatter"}.get(g("distribution"))
        if dist is None:
            raise ValueError(f"{self.where}: principled_bsdf distribution {g('distribution')!r}")
        method = g("subsurface_method")
        em = g("emission")
        if nodes.is_linked(em) or tuple(em) != (0.0, 0.0, 0.0):
            raise ValueError(f"{self.where}: principled_bsdf emission (an add closure) is not supported")
        params = {key: g(key) for key in sc.PRINCIPLED_DEFAULTS}
        for key in sc.PRINCIPLED_VECTORS:
            if g(key) is not None:
                params[key] = g(key)
        bsdf = sc.principled(dist, subsurface_method=method, **params)
        alpha = g("alpha")
        if nodes.is_linked(alpha) or float(alpha) != 1.0:
            return sc.mix(alpha, sc.transparent((1.0, 1.0, 1.0)), bsdf)
        return bsdf

    def shader(self):
        """(surface closure or None, volume closure or None) at the output node."""
        outn = self.nodes["output"]
        surf = self.output(*outn.links["surface"]) if "surface" in outn.links else None
        vol = self.output(*outn.links["volume"]) if "volume" in outn.links else None
        for v, what in ((surf, "surface"), (vol, "volume")):
            if v is not None and not isinstance(v, sc.Closure):
                raise ValueError(f"{self.where}: output {what} must be linked to a closure")
        return surf, vol


# --------------------------------------------------------------------------
# the reader


@dataclass
class _State:
    """XMLReadState (cycles_xml.cpp:48-62)."""
    tfm: np.ndarray
    shader: str | None  # None: the scene's default_surface
    smooth: bool
    base: str


class XMLReader:
    def __init__(self, samples: int):
        self.samples = samples
        self.width, self.height = 0, 0
        self.camera = sc.Camera()
        self.camera_set = False
        self.shaders = {}  # name -> (surface, volume)
        self.materials = []  # scene materials in first-use order
        self.material_of = {}
        self.instances = []
        self.lamps = []
        self.film = {}
        self.integrator = {}
        self.world = None  # (surface, volume) of <background>
        self.background_light = None  # map resolution of a <light type="background">

    # -- materials ---------------------------------------------------------------
    def _material(self, shader: str | None) -> int:
        key = shader if shader is not None else "<default_surface>"
        if key not in self.material_of:
            if shader is None:
                m = sc.diffuse((0.8, 0.8, 0.8))
            else:
                surf, vol = self.shaders[shader]
                if surf is None:
                    if vol is None:
                        raise ValueError(f"shader {shader!r} has neither surface nor volume")
                    # a volume-only shader: no surface closure (shader.cpp:533)
                    surf = None
                m = sc.material(surf, vol) if vol is not None else surf
            self.material_of[key] = len(self.materials)
            self.materials.append(m)
        return self.material_of[key]

    # -- elements ----------------------------------------------------------------
    def read_scene(self, st: _State, root):
        for el in root:
            tag = el.tag.lower()  # string_iequals
            if tag == "film":
                self.film.update(el.attrib)
            elif tag == "integrator":
                self.integrator.update(el.attrib)
            elif tag == "camera":
                self.read_camera(st, el)
            elif tag == "shader":
                name = el.attrib.get("name")
                if not name:
                    raise ValueError("shader without a name")
                self.shaders[name] = ShaderGraph(el, f"shader {name!r}", st.base).shader()
            elif tag == "background":
                self.world = ShaderGraph(el, "background", st.base).shader()
            elif tag == "mesh":
                self.read_mesh(st, el)
            elif tag == "light":
                self.read_light(st, el)
            elif tag == "transform":
                self.read_scene(_State(read_transform(el, st.tfm), st.shader, st.smooth, st.base), el)
            elif tag == "state":
                sub = _State(st.tfm, st.shader, st.smooth, st.base)
                name = el.attrib.get("shader")
                if name is not None:
                    if name not in self.shaders:
                        raise ValueError(f"unknown shader {name!r}")
                    sub.shader = name
                interp = (el.attrib.get("interpolation") or "").lower()
                if interp == "smooth":
                    sub.smooth = True
                elif interp == "flat":
                    sub.smooth = False
                self.read_scene(sub, el)
            elif tag == "include":
                src = el.attrib.get("src")
                if src:
                    self.read_include(st, src)
            else:
                raise ValueError(f"unknown node {el.tag!r}")

    def read_include(self, st: _State, src: str):
        path = os.path.join(st.base, src)
        # a file may be included several times (e.g. under different
        # transforms), but not from inside itself
        real = os.path.realpath(path)
        active = self.__dict__.setdefault("_including", [])
        if real in active:
            chain = " -> ".join(os.path.basename(p) for p in active + [real])
            raise ValueError(f"{src}: include cycle ({chain})")
        root = ET.parse(path).getroot()
        if root.tag != "cycles":
            raise ValueError(f"{src}: the document element must be <cycles>")
        active.append(real)
        try:
            self.read_scene(_State(st.tfm, st.shader, st.smooth, os.path.dirname(path)), root)
        finally:
            active.pop()

    def read_camera(self, st: _State, el):
        a = el.attrib
        if "width" in a:
            self.width = int(a["width"])
        if "height" in a:
            self.height = int(a["height"])
        cam = sc.Camera()
        types = {"perspective": "perspective", "orthograph": "orthographic", "panorama": "panorama"}
        if "type" in a:
            if a["type"] not in types:
                raise ValueError(f"camera type {a['type']!r}")
            cam.type = types[a["type"]]
        cam.fov = float(a.get("fov", math.pi / 4))
        for key in ("nearclip", "farclip", "aperturesize", "focaldistance", "bladesrotation", "aperture_ratio",
                    "fisheye_fov", "fisheye_lens", "sensorwidth", "sensorheight", "latitude_min", "latitude_max",
                    "longitude_min", "longitude_max"):
            if key in a:
                setattr(cam, key, float(a[key]))
        if "sensorwidth" not in a:
            cam.sensorwidth = 0.036
        if "sensorheight" not in a:
            cam.sensorheight = 0.024
        if "blades" in a:
            cam.blades = int(a["blades"])
        if "panorama_type" in a:
            if a["panorama_type"] not in sc.PANORAMA_TYPES:
                raise ValueError(f"camera panorama_type {a['panorama_type']!r}")
            cam.panorama_type = a["panorama_type"]
        for key in ("motion", "shuttertime", "stereo_eye", "use_spherical_stereo"):
            if key in a:
                raise ValueError(f"camera {key} is not supported")
        cam.matrix = st.tfm.astype(np.float64)
        self.camera = cam
        self.camera_set = True

    def read_mesh(self, st: _State, el):
        a = el.attrib
        if (a.get("subdivision") or "").lower() in ("catmull-clark", "linear"):
            raise ValueError("mesh subdivision is not supported")
        P = np.asarray(_floats(a.get("P", "")), dtype=f32).reshape(-1, 3)
        verts = _ints(a.get("verts", ""))
        nverts = _ints(a.get("nverts", ""))
        tris, corners = [], []
        off = 0
        for nv in nverts:
            for j in range(nv - 2):
                tris.append((verts[off], verts[off + j + 1], verts[off + j + 2]))
                corners.append((off, off + j + 1, off + j + 2))
            off += nv
        tris = np.asarray(tris, dtype=np.int64).reshape(-1, 3)
        if len(tris) and (tris.max() >= len(P) or tris.min() < 0):
            raise ValueError("mesh vertex index out of range")
        uv = None
        if "UV" in a:
            uvs = np.asarray(_floats(a["UV"]), dtype=f32).reshape(-1, 2)
            uv = uvs[np.asarray(corners, dtype=np.int64)] if len(corners) else np.zeros((0, 3, 2), f32)
        mesh = sc.Mesh(verts=P, tris=tris, shader=self._material(st.shader), smooth=st.smooth, uv=uv)
        self.instances.append(sc.Instance(mesh, st.tfm[:3].astype(np.float64)))

    def read_light(self, st: _State, el):
        a = el.attrib
        kinds = {"point": "point", "distant": "sun", "area": "area", "spot": "spot"}
        kind = a.get("type", "point")
        if kind == "background":
            # the world's importance-sampled light (light.cpp:210-243): world
            # MIS with the light's map resolution
            self.background_light = int(a.get("map_resolution", 0))
            return
        if kind not in kinds:
            raise ValueError(f"light type {kind!r} is not supported")

        def v3(key, d):
            return tuple(_floats(a[key])) if key in a else d

        lamp = sc.Lamp(kinds[kind])
        lamp.color = v3("strength", (1.0, 1.0, 1.0))
        lamp.strength = 1.0
        lamp.co = v3("co", (0.0, 0.0, 0.0))
        lamp.direction = v3("dir", (0.0, 0.0, 0.0))
        lamp.size = float(a.get("size", 0.0))
        lamp.angle = float(a.get("angle", 0.0))
        lamp.axisu = v3("axisu", (0.0, 0.0, 0.0))
        lamp.axisv = v3("axisv", (0.0, 0.0, 0.0))
        lamp.sizeu = float(a.get("sizeu", 1.0))
        lamp.sizev = float(a.get("sizev", 1.0))
        lamp.round = _bool(a.get("round", "false"))
        lamp.spot_angle = float(a.get("spot_angle", math.pi / 4))
        lamp.spot_smooth = float(a.get("spot_smooth", 0.0))
        lamp.cast_shadow = _bool(a.get("cast_shadow", "true"))
        lamp.use_mis = _bool(a.get("use_mis", "false"))
        lamp.max_bounces = int(a.get("max_bounces", 1024))
        for key in ("is_portal", "use_diffuse", "use_glossy", "use_transmission", "use_scatter"):
            if key in a and _bool(a[key]) != (key != "is_portal"):
                raise ValueError(f"light {key} is not supported")
        # the light's shader: the state's (default_light when none is set)
        if st.shader is None:
            lamp.shader = sc.emission((0.8, 0.8, 0.8), 0.0)
        else:
            surf, _ = self.shaders[st.shader]
            if surf is None:
                raise ValueError(f"light shader {st.shader!r} has no surface")
            lamp.shader = surf
        self.lamps.append(lamp)

    # -- assembly -----------------------------------------------------------------
    def scene(self, name: str) -> sc.Scene:
        if not self.camera_set or self.width <= 0 or self.height <= 0:
            raise ValueError("the XML scene has no camera with width and height")
        s = sc.Scene(width=self.width, height=self.height, camera=self.camera, meshes=[],
                     materials=self.materials, samples=self.samples, name=name)
        s.instances = self.instances
        s.lamps = self.lamps
        # film (film.cpp:360-385 sockets; exposure default 0.8)
        f = self.film
        s.exposure = float(f.get("exposure", 0.8))
        ft = f.get("filter_type", "box")
        if ft not in ("box", "gaussian", "blackman_harris"):
            raise ValueError(f"film filter_type {ft!r}")
        s.filter_type = ft
        s.filter_width = float(f.get("filter_width", 1.0))
        # integrator (integrator.cpp:38-95 sockets)
        it = self.integrator
        for key in ("min_bounce", "max_bounce", "max_diffuse_bounce", "max_glossy_bounce",
                    "max_transmission_bounce", "transparent_max_bounce", "seed"):
            if key in it:
                setattr(s, key, int(it[key]))
        for key in ("filter_glossy", "light_sampling_threshold"):
            if key in it:
                setattr(s, key, float(it[key]))
        for key in ("caustics_reflective", "caustics_refractive"):
            if key in it:
                setattr(s, key, _bool(it[key]))
        for key, ok in (("method", "path"), ("sampling_pattern", "sobol"), ("motion_blur", "false")):
            if key in it and it[key].lower() != ok:
                raise ValueError(f"integrator {key}={it[key]!r} is not supported")
        # world: the <background> graph, or default_background (empty: black)
        if self.world is None or self.world[0] is None:
            s.world_color, s.world_strength = (0.0, 0.0, 0.0), 0.0
        else:
            bg = self.world[0]
            if bg.kind != "background":
                raise ValueError("background: output surface must be a background closure")
            s.world_color, s.world_strength = bg.color, bg.strength
        # a background light exists only when the file declares one
        s.world_mis = self.background_light is not None
        s.world_map_resolution = self.background_light or 0
        if self.world is not None and self.world[1] is not None:
            s.world_volume = self.world[1]
        return s


def read_file(path: str, samples: int = 16) -> sc.Scene:
    """xml_read_file (cycles_xml.cpp:687-700): the file and its includes."""
    r = XMLReader(samples)
    r.read_include(_State(np.eye(4, dtype=f32), None, False, os.path.dirname(os.path.abspath(path))),
                   os.path.basename(path))
    return r.scene(os.path.splitext(os.path.basename(path))[0])


def read_string(text: str, samples: int = 16, base: str = ".") -> sc.Scene:
    r = XMLReader(samples)
    root = ET.fromstring(text)
    if root.tag != "cycles":
        raise ValueError("the document element must be <cycles>")
    r.read_scene(_State(np.eye(4, dtype=f32), None, False, base), root)
    return r.scene("xml")
