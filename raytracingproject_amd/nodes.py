"""Shader node graph: texture, converter and input nodes feeding closure inputs.

The host side of the SVM nodes in csrc/kernel/cy_svm_nodes.h.  A node is built
with one of the constructors below; indexing it by an output name gives a
`Socket` that can be passed wherever a closure (scene.Closure) or another node
takes an input.  Plain numbers / 3-tuples stay constants.

Encodings follow the reference's ShaderNode::compile (render/nodes.cpp) and the
kernel decoders (kernel/svm/svm_*.h):
  * every linked or constant input gets a stack slot (SVMCompiler::stack_assign,
    render/svm.cpp:140-200; constants through NODE_VALUE_F / NODE_VALUE_V);
  * inputs the kernel reads with stack_load_float_default (checker scale,
    clamp min/max, map-range bounds) pass SVM_STACK_INVALID plus the value when
    unlinked (stack_assign_if_linked);
  * implicit socket conversions insert NODE_CONVERT (render/graph.cpp:250-300
    ConvertNode): float -> color/vector (FV), color -> float (CF, film rgb_to_y),
    vector -> float (VF).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

SVM_STACK_INVALID = 255

# svm_types.h node ids
NODE_GEOMETRY = 11
NODE_CONVERT = 12
NODE_TEX_COORD = 13
NODE_VALUE_F = 14
NODE_VALUE_V = 15
NODE_HSV = 36
NODE_MATH = 42
NODE_VECTOR_MATH = 43
NODE_RGB_RAMP = 44
NODE_GAMMA = 45
NODE_BRIGHTCONTRAST = 46
NODE_LIGHT_PATH = 47
NODE_MAPPING = 52
NODE_TEX_GRADIENT = 57
NODE_TEX_CHECKER = 62
# procedural noise textures (svm_types.h:89-128)
NODE_TEX_NOISE, NODE_TEX_MUSGRAVE, NODE_TEX_WAVE, NODE_TEX_MAGIC = 25, 59, 60, 61
NODE_TEX_BRICK, NODE_TEX_WHITE_NOISE, NODE_TEX_VORONOI = 63, 64, 58
VORONOI_FEATURES = {"f1": 0, "f2": 1, "smooth_f1": 2, "distance_to_edge": 3, "n_sphere_radius": 4}
VORONOI_METRICS = {"euclidean": 0, "manhattan": 1, "chebychev": 2, "minkowski": 3}
MUSGRAVE_TYPES = {"multifractal": 0, "fBm": 1, "hybrid_multifractal": 2, "ridged_multifractal": 3,
                  "hetero_terrain": 4}
WAVE_TYPES = {"bands": 0, "rings": 1}
WAVE_DIRECTIONS = {"x": 0, "y": 1, "z": 2, "diagonal": 3, "spherical": 3}
WAVE_PROFILES = {"sin": 0, "saw": 1, "tri": 2}
NODE_LIGHT_FALLOFF = 66
NODE_INVERT = 72
NODE_MIX = 73
NODE_SEPARATE_VECTOR = 74
NODE_COMBINE_VECTOR = 75
NODE_SEPARATE_HSV = 76
NODE_COMBINE_HSV = 77
NODE_MAP_RANGE = 83
NODE_CLAMP = 84
NODE_ATTR, NODE_VERTEX_COLOR = 16, 17
# bump evaluation (svm_types.h): the *_BUMP_DX / _DY forms of the geometry,
# attribute, vertex colour and texture coordinate nodes, and NODE_SET_BUMP
NODE_GEOMETRY_BUMP_DX, NODE_GEOMETRY_BUMP_DY = 18, 19
NODE_SET_BUMP, NODE_ATTR_BUMP_DX, NODE_ATTR_BUMP_DY = 26, 27, 28
NODE_VERTEX_COLOR_BUMP_DX, NODE_VERTEX_COLOR_BUMP_DY = 29, 30
NODE_TEX_COORD_BUMP_DX, NODE_TEX_COORD_BUMP_DY = 31, 32
NODE_CLOSURE_SET_NORMAL = 33
NODE_BEVEL, NODE_AMBIENT_OCCLUSION = 85, 86
NODE_WIREFRAME = 80
NODE_AO_ONLY_LOCAL, NODE_AO_INSIDE, NODE_AO_GLOBAL_RADIUS = 1, 2, 4
NODE_OBJECT_INFO, NODE_TANGENT, NODE_NORMAL_MAP = 48, 70, 71
NODE_FRESNEL, NODE_LAYER_WEIGHT = 38, 39
NODE_CAMERA, NODE_NORMAL, NODE_RGB_CURVES, NODE_VECTOR_CURVES = 54, 65, 68, 69
NODE_VECTOR_ROTATE, NODE_VECTOR_TRANSFORM = 78, 79
VECTOR_ROTATE_TYPES = {"axis": 0, "x": 1, "y": 2, "z": 3, "euler_xyz": 4}
VECTOR_TRANSFORM_TYPES = {"vector": 0, "point": 1, "normal": 2}
VECTOR_TRANSFORM_SPACES = {"world": 0, "object": 1, "camera": 2}
CAMERA_OUTPUTS = {"View Vector": "vector", "View Z Depth": "float", "View Distance": "float"}
NORMAL_MAP_SPACES = {"tangent": 0, "object": 1, "world": 2, "blender_object": 3, "blender_world": 4}
TANGENT_DIRECTIONS = {"radial": 0, "uv_map": 1}
TANGENT_AXES = {"x": 0, "y": 1, "z": 2}
OBJECT_INFO_OUTPUTS = {"Location": ("vector", 0), "Color": ("color", 1), "Object Index": ("float", 2),
                       "Material Index": ("float", 3), "Random": ("float", 4)}
# Particle Info / Hair Info (svm_types.h:185-205, nodes.cpp:4247-4426)
NODE_PARTICLE_INFO, NODE_HAIR_INFO, NODE_TEXTURE_MAPPING, NODE_MIN_MAX = 49, 50, 51, 53
PARTICLE_INFO_OUTPUTS = {"Index": ("float", 0), "Random": ("float", 1), "Age": ("float", 2),
                         "Lifetime": ("float", 3), "Location": ("vector", 4), "Size": ("float", 6),
                         "Velocity": ("vector", 7), "Angular Velocity": ("vector", 8)}
HAIR_INFO_OUTPUTS = {"Is Strand": "float", "Intercept": "float", "Thickness": "float",
                     "Tangent Normal": "vector", "Random": "float"}
NODE_INFO_CURVE_IS_STRAND, NODE_INFO_CURVE_THICKNESS, NODE_INFO_CURVE_TANGENT_NORMAL = 0, 2, 3
ATTR_STD_CURVE_INTERCEPT, ATTR_STD_CURVE_RANDOM = 14, 15
# NodeAttributeType (svm_types.h:160-166)
NODE_ATTR_FLOAT, NODE_ATTR_FLOAT2, NODE_ATTR_FLOAT3, NODE_ATTR_RGBA = 0, 1, 2, 3
# AttributeStandard (kernel_types.h:750-779) of the attributes this host packs;
# Attribute::standard_name (render/attribute.cpp:279-330) for the name lookup
ATTR_STD_UV, ATTR_STD_VERTEX_COLOR, ATTR_STD_GENERATED, ATTR_STD_NUM = 3, 6, 7, 26
ATTR_STD_VERTEX_NORMAL, ATTR_STD_UV_TANGENT, ATTR_STD_UV_TANGENT_SIGN = 1, 4, 5
ATTR_STD_NAMES = {"uv": ATTR_STD_UV, "vertex_color": ATTR_STD_VERTEX_COLOR, "generated": ATTR_STD_GENERATED,
                  "N": ATTR_STD_VERTEX_NORMAL, "tangent": ATTR_STD_UV_TANGENT, "tangent_sign": ATTR_STD_UV_TANGENT_SIGN}

# svm_types.h enums (the names are the Blender UI's, lower-cased)
MATH_OPS = ["add", "subtract", "multiply", "divide", "sine", "cosine", "tangent", "arcsine", "arccosine",
            "arctangent", "power", "logarithm", "minimum", "maximum", "round", "less_than", "greater_than",
            "modulo", "absolute", "arctan2", "floor", "ceil", "fraction", "sqrt", "inv_sqrt", "sign",
            "exponent", "radians", "degrees", "sinh", "cosh", "tanh", "trunc", "snap", "wrap", "compare",
            "multiply_add", "pingpong", "smooth_min", "smooth_max"]
# the shading_math golden grid: every op but the libm tan / sinh / cosh / tanh,
# which the shading_math_libm case covers (all restated bit-exactly)
MATH_OPS_GRID = [op for op in MATH_OPS if op not in ("tangent", "sinh", "cosh", "tanh")]
VECTOR_MATH_OPS = ["add", "subtract", "multiply", "divide", "cross_product", "project", "reflect",
                   "dot_product", "distance", "length", "scale", "normalize", "snap", "floor", "ceil",
                   "modulo", "fraction", "absolute", "minimum", "maximum", "wrap", "sine", "cosine",
                   "tangent"]
VECTOR_MATH_VALUE_OPS = ("dot_product", "distance", "length")
MIX_TYPES = ["mix", "add", "multiply", "subtract", "screen", "divide", "difference", "darken", "lighten",
             "overlay", "dodge", "burn", "hue", "saturation", "value", "color", "soft_light", "linear_light"]
NODE_MIX_CLAMP = 18
GRADIENT_TYPES = ["linear", "quadratic", "easing", "diagonal", "radial", "quadratic_sphere", "spherical"]
TEXCO_OUTPUTS = {"Normal": 0, "Object": 1, "Camera": 2, "Window": 3, "Reflection": 4}
GEOMETRY_OUTPUTS = {"Position": 0, "Normal": 1, "Tangent": 2, "Incoming": 3, "True Normal": 4, "Parametric": 5}
LIGHT_PATH_OUTPUTS = ["Is Camera Ray", "Is Shadow Ray", "Is Diffuse Ray", "Is Glossy Ray", "Is Singular Ray",
                      "Is Reflection Ray", "Is Transmission Ray", "Is Volume Scatter Ray", "Is Backfacing",
                      "Ray Length", "Ray Depth", "Diffuse Depth", "Glossy Depth", "Transparent Depth",
                      "Transmission Depth"]
LIGHT_FALLOFF_OUTPUTS = {"Quadratic": 0, "Linear": 1, "Constant": 2}
MAPPING_TYPES = ["point", "texture", "vector", "normal"]
CLAMP_TYPES = ["minmax", "range"]
MAP_RANGE_TYPES = ["linear", "stepped", "smoothstep", "smootherstep"]

CONVERT_FV, CONVERT_CF, CONVERT_VF = 0, 2, 4


def f32bits(x: float) -> int:
    return int(np.array([x], dtype=np.float32).view(np.uint32)[0])


def uchar4(x, y=0, z=0, w=0) -> int:
    return (x & 0xFF) | ((y & 0xFF) << 8) | ((z & 0xFF) << 16) | ((w & 0xFF) << 24)


@dataclass(eq=False)
class Node:
    kind: str
    inputs: dict = field(default_factory=dict)
    params: dict = field(default_factory=dict)

    def __getitem__(self, name: str) -> "Socket":
        if name not in _outputs(self):
            raise KeyError(f"{self.kind} node has no output {name!r}; outputs: {sorted(_outputs(self))}")
        return Socket(self, name)


@dataclass(frozen=True, eq=False)
class Socket:
    node: Node
    name: str

    @property
    def type(self) -> str:
        return _outputs(self.node)[self.name]


def is_linked(v) -> bool:
    return isinstance(v, Socket)


# ---------------------------------------------------------------------------
# constructors (render/nodes.cpp socket names and defaults)


def value(v: float) -> Socket:
    return Node("value", params={"value": float(v)})["Value"]


def rgb(c) -> Socket:
    return Node("rgb", params={"value": tuple(float(x) for x in c)})["Color"]


def tex_coord() -> Node:
    """Texture Coordinate node (nodes.cpp:3818-3923): Generated and UV read the
    mesh attributes (render/attribute.cpp: generated = vertex float3, uv =
    corner float2), the others NODE_TEX_COORD."""
    return Node("tex_coord")


def attribute(name: str) -> Node:
    """Attribute node (nodes.cpp:5394-5436): the named (or standard: "uv",
    "generated", "vertex_color") geometry attribute as Color / Vector / Fac."""
    return Node("attribute", params={"name": str(name)})


def vertex_color(layer: str = "") -> Node:
    """Vertex Color node (nodes.cpp:4532-4568): a byte-colour corner attribute
    (the active layer when `layer` is empty) as Color and Alpha."""
    return Node("vertex_color", params={"layer": str(layer)})


def normal_map(color=(0.5, 0.5, 1.0), strength=1.0, space: str = "tangent", uv_map: str = "") -> Socket:
    """Normal Map node (nodes.cpp:6717-6761, svm_tex_coord.h:255-345): a
    tangent-space map reads the UV tangent, its sign and the vertex normal
    (attributes `uv_map`.tangent / .tangent_sign, or the standard ones when
    `uv_map` is empty); object / world spaces transform the colour directly."""
    if space not in NORMAL_MAP_SPACES:
        raise ValueError(f"normal_map space one of {sorted(NORMAL_MAP_SPACES)}")
    return Node("normal_map", {"Color": color, "Strength": strength}, {"space": space, "uv_map": uv_map})["Normal"]


def tangent(direction: str = "radial", axis: str = "z", uv_map: str = "") -> Socket:
    """Tangent node (nodes.cpp:6813-6847, svm_tex_coord.h:347-390): radial
    around an axis of the generated coordinates, or the UV map's tangent."""
    if direction not in TANGENT_DIRECTIONS or axis not in TANGENT_AXES:
        raise ValueError("tangent: direction radial | uv_map, axis x | y | z")
    return Node("tangent", params={"direction": direction, "axis": axis, "uv_map": uv_map})["Tangent"]


def fresnel(ior=1.45, normal=None) -> Socket:
    """Fresnel node (nodes.cpp FresnelNode, svm_fresnel.h:21-38): Fac."""
    return Node("fresnel", {"IOR": ior, "Normal": normal})["Fac"]


def layer_weight(blend=0.5, normal=None) -> Node:
    """Layer Weight node (nodes.cpp LayerWeightNode, svm_fresnel.h:40-75):
    Fresnel and Facing (blend != 0.5 bends Facing through powf)."""
    return Node("layer_weight", {"Blend": blend, "Normal": normal})


def camera_data() -> Node:
    """Camera Data node (nodes.cpp CameraNode, svm_camera.h): View Vector,
    View Z Depth, View Distance."""
    return Node("camera_data")


def normal(direction=(0.0, 0.0, 1.0), normal_in=(0.0, 0.0, 1.0)) -> Node:
    """Normal node (nodes.cpp NormalNode, svm_normal.h): the node's direction
    and its Dot with the normalised input."""
    return Node("normal", {"Normal": normal_in}, {"direction": tuple(float(x) for x in direction)})


def _curve_table(points, table_size, min_x, max_x):
    """Piecewise-linear curve through (x, y) control points sampled at
    table_size positions over [min_x, max_x] (the host bakes Blender's curve
    mapping to such a table, CurvesNode / curvemapping_table_RGBA)."""
    pts = sorted((float(x), float(y)) for x, y in points)
    xs = np.array([p for p, _ in pts]), np.array([q for _, q in pts])
    x = min_x + (max_x - min_x) * np.arange(table_size, dtype=np.float64) / (table_size - 1)
    return np.interp(x, xs[0], xs[1])


def rgb_curves(color, r=((0, 0), (1, 1)), g=((0, 0), (1, 1)), b=((0, 0), (1, 1)), fac=1.0,
               table_size: int = 257, min_x: float = 0.0, max_x: float = 1.0) -> Socket:
    """RGB Curves node (nodes.cpp RGBCurvesNode / CurvesNode::compile,
    svm_ramp.h svm_node_curves): per-channel curves with linear extrapolation
    outside [min_x, max_x]."""
    table = np.stack([_curve_table(c, table_size, min_x, max_x) for c in (r, g, b)], axis=1)
    return Node("rgb_curves", {"Fac": fac, "Color": color},
                {"table": table, "min_x": float(min_x), "max_x": float(max_x)})["Color"]


def vector_curves(vector, x=((-1, -1), (1, 1)), y=((-1, -1), (1, 1)), z=((-1, -1), (1, 1)), fac=1.0,
                  table_size: int = 257, min_x: float = -1.0, max_x: float = 1.0) -> Socket:
    """Vector Curves node (nodes.cpp VectorCurvesNode): per-component curves."""
    table = np.stack([_curve_table(c, table_size, min_x, max_x) for c in (x, y, z)], axis=1)
    return Node("vector_curves", {"Fac": fac, "Vector": vector},
                {"table": table, "min_x": float(min_x), "max_x": float(max_x)})["Vector"]


def vector_rotate(vector, kind: str = "axis", center=(0.0, 0.0, 0.0), axis=(0.0, 0.0, 1.0), angle=0.0,
                  rotation=(0.0, 0.0, 0.0), invert: bool = False) -> Socket:
    """Vector Rotate node (nodes.cpp VectorRotateNode, svm_vector_rotate.h)."""
    if kind not in VECTOR_ROTATE_TYPES:
        raise ValueError(f"vector_rotate type one of {sorted(VECTOR_ROTATE_TYPES)}")
    return Node("vector_rotate", {"Vector": vector, "Rotation": rotation, "Center": center, "Axis": axis,
                                  "Angle": angle}, {"type": kind, "invert": bool(invert)})["Vector"]


def vector_transform(vector, kind: str = "vector", convert_from: str = "world", convert_to: str = "object") -> Socket:
    """Vector Transform node (nodes.cpp VectorTransformNode, svm_vector_transform.h)."""
    if kind not in VECTOR_TRANSFORM_TYPES or convert_from not in VECTOR_TRANSFORM_SPACES or \
            convert_to not in VECTOR_TRANSFORM_SPACES:
        raise ValueError("vector_transform: type vector | point | normal, spaces world | object | camera")
    return Node("vector_transform", {"Vector": vector}, {"type": kind, "from": convert_from,
                                                         "to": convert_to})["Vector"]


def object_info() -> Node:
    """Object Info node (nodes.cpp:4211-4237, svm_geometry.h:104-139): Location,
    Color, Object Index, Material Index, Random."""
    return Node("object_info")


def particle_info() -> Node:
    """Particle Info node (nodes.cpp:4247-4347, svm_geometry.h:141-202): the
    instancing object's particle (KernelObject.particle_index into __particles):
    Index, Random, Age, Lifetime, Location, Size, Velocity, Angular Velocity."""
    return Node("particle_info")


def hair_info() -> Node:
    """Hair Info node (nodes.cpp:4354-4426, svm_geometry.h:204-243): Is Strand,
    Thickness and Tangent Normal from the hit curve segment; Intercept and
    Random read the curves' ATTR_STD_CURVE_INTERCEPT / _RANDOM attributes."""
    return Node("hair_info")


def texture_mapping(vector, tfm, min_=None, max_=None, normalize: bool = False) -> Socket:
    """A texture node's TextureMapping (nodes.cpp:155-176 compile, the mapping
    Blender's legacy texture settings carry): the vector through the 3x4
    matrix `tfm` (TextureMapping::compute_transform's result, any affine map
    here), then clamped to [min_, max_] per component (use_minmax), then
    normalized (type NORMAL)."""
    t = np.asarray(tfm, dtype=np.float32).reshape(3, 4)
    mm = None if min_ is None else (tuple(float(v) for v in min_), tuple(float(v) for v in max_))
    return Node("texture_mapping", inputs={"Vector": vector},
                params={"tfm": t, "minmax": mm, "normalize": bool(normalize)})["Vector"]


def _default_vector(vector, kind: str = "generated"):
    """ShaderGraph::default_inputs (render/graph.cpp:830-880): an unlinked
    texture vector reads the generated coordinates (LINK_TEXTURE_GENERATED) or
    the UV map (LINK_TEXTURE_UV)."""
    if vector is not None:
        return vector
    return tex_coord()["UV" if kind == "uv" else "Generated"]


def geometry() -> Node:
    return Node("geometry")


def light_path() -> Node:
    return Node("light_path")


def light_falloff(strength=100.0, smooth=0.0) -> Node:
    return Node("light_falloff", {"Strength": strength, "Smooth": smooth})


def math(op: str, a=0.5, b=0.5, c=0.0, clamp: bool = False) -> Socket:
    if op not in MATH_OPS:
        raise ValueError(f"unknown math op {op!r}")
    return Node("math", {"Value1": a, "Value2": b, "Value3": c}, {"op": op, "clamp": clamp})["Value"]


def vector_math(op: str, a=(0.0, 0.0, 0.0), b=(0.0, 0.0, 0.0), c=(0.0, 0.0, 0.0), scale=1.0) -> Node:
    if op not in VECTOR_MATH_OPS:
        raise ValueError(f"unknown vector math op {op!r}")
    return Node("vector_math", {"Vector1": a, "Vector2": b, "Vector3": c, "Scale": scale}, {"op": op})


def mix_rgb(blend: str, fac, color1, color2, clamp: bool = False) -> Socket:
    if blend not in MIX_TYPES:
        raise ValueError(f"unknown mix type {blend!r}")
    return Node("mix", {"Fac": fac, "Color1": color1, "Color2": color2}, {"type": blend, "clamp": clamp})["Color"]


def hsv(color, hue=0.5, saturation=1.0, value_=1.0, fac=1.0) -> Socket:
    return Node("hsv", {"Hue": hue, "Saturation": saturation, "Value": value_, "Fac": fac, "Color": color})["Color"]


def gamma(color, g=1.0) -> Socket:
    return Node("gamma", {"Color": color, "Gamma": g})["Color"]


def bright_contrast(color, bright=0.0, contrast=0.0) -> Socket:
    return Node("brightcontrast", {"Color": color, "Bright": bright, "Contrast": contrast})["Color"]


def invert(color, fac=1.0) -> Socket:
    return Node("invert", {"Fac": fac, "Color": color})["Color"]


def checker(vector=None, color1=(0.8, 0.8, 0.8), color2=(0.2, 0.2, 0.2), scale=5.0) -> Node:
    return Node("checker", {"Vector": _default_vector(vector), "Color1": color1, "Color2": color2, "Scale": scale})


IMAGE_DATA_TYPES = ("float4", "byte4", "half4", "float", "byte", "half", "ushort4", "ushort")
INTERPOLATIONS = ("linear", "closest", "cubic", "smart")
EXTENSIONS = ("repeat", "extend", "clip")
IMAGE_PROJECTIONS = {"flat": 0, "sphere": 2, "tube": 3}
ENVIRONMENT_PROJECTIONS = {"equirectangular": 0, "mirror_ball": 1}
NODE_TEX_IMAGE, NODE_TEX_ENVIRONMENT = 23, 55
NODE_TEX_VOXEL = 87  # svm_types.h
ATTR_STD_GENERATED_TRANSFORM = 8  # kernel_types.h AttributeStandard
NODE_IMAGE_COMPRESS_AS_SRGB, NODE_IMAGE_ALPHA_UNASSOCIATE = 1, 2


@dataclass(eq=False)
class Image:
    """One image of the ImageManager (render/image.cpp): texels in one of the
    ImageDataTypes (util_texture.h:51-62), uploaded to an SVM image slot by
    the device's tex_alloc.  `pixels` is (H, W, C) with C = 4 for the
    *4 types and 1 (or 2-D) for the single-channel ones; row 0 is v = 0.
    `tiles` maps UDIM tile numbers (1001, 1002, ...) to Images for a tiled
    image; then `pixels` is unused.  A 3D image (volume grids, the Point
    Density node's voxels) has `depth` > 1 and pixels (D, H, W, C);
    `transform_3d` (3, 4) sets TextureInfo::use_transform_3d / transform_3d."""
    pixels: object = None
    data_type: str = "byte4"
    interpolation: str = "linear"
    extension: str = "repeat"
    compress_as_srgb: bool = False  # byte images stored in sRGB (ImageMetaData)
    tiles: dict | None = None
    depth: int = 1
    transform_3d: object = None

    def texel_array(self) -> np.ndarray:
        dt = {"float4": np.float32, "float": np.float32, "byte4": np.uint8, "byte": np.uint8,
              "half4": np.uint16, "half": np.uint16, "ushort4": np.uint16, "ushort": np.uint16}[self.data_type]
        a = np.ascontiguousarray(self.pixels, dtype=dt)
        ch = 4 if self.data_type.endswith("4") else 1
        nd = 4 if self.depth > 1 else 3
        if a.ndim == nd - 1 and ch == 1:
            a = a[..., None]
        if a.ndim != nd or a.shape[-1] != ch or (nd == 4 and a.shape[0] != self.depth):
            want = f"(D={self.depth}, H, W, {ch})" if nd == 4 else f"(H, W, {ch})"
            raise ValueError(f"{self.data_type} image needs shape {want}, got {a.shape}")
        return a

    def dims(self) -> tuple:
        """(width, height, depth) of the texel array"""
        a = self.texel_array()
        return (a.shape[2], a.shape[1], a.shape[0]) if self.depth > 1 else (a.shape[1], a.shape[0], 1)


def image_texture(image: Image, vector=None, projection: str = "flat", alpha_unassociate: bool = False) -> Node:
    """Image Texture node (nodes.cpp ImageTextureNode, svm_image.h:43-112).
    An unlinked vector reads the UV map (LINK_TEXTURE_UV); box projection is
    not implemented.  alpha_unassociate sets NODE_IMAGE_ALPHA_UNASSOCIATE (the
    reference sets it when the Alpha output is used on a non-data image)."""
    return Node("image_texture", {"Vector": _default_vector(vector, "uv")},
                params={"image": image, "projection": IMAGE_PROJECTIONS[projection],
                        "alpha_unassociate": alpha_unassociate})


def point_density(image: Image, vector=None, space: str = "object", tfm=None) -> Node:
    """Point Density texture node (nodes.cpp:1810-1852 PointDensityTextureNode::
    compile, svm_voxel.h): the host-built voxel grid `image` (3D, float4:
    colour in rgb, density in alpha) looked up at the input point, in object
    space (volume_normalized_position) or through `tfm` (3x4, world space).
    The vector defaults to the shading position."""
    if space not in ("object", "world"):
        raise ValueError(f"point density space {space!r}: object or world")
    if image.depth <= 1:
        raise ValueError("point density needs a 3D image (depth > 1)")
    t = np.eye(4)[:3] if tfm is None else np.asarray(tfm, dtype=np.float64).reshape(3, 4)
    return Node("point_density", {"Vector": vector if vector is not None else geometry()["Position"]},
                params={"image": image, "space": space, "tfm": t})


def environment_texture(image: Image, vector, projection: str = "equirectangular") -> Node:
    """Environment Texture node (nodes.cpp EnvironmentTextureNode,
    svm_image.h:218-245); in a world shader geometry()["Position"] is the ray
    direction."""
    return Node("environment_texture", {"Vector": vector},
                params={"image": image, "projection": ENVIRONMENT_PROJECTIONS[projection]})


SKY_TYPES = {"preetham": 0, "hosek_wilkie": 1, "nishita_improved": 2}
NODE_TEX_SKY = 56


def _sky_preetham(sun_direction, turbidity):
    """nodes.cpp:624-705 sky_texture_precompute_preetham, in float32: the sun's
    (theta, phi), zenith Y / x / y (radiance_x/y/z) and the Perez
    coefficients (config_x/y/z[0..4]) normalised at the zenith."""
    f = np.float32
    d = np.asarray(sun_direction, dtype=np.float32)
    theta, phi = f(np.arccos(d[2])), f(np.arctan2(d[0], d[1]))
    theta2 = f(theta * theta)
    theta3 = f(theta2 * theta)
    T = f(turbidity)
    T2 = f(T * T)
    chi = f(f(f(4.0 / 9.0) - f(T / f(120.0))) * f(f(np.pi) - f(2.0) * theta))
    rx = f(f(f(f(4.0453) * T - f(4.9710)) * f(np.tan(chi)) - f(0.2155) * T) + f(2.4192))
    rx = f(rx * f(0.06))

    def poly(a, b, c, d_, e, g, h, i, j, k, l_):
        t1 = f(f(f(a) * theta3 - f(b) * theta2) + f(c) * theta)
        t2 = f(f(f(f(d_) * theta3 + f(e) * theta2) - f(g) * theta) + f(h))
        t3 = f(f(f(f(i) * theta3 - f(j) * theta2) + f(k) * theta) + f(l_))
        return f(f(t1 * T2 + t2 * T) + t3)

    ry = poly(0.00166, 0.00375, 0.00209, -0.02903, 0.06377, 0.03202, 0.00394, 0.11693, 0.21196, 0.06052, 0.25886)
    rz = poly(0.00275, 0.00610, 0.00317, -0.04214, 0.08970, 0.04153, 0.00516, 0.15346, 0.26756, 0.06670, 0.26688)
    lin = lambda a, b: f(f(a) * T + f(b))  # noqa: E731
    cx = [lin(0.1787, -1.4630), lin(-0.3554, 0.4275), lin(-0.0227, 5.3251), lin(0.1206, -2.5771),
          lin(-0.0670, 0.3703)] + [f(0.0)] * 4
    cy = [lin(-0.0193, -0.2592), lin(-0.0665, 0.0008), lin(-0.0004, 0.2125), lin(-0.0641, -0.8989),
          lin(-0.0033, 0.0452)] + [f(0.0)] * 4
    cz = [lin(-0.0167, -0.2608), lin(-0.0950, 0.0092), lin(-0.0079, 0.2102), lin(-0.0441, -1.6537),
          lin(-0.0109, 0.0529)] + [f(0.0)] * 4

    def perez(lam, th, gamma):
        a = f(f(1.0) + f(lam[0] * f(np.exp(f(lam[1] / f(np.cos(th)))))))
        cg = f(np.cos(gamma))
        b = f(f(f(1.0) + f(lam[2] * f(np.exp(f(lam[3] * gamma))))) + f(f(lam[4] * cg) * cg))
        return f(a * b)

    rx = f(rx / perez(cx, f(0.0), theta))
    ry = f(ry / perez(cy, f(0.0), theta))
    rz = f(rz / perez(cz, f(0.0), theta))
    return theta, phi, (rx, ry, rz), (cx, cy, cz)


def sky_texture(vector, kind: str = "nishita_improved", sun_direction=(0.0, 0.0, 1.0), turbidity: float = 2.2,
                ground_albedo: float = 0.3, sun_disc: bool = True, sun_size: float = 0.009512,
                sun_intensity: float = 1.0, sun_elevation: float = 15.0 * np.pi / 180.0, sun_rotation: float = 0.0,
                model=None) -> Node:
    """Sky Texture node (nodes.cpp:708-914 SkyTextureNode, svm_sky.h).  The
    Preetham parameters are computed here (nodes.cpp:645-705).  The other two
    models take their precomputed data from Blender's intern/sky library, which
    the host runs (outside the device path): `model` is, for hosek_wilkie,
    {"configs": (3, 9), "radiances": (3,)} of SKY_arhosek_xyz_skymodelstate at
    (turbidity, ground_albedo, the sun's elevation) — theta / phi of
    `sun_direction` come from sky_spherical_coordinates here; for
    nishita_improved, {"pixel_bottom": (3,), "pixel_top": (3,), "image": Image}
    (SKY_nishita_skymodel_precompute_sun / _texture; the image is the 512 x 128
    float4 SkyLoader texture, linear interpolation, extend).  In a world shader
    geometry()["Position"] is the ray direction."""
    if kind not in SKY_TYPES:
        raise ValueError("sky_texture: preetham | hosek_wilkie | nishita_improved")
    if kind != "preetham" and model is None:
        raise ValueError(f"sky_texture {kind}: needs the host-precomputed model data")
    return Node("sky_texture", {"Vector": vector},
                params={"type": SKY_TYPES[kind], "sun_direction": tuple(float(c) for c in sun_direction),
                        "turbidity": float(turbidity), "ground_albedo": float(ground_albedo),
                        "sun_disc": bool(sun_disc), "sun_size": float(sun_size),
                        "sun_intensity": float(sun_intensity), "sun_elevation": float(sun_elevation),
                        "sun_rotation": float(sun_rotation), "model": model})


NODE_IES = 67


NODE_WAVELENGTH, NODE_BLACKBODY = 81, 82


def wavelength(value=500.0) -> Socket:
    """Wavelength node (nodes.cpp WavelengthNode, svm_wavelength.h): the CIE
    colour of a wavelength in nm through the film's XYZ -> RGB rows."""
    return Node("wavelength", {"Wavelength": value})["Color"]


def blackbody(temperature=1500.0) -> Socket:
    """Blackbody node (nodes.cpp BlackbodyNode, svm_blackbody.h): the colour of
    a black body at `temperature` Kelvin.  (The reference host folds a
    constant temperature to a colour; link it to keep the node.)"""
    return Node("blackbody", {"Temperature": temperature})["Color"]




def ies_texture(vector, ies, strength=1.0) -> Node:
    """IES Texture node (nodes.cpp:1213-1300 IESLightNode, svm_ies.h): the
    light's intensity towards `vector` from an IES photometric file (its text,
    or an ies.IESFile), times Strength; outputs Fac.  The file gets a slot of
    the scene's __ies table (LightManager::add_ies: one slot per distinct
    content)."""
    from .ies import IESFile

    f = ies if isinstance(ies, IESFile) else IESFile(ies)
    return Node("ies_texture", {"Vector": vector, "Strength": strength}, params={"ies": f})


def noise_texture(vector=None, w=0.0, scale=5.0, detail=2.0, roughness=0.5, distortion=0.0, dimensions=3) -> Node:
    """Noise Texture (nodes.cpp NoiseTextureNode): fractal Perlin noise in 1-4
    dimensions (1D uses W, 4D the vector and W); outputs Fac, Color.  An
    unlinked vector reads the generated coordinates."""
    if dimensions not in (1, 2, 3, 4):
        raise ValueError("noise dimensions: 1..4")
    return Node("noise_texture", {"Vector": _default_vector(vector), "W": w, "Scale": scale, "Detail": detail,
                                  "Roughness": roughness, "Distortion": distortion}, {"dimensions": dimensions})


def musgrave_texture(vector=None, kind="fBm", w=0.0, scale=5.0, detail=2.0, dimension=2.0, lacunarity=2.0, offset=0.0,
                     gain=1.0, dimensions=3) -> Node:
    """Musgrave Texture (nodes.cpp MusgraveTextureNode): multifractal / fBm /
    hybrid multifractal / ridged multifractal / hetero terrain, 1-4 D."""
    if kind not in MUSGRAVE_TYPES or dimensions not in (1, 2, 3, 4):
        raise ValueError(f"musgrave: type one of {sorted(MUSGRAVE_TYPES)}, dimensions 1..4")
    return Node("musgrave_texture", {"Vector": _default_vector(vector), "W": w, "Scale": scale, "Detail": detail,
                                     "Dimension": dimension, "Lacunarity": lacunarity, "Offset": offset, "Gain": gain},
                {"type": kind, "dimensions": dimensions})


def wave_texture(vector=None, kind="bands", direction="x", profile="sin", scale=5.0, distortion=0.0, detail=2.0,
                 detail_scale=1.0, detail_roughness=0.5, phase=0.0) -> Node:
    """Wave Texture (nodes.cpp WaveTextureNode): bands or rings, sine / saw /
    triangle profile, optional noise distortion."""
    if kind not in WAVE_TYPES or direction not in WAVE_DIRECTIONS or profile not in WAVE_PROFILES:
        raise ValueError("wave: unknown type / direction / profile")
    return Node("wave_texture", {"Vector": _default_vector(vector), "Scale": scale, "Distortion": distortion, "Detail": detail,
                                 "Detail Scale": detail_scale, "Detail Roughness": detail_roughness,
                                 "Phase Offset": phase}, {"type": kind, "direction": direction, "profile": profile})


def magic_texture(vector=None, depth=2, scale=5.0, distortion=1.0) -> Node:
    """Magic Texture (nodes.cpp MagicTextureNode)."""
    return Node("magic_texture", {"Vector": _default_vector(vector), "Scale": scale, "Distortion": distortion}, {"depth": int(depth)})


def brick_texture(vector=None, color1=(0.8, 0.8, 0.8), color2=(0.2, 0.2, 0.2), mortar=(0.0, 0.0, 0.0), scale=5.0,
                  mortar_size=0.02, mortar_smooth=0.1, bias=0.0, brick_width=0.5, row_height=0.25, offset=0.5,
                  offset_frequency=2, squash=1.0, squash_frequency=2) -> Node:
    """Brick Texture (nodes.cpp BrickTextureNode)."""
    return Node("brick_texture", {"Vector": _default_vector(vector), "Color1": color1, "Color2": color2, "Mortar": mortar,
                                  "Scale": scale, "Mortar Size": mortar_size, "Mortar Smooth": mortar_smooth,
                                  "Bias": bias, "Brick Width": brick_width, "Row Height": row_height},
                {"offset": float(offset), "offset_frequency": int(offset_frequency), "squash": float(squash),
                 "squash_frequency": int(squash_frequency)})


def voronoi_texture(vector=None, feature="f1", metric="euclidean", w=0.0, scale=5.0, smoothness=1.0, exponent=0.5,
                    randomness=1.0, dimensions=3) -> Node:
    """Voronoi Texture (nodes.cpp VoronoiTextureNode): F1 / F2 / smooth F1 /
    distance to edge / n-sphere radius in 1-4 D with euclidean, manhattan,
    chebychev or minkowski distances; outputs Distance, Color, Position, W,
    Radius."""
    if feature not in VORONOI_FEATURES or metric not in VORONOI_METRICS or dimensions not in (1, 2, 3, 4):
        raise ValueError("voronoi: unknown feature / metric / dimensions")
    return Node("voronoi_texture", {"Vector": _default_vector(vector), "W": w, "Scale": scale, "Smoothness": smoothness,
                                    "Exponent": exponent, "Randomness": randomness},
                {"feature": feature, "metric": metric, "dimensions": dimensions})


def white_noise_texture(vector=None, w=0.0, dimensions=3) -> Node:
    """White Noise Texture (nodes.cpp WhiteNoiseTextureNode): hashes of the
    coordinates; outputs Value, Color."""
    if dimensions not in (1, 2, 3, 4):
        raise ValueError("white noise dimensions: 1..4")
    return Node("white_noise_texture", {"Vector": _default_vector(vector), "W": w}, {"dimensions": dimensions})


def gradient(vector=None, kind: str = "linear") -> Node:
    if kind not in GRADIENT_TYPES:
        raise ValueError(f"unknown gradient type {kind!r}")
    return Node("gradient", {"Vector": _default_vector(vector)}, {"type": kind})


def mapping(vector, location=(0.0, 0.0, 0.0), rotation=(0.0, 0.0, 0.0), scale=(1.0, 1.0, 1.0),
            kind: str = "point") -> Socket:
    if kind not in MAPPING_TYPES:
        raise ValueError(f"unknown mapping type {kind!r}")
    return Node("mapping", {"Vector": vector, "Location": location, "Rotation": rotation, "Scale": scale},
                {"type": kind})["Vector"]


def separate_xyz(vector) -> Node:
    return Node("separate_xyz", {"Vector": vector})


def combine_xyz(x=0.0, y=0.0, z=0.0) -> Socket:
    return Node("combine_xyz", {"X": x, "Y": y, "Z": z})["Vector"]


def separate_hsv(color) -> Node:
    return Node("separate_hsv", {"Color": color})


def combine_hsv(h=0.0, s=0.0, v=0.0) -> Socket:
    return Node("combine_hsv", {"H": h, "S": s, "V": v})["Color"]


def clamp(value_, min_=0.0, max_=1.0, kind: str = "minmax") -> Socket:
    return Node("clamp", {"Value": value_, "Min": min_, "Max": max_}, {"type": kind})["Result"]


def map_range(value_, from_min=0.0, from_max=1.0, to_min=0.0, to_max=1.0, steps=4.0,
              kind: str = "linear") -> Socket:
    return Node("map_range", {"Value": value_, "From Min": from_min, "From Max": from_max, "To Min": to_min,
                              "To Max": to_max, "Steps": steps}, {"type": kind})["Result"]


def color_ramp(fac, stops, interpolation: str = "linear", table_size: int = 256) -> Node:
    """ColorRamp: `stops` = [(position, (r, g, b, a)), ...] baked to a table of
    `table_size` entries the way the host does (RGBRampNode, BKE colorband
    evaluation at i / (size - 1)); constant interpolation looks up the stop at
    or before the position."""
    pts = sorted(stops, key=lambda s: s[0])
    pos = np.array([p for p, _ in pts], dtype=np.float64)
    col = np.array([c for _, c in pts], dtype=np.float64)
    x = np.arange(table_size, dtype=np.float64) / (table_size - 1)
    if interpolation == "constant":
        idx = np.clip(np.searchsorted(pos, x, side="right") - 1, 0, len(pos) - 1)
        table = col[idx]
    else:
        table = np.stack([np.interp(x, pos, col[:, k]) for k in range(4)], axis=1)
    return Node("rgb_ramp", {"Fac": fac}, {"table": table.astype(np.float32), "interpolate": interpolation != "constant"})


# ---------------------------------------------------------------------------
# socket types


DISPLACEMENT_SPACES = {"object": 1, "world": 2}  # NodeNormalMapSpace (svm_types.h:455-461)
NODE_DISPLACEMENT, NODE_VECTOR_DISPLACEMENT = 21, 22


def _bump_copy(s: Socket, mode: str, memo: dict) -> Socket:
    """A copy of the node graph feeding `s` with every node marked for the
    bump offset `mode` ("dx" / "dy"): ShaderGraph::refine_bump_nodes
    (graph.cpp:1003-1054) copies the Height input's dependencies twice and
    sets node->bump to SHADER_BUMP_DX / DY."""
    n = s.node
    if id(n) not in memo:
        inputs = {k: (_bump_copy(v, mode, memo) if is_linked(v) else v) for k, v in n.inputs.items()}
        memo[id(n)] = Node(n.kind, inputs, {**n.params, "bump": mode})
    return Socket(memo[id(n)], s.name)


def bump(height=1.0, strength=1.0, distance=0.1, invert=False, normal=None, object_space=False) -> Socket:
    """Bump node (nodes.cpp BumpNode, svm_displace.h svm_node_set_bump): the
    height at the shading point and, through copies of its node graph that
    sample one ray differential away (geometry, texture coordinate, attribute
    and vertex colour nodes in their *_BUMP_DX / _DY forms), at the
    neighbouring points; the perturbed normal (needs the device's ray
    differentials).  An unlinked height leaves the three samples at 0."""
    inputs = {"Strength": strength, "Distance": distance}
    if normal is not None:
        inputs["Normal"] = normal
    if is_linked(height):
        inputs["SampleCenter"] = height
        inputs["SampleX"] = _bump_copy(height, "dx", {})
        inputs["SampleY"] = _bump_copy(height, "dy", {})
    else:
        inputs.update({"SampleCenter": 0.0, "SampleX": 0.0, "SampleY": 0.0})
    return Node("bump", inputs, {"invert": bool(invert), "object_space": bool(object_space)})["Normal"]


def ambient_occlusion(color=(1.0, 1.0, 1.0), distance=1.0, normal=None, samples=16, inside=False,
                      only_local=False) -> Node:
    """Ambient Occlusion node (nodes.cpp:3210-3256, svm_ao.h): the fraction of
    `samples` cosine-distributed rays from the shading point that reach
    `distance` (0 unlinked: the world's AO distance) without a hit -- of the
    same object only with only_local -- as AO and times Color.  An unset Normal
    is the Geometry normal (graph.cpp default_inputs, LINK_NORMAL)."""
    if normal is None:
        normal = geometry()["Normal"]
    return Node("ambient_occlusion", {"Color": color, "Distance": distance, "Normal": normal},
                {"samples": int(samples), "inside": bool(inside), "only_local": bool(only_local)})


def wireframe(size=0.01, use_pixel_size=False) -> Socket:
    """Wireframe node (nodes.cpp:5583-5613, svm_wireframe.h): Fac 1 within
    size / 2 of the shading triangle's edges (in pixels, through the ray
    differentials, with use_pixel_size)."""
    return Node("wireframe", {"Size": size}, {"use_pixel_size": bool(use_pixel_size)})["Fac"]


def bevel(radius=0.05, normal=None, samples=4) -> Socket:
    """Bevel node (nodes.cpp:6865-6894, svm_bevel.h): the normal averaged over
    nearby points of the same object within `radius` (local probe rays); an
    unset Normal input is the Geometry normal (LINK_NORMAL), which the node
    adds its change to."""
    if normal is None:
        normal = geometry()["Normal"]
    return Node("bevel", {"Radius": radius, "Normal": normal}, {"samples": int(samples)})["Normal"]


def bump_from_displacement(disp: Socket, object_space: bool = False) -> Socket:
    """ShaderGraph::bump_from_displacement (graph.cpp:956-1050), the
    displacement method "bump": three copies of the displacement graph (centre,
    dx, dy), each projected on the Geometry normal by a dot product, feed a
    Bump node (distance 1) whose normal a Set Normal node makes the shading
    normal.  Compiled as the shader's bump program, which falls through into
    its surface program (svm.cpp:864-880)."""
    geom_n = geometry()["Normal"]

    def height(v):
        return vector_math("dot_product", v, geom_n)["Value"]

    b = Node("bump", {"Strength": 1.0, "Distance": 1.0, "SampleCenter": height(disp),
                      "SampleX": height(_bump_copy(disp, "dx", {})), "SampleY": height(_bump_copy(disp, "dy", {}))},
             {"invert": False, "object_space": bool(object_space)})["Normal"]
    return Node("set_normal", {"Direction": b})["Normal"]


def displacement(height, midlevel=0.5, scale=1.0, normal=None, space: str = "object") -> Socket:
    """Displacement node (nodes.cpp:6905-6952): (height - midlevel) * scale along
    the normal (sd->N when unlinked), in object or world space."""
    if space not in DISPLACEMENT_SPACES:
        raise ValueError(f"displacement space {space!r}: object or world")
    inputs = {"Height": height, "Midlevel": midlevel, "Scale": scale}
    if normal is not None:
        inputs["Normal"] = normal
    return Node("displacement", inputs, {"space": space})["Displacement"]


def vector_displacement(vector, midlevel=0.0, scale=1.0, space: str = "object") -> Socket:
    """Vector Displacement node (nodes.cpp:6962-7043) in object or world space
    (tangent space needs the UV tangent attributes: not supported)."""
    if space not in DISPLACEMENT_SPACES:
        raise ValueError(f"vector displacement space {space!r}: object or world (tangent is not supported)")
    return Node("vector_displacement", {"Vector": vector, "Midlevel": midlevel, "Scale": scale},
                {"space": space})["Displacement"]


def _outputs(node: Node) -> dict:
    k = node.kind
    if k == "value":
        return {"Value": "float"}
    if k == "rgb":
        return {"Color": "color"}
    if k == "tex_coord":
        return {n: "vector" for n in ("Generated", *TEXCO_OUTPUTS, "UV")}
    if k == "attribute":
        return {"Color": "color", "Vector": "vector", "Fac": "float"}
    if k == "vertex_color":
        return {"Color": "color", "Alpha": "float"}
    if k == "normal_map":
        return {"Normal": "vector"}
    if k == "fresnel":
        return {"Fac": "float"}
    if k == "camera_data":
        return dict(CAMERA_OUTPUTS)
    if k == "normal":
        return {"Normal": "vector", "Dot": "float"}
    if k == "rgb_curves":
        return {"Color": "color"}
    if k in ("vector_curves", "vector_rotate", "vector_transform"):
        return {"Vector": "vector"}
    if k == "layer_weight":
        return {"Fresnel": "float", "Facing": "float"}
    if k == "tangent":
        return {"Tangent": "vector"}
    if k == "object_info":
        return {n: t for n, (t, _) in OBJECT_INFO_OUTPUTS.items()}
    if k == "particle_info":
        return {n: t for n, (t, _) in PARTICLE_INFO_OUTPUTS.items()}
    if k == "hair_info":
        return dict(HAIR_INFO_OUTPUTS)
    if k == "texture_mapping":
        return {"Vector": "vector"}
    if k == "geometry":
        return {n: "vector" for n in GEOMETRY_OUTPUTS}
    if k == "light_path":
        return {n: "float" for n in LIGHT_PATH_OUTPUTS}
    if k == "light_falloff":
        return {n: "float" for n in LIGHT_FALLOFF_OUTPUTS}
    if k == "math":
        return {"Value": "float"}
    if k == "vector_math":
        return {"Vector": "vector", "Value": "float"}
    if k in ("mix", "hsv", "gamma", "brightcontrast", "invert", "combine_hsv"):
        return {"Color": "color"}
    if k in ("checker", "gradient", "noise_texture", "wave_texture", "magic_texture", "brick_texture"):
        return {"Color": "color", "Fac": "float"}
    if k == "musgrave_texture":
        return {"Fac": "float"}
    if k == "white_noise_texture":
        return {"Value": "float", "Color": "color"}
    if k == "voronoi_texture":
        return {"Distance": "float", "Color": "color", "Position": "vector", "W": "float", "Radius": "float"}
    if k in ("mapping", "combine_xyz"):
        return {"Vector": "vector"}
    if k == "separate_xyz":
        return {"X": "float", "Y": "float", "Z": "float"}
    if k == "separate_hsv":
        return {"H": "float", "S": "float", "V": "float"}
    if k in ("clamp", "map_range"):
        return {"Result": "float"}
    if k in ("rgb_ramp", "image_texture", "environment_texture"):
        return {"Color": "color", "Alpha": "float"}
    if k == "point_density":
        return {"Color": "color", "Density": "float"}
    if k == "sky_texture":
        return {"Color": "color"}
    if k == "ies_texture":
        return {"Fac": "float"}
    if k in ("wavelength", "blackbody"):
        return {"Color": "color"}
    if k in ("displacement", "vector_displacement"):
        return {"Displacement": "vector"}
    if k in ("bump", "set_normal", "bevel"):
        return {"Normal": "vector"}
    if k == "ambient_occlusion":
        return {"Color": "color", "AO": "float"}
    if k == "wireframe":
        return {"Fac": "float"}
    raise ValueError(f"unknown node kind {k!r}")


_INPUT_TYPES = {
    "texture_mapping": {"Vector": "vector"},
    "light_falloff": {"Strength": "float", "Smooth": "float"},
    "math": {"Value1": "float", "Value2": "float", "Value3": "float"},
    "vector_math": {"Vector1": "vector", "Vector2": "vector", "Vector3": "vector", "Scale": "float"},
    "mix": {"Fac": "float", "Color1": "color", "Color2": "color"},
    "hsv": {"Hue": "float", "Saturation": "float", "Value": "float", "Fac": "float", "Color": "color"},
    "gamma": {"Color": "color", "Gamma": "float"},
    "brightcontrast": {"Color": "color", "Bright": "float", "Contrast": "float"},
    "invert": {"Fac": "float", "Color": "color"},
    "checker": {"Vector": "vector", "Color1": "color", "Color2": "color", "Scale": "float"},
    "gradient": {"Vector": "vector"},
    "noise_texture": {"Vector": "vector", "W": "float", "Scale": "float", "Detail": "float", "Roughness": "float",
                      "Distortion": "float"},
    "musgrave_texture": {"Vector": "vector", "W": "float", "Scale": "float", "Detail": "float", "Dimension": "float",
                         "Lacunarity": "float", "Offset": "float", "Gain": "float"},
    "wave_texture": {"Vector": "vector", "Scale": "float", "Distortion": "float", "Detail": "float",
                     "Detail Scale": "float", "Detail Roughness": "float", "Phase Offset": "float"},
    "magic_texture": {"Vector": "vector", "Scale": "float", "Distortion": "float"},
    "brick_texture": {"Vector": "vector", "Color1": "color", "Color2": "color", "Mortar": "color", "Scale": "float",
                      "Mortar Size": "float", "Mortar Smooth": "float", "Bias": "float", "Brick Width": "float",
                      "Row Height": "float"},
    "white_noise_texture": {"Vector": "vector", "W": "float"},
    "voronoi_texture": {"Vector": "vector", "W": "float", "Scale": "float", "Smoothness": "float",
                        "Exponent": "float", "Randomness": "float"},
    "mapping": {"Vector": "vector", "Location": "vector", "Rotation": "vector", "Scale": "vector"},
    "separate_xyz": {"Vector": "vector"},
    "combine_xyz": {"X": "float", "Y": "float", "Z": "float"},
    "separate_hsv": {"Color": "color"},
    "combine_hsv": {"H": "float", "S": "float", "V": "float"},
    "clamp": {"Value": "float", "Min": "float", "Max": "float"},
    "map_range": {"Value": "float", "From Min": "float", "From Max": "float", "To Min": "float",
                  "To Max": "float", "Steps": "float"},
    "rgb_ramp": {"Fac": "float"},
    "image_texture": {"Vector": "vector"},
    "environment_texture": {"Vector": "vector"},
    "point_density": {"Vector": "vector"},
    "sky_texture": {"Vector": "vector"},
    "ies_texture": {"Vector": "vector", "Strength": "float"},
    "wavelength": {"Wavelength": "float"},
    "blackbody": {"Temperature": "float"},
    "displacement": {"Height": "float", "Midlevel": "float", "Scale": "float", "Normal": "vector"},
    "normal_map": {"Color": "color", "Strength": "float"},
    "fresnel": {"IOR": "float", "Normal": "vector"},
    "normal": {"Normal": "vector"},
    "rgb_curves": {"Fac": "float", "Color": "color"},
    "vector_curves": {"Fac": "float", "Vector": "vector"},
    "vector_rotate": {"Vector": "vector", "Rotation": "vector", "Center": "vector", "Axis": "vector",
                      "Angle": "float"},
    "vector_transform": {"Vector": "vector"},
    "layer_weight": {"Blend": "float", "Normal": "vector"},
    "vector_displacement": {"Vector": "color", "Midlevel": "float", "Scale": "float"},
    "bump": {"SampleCenter": "float", "SampleX": "float", "SampleY": "float", "Normal": "vector",
             "Strength": "float", "Distance": "float"},
    "set_normal": {"Direction": "vector"},
    "ambient_occlusion": {"Color": "color", "Distance": "float", "Normal": "vector"},
    "bevel": {"Radius": "float", "Normal": "vector"},
    "wireframe": {"Size": "float"},
}


def _width(t: str) -> int:
    return 1 if t == "float" else 3


# ShaderNode::has_spatial_varying (render/nodes.h): nodes whose value depends on
# the shading point or direction (texture coordinate, geometry, textures)
SPATIAL_KINDS = ("tex_coord", "geometry", "checker", "gradient", "image_texture", "environment_texture", "sky_texture", "ies_texture",
                 "point_density",
                 "attribute", "vertex_color", "normal_map", "tangent", "object_info", "camera_data")


def has_spatial_varying(values) -> bool:
    """ShaderGraph has_surface_spatial_varying for the sockets feeding a shader."""
    return any(n.kind in SPATIAL_KINDS for v in values for n in upstream(v))


def upstream(v) -> list[Node]:
    """Nodes a value depends on, dependencies first."""
    order: list[Node] = []
    seen: set[int] = set()

    def visit(n: Node):
        if id(n) in seen:
            return
        seen.add(id(n))
        for x in n.inputs.values():
            if is_linked(x):
                visit(x.node)
        order.append(n)

    if is_linked(v):
        visit(v.node)
    return order


# ---------------------------------------------------------------------------
# compiler


class NodeCompiler:
    """Assigns stack slots and emits the node code of one shader.

    `alloc(n)` / `free(off, n)` are the owning SVMCompiler's slot allocator;
    `emit` appends to its code.  Like the reference compiler (svm.cpp
    stack_clear_users / stack_clear_temporary), a node output's slot is
    released once every node reading it has been emitted, and constants /
    conversions materialised for one node's inputs right after that node;
    outputs feeding the closures (`roots`) stay live."""

    def __init__(self, alloc, emit, roots=(), free=None, images=None, attribute=None, background=False,
                 volume=False, features=None, ies_slots=None):
        self.images = images if images is not None else []  # SVM image slots (shared per scene)
        self.ies_slots = ies_slots if ies_slots is not None else []  # __ies slots (shared per scene)
        # scene-wide needs of the compiled nodes (e.g. "xyz_to_rgb": film colour matrices)
        self.features = features if features is not None else set()
        # SVMCompiler::attribute (svm.cpp): attribute id of a standard id or a
        # name, recording the shader's attribute request
        self.attribute = attribute or (lambda key: (_ for _ in ()).throw(
            ValueError("attribute nodes need the scene's SVM compiler")))
        self.background = background  # compiler.background: the world shader
        self.volume = volume  # compiler.output_type() == SHADER_TYPE_VOLUME
        self.alloc = alloc
        self.free = free or (lambda off, n: None)
        self.emit = emit
        self.slots: dict[tuple[int, str], int] = {}  # (id(node), output) -> slot
        self.done: set[int] = set()
        self.temps: list[tuple[int, int]] = []
        # outputs some input links to: only those get a slot (stack_assign_if_linked)
        self.used: set[tuple[int, str]] = set()
        self.users: dict[tuple[int, str], int] = {}
        seen: set[int] = set()
        for v in roots:
            for n in upstream(v):
                if id(n) in seen:
                    continue
                seen.add(id(n))
                for x in n.inputs.values():
                    if is_linked(x):
                        key = (id(x.node), x.name)
                        self.used.add(key)
                        self.users[key] = self.users.get(key, 0) + 1
            if is_linked(v):
                key = (id(v.node), v.name)
                self.used.add(key)
                self.users[key] = self.users.get(key, 0) + (1 << 30)  # pinned

    # -- inputs
    def constant(self, v, t: str) -> int:
        if t == "float":
            off = self.alloc(1)
            self.emit((NODE_VALUE_F, f32bits(float(v)), off, 0))
            return off
        vv = (float(v),) * 3 if np.isscalar(v) else tuple(float(x) for x in v)
        off = self.alloc(3)
        self.emit((NODE_VALUE_V, off, 0, 0))
        self.emit((NODE_VALUE_V, *(f32bits(x) for x in vv)))
        return off

    def link(self, s: Socket, t: str, temps: list | None = None) -> int:
        """Stack slot of socket `s` converted to type `t`; a conversion slot is
        appended to `temps` (or kept for the shader's lifetime when None)."""
        self.compile_node(s.node)
        off = self.slots[(id(s.node), s.name)]
        st = s.type
        if st == t or (st != "float" and t != "float"):
            return off  # color <-> vector share the layout
        if st == "float":
            out = self.alloc(3)
            self.emit((NODE_CONVERT, CONVERT_FV, off, out))
            n = 3
        else:
            out = self.alloc(1)
            self.emit((NODE_CONVERT, CONVERT_CF if st == "color" else CONVERT_VF, off, out))
            n = 1
        if temps is not None:
            temps.append((out, n))
        return out

    def assign(self, v, t: str, temps: list | None = None) -> int:
        """stack_assign: linked sockets by slot, constants materialised."""
        if is_linked(v):
            return self.link(v, t, temps)
        off = self.constant(v, t)
        if temps is not None:
            temps.append((off, _width(t)))
        return off

    def assign_if_linked(self, v, t: str) -> int:
        return self.link(v, t, self.temps) if is_linked(v) else SVM_STACK_INVALID

    def inp(self, node: Node, name: str) -> int:
        return self.assign(node.inputs[name], _INPUT_TYPES[node.kind][name], self.temps)

    def out(self, node: Node, name: str) -> int:
        key = (id(node), name)
        if key not in self.used:
            return SVM_STACK_INVALID
        if key not in self.slots:
            self.slots[key] = self.alloc(_width(_outputs(node)[name]))
        return self.slots[key]

    def _release(self, n: Node):
        for off, w in self.temps:
            self.free(off, w)
        self.temps = []
        for x in n.inputs.values():
            if is_linked(x):
                key = (id(x.node), x.name)
                self.users[key] -= 1
                if self.users[key] == 0:
                    self.free(self.slots[key], _width(x.type))

    # -- nodes
    def compile_node(self, n: Node):
        if id(n) in self.done:
            return
        for x in n.inputs.values():
            if is_linked(x):
                self.compile_node(x.node)
        self.done.add(id(n))
        self.temps = []
        getattr(self, "_n_" + n.kind)(n)
        self._release(n)

    def _n_value(self, n):
        self.emit((NODE_VALUE_F, f32bits(n.params["value"]), self.out(n, "Value"), 0))

    def _n_rgb(self, n):
        off = self.out(n, "Color")
        self.emit((NODE_VALUE_V, off, 0, 0))
        self.emit((NODE_VALUE_V, *(f32bits(x) for x in n.params["value"])))

    @staticmethod
    def _bump_kind(n, center, dx, dy):
        """The node type of `n`'s bump copy (ShaderNode::bump, nodes.cpp)."""
        return {"dx": dx, "dy": dy}.get(n.params.get("bump"), center)

    def _n_tex_coord(self, n):  # nodes.cpp:3840-3923 TextureCoordinateNode::compile
        used = lambda name: (id(n), name) in self.used  # noqa: E731
        texco = self._bump_kind(n, NODE_TEX_COORD, NODE_TEX_COORD_BUMP_DX, NODE_TEX_COORD_BUMP_DY)
        attr = self._bump_kind(n, NODE_ATTR, NODE_ATTR_BUMP_DX, NODE_ATTR_BUMP_DY)
        geom = self._bump_kind(n, NODE_GEOMETRY, NODE_GEOMETRY_BUMP_DX, NODE_GEOMETRY_BUMP_DY)
        if used("Generated"):
            if self.background:
                self.emit((geom, GEOMETRY_OUTPUTS["Position"], self.out(n, "Generated"), 0))
            elif self.volume:
                raise ValueError("tex_coord Generated in a volume shader (NODE_TEXCO_VOLUME_GENERATED needs the "
                                 "generated-transform attribute) is not supported")
            else:
                self.emit((attr, self.attribute(ATTR_STD_GENERATED), self.out(n, "Generated"), NODE_ATTR_FLOAT3))
        if used("Normal"):
            self.emit((texco, TEXCO_OUTPUTS["Normal"], self.out(n, "Normal"), 0))
        if used("UV"):
            self.emit((attr, self.attribute(ATTR_STD_UV), self.out(n, "UV"), NODE_ATTR_FLOAT3))
        for name in ("Object", "Camera", "Window"):
            if used(name):
                self.emit((texco, TEXCO_OUTPUTS[name], self.out(n, name), 0))
        if used("Reflection"):
            if self.background:
                self.emit((geom, GEOMETRY_OUTPUTS["Incoming"], self.out(n, "Reflection"), 0))
            else:
                self.emit((texco, TEXCO_OUTPUTS["Reflection"], self.out(n, "Reflection"), 0))

    def _n_attribute(self, n):  # nodes.cpp:5411-5436 AttributeNode::compile
        attr = self.attribute(ATTR_STD_NAMES.get(n.params["name"], n.params["name"]))
        node = self._bump_kind(n, NODE_ATTR, NODE_ATTR_BUMP_DX, NODE_ATTR_BUMP_DY)
        for name in ("Color", "Vector"):
            if (id(n), name) in self.used:
                self.emit((node, attr, self.out(n, name), NODE_ATTR_FLOAT3))
        if (id(n), "Fac") in self.used:
            self.emit((node, attr, self.out(n, "Fac"), NODE_ATTR_FLOAT))

    def _n_normal_map(self, n):  # nodes.cpp:6717-6761 NormalMapNode::attributes / compile
        space = NORMAL_MAP_SPACES[n.params["space"]]
        attr = attr_sign = 0
        if space == 0 and not self.volume:
            uvm = n.params["uv_map"]
            attr = self.attribute(f"{uvm}.tangent" if uvm else ATTR_STD_UV_TANGENT)
            attr_sign = self.attribute(f"{uvm}.tangent_sign" if uvm else ATTR_STD_UV_TANGENT_SIGN)
            self.attribute(ATTR_STD_VERTEX_NORMAL)  # requested by attributes(), looked up by id
        col, strength = self.inp(n, "Color"), self.inp(n, "Strength")
        out = self.out(n, "Normal")
        self.emit((NODE_NORMAL_MAP, uchar4(col, strength, out, space), attr, attr_sign))

    def _n_tangent(self, n):  # nodes.cpp:6813-6847 TangentNode::attributes / compile
        uvm = n.params["uv_map"]
        if n.params["direction"] == "uv_map":
            attr = self.attribute(f"{uvm}.tangent" if uvm else ATTR_STD_UV_TANGENT)
        else:
            attr = self.attribute(ATTR_STD_GENERATED)
        self.emit((NODE_TANGENT, uchar4(self.out(n, "Tangent"), TANGENT_DIRECTIONS[n.params["direction"]],
                                        TANGENT_AXES[n.params["axis"]]), attr, 0))

    def _n_camera_data(self, n):  # nodes.cpp CameraNode::compile
        self.emit((NODE_CAMERA, *(self.out(n, k) for k in CAMERA_OUTPUTS)))

    def _n_normal(self, n):  # nodes.cpp NormalNode::compile
        nin = self.inp(n, "Normal")
        self.emit((NODE_NORMAL, nin, self.out(n, "Normal"), self.out(n, "Dot")))
        self.emit(tuple(f32bits(x) for x in n.params["direction"]) + (0,))

    def _curves(self, n, ntype, value):  # nodes.cpp CurvesNode::compile
        fac, val = self.inp(n, "Fac"), self.inp(n, value)
        table = n.params["table"]
        self.emit((ntype, uchar4(fac, val, self.out(n, value)), f32bits(n.params["min_x"]),
                   f32bits(n.params["max_x"])))
        self.emit((len(table), 0, 0, 0))
        for row in table:
            self.emit((f32bits(row[0]), f32bits(row[1]), f32bits(row[2]), 0))

    def _n_rgb_curves(self, n):
        self._curves(n, NODE_RGB_CURVES, "Color")

    def _n_vector_curves(self, n):
        self._curves(n, NODE_VECTOR_CURVES, "Vector")

    def _n_vector_rotate(self, n):  # nodes.cpp VectorRotateNode::compile
        v, rot, c, ax, ang = (self.inp(n, k) for k in ("Vector", "Rotation", "Center", "Axis", "Angle"))
        self.emit((NODE_VECTOR_ROTATE, uchar4(VECTOR_ROTATE_TYPES[n.params["type"]], v, rot,
                                              int(n.params["invert"])),
                   uchar4(c, ax, ang), self.out(n, "Vector")))

    def _n_vector_transform(self, n):  # nodes.cpp VectorTransformNode::compile
        v = self.inp(n, "Vector")
        self.emit((NODE_VECTOR_TRANSFORM, uchar4(VECTOR_TRANSFORM_TYPES[n.params["type"]],
                                                 VECTOR_TRANSFORM_SPACES[n.params["from"]],
                                                 VECTOR_TRANSFORM_SPACES[n.params["to"]]),
                   uchar4(v, self.out(n, "Vector")), 0))

    def _n_fresnel(self, n):  # nodes.cpp FresnelNode::compile
        ior = self.assign_if_linked(n.inputs["IOR"], "float")
        nrm = self.assign_if_linked(n.inputs["Normal"], "vector")
        val = 0.0 if is_linked(n.inputs["IOR"]) else float(n.inputs["IOR"])
        self.emit((NODE_FRESNEL, ior, f32bits(val), uchar4(nrm, self.out(n, "Fac"))))

    def _n_layer_weight(self, n):  # nodes.cpp LayerWeightNode::compile
        blend = self.assign_if_linked(n.inputs["Blend"], "float")
        nrm = self.assign_if_linked(n.inputs["Normal"], "vector")
        val = 0.0 if is_linked(n.inputs["Blend"]) else float(n.inputs["Blend"])
        for t, name in enumerate(("Fresnel", "Facing")):
            if (id(n), name) in self.used:
                self.emit((NODE_LAYER_WEIGHT, blend, f32bits(val), uchar4(t, nrm, self.out(n, name))))

    def _n_object_info(self, n):  # nodes.cpp:4211-4237 ObjectInfoNode::compile
        for name, (_, t) in OBJECT_INFO_OUTPUTS.items():
            if (id(n), name) in self.used:
                self.emit((NODE_OBJECT_INFO, t, self.out(n, name), 0))

    def _n_particle_info(self, n):  # nodes.cpp:4295-4347 ParticleInfoNode::compile
        for name, (_, t) in PARTICLE_INFO_OUTPUTS.items():
            if (id(n), name) in self.used:
                self.emit((NODE_PARTICLE_INFO, t, self.out(n, name), 0))

    def _n_hair_info(self, n):  # nodes.cpp:4391-4426 HairInfoNode::compile
        for name in HAIR_INFO_OUTPUTS:
            if (id(n), name) not in self.used:
                continue
            if name == "Intercept":
                self.emit((NODE_ATTR, self.attribute(ATTR_STD_CURVE_INTERCEPT), self.out(n, name), NODE_ATTR_FLOAT))
            elif name == "Random":
                self.emit((NODE_ATTR, self.attribute(ATTR_STD_CURVE_RANDOM), self.out(n, name), NODE_ATTR_FLOAT))
            else:
                t = {"Is Strand": NODE_INFO_CURVE_IS_STRAND, "Thickness": NODE_INFO_CURVE_THICKNESS,
                     "Tangent Normal": NODE_INFO_CURVE_TANGENT_NORMAL}[name]
                self.emit((NODE_HAIR_INFO, t, self.out(n, name), 0))

    def _n_texture_mapping(self, n):  # nodes.cpp:155-176 TextureMapping::compile
        v = self.inp(n, "Vector")
        out = self.out(n, "Vector")
        self.emit((NODE_TEXTURE_MAPPING, v, out, 0))
        for row in n.params["tfm"]:
            self.emit(tuple(f32bits(float(x)) for x in row))
        if n.params["minmax"] is not None:
            self.emit((NODE_MIN_MAX, out, out, 0))
            for vec in n.params["minmax"]:
                self.emit((*(f32bits(x) for x in vec), f32bits(0.0)))
        if n.params["normalize"]:
            self.emit((NODE_VECTOR_MATH, VECTOR_MATH_OPS.index("normalize"), uchar4(out, out, out),
                       uchar4(SVM_STACK_INVALID, out)))

    def _n_vertex_color(self, n):  # nodes.cpp:4543-4568 VertexColorNode::compile
        layer = n.params["layer"]
        attr = self.attribute(ATTR_STD_NAMES.get(layer, layer) if layer else ATTR_STD_VERTEX_COLOR)
        # both outputs are stack-assigned (stack_assign): an unread one gets a
        # slot released after the node
        offs = []
        for name, w in (("Color", 3), ("Alpha", 1)):
            off = self.out(n, name)
            if off == SVM_STACK_INVALID:
                off = self.alloc(w)
                self.temps.append((off, w))
            offs.append(off)
        self.emit((self._bump_kind(n, NODE_VERTEX_COLOR, NODE_VERTEX_COLOR_BUMP_DX, NODE_VERTEX_COLOR_BUMP_DY), attr,
                   offs[0], offs[1]))

    def _n_geometry(self, n):  # nodes.cpp GeometryNode::attributes / compile
        if (id(n), "Tangent") in self.used and not self.background:
            self.attribute(ATTR_STD_GENERATED)  # primitive_tangent reads the generated coordinates
        geom = self._bump_kind(n, NODE_GEOMETRY, NODE_GEOMETRY_BUMP_DX, NODE_GEOMETRY_BUMP_DY)
        for name, t in GEOMETRY_OUTPUTS.items():
            if (id(n), name) in self.used:
                self.emit((geom, t, self.out(n, name), 0))

    def _n_bump(self, n):  # nodes.cpp BumpNode::compile
        nrm = self.assign_if_linked(n.inputs.get("Normal"), "vector")
        dist = self.inp(n, "Distance")
        c, x, y = self.inp(n, "SampleCenter"), self.inp(n, "SampleX"), self.inp(n, "SampleY")
        strength = self.inp(n, "Strength")
        self.emit((NODE_SET_BUMP, uchar4(nrm, dist, int(n.params["invert"]), int(n.params["object_space"])),
                   uchar4(c, x, y, strength), self.out(n, "Normal")))

    def _n_ambient_occlusion(self, n):  # nodes.cpp:3233-3256 AmbientOcclusionNode::compile
        dist = n.inputs["Distance"]
        flags = (NODE_AO_INSIDE if n.params["inside"] else 0) | (NODE_AO_ONLY_LOCAL if n.params["only_local"] else 0)
        if not is_linked(dist) and float(dist) == 0.0:
            flags |= NODE_AO_GLOBAL_RADIUS
        self.emit((NODE_AMBIENT_OCCLUSION,
                   uchar4(flags, self.assign_if_linked(dist, "float"), self.assign_if_linked(n.inputs["Normal"], "vector"),
                          self.out(n, "AO")),
                   uchar4(self.inp(n, "Color"), self.out(n, "Color"), n.params["samples"]),
                   f32bits(0.0 if is_linked(dist) else float(dist))))

    def _n_wireframe(self, n):  # nodes.cpp:5598-5613 WireframeNode::compile
        offset = {"dx": 1, "dy": 2}.get(n.params.get("bump"), 0)
        self.emit((NODE_WIREFRAME, self.inp(n, "Size"), self.out(n, "Fac"),
                   uchar4(int(n.params["use_pixel_size"]), offset)))

    def _n_bevel(self, n):  # nodes.cpp:6883-6894 BevelNode::compile
        self.emit((NODE_BEVEL, uchar4(n.params["samples"], self.inp(n, "Radius"),
                                      self.assign_if_linked(n.inputs["Normal"], "vector"), self.out(n, "Normal")),
                   0, 0))

    def _n_set_normal(self, n):  # nodes.cpp SetNormalNode::compile
        self.emit((NODE_CLOSURE_SET_NORMAL, self.inp(n, "Direction"), self.out(n, "Normal"), 0))

    def _n_light_path(self, n):  # nodes.cpp LightPathNode::compile
        for t, name in enumerate(LIGHT_PATH_OUTPUTS):
            if (id(n), name) in self.used:
                self.emit((NODE_LIGHT_PATH, t, self.out(n, name), 0))

    def _n_light_falloff(self, n):
        s, sm = self.inp(n, "Strength"), self.inp(n, "Smooth")
        for name, t in LIGHT_FALLOFF_OUTPUTS.items():
            if (id(n), name) not in self.used:
                continue
            self.emit((NODE_LIGHT_FALLOFF, t, uchar4(s, sm, self.out(n, name)), 0))

    def _n_math(self, n):  # nodes.cpp MathNode::compile (+ expand: use_clamp -> ClampNode 0..1)
        a, b, c = self.inp(n, "Value1"), self.inp(n, "Value2"), self.inp(n, "Value3")
        out = self.out(n, "Value")
        self.emit((NODE_MATH, MATH_OPS.index(n.params["op"]), uchar4(a, b, c), out))
        if n.params.get("clamp"):
            self.emit((NODE_CLAMP, out, uchar4(SVM_STACK_INVALID, SVM_STACK_INVALID, 0), out))
            self.emit((f32bits(0.0), f32bits(1.0), 0, 0))

    def _n_vector_math(self, n):  # nodes.cpp VectorMathNode::compile
        op = n.params["op"]
        wrong = "Vector" if op in VECTOR_MATH_VALUE_OPS else "Value"
        if (id(n), wrong) in self.used:
            raise ValueError(f"vector math {op!r} does not write its {wrong!r} output")
        a, b, s = self.inp(n, "Vector1"), self.inp(n, "Vector2"), self.inp(n, "Scale")
        value_off = self.out(n, "Value") if op in VECTOR_MATH_VALUE_OPS else SVM_STACK_INVALID
        vector_off = SVM_STACK_INVALID if op in VECTOR_MATH_VALUE_OPS else self.out(n, "Vector")
        if op == "wrap":
            c = self.inp(n, "Vector3")
            self.emit((NODE_VECTOR_MATH, VECTOR_MATH_OPS.index(op), uchar4(a, b, s), uchar4(value_off, vector_off)))
            self.emit((c, 0, 0, 0))
        else:
            self.emit((NODE_VECTOR_MATH, VECTOR_MATH_OPS.index(op), uchar4(a, b, s), uchar4(value_off, vector_off)))

    def _n_mix(self, n):  # nodes.cpp MixNode::compile
        fac, c1, c2 = self.inp(n, "Fac"), self.inp(n, "Color1"), self.inp(n, "Color2")
        out = self.out(n, "Color")
        self.emit((NODE_MIX, fac, c1, c2))
        self.emit((NODE_MIX, MIX_TYPES.index(n.params["type"]), out, 0))
        if n.params.get("clamp"):
            self.emit((NODE_MIX, 0, out, 0))
            self.emit((NODE_MIX, NODE_MIX_CLAMP, out, 0))

    def _n_hsv(self, n):
        h, s, v = self.inp(n, "Hue"), self.inp(n, "Saturation"), self.inp(n, "Value")
        fac, col = self.inp(n, "Fac"), self.inp(n, "Color")
        self.emit((NODE_HSV, uchar4(col, fac, self.out(n, "Color")), uchar4(h, s, v), 0))

    def _n_gamma(self, n):
        g, col = self.inp(n, "Gamma"), self.inp(n, "Color")
        self.emit((NODE_GAMMA, g, col, self.out(n, "Color")))

    def _n_brightcontrast(self, n):
        col, br, co = self.inp(n, "Color"), self.inp(n, "Bright"), self.inp(n, "Contrast")
        self.emit((NODE_BRIGHTCONTRAST, col, self.out(n, "Color"), uchar4(br, co)))

    def _n_invert(self, n):
        fac, col = self.inp(n, "Fac"), self.inp(n, "Color")
        self.emit((NODE_INVERT, fac, col, self.out(n, "Color")))

    def _n_checker(self, n):  # nodes.cpp CheckerTextureNode::compile (identity texture mapping)
        vec, c1, c2 = self.inp(n, "Vector"), self.inp(n, "Color1"), self.inp(n, "Color2")
        scale = self.assign_if_linked(n.inputs["Scale"], "float")
        sval = 0.0 if is_linked(n.inputs["Scale"]) else float(n.inputs["Scale"])
        self.emit((NODE_TEX_CHECKER, uchar4(vec, c1, c2, scale),
                   uchar4(self.out(n, "Color"), self.out(n, "Fac")), f32bits(sval)))

    def image_slot(self, image: Image) -> int:
        """ImageManager::add_image: one slot per distinct image."""
        for i, im in enumerate(self.images):
            if im is image:
                return i
        self.images.append(image)
        return len(self.images) - 1

    def _image_flags(self, n, image: Image) -> int:
        flags = NODE_IMAGE_COMPRESS_AS_SRGB if image.compress_as_srgb else 0
        if n.params.get("alpha_unassociate"):
            flags |= NODE_IMAGE_ALPHA_UNASSOCIATE
        return flags

    def _n_image_texture(self, n):  # nodes.cpp:359-426 ImageTextureNode::compile (identity mapping)
        image = n.params["image"]
        vec = self.inp(n, "Vector")
        flags = self._image_flags(n, image)
        col, alpha = self.out(n, "Color"), self.out(n, "Alpha")
        if image.tiles:
            tiles = sorted(image.tiles)
            slots = [self.image_slot(image.tiles[t]) for t in tiles]
            num_nodes = -(-len(tiles) // 2)
            self.emit((NODE_TEX_IMAGE, num_nodes, uchar4(vec, col, alpha, flags), n.params["projection"]))
            for i in range(num_nodes):
                a = (tiles[2 * i], slots[2 * i])
                b = (tiles[2 * i + 1], slots[2 * i + 1]) if 2 * i + 1 < len(tiles) else (-1, -1)
                self.emit(tuple(int(x) & 0xFFFFFFFF for x in (*a, *b)))
        else:
            slot = self.image_slot(image)
            self.emit((NODE_TEX_IMAGE, (-slot) & 0xFFFFFFFF, uchar4(vec, col, alpha, flags), n.params["projection"]))

    def _n_point_density(self, n):  # nodes.cpp:1810-1852 PointDensityTextureNode::compile
        p = n.params
        dens, col = self.out(n, "Density"), self.out(n, "Color")
        if dens == SVM_STACK_INVALID and col == SVM_STACK_INVALID:
            return
        vec = self.inp(n, "Vector")
        space = 0 if p["space"] == "object" else 1
        self.emit((NODE_TEX_VOXEL, self.image_slot(p["image"]), uchar4(vec, dens, col, space), 0))
        if space == 1:
            t = np.asarray(p["tfm"], dtype=np.float32)
            for r in range(3):
                self.emit(tuple(int(x) for x in t[r].view(np.uint32)))
        if space == 0:
            # PointDensityTextureNode::attributes: the mesh's generated transform
            self.attribute(ATTR_STD_GENERATED_TRANSFORM)

    def _n_environment_texture(self, n):  # nodes.cpp EnvironmentTextureNode::compile
        image = n.params["image"]
        vec = self.inp(n, "Vector")
        flags = self._image_flags(n, image)
        self.emit((NODE_TEX_ENVIRONMENT, self.image_slot(image),
                   uchar4(vec, self.out(n, "Color"), self.out(n, "Alpha"), flags), n.params["projection"]))

    def _n_sky_texture(self, n):  # nodes.cpp:837-914 SkyTextureNode::compile (identity texture mapping)
        p = n.params
        vec = self.inp(n, "Vector")
        col = self.out(n, "Color")
        if col == SVM_STACK_INVALID:
            col = self.alloc(3)
            self.temps.append((col, 3))
        self.emit((NODE_TEX_SKY, vec, col, p["type"]))
        self.features.add("xyz_to_rgb")
        f = np.float32
        if p["type"] != SKY_TYPES["nishita_improved"]:
            if p["type"] == SKY_TYPES["preetham"]:
                theta, phi, rad, cfg = _sky_preetham(p["sun_direction"], p["turbidity"])
            else:  # sky_texture_precompute_hosek: clamped theta, the library's state cast to float
                d = np.asarray(p["sun_direction"], dtype=np.float32)
                theta = f(min(max(f(np.arccos(d[2])), f(0.0)), f(np.pi / 2)))
                phi = f(np.arctan2(d[0], d[1]))
                m = p["model"]
                cfg = np.asarray(m["configs"], dtype=np.float32).reshape(3, 9)
                rad = np.asarray(m["radiances"], dtype=np.float32).reshape(3)
            vals = [phi, theta, rad[0], rad[1], rad[2], *cfg[0], *cfg[1], *cfg[2]]
        else:  # sky_texture_precompute_nishita
            m = p["model"]
            rot = f(np.fmod(f(p["sun_rotation"]), f(2.0 * np.pi)))
            if rot < 0.0:
                rot = f(rot + f(2.0 * np.pi))
            rot = f(f(2.0 * np.pi) - rot)
            size = f(max(f(p["sun_size"]), f(0.0005)))  # get_sun_size
            vals = [*np.asarray(m["pixel_bottom"], dtype=np.float32), *np.asarray(m["pixel_top"], dtype=np.float32),
                    f(p["sun_elevation"]), rot, size if p["sun_disc"] else f(-1.0), f(p["sun_intensity"])]
        words = [f32bits(float(v)) for v in vals]
        if p["type"] == SKY_TYPES["nishita_improved"]:
            words = words + [self.image_slot(p["model"]["image"]), 0]
        for i in range(0, len(words), 4):
            self.emit(tuple(words[i:i + 4]))

    def _n_wavelength(self, n):  # nodes.cpp:5645-5653 WavelengthNode::compile
        self.features.add("xyz_to_rgb")
        self.emit((NODE_WAVELENGTH, self.inp(n, "Wavelength"), self._out_assigned(n, "Color", 3), 0))

    def _n_blackbody(self, n):  # nodes.cpp:5680-5690 BlackbodyNode::compile
        self.emit((NODE_BLACKBODY, self.inp(n, "Temperature"), self._out_assigned(n, "Color", 3), 0))

    def _out_assigned(self, n, name, width):
        """compiler.stack_assign(output): a slot even when nothing reads it."""
        off = self.out(n, name)
        if off == SVM_STACK_INVALID:
            off = self.alloc(width)
            self.temps.append((off, width))
        return off

    def _n_ies_texture(self, n):  # nodes.cpp:1279-1295 IESLightNode::compile (identity texture mapping)
        f = n.params["ies"]
        slot = next((i for i, g in enumerate(self.ies_slots) if g.content == f.content), None)
        if slot is None:  # LightManager::add_ies: a new slot per distinct file
            self.ies_slots.append(f)
            slot = len(self.ies_slots) - 1
        strength = self.assign_if_linked(n.inputs["Strength"], "float")
        vec = self.inp(n, "Vector")
        fac = self.out(n, "Fac")
        if fac == SVM_STACK_INVALID:
            fac = self.alloc(1)
            self.temps.append((fac, 1))
        sval = 0.0 if is_linked(n.inputs["Strength"]) else float(n.inputs["Strength"])
        self.emit((NODE_IES, uchar4(strength, vec, fac, 0), slot, f32bits(sval)))

    # -- procedural noise textures (nodes.cpp *TextureNode::compile, identity
    # texture mapping: tex_mapping.compile_begin = stack_assign(vector))
    def _lin(self, n, name):
        return self.assign_if_linked(n.inputs[name], _INPUT_TYPES[n.kind][name])

    def _val(self, n, name):
        v = n.inputs[name]
        return f32bits(0.0 if is_linked(v) else float(v))

    def _vector(self, n):
        return self.inp(n, "Vector")

    def _n_noise_texture(self, n):  # nodes.cpp:1061-1095
        vec = self._vector(n)
        offs = [self._lin(n, k) for k in ("W", "Scale", "Detail", "Roughness", "Distortion")]
        self.emit((NODE_TEX_NOISE, n.params["dimensions"], uchar4(vec, offs[0], offs[1], offs[2]),
                   uchar4(offs[3], offs[4], self.out(n, "Fac"), self.out(n, "Color"))))
        self.emit(tuple(self._val(n, k) for k in ("W", "Scale", "Detail", "Roughness")))
        self.emit((self._val(n, "Distortion"), SVM_STACK_INVALID, SVM_STACK_INVALID, SVM_STACK_INVALID))

    def _n_musgrave_texture(self, n):  # nodes.cpp:1393-1428 (Fac always stack-assigned)
        vec = self._vector(n)
        offs = [self._lin(n, k) for k in ("W", "Scale", "Detail", "Dimension", "Lacunarity", "Offset", "Gain")]
        fac = self.out(n, "Fac")
        if fac == SVM_STACK_INVALID:
            fac = self.alloc(1)
            self.temps.append((fac, 1))
        self.emit((NODE_TEX_MUSGRAVE, uchar4(MUSGRAVE_TYPES[n.params["type"]], n.params["dimensions"], vec, offs[0]),
                   uchar4(offs[1], offs[2], offs[3], offs[4]), uchar4(offs[5], offs[6], fac)))
        self.emit(tuple(self._val(n, k) for k in ("W", "Scale", "Detail", "Dimension")))
        self.emit((self._val(n, "Lacunarity"), self._val(n, "Offset"), self._val(n, "Gain"), 0))

    def _n_wave_texture(self, n):  # nodes.cpp:1492-1528
        vec = self._vector(n)
        d = WAVE_DIRECTIONS[n.params["direction"]]
        self.emit((NODE_TEX_WAVE, uchar4(WAVE_TYPES[n.params["type"]], d, d, WAVE_PROFILES[n.params["profile"]]),
                   uchar4(vec, self._lin(n, "Scale"), self._lin(n, "Distortion")),
                   uchar4(self._lin(n, "Detail"), self._lin(n, "Detail Scale"), self._lin(n, "Detail Roughness"),
                          self._lin(n, "Phase Offset"))))
        self.emit((uchar4(self.out(n, "Color"), self.out(n, "Fac")), self._val(n, "Scale"),
                   self._val(n, "Distortion"), self._val(n, "Detail")))
        self.emit((self._val(n, "Detail Scale"), self._val(n, "Detail Roughness"), self._val(n, "Phase Offset"),
                   SVM_STACK_INVALID))

    def _n_magic_texture(self, n):  # nodes.cpp:1567-1587
        vec = self._vector(n)
        self.emit((NODE_TEX_MAGIC, uchar4(n.params["depth"], self.out(n, "Color"), self.out(n, "Fac")),
                   uchar4(vec, self._lin(n, "Scale"), self._lin(n, "Distortion")), 0))
        self.emit((self._val(n, "Scale"), self._val(n, "Distortion"), 0, 0))

    def _n_brick_texture(self, n):  # nodes.cpp:1688-1734
        vec = self._vector(n)
        c1, c2, mortar = self.inp(n, "Color1"), self.inp(n, "Color2"), self.inp(n, "Mortar")
        p = n.params
        self.emit((NODE_TEX_BRICK, uchar4(vec, c1, c2, mortar),
                   uchar4(self._lin(n, "Scale"), self._lin(n, "Mortar Size"), self._lin(n, "Bias"),
                          self._lin(n, "Brick Width")),
                   uchar4(self._lin(n, "Row Height"), self.out(n, "Color"), self.out(n, "Fac"),
                          self._lin(n, "Mortar Smooth"))))
        self.emit((uchar4(p["offset_frequency"], p["squash_frequency"]), self._val(n, "Scale"),
                   self._val(n, "Mortar Size"), self._val(n, "Bias")))
        self.emit((self._val(n, "Brick Width"), self._val(n, "Row Height"), f32bits(p["offset"]),
                   f32bits(p["squash"])))
        self.emit((self._val(n, "Mortar Smooth"), SVM_STACK_INVALID, SVM_STACK_INVALID, SVM_STACK_INVALID))

    def _n_voronoi_texture(self, n):  # nodes.cpp:1155-1199
        vec = self._vector(n)
        offs = [self._lin(n, k) for k in ("W", "Scale", "Smoothness", "Exponent", "Randomness")]
        p = n.params
        self.emit((NODE_TEX_VORONOI, p["dimensions"], VORONOI_FEATURES[p["feature"]], VORONOI_METRICS[p["metric"]]))
        self.emit((uchar4(vec, offs[0], offs[1], offs[2]),
                   uchar4(offs[3], offs[4], self.out(n, "Distance"), self.out(n, "Color")),
                   uchar4(self.out(n, "Position"), self.out(n, "W"), self.out(n, "Radius")), self._val(n, "W")))
        self.emit(tuple(self._val(n, k) for k in ("Scale", "Smoothness", "Exponent", "Randomness")))

    def _n_white_noise_texture(self, n):  # nodes.cpp:1327-1343 (every socket stack-assigned)
        vec = self._vector(n)
        w = self.inp(n, "W")
        outs = []
        for name in ("Value", "Color"):
            off = self.out(n, name)
            if off == SVM_STACK_INVALID:
                width = 1 if name == "Value" else 3
                off = self.alloc(width)
                self.temps.append((off, width))
            outs.append(off)
        self.emit((NODE_TEX_WHITE_NOISE, n.params["dimensions"], uchar4(vec, w), uchar4(outs[0], outs[1])))

    def _n_gradient(self, n):  # nodes.cpp GradientTextureNode::compile
        vec = self.inp(n, "Vector")
        self.emit((NODE_TEX_GRADIENT, uchar4(GRADIENT_TYPES.index(n.params["type"]), vec, self.out(n, "Fac"),
                                             self.out(n, "Color")), 0, 0))

    def _n_displacement(self, n):  # nodes.cpp:6937-6952 DisplacementNode::compile
        h, m, sc = self.inp(n, "Height"), self.inp(n, "Midlevel"), self.inp(n, "Scale")
        nrm = self.assign_if_linked(n.inputs.get("Normal"), "vector")
        self.emit((NODE_DISPLACEMENT, uchar4(h, m, sc, nrm), self.out(n, "Displacement"),
                   DISPLACEMENT_SPACES[n.params["space"]]))

    def _n_vector_displacement(self, n):  # nodes.cpp:7014-7043 VectorDisplacementNode::compile
        v, m, sc = self.inp(n, "Vector"), self.inp(n, "Midlevel"), self.inp(n, "Scale")
        self.emit((NODE_VECTOR_DISPLACEMENT, uchar4(v, m, sc, self.out(n, "Displacement")), 0, 0))
        self.emit((DISPLACEMENT_SPACES[n.params["space"]], 0, 0, 0))

    def _n_mapping(self, n):  # nodes.cpp MappingNode::compile
        v, loc = self.inp(n, "Vector"), self.inp(n, "Location")
        rot, sc = self.inp(n, "Rotation"), self.inp(n, "Scale")
        self.emit((NODE_MAPPING, MAPPING_TYPES.index(n.params["type"]), uchar4(v, loc, rot, sc),
                   self.out(n, "Vector")))

    def _n_separate_xyz(self, n):
        v = self.inp(n, "Vector")
        for i, name in enumerate("XYZ"):
            if (id(n), name) in self.used:
                self.emit((NODE_SEPARATE_VECTOR, v, i, self.out(n, name)))

    def _n_combine_xyz(self, n):
        out = self.out(n, "Vector")
        for i, name in enumerate("XYZ"):
            self.emit((NODE_COMBINE_VECTOR, self.inp(n, name), i, out))

    def _n_separate_hsv(self, n):
        col = self.inp(n, "Color")
        self.emit((NODE_SEPARATE_HSV, col, self.out(n, "H"), self.out(n, "S")))
        self.emit((NODE_SEPARATE_HSV, self.out(n, "V"), 0, 0))

    def _n_combine_hsv(self, n):
        h, s, v = self.inp(n, "H"), self.inp(n, "S"), self.inp(n, "V")
        self.emit((NODE_COMBINE_HSV, h, s, v))
        self.emit((NODE_COMBINE_HSV, self.out(n, "Color"), 0, 0))

    def _defaults(self, n, names):
        return [0.0 if is_linked(n.inputs[k]) else float(n.inputs[k]) for k in names]

    def _n_clamp(self, n):  # nodes.cpp ClampNode::compile
        v = self.inp(n, "Value")
        mn = self.assign_if_linked(n.inputs["Min"], "float")
        mx = self.assign_if_linked(n.inputs["Max"], "float")
        dmin, dmax = self._defaults(n, ["Min", "Max"])
        self.emit((NODE_CLAMP, v, uchar4(mn, mx, CLAMP_TYPES.index(n.params["type"])), self.out(n, "Result")))
        self.emit((f32bits(dmin), f32bits(dmax), 0, 0))

    def _n_map_range(self, n):  # nodes.cpp MapRangeNode::compile
        names = ["From Min", "From Max", "To Min", "To Max"]
        v = self.inp(n, "Value")
        offs = [self.assign_if_linked(n.inputs[k], "float") for k in names]
        steps = self.assign_if_linked(n.inputs["Steps"], "float")
        d = self._defaults(n, names)
        (dsteps,) = self._defaults(n, ["Steps"])
        self.emit((NODE_MAP_RANGE, v, uchar4(*offs),
                   uchar4(MAP_RANGE_TYPES.index(n.params["type"]), steps, self.out(n, "Result"))))
        self.emit(tuple(f32bits(x) for x in d))
        self.emit((f32bits(dsteps), 0, 0, 0))

    def _n_rgb_ramp(self, n):  # nodes.cpp RGBRampNode::compile + SVMCompiler::add_node(float4 table)
        fac = self.inp(n, "Fac")
        table = n.params["table"]
        self.emit((NODE_RGB_RAMP, uchar4(fac, self.out(n, "Color"), self.out(n, "Alpha")),
                   int(n.params["interpolate"]), 0))
        self.emit((len(table), 0, 0, 0))
        for row in table:
            self.emit(tuple(f32bits(float(x)) for x in row))
