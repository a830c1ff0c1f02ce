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

from . import abi, native, nodes, sobol
from . import nodes as _nodes  # compile_scene has a local "nodes" (BVH nodes)

# ---------------------------------------------------------------------------
# constants of the device ABI (kernel_types.h / svm_types.h)
PATH_RAY_ALL_VISIBILITY = (1 << 14) - 1
PATH_RAY_SHADOW_OPAQUE_NON_CATCHER = 1 << 7
PATH_RAY_SHADOW_OPAQUE_CATCHER = 1 << 8
PATH_RAY_SHADOW_TRANSPARENT_NON_CATCHER = 1 << 9
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
PRIMITIVE_CURVE_THICK = 1 << 2
PRIMITIVE_CURVE_RIBBON = 1 << 4
PRIMITIVE_ALL_CURVE = (1 << 2) | (1 << 3) | (1 << 4) | (1 << 5)
PRIMITIVE_NUM_TOTAL = 6  # kernel_types.h:713: the segment index is packed above the type bits
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
NODE_SET_DISPLACEMENT = 20
NODE_ENTER_BUMP_EVAL, NODE_LEAVE_BUMP_EVAL = 34, 35  # svm_types.h ShaderNodeType
NODE_AOV_START, NODE_AOV_COLOR, NODE_AOV_VALUE = 88, 89, 90
SVM_BUMP_EVAL_STATE_SIZE = 9  # svm_types.h
ATTR_STD_POSITION_UNDISPLACED = 10  # kernel_types.h AttributeStandard
NODE_CLOSURE_BACKGROUND, NODE_CLOSURE_SET_WEIGHT = 4, 5
NODE_CLOSURE_HOLDOUT = 37  # svm_types.h ShaderNodeType
NODE_CLOSURE_WEIGHT, NODE_EMISSION_WEIGHT = 6, 7
NODE_MIX_CLOSURE, NODE_JUMP_IF_ZERO, NODE_VALUE_F = 8, 9, 14
SVM_STACK_INVALID = 255
SVM_STACK_SIZE = 32  # CY_SVM_STACK (cy_types.h)

CLOSURE_BSDF_DIFFUSE_ID = 2
CLOSURE_BSDF_DIFFUSE_TOON_ID = 7
CLOSURE_BSDF_TRANSLUCENT_ID = 8
CLOSURE_BSDF_REFLECTION_ID = 9
CLOSURE_BSDF_MICROFACET_GGX_ID = 10
CLOSURE_BSDF_MICROFACET_BECKMANN_ID = 13
CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID = 16
CLOSURE_BSDF_ASHIKHMIN_VELVET_ID = 17
CLOSURE_BSDF_GLOSSY_TOON_ID = 20
CLOSURE_BSDF_REFRACTION_ID = 22
CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID = 23
CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID = 24
CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID = 26
CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID = 27
CLOSURE_BSDF_SHARP_GLASS_ID = 29
CLOSURE_BSDF_TRANSPARENT_ID = 34
CLOSURE_BSDF_HAIR_REFLECTION_ID = 21
CLOSURE_BSDF_HAIR_PRINCIPLED_ID = 30
CLOSURE_BSDF_HAIR_TRANSMISSION_ID = 31
ATTR_STD_CURVE_INTERCEPT, ATTR_STD_CURVE_RANDOM = 14, 15  # kernel_types.h AttributeStandard
# PrincipledHairBsdfNode (nodes.cpp:3474-3512): parametrization enum
# (svm_types.h:509-513) and socket defaults
PRINCIPLED_HAIR_PARAMETRIZATIONS = {"color": 0, "melanin": 1, "absorption": 2}
PRINCIPLED_HAIR_DEFAULTS = {
    "color": (0.017513, 0.005763, 0.002059), "melanin": 0.8, "melanin_redness": 1.0, "tint": (1.0, 1.0, 1.0),
    "absorption_coefficient": (0.245531, 0.52, 1.365), "offset": 2.0 * 3.14159265358979 / 180.0, "roughness": 0.3,
    "radial_roughness": 0.3, "coat": 0.0, "ior": 1.55, "random_roughness": 0.0, "random_color": 0.0,
    "random": 0.0, "normal": None}
# HairBsdfNode (nodes.cpp:3603-3635)
HAIR_DEFAULTS = {"offset": 0.0, "roughness_u": 0.2, "roughness_v": 0.2}
# Subsurface Scattering node falloffs (nodes.cpp SubsurfaceScatteringNode)
SUBSURFACE_FALLOFFS = {"cubic": 35, "gaussian": 36, "burley": 38, "random_walk": 39}
CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID = 40

# Distribution enums of the glossy / anisotropic / glass / refraction nodes
# (nodes.cpp GlossyBsdfNode, GlassBsdfNode, RefractionBsdfNode NODE_DEFINE)
CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID = 14
GLOSSY_DISTRIBUTIONS = {"sharp": CLOSURE_BSDF_REFLECTION_ID, "ggx": CLOSURE_BSDF_MICROFACET_GGX_ID,
                        "beckmann": CLOSURE_BSDF_MICROFACET_BECKMANN_ID,
                        "ashikhmin_shirley": CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID,
                        "multi_ggx": CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID}
CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID = 25
GLASS_DISTRIBUTIONS = {"sharp": CLOSURE_BSDF_SHARP_GLASS_ID, "ggx": CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID,
                       "beckmann": CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID,
                       "multi_ggx": CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID}
REFRACTION_DISTRIBUTIONS = {"sharp": CLOSURE_BSDF_REFRACTION_ID, "ggx": CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID,
                            "beckmann": CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID}
CLOSURE_BSDF_PRINCIPLED_ID = 45
CLOSURE_BSSRDF_PRINCIPLED_ID = 37
# PrincipledBsdfNode subsurface_method (nodes.cpp:2706-2711)
PRINCIPLED_SUBSURFACE_METHODS = {"burley": 37, "random_walk": 40}
PRINCIPLED_DISTRIBUTIONS = {"ggx": CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID, "multiscatter": 25}
# PrincipledBsdfNode sockets and defaults (render/nodes.cpp:2720-2770)
PRINCIPLED_DEFAULTS = {
    "base_color": (0.8, 0.8, 0.8), "subsurface_color": (0.8, 0.8, 0.8), "metallic": 0.0, "subsurface": 0.0,
    "subsurface_radius": (0.1, 0.1, 0.1), "specular": 0.0, "roughness": 0.5, "specular_tint": 0.0,
    "anisotropic": 0.0, "sheen": 0.0, "sheen_tint": 0.0, "clearcoat": 0.0, "clearcoat_roughness": 0.03,
    "ior": 0.0, "transmission": 0.0, "transmission_roughness": 0.0, "anisotropic_rotation": 0.0,
}
PRINCIPLED_VECTORS = ("normal", "clearcoat_normal", "tangent")
BECKMANN_CLOSURES = (CLOSURE_BSDF_MICROFACET_BECKMANN_ID, CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID,
                     CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID)
SD_HAS_TRANSPARENT_SHADOW = 1 << 17
SD_HAS_DISPLACEMENT = 1 << 26
SD_HAS_BSSRDF_BUMP = 1 << 21
SD_HAS_BUMP = 1 << 25
# volumes (kernel_types.h:832-931, svm_types.h:577-579, 105-106)
SD_HAS_VOLUME = 1 << 18
SD_HAS_ONLY_VOLUME = 1 << 19
SD_HETEROGENEOUS_VOLUME = 1 << 20
SD_VOLUME_EQUIANGULAR, SD_VOLUME_MIS = 1 << 22, 1 << 23  # kernel_types.h:887-889 ShaderDataFlag
SD_NEED_VOLUME_ATTRIBUTES = 1 << 28
SD_OBJECT_HAS_VOLUME = 1 << 4
SD_OBJECT_INTERSECTS_VOLUME = 1 << 5
SD_OBJECT_HOLDOUT_MASK = 1 << 0  # kernel_types.h ShaderDataObjectFlag; object.cpp:547-548 use_holdout
SD_OBJECT_SHADOW_CATCHER = 1 << 7  # object.cpp:714-719 is_shadow_catcher
CLOSURE_VOLUME_ABSORPTION_ID = 43
CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID = 44
NODE_CLOSURE_VOLUME, NODE_PRINCIPLED_VOLUME = 40, 41
VOLUME_STACK_SIZE = 32  # kernel_types.h:64
ATTR_STD_VOLUME_DENSITY, ATTR_STD_VOLUME_TEMPERATURE, ATTR_STD_NUM = 18, 22, 26
# PrincipledVolumeNode sockets and defaults (render/nodes.cpp:3376-3410)
PRINCIPLED_VOLUME_DEFAULTS = {"absorption_color": (0.0, 0.0, 0.0), "emission_strength": 0.0,
                              "emission_color": (1.0, 1.0, 1.0)}


def f32bits(x: float) -> int:
    return int(np.array([x], dtype=np.float32).view(np.uint32)[0])


# ---------------------------------------------------------------------------
# Shader description (a tiny node graph: one closure tree per material)


@dataclass
class Closure:
    """One closure tree node.  `color`, `roughness`, `ior`, `strength`, `fac`
    and `normal` take constants or node sockets (nodes.py)."""

    # diffuse | translucent | glossy | anisotropic | glass | refraction | velvet |
    # diffuse_toon | glossy_toon | transparent | emission | background | mix
    kind: str
    color: object = (0.8, 0.8, 0.8)
    roughness: object = 0.0  # roughness; velvet: sigma; toon: size
    ior: object = 1.45  # glass / refraction: IOR; toon: smooth
    strength: object = 1.0
    fac: object = 0.5
    a: "Closure | None" = None
    b: "Closure | None" = None
    normal: object = None
    distribution: str = "ggx"  # glossy / anisotropic / glass / refraction
    anisotropy: object = 0.0
    rotation: object = 0.0
    tangent: object = None
    params: dict | None = None  # principled: PRINCIPLED_DEFAULTS keys + normals
    # subsurface: radius (vector), sharpness, texture blur (strength = scale)
    radius: object = (0.1, 0.1, 0.1)
    sharpness: object = 0.0
    texture_blur: object = 0.0
    subsurface_method: str = "burley"  # principled
    # material output "Displacement" (a vector socket, e.g. nodes.displacement)
    # and the material's displacement method (shader.cpp:184-188): "true" (its
    # own SVM program, run by SHADER_EVAL_DISPLACE) or "bump" (a bump program
    # from the displacement graph ahead of the surface program, through ray
    # differentials; Blender's default).  "both" needs the mesh displaced with
    # its undisplaced positions kept (ATTR_STD_POSITION_UNDISPLACED, Mesh.undisplaced)
    # and adds a bump program evaluated at them (NODE_ENTER / LEAVE_BUMP_EVAL).
    displacement: object = None
    displacement_method: str = "true"
    # material output "Volume": a tree of volume closures (volume_absorption,
    # volume_scatter, principled_volume, emission, mix), its own SVM program
    volume: "Closure | None" = None
    pass_index: int = 0  # Material pass index (KernelShader.pass_id, Object Info "Material Index")
    density: object = 1.0  # volume closures
    # AOV Output nodes of the material (OutputAOVNode, nodes.cpp): AOV name ->
    # a colour or value (constant or socket) written to the film's AOV pass of
    # that name at the camera path's first hit (svm_aov.h); names without a
    # pass in Scene.aovs are dropped, as OutputAOVNode::simplify drops them
    aovs: dict | None = None
    # Shader::volume_sampling_method of the material's volume: "distance",
    # "equiangular" or "multiple_importance" (SD_VOLUME_EQUIANGULAR / _MIS)
    volume_sampling: str = "distance"

    def closure_type(self) -> int:
        """The ClosureType the node compiles to, after simplify_settings
        (nodes.cpp:2373-2581: an unlinked roughness <= 1e-4 selects the sharp
        distribution when filter_glossy is 0)."""
        sharp = not nodes.is_linked(self.roughness) and self.roughness <= 1e-4
        if self.kind == "glossy":
            return GLOSSY_DISTRIBUTIONS["sharp" if sharp else self.distribution]
        if self.kind == "anisotropic":
            return GLOSSY_DISTRIBUTIONS[self.distribution]
        if self.kind == "glass":
            return GLASS_DISTRIBUTIONS["sharp" if sharp else self.distribution]
        if self.kind == "refraction":
            return REFRACTION_DISTRIBUTIONS["sharp" if sharp else self.distribution]
        if self.kind == "subsurface":
            return SUBSURFACE_FALLOFFS[self.distribution]
        if self.kind == "hair":
            return CLOSURE_BSDF_HAIR_TRANSMISSION_ID if self.distribution == "transmission" else \
                CLOSURE_BSDF_HAIR_REFLECTION_ID
        if self.kind == "principled_hair":
            return CLOSURE_BSDF_HAIR_PRINCIPLED_ID
        return {"diffuse": CLOSURE_BSDF_DIFFUSE_ID, "translucent": CLOSURE_BSDF_TRANSLUCENT_ID,
                "velvet": CLOSURE_BSDF_ASHIKHMIN_VELVET_ID, "diffuse_toon": CLOSURE_BSDF_DIFFUSE_TOON_ID,
                "glossy_toon": CLOSURE_BSDF_GLOSSY_TOON_ID, "transparent": CLOSURE_BSDF_TRANSPARENT_ID}[self.kind]

    def num_closures(self) -> int:
        """ShaderGraph::get_num_closures (render/graph.cpp:1130-1161)."""
        if self.kind == "mix":
            return self.a.num_closures() + self.b.num_closures()
        if self.kind == "glass":
            return 2
        if self.kind in ("glossy", "anisotropic") and self.closure_type() == CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
            return 2  # CLOSURE_IS_BSDF_MULTISCATTER
        if self.kind == "principled":
            return 8  # CLOSURE_IS_PRINCIPLED
        if self.kind == "subsurface":
            return 3  # CLOSURE_IS_BSSRDF
        if self.kind == "principled_hair":
            return 4  # graph.cpp:1153-1155
        if self.kind in VOLUME_KINDS:
            return VOLUME_STACK_SIZE  # CLOSURE_IS_VOLUME
        if self.kind in ("none", "emission", "background"):
            return 0 if self.kind == "none" else 1
        return 1

    def material_closures(self) -> int:
        """ShaderGraph::get_num_closures over both outputs of a material."""
        return self.num_closures() + (self.volume.num_closures() if self.volume is not None else 0)

    def closure_types(self) -> set:
        if self.kind == "mix":
            return self.a.closure_types() | self.b.closure_types()
        if self.kind in ("emission", "background", "none", "holdout") or self.kind in VOLUME_KINDS:
            return set()
        if self.kind == "principled":
            return {CLOSURE_BSDF_PRINCIPLED_ID}
        return {self.closure_type()}

    def has_emission(self) -> bool:
        if self.kind == "mix":
            return self.a.has_emission() or self.b.has_emission()
        return self.kind == "emission"

    def has_transparent(self) -> bool:
        """Shader::has_surface_transparent (svm.cpp:515)."""
        if self.kind == "mix":
            return self.a.has_transparent() or self.b.has_transparent()
        return self.kind == "transparent"

    def sockets(self) -> list:
        """Every linked input of the tree (nodes.Socket), with its socket type."""
        out = []
        for name, t in (("color", "color"), ("roughness", "float"), ("ior", "float"), ("strength", "float"),
                        ("fac", "float"), ("normal", "vector"), ("anisotropy", "float"), ("rotation", "float"),
                        ("tangent", "vector"), ("radius", "vector"), ("sharpness", "float"),
                        ("texture_blur", "float"), ("density", "float")):
            v = getattr(self, name)
            if nodes.is_linked(v) and (self.kind == "mix") == (name == "fac"):
                out.append((v, t))
        if self.kind in ("principled", "principled_volume", "principled_hair", "hair"):
            for name, v in self.params.items():
                if nodes.is_linked(v):
                    vec = name in PRINCIPLED_VECTORS or name in ("subsurface_radius", "absorption_coefficient")
                    col = name.endswith("color") and name != "random_color" or name == "tint"
                    out.append((v, "color" if col else "vector" if vec else "float"))
        for sub in (self.a, self.b):
            if sub is not None:
                out.extend(sub.sockets())
        return out

    def constant_emission(self):
        """ShaderManager constant emission (shader.cpp:462-475, nodes.cpp
        EmissionNode/BackgroundNode::constant_emission): color * strength when
        neither input is linked."""
        if self.kind not in ("emission", "background"):
            return None
        if nodes.is_linked(self.color) or nodes.is_linked(self.strength):
            return None
        return np.array(self.color, dtype=np.float32) * np.float32(self.strength)


def diffuse(color, roughness=0.0, normal=None):
    return Closure("diffuse", _const_or_socket(color), roughness=roughness, normal=normal)


def glossy(color, roughness, normal=None, distribution="ggx"):
    """Glossy BSDF: distribution ggx | beckmann | ashikhmin_shirley | sharp |
    multi_ggx (multiple-scattering GGX, bsdf_microfacet_multi.h)."""
    return Closure("glossy", _const_or_socket(color), roughness=roughness, normal=normal, distribution=distribution)


def anisotropic(color, roughness, anisotropy, rotation, tangent=None, normal=None, distribution="ggx"):
    """Anisotropic BSDF (nodes.cpp AnisotropicBsdfNode).  An unset tangent is
    the reference's default link (graph.cpp:885-889): the Geometry node's
    Tangent, the radial tangent of the generated coordinates."""
    if tangent is None:
        tangent = nodes.geometry()["Tangent"]
    if not nodes.is_linked(tangent):
        raise ValueError("anisotropic BSDF: link the tangent input to a vector socket")
    return Closure("anisotropic", _const_or_socket(color), roughness=roughness, anisotropy=anisotropy,
                   rotation=rotation, tangent=tangent, normal=normal, distribution=distribution)


def glass(color, roughness, ior=1.45, normal=None, distribution="ggx"):
    """Glass BSDF: distribution ggx | beckmann | sharp | multi_ggx
    (multiple-scattering GGX glass, bsdf_microfacet_multi.h)."""
    return Closure("glass", _const_or_socket(color), roughness=roughness, ior=ior, normal=normal,
                   distribution=distribution)


def refraction(color, roughness, ior=1.45, normal=None, distribution="ggx"):
    """Refraction BSDF: distribution ggx | beckmann | sharp."""
    return Closure("refraction", _const_or_socket(color), roughness=roughness, ior=ior, normal=normal,
                   distribution=distribution)


def principled(distribution="ggx", subsurface_method="burley", **params):
    """Principled BSDF (nodes.cpp PrincipledBsdfNode, svm_closure.h:100-463).
    Parameters are PRINCIPLED_DEFAULTS keys (constants or sockets) plus the
    normal / clearcoat_normal / tangent vector sockets.  distribution is
    "ggx" or "multiscatter" (Blender's default: multiple-scattering GGX for the
    specular layer and for rough transmission); subsurface > 0 adds a BSSRDF.  The node's Emission and Alpha inputs (expanded
    into separate closures by the reference graph) are expressed here with
    emission() / transparent() and mix()."""
    unknown = set(params) - set(PRINCIPLED_DEFAULTS) - set(PRINCIPLED_VECTORS)
    if unknown:
        raise ValueError(f"principled: unknown parameters {sorted(unknown)}")
    p = dict(PRINCIPLED_DEFAULTS)
    p.update(params)
    if subsurface_method not in PRINCIPLED_SUBSURFACE_METHODS:
        raise ValueError(f"principled: unknown subsurface_method {subsurface_method}")
    if "tangent" not in params and (_nodes.is_linked(p["anisotropic"]) or float(p["anisotropic"]) != 0.0):
        # graph.cpp:885-889 default link of the Tangent input (only read when
        # the roughness is anisotropic)
        p["tangent"] = _nodes.geometry()["Tangent"]
    if distribution not in PRINCIPLED_DISTRIBUTIONS:
        raise ValueError(f"principled: distribution one of {sorted(PRINCIPLED_DISTRIBUTIONS)}")
    return Closure("principled", distribution=distribution, params=p, subsurface_method=subsurface_method)


def subsurface(color, scale=0.01, radius=(0.1, 0.1, 0.1), falloff="burley", texture_blur=1.0, sharpness=0.0,
               normal=None):
    """Subsurface Scattering node (nodes.cpp:3025-3045 SubsurfaceScatteringNode,
    a BSSRDF closure, svm_closure.h:880-905), with the node's defaults:
    falloff burley | cubic | gaussian (disk profiles, up to four exit points)
    | random_walk; texture_blur re-evaluates the shader at the exit point and
    blends the two points' colours (kernel_subsurface.h:132-158)."""
    if falloff not in SUBSURFACE_FALLOFFS:
        raise ValueError(f"subsurface: unknown falloff {falloff}")
    return Closure("subsurface", _const_or_socket(color), strength=scale, radius=radius, distribution=falloff,
                   texture_blur=texture_blur, sharpness=sharpness, normal=normal)


def principled_hair(parametrization="color", **params):
    """Principled Hair BSDF node (nodes.cpp:3474-3593 PrincipledHairBsdfNode,
    closure/bsdf_hair_principled.h): parametrization "color" (direct
    colouring), "melanin" (pigment concentration, with tint and random
    colour) or "absorption" (absorption coefficient); parameters are
    PRINCIPLED_HAIR_DEFAULTS keys (constants or sockets).  Random defaults to
    the curves' ATTR_STD_CURVE_RANDOM attribute when unlinked (absent here:
    the node's Random value is used)."""
    unknown = set(params) - set(PRINCIPLED_HAIR_DEFAULTS)
    if unknown:
        raise ValueError(f"principled_hair: unknown parameters {sorted(unknown)}")
    if parametrization not in PRINCIPLED_HAIR_PARAMETRIZATIONS:
        raise ValueError(f"principled_hair: parametrization one of {sorted(PRINCIPLED_HAIR_PARAMETRIZATIONS)}")
    p = dict(PRINCIPLED_HAIR_DEFAULTS)
    p.update(params)
    return Closure("principled_hair", distribution=parametrization, params=p)


def hair(color=(0.8, 0.8, 0.8), component="reflection", tangent=None, normal=None, **params):
    """Hair BSDF node (nodes.cpp:3603-3635 HairBsdfNode, closure/bsdf_hair.h):
    component "reflection" or "transmission"; offset, roughness_u,
    roughness_v (HAIR_DEFAULTS keys); the tangent defaults to the curve's
    dPdu (dPdv on meshes, offset 0)."""
    unknown = set(params) - set(HAIR_DEFAULTS)
    if unknown:
        raise ValueError(f"hair: unknown parameters {sorted(unknown)}")
    if component not in ("reflection", "transmission"):
        raise ValueError("hair: component is reflection or transmission")
    p = dict(HAIR_DEFAULTS)
    p.update(params)
    return Closure("hair", _const_or_socket(color), distribution=component, params=p, tangent=tangent, normal=normal)


VOLUME_KINDS = ("volume_absorption", "volume_scatter", "principled_volume")


def volume_absorption(color=(0.8, 0.8, 0.8), density=1.0):
    """Volume Absorption node (nodes.cpp AbsorptionVolumeNode)."""
    return Closure("volume_absorption", _const_or_socket(color), density=density)


def volume_scatter(color=(0.8, 0.8, 0.8), density=1.0, anisotropy=0.0):
    """Volume Scatter node (nodes.cpp ScatterVolumeNode): Henyey-Greenstein."""
    return Closure("volume_scatter", _const_or_socket(color), density=density, anisotropy=anisotropy)


def principled_volume(color=(0.5, 0.5, 0.5), density=1.0, anisotropy=0.0, **params):
    """Principled Volume node (nodes.cpp PrincipledVolumeNode) without volume
    attributes (no voxel grids: the density and color attributes are never
    found) and without blackbody emission.  params: absorption_color,
    emission_strength, emission_color."""
    unknown = set(params) - set(PRINCIPLED_VOLUME_DEFAULTS)
    if unknown:
        raise ValueError(f"principled_volume: unknown parameters {sorted(unknown)}")
    p = dict(PRINCIPLED_VOLUME_DEFAULTS)
    p.update(params)
    return Closure("principled_volume", _const_or_socket(color), density=density, anisotropy=anisotropy, params=p)


def material(surface=None, volume=None):
    """A material with a Surface and / or a Volume output.  Without a surface
    the mesh only bounds its volume (SD_HAS_ONLY_VOLUME: rays pass through)."""
    m = surface if surface is not None else Closure("none")
    m.volume = volume
    return m


def translucent(color, normal=None):
    return Closure("translucent", _const_or_socket(color), normal=normal)


def velvet(color, sigma=1.0, normal=None):
    return Closure("velvet", _const_or_socket(color), roughness=sigma, normal=normal)


def toon(color, size=0.5, smooth=0.0, glossy=False, normal=None):
    return Closure("glossy_toon" if glossy else "diffuse_toon", _const_or_socket(color), roughness=size,
                   ior=smooth, normal=normal)


def transparent(color=(1.0, 1.0, 1.0)):
    """Transparent BSDF (nodes.cpp TransparentBsdfNode): light passes straight
    through, weighted by color; its shadows are transparent too."""
    return Closure("transparent", _const_or_socket(color))


def emission(color, strength):
    return Closure("emission", _const_or_socket(color), strength=strength)


def holdout():
    """Holdout closure (nodes.cpp:3177-3201 HoldoutNode): with a transparent
    film the surface cuts the pixel's alpha by its mix weight; the path ends
    where the holdout weight is 1 (kernel_path.h:285-296)."""
    return Closure("holdout", (1.0, 1.0, 1.0))


def background(color, strength=1.0):
    return Closure("background", _const_or_socket(color), strength=strength)


def mix(fac, a, b):
    return Closure("mix", fac=fac, a=a, b=b)


def _const_or_socket(v):
    return v if nodes.is_linked(v) else tuple(v)


class SVMCompiler:
    """Emits SVM bytecode with the node encodings of svm/svm.h + svm_closure.h
    (the reference host compiler is render/svm.cpp + nodes.cpp compile())."""

    def __init__(self):
        self.images: list = []  # SVM image slots, shared by every shader of the scene
        self.features: set = set()  # scene-wide needs of the compiled nodes (NodeCompiler.features)
        self.ies_slots: list = []  # IES files of the IES Texture nodes (LightManager ies_slots)
        self.nodes: list[tuple[int, int, int, int]] = []
        self.stack_top = 0
        self.stack_used = [False] * SVM_STACK_SIZE
        self.nc: nodes.NodeCompiler | None = None
        # ShaderManager::get_attribute_id (shader.cpp:442-460): standard
        # attributes by their id, names from ATTR_STD_NUM in first-use order
        self.attribute_ids: dict[str, int] = {}
        # per shader: the attribute requests of its nodes (ShaderNode::attributes),
        # as standard ids or names, in first-use order
        self.requests: list[list] = []
        self._shader = 0
        # Film::get_aov_offset (film.cpp:691-712): AOV name -> (is_color, index
        # among the film's colour / value AOV passes)
        self.aov_slots: dict[str, tuple[bool, int]] = {}

    def attribute(self, key) -> int:
        """SVMCompiler::attribute: the kernel's id for a standard attribute
        (int) or a name, recorded as a request of the shader being compiled."""
        if isinstance(key, str):
            if key not in self.attribute_ids:
                self.attribute_ids[key] = nodes.ATTR_STD_NUM + len(self.attribute_ids)
            aid = self.attribute_ids[key]
        else:
            aid = int(key)
        reqs = self.requests[self._shader]
        if key not in reqs:
            reqs.append(key)
        return aid

    def _node_compiler(self, roots, background=False, volume=False):
        return nodes.NodeCompiler(self.alloc, self.nodes.append, roots, self.free, images=self.images,
                                  attribute=self.attribute, background=background, volume=volume,
                                  features=self.features, ies_slots=self.ies_slots)

    def alloc(self, n=1) -> int:
        """First fit over the free slots (svm.cpp stack_find_offset)."""
        for off in range(SVM_STACK_SIZE - n + 1):
            if not any(self.stack_used[off:off + n]):
                self.stack_used[off:off + n] = [True] * n
                self.stack_top = max(self.stack_top, off + n)
                return off
        raise ValueError(f"SVM stack exceeds the HIP device's {SVM_STACK_SIZE} slots")

    def free(self, off: int, n: int = 1):
        self.stack_used[off:off + n] = [False] * n

    @staticmethod
    def uchar4(x, y, z, w) -> int:
        return (x & 0xFF) | ((y & 0xFF) << 8) | ((z & 0xFF) << 16) | ((w & 0xFF) << 24)

    def _float_param(self, v):
        """(stack offset, inline value) of a BSDF float parameter."""
        if nodes.is_linked(v):
            return self.nc.link(v, "float"), 0.0
        return SVM_STACK_INVALID, float(v)

    def emit_closure(self, c: Closure, mix_weight: int) -> list:
        out = []
        emit = out.append
        if c.kind == "mix":
            if nodes.is_linked(c.fac):
                fac_off = self.nc.link(c.fac, "float")
            else:
                fac_off = self.alloc()
                emit((NODE_VALUE_F, f32bits(c.fac), fac_off, 0))
            w1, w2 = self.alloc(), self.alloc()
            emit((NODE_MIX_CLOSURE, self.uchar4(fac_off, mix_weight, w1, w2), 0, 0))
            for sub, w in ((c.a, w1), (c.b, w2)):
                code = self.emit_closure(sub, w)
                emit((NODE_JUMP_IF_ZERO, len(code), w, 0))
                out.extend(code)
            return out
        if c.kind in ("emission", "background"):
            # nodes.cpp EmissionNode/BackgroundNode::compile
            const = c.constant_emission()
            if const is None:
                emit((NODE_EMISSION_WEIGHT, self.nc.assign(c.color, "color"), self.nc.assign(c.strength, "float"), 0))
            else:
                emit((NODE_CLOSURE_SET_WEIGHT, *(f32bits(v) for v in const)))
            emit((NODE_CLOSURE_EMISSION if c.kind == "emission" else NODE_CLOSURE_BACKGROUND, mix_weight, 0, 0))
            return out
        if c.kind == "holdout":
            # nodes.cpp:3195-3201 HoldoutNode::compile
            emit((NODE_CLOSURE_SET_WEIGHT, *(f32bits(1.0) for _ in range(3))))
            emit((NODE_CLOSURE_HOLDOUT, mix_weight, 0, 0))
            return out
        if c.kind == "principled":
            return self.emit_principled(c, mix_weight)
        if c.kind == "principled_hair":
            return self.emit_principled_hair(c, mix_weight)
        if c.kind == "none":
            return out
        if c.kind in VOLUME_KINDS:
            return self.emit_volume(c, mix_weight)
        ctype = c.closure_type()
        # nodes.cpp BsdfNode::compile: linked color -> NODE_CLOSURE_WEIGHT
        if nodes.is_linked(c.color):
            emit((NODE_CLOSURE_WEIGHT, self.nc.link(c.color, "color"), 0, 0))
        else:
            emit((NODE_CLOSURE_SET_WEIGHT, *(f32bits(v) for v in c.color)))
        normal_off = self.nc.link(c.normal, "vector") if nodes.is_linked(c.normal) else SVM_STACK_INVALID
        tangent_off, param3_off, param4_off = SVM_STACK_INVALID, SVM_STACK_INVALID, SVM_STACK_INVALID
        # per node: (param1, param2) of BsdfNode::compile (nodes.cpp:2200-2800)
        if c.kind in ("diffuse", "velvet"):
            params = (c.roughness, None)
        elif c.kind in ("translucent", "transparent") or ctype in (CLOSURE_BSDF_REFLECTION_ID,):
            params = (None, None)
        elif c.kind == "anisotropic":
            params = (c.roughness, c.anisotropy)
            tangent_off = self.nc.link(c.tangent, "vector")
            # param3 (rotation) is always stack-assigned (BsdfNode::compile)
            param3_off = self.nc.assign(c.rotation, "float")
            if ctype == CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
                param4_off = self.nc.assign(c.color, "color")  # nodes.cpp:2330-2332
        elif c.kind == "glossy":
            params = (c.roughness, None)
            if ctype == CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
                # GlossyBsdfNode::compile (nodes.cpp:2423-2424): the colour
                # goes to the multiscatter walk as param4 (stack-assigned)
                param4_off = self.nc.assign(c.color, "color")
        elif c.kind == "hair":
            # HairBsdfNode::compile: BsdfNode::compile(RoughnessU, RoughnessV, Offset)
            params = (c.params["roughness_u"], c.params["roughness_v"])
            param3_off = self.nc.assign(c.params["offset"], "float")
            if nodes.is_linked(c.tangent):
                tangent_off = self.nc.link(c.tangent, "vector")
        elif c.kind == "subsurface":
            # BsdfNode::compile(Scale, Texture Blur, Radius, Sharpness): radius and
            # sharpness always stack-assigned
            params = (c.strength, c.texture_blur)
            param3_off = self.nc.assign(c.radius, "vector")
            param4_off = self.nc.assign(c.sharpness, "float")
        else:  # glass, refraction (roughness, IOR); toons (size, smooth)
            params = (c.roughness, c.ior)
            if ctype == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID:
                # GlassBsdfNode::compile (nodes.cpp:2516-2517): the colour as param3
                param3_off = self.nc.assign(c.color, "color")
        p1, v1 = self._float_param(params[0]) if params[0] is not None else (SVM_STACK_INVALID, 0.0)
        p2, v2 = self._float_param(params[1]) if params[1] is not None else (SVM_STACK_INVALID, 0.0)
        emit((NODE_CLOSURE_BSDF, self.uchar4(ctype, p1, p2, mix_weight), f32bits(v1), f32bits(v2)))
        # data node: normal, tangent, param3, param4
        emit((normal_off, tangent_off, param3_off, param4_off))
        return out

    def emit_volume(self, c: Closure, mix_weight: int) -> list:
        """nodes.cpp:3273-3290 VolumeNode::compile (absorption: density;
        scatter: density, anisotropy) and 3417-3455 PrincipledVolumeNode::compile
        (closure node, value node, attribute node)."""
        out = []
        emit = out.append
        if nodes.is_linked(c.color):
            emit((NODE_CLOSURE_WEIGHT, self.nc.link(c.color, "color"), 0, 0))
        else:
            emit((NODE_CLOSURE_SET_WEIGHT, *(f32bits(v) for v in c.color)))
        if c.kind in ("volume_absorption", "volume_scatter"):
            ctype = CLOSURE_VOLUME_ABSORPTION_ID if c.kind == "volume_absorption" else \
                CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID
            d_off, d_val = self._float_param(c.density)
            a_off, a_val = (self._float_param(c.anisotropy) if c.kind == "volume_scatter"
                            else (SVM_STACK_INVALID, 0.0))
            emit((NODE_CLOSURE_VOLUME, self.uchar4(ctype, d_off, a_off, mix_weight), f32bits(d_val), f32bits(a_val)))
            return out
        p = c.params
        nc = self.nc
        temps: list = []
        saved_emit, nc.emit = nc.emit, emit
        try:
            d_off = nc.link(c.density, "float") if nodes.is_linked(c.density) else SVM_STACK_INVALID
            a_off = nc.link(c.anisotropy, "float") if nodes.is_linked(c.anisotropy) else SVM_STACK_INVALID
            ac_off = nc.assign(p["absorption_color"], "color", temps)
            e_off = (nc.link(p["emission_strength"], "float") if nodes.is_linked(p["emission_strength"])
                     else SVM_STACK_INVALID)
            ec_off = nc.assign(p["emission_color"], "color", temps)
        finally:
            nc.emit = saved_emit

        def const(v):
            return 0.0 if nodes.is_linked(v) else float(v)

        emit((NODE_PRINCIPLED_VOLUME, self.uchar4(d_off, a_off, ac_off, mix_weight),
              self.uchar4(e_off, ec_off, SVM_STACK_INVALID, SVM_STACK_INVALID), SVM_STACK_INVALID))
        emit((f32bits(const(c.density)), f32bits(const(c.anisotropy)), f32bits(const(p["emission_strength"])),
              f32bits(0.0)))
        emit((ATTR_STD_VOLUME_DENSITY, ATTR_STD_NUM, ATTR_STD_VOLUME_TEMPERATURE, 0))
        for off, w in temps:
            self.free(off, w)
        return out

    def emit_principled(self, c: Closure, mix_weight: int) -> list:
        """nodes.cpp:2839-2925 PrincipledBsdfNode::compile: weight (1,1,1), every
        float input stack-assigned (constants materialised as temporaries,
        released after the node like svm.cpp stack_clear_temporary), the
        closure node, its data node and four parameter nodes."""
        out = []
        emit = out.append
        p = c.params
        nc = self.nc
        emit((NODE_CLOSURE_SET_WEIGHT, f32bits(1.0), f32bits(1.0), f32bits(1.0)))
        temps: list = []

        def vec_if_linked(name):
            v = p.get(name)
            return nc.link(v, "vector") if nodes.is_linked(v) else SVM_STACK_INVALID

        # NodeCompiler.assign emits through self.nc.emit (the shader's code);
        # route it into this closure's code while the inputs are assigned
        saved_emit, nc.emit = nc.emit, emit
        try:
            normal_off = vec_if_linked("normal")
            cc_normal_off = vec_if_linked("clearcoat_normal")
            tangent_off = vec_if_linked("tangent")
            offs = {}
            for name in ("specular", "roughness", "specular_tint", "anisotropic", "sheen", "sheen_tint", "clearcoat",
                         "clearcoat_roughness", "ior", "transmission", "transmission_roughness",
                         "anisotropic_rotation"):
                offs[name] = nc.assign(p[name], "float", temps)
            radius_off = nc.assign(p["subsurface_radius"], "vector", temps)
            metallic_off = nc.assign(p["metallic"], "float", temps)
            subsurface_off = nc.assign(p["subsurface"], "float", temps)
            base_off = nc.link(p["base_color"], "color") if nodes.is_linked(p["base_color"]) else SVM_STACK_INVALID
            ss_off = (nc.link(p["subsurface_color"], "color") if nodes.is_linked(p["subsurface_color"])
                      else SVM_STACK_INVALID)
        finally:
            nc.emit = saved_emit

        def const(v, default):
            return default if nodes.is_linked(v) else v

        emit((NODE_CLOSURE_BSDF, self.uchar4(CLOSURE_BSDF_PRINCIPLED_ID, metallic_off, subsurface_off, mix_weight),
              f32bits(const(p["metallic"], 0.0)), f32bits(const(p["subsurface"], 0.0))))
        emit((normal_off, tangent_off,
              self.uchar4(offs["specular"], offs["roughness"], offs["specular_tint"], offs["anisotropic"]),
              self.uchar4(offs["sheen"], offs["sheen_tint"], offs["clearcoat"], offs["clearcoat_roughness"])))
        emit((self.uchar4(offs["ior"], offs["transmission"], offs["anisotropic_rotation"],
                          offs["transmission_roughness"]),
              PRINCIPLED_DISTRIBUTIONS[c.distribution], PRINCIPLED_SUBSURFACE_METHODS[c.subsurface_method],
              SVM_STACK_INVALID))
        bc = const(p["base_color"], PRINCIPLED_DEFAULTS["base_color"])
        emit((base_off, *(f32bits(x) for x in bc)))
        emit((cc_normal_off, radius_off, SVM_STACK_INVALID, SVM_STACK_INVALID))
        ssc = const(p["subsurface_color"], PRINCIPLED_DEFAULTS["subsurface_color"])
        emit((ss_off, *(f32bits(x) for x in ssc)))
        for off, w in temps:
            self.free(off, w)
        return out

    def emit_principled_hair(self, c: Closure, mix_weight: int) -> list:
        """nodes.cpp:3529-3593 PrincipledHairBsdfNode::compile: weight (1,1,1),
        Color / Tint / Absorption Coefficient stack-assigned (temporaries),
        the other inputs by slot when linked and inline otherwise, the Random
        attribute request when Random is unlinked; the closure node and four
        data nodes."""
        out = []
        emit = out.append
        p = c.params
        nc = self.nc
        emit((NODE_CLOSURE_SET_WEIGHT, f32bits(1.0), f32bits(1.0), f32bits(1.0)))
        temps: list = []
        saved_emit, nc.emit = nc.emit, emit
        try:
            color_off = nc.assign(p["color"], "color", temps)
            tint_off = nc.assign(p["tint"], "color", temps)
            absorption_off = nc.assign(p["absorption_coefficient"], "vector", temps)

            def lk(name, t="float"):
                v = p.get(name)
                return nc.link(v, t) if nodes.is_linked(v) else SVM_STACK_INVALID

            offs = {k: lk(k) for k in ("roughness", "radial_roughness", "offset", "ior", "coat", "melanin",
                                       "melanin_redness", "random", "random_color", "random_roughness")}
            normal_off = lk("normal", "vector")
        finally:
            nc.emit = saved_emit
        attr_random = SVM_STACK_INVALID if nodes.is_linked(p["random"]) else self.attribute(ATTR_STD_CURVE_RANDOM)

        def f(name):
            v = p[name]
            return f32bits(0.0 if nodes.is_linked(v) else float(v))

        emit((NODE_CLOSURE_BSDF,
              self.uchar4(CLOSURE_BSDF_HAIR_PRINCIPLED_ID, offs["roughness"], offs["radial_roughness"], mix_weight),
              f("roughness"), f("radial_roughness")))
        emit((normal_off,
              self.uchar4(offs["offset"], offs["ior"], color_off, PRINCIPLED_HAIR_PARAMETRIZATIONS[c.distribution]),
              f("offset"), f("ior")))
        emit((self.uchar4(offs["coat"], offs["melanin"], offs["melanin_redness"], absorption_off),
              f("coat"), f("melanin"), f("melanin_redness")))
        emit((self.uchar4(tint_off, offs["random"], offs["random_color"], offs["random_roughness"]),
              f("random"), f("random_color"), f("random_roughness")))
        emit((self.uchar4(SVM_STACK_INVALID, SVM_STACK_INVALID, SVM_STACK_INVALID, SVM_STACK_INVALID), attr_random,
              SVM_STACK_INVALID, SVM_STACK_INVALID))
        for off, w in temps:
            self.free(off, w)
        return out

    def compile(self, surfaces: list[Closure], world: Closure) -> np.ndarray:
        """Shader i's code starts with the jump node at index i (svm.cpp
        SVMShaderManager::device_update: shader ids index the jump table).
        Node inputs are compiled ahead of the closure tree so both branches of
        a mix closure see them (svm.cpp generate_multi_closure shared deps)."""
        shaders = list(surfaces) + [world]
        n = len(shaders)
        self.nodes = [(NODE_SHADER_JUMP, 0, 0, 0)] * n
        self.requests = [[] for _ in shaders]
        for i, sh in enumerate(shaders):
            self._shader = i
            self.stack_top = 0
            self.stack_used = [False] * SVM_STACK_SIZE
            start = len(self.nodes)
            self.nodes[i] = (NODE_SHADER_JUMP, start, 0, 0)
            if _has_bump(sh):
                # the bump program (svm.cpp:864-868, compile_type SHADER_TYPE_BUMP:
                # the graph feeding the output's Normal, no NODE_END) falls
                # through into the surface program.  Method "both" (svm.cpp:744-750,
                # 811-813): the graph is finalized with the bump in object space
                # (graph.cpp bump_from_displacement(use_object_space)) and wrapped
                # in NODE_ENTER_BUMP_EVAL / NODE_LEAVE_BUMP_EVAL, which evaluate it
                # at the undisplaced position (SVM_BUMP_EVAL_STATE_SIZE = 9 floats
                # of saved P, dP.dx, dP.dy, reserved first)
                both = _displacement_method(sh) == "both"
                state = self.alloc(SVM_BUMP_EVAL_STATE_SIZE) if both else SVM_STACK_INVALID
                if both:
                    self.nodes.append((NODE_ENTER_BUMP_EVAL, state, 0, 0))
                setn = nodes.bump_from_displacement(sh.displacement, object_space=both)
                self.nc = self._node_compiler([setn], background=False)
                self.nc.link(setn, "vector")
                if both:
                    self.nodes.append((NODE_LEAVE_BUMP_EVAL, state, 0, 0))
                self.stack_top = 0
                self.stack_used = [False] * SVM_STACK_SIZE
            socks = sh.sockets()
            # AOV outputs with a pass (OutputAOVNode::simplify: slot >= 0)
            aovs = [(name, v) for name, v in (getattr(sh, "aovs", None) or {}).items() if name in self.aov_slots]
            self.nc = self._node_compiler([v for v, _ in socks] + [v for _, v in aovs if nodes.is_linked(v)],
                                          background=sh is world)
            for v, t in socks:
                self.nc.link(v, t)
            self.nodes.extend(self.emit_closure(sh, SVM_STACK_INVALID))
            if aovs and sh is not world:
                # svm.cpp:782-806: NODE_AOV_START (the kernel stops here unless
                # the camera path's first hit), then each AOV output's
                # dependencies and its OutputAOVNode::compile
                self.nodes.append((NODE_AOV_START, 0, 0, 0))
                for name, v in aovs:
                    is_color, slot = self.aov_slots[name]
                    off = self.nc.assign(v, "color" if is_color else "float")
                    self.nodes.append((NODE_AOV_COLOR if is_color else NODE_AOV_VALUE, off, slot, 0))
            self.nodes.append((NODE_END, 0, 0, 0))
            vol = getattr(sh, "volume", None)
            vol_start = 0
            if vol is not None:
                # svm.cpp SVMCompiler::compile: the volume program's start in
                # the jump node's z
                vol_start = len(self.nodes)
                self.nodes[i] = (NODE_SHADER_JUMP, start, vol_start, 0)
                self.stack_top = 0
                self.stack_used = [False] * SVM_STACK_SIZE
                vsocks = vol.sockets()
                self.nc = self._node_compiler([v for v, _ in vsocks], background=sh is world, volume=True)
                for v, t in vsocks:
                    self.nc.link(v, t)
                self.nodes.extend(self.emit_closure(vol, SVM_STACK_INVALID))
                self.nodes.append((NODE_END, 0, 0, 0))
            disp = getattr(sh, "displacement", None)
            if nodes.is_linked(disp):
                # svm.cpp SVMCompiler::compile: the displacement program's start
                # in the jump node's w; OutputNode::compile emits
                # NODE_SET_DISPLACEMENT of the "Displacement" input (nodes.cpp)
                self.nodes[i] = (NODE_SHADER_JUMP, start, vol_start, len(self.nodes))
                self.stack_top = 0
                self.stack_used = [False] * SVM_STACK_SIZE
                self.nc = self._node_compiler([disp], background=sh is world)
                off = self.nc.link(disp, "vector")
                self.nodes.append((NODE_SET_DISPLACEMENT, off, 0, 0))
                self.nodes.append((NODE_END, 0, 0, 0))
            if nodes.is_linked(disp) and _displacement_method(sh) == "both":
                # Shader::attributes (shader.cpp:349-350): after the nodes' requests
                self.attribute(ATTR_STD_POSITION_UNDISPLACED)
        self.nc = None
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
    # geometry attributes (render/attribute.h AttributeSet), read by the
    # Attribute, Texture Coordinate (UV, Generated) and Vertex Color nodes:
    uv: np.ndarray | None = None  # (T, 3, 2) per-corner UV map "UVMap" (ATTR_STD_UV)
    # name -> (T, 3, 4) per-corner RGBA in [0, 1], stored as bytes
    # (ATTR_ELEMENT_CORNER_BYTE); the first layer is the active one (ATTR_STD_VERTEX_COLOR)
    vertex_colors: dict | None = None
    # name -> (element, data): element "vertex" (V rows), "face" (T rows) or
    # "corner" (3T rows), data (N,) float, (N, 2) float2 or (N, 3) float3
    attributes: dict | None = None
    # object properties (render/object.h Object: color, pass_id, random_id;
    # Object Info node); unset ones pack as 0
    object_color: tuple | None = None
    pass_index: int = 0
    object_random: float | None = None  # Object::random_id / 0xFFFFFFFF
    # Object::use_holdout (SD_OBJECT_HOLDOUT_MASK, object.cpp:547-548)
    holdout: bool = False
    # Object::is_shadow_catcher (SD_OBJECT_SHADOW_CATCHER, object.cpp:714-719;
    # hidden from the shadow rays of paths behind a catcher,
    # Object::visibility_for_tracing, object.cpp:260-270); meshes drawn once
    shadow_catcher: bool = False
    # the particle this object instances (Object::particle_system /
    # particle_index, object.cpp:440-452; ParticleInfo node): a dict of
    # KernelParticle fields index, age, lifetime, size, rotation (4),
    # location, velocity, angular_velocity (3 each); None: particle 0
    particle: dict | None = None
    # (V, 3) vertex positions before true displacement moved them
    # (Mesh::add_undisplaced, mesh.cpp:535-560, copies the verts before
    # MeshManager::displace runs): ATTR_STD_POSITION_UNDISPLACED, requested by
    # shaders with displacement method "both" (shader.cpp:349-350); None: the
    # verts themselves (nothing displaced them)
    undisplaced: np.ndarray | None = None
    # (3, 4) ATTR_STD_GENERATED_TRANSFORM (element MESH, three float4 rows; the
    # texture space of volume meshes, read by volume_normalized_position for
    # an object-space Point Density node); None: no such attribute
    generated_transform: np.ndarray | None = None


@dataclass
class Hair:
    """A curves object (render/hair.h Hair): Catmull-Rom curves through keys
    (K, 3, world space) with a radius per key; curve c uses keys
    curve_first[c] .. curve_first[c] + curve_nkeys[c] - 1 and has
    curve_nkeys[c] - 1 segments (Hair::Curve::num_segments)."""

    keys: np.ndarray
    radius: np.ndarray
    curve_first: np.ndarray
    curve_nkeys: np.ndarray
    shader: np.ndarray | int = 0  # per curve, or one material index
    # curve attributes (Hair's AttributeSet, blender_curves.cpp ExportCurveSegments):
    # key -> (element, data) with element "curve" (one value per curve) or
    # "curve_key" (one per key), data (N,) float, (N, 2) float2 or (N, 3) float3;
    # key an AttributeStandard id (ATTR_STD_CURVE_INTERCEPT, ATTR_STD_CURVE_RANDOM)
    # or a name.  Absent attributes read 0, as on a host that exports none.
    attributes: dict | None = None
    holdout: bool = False


@dataclass
class Instance:
    """An object placing geometry with a transform (render/object.h).  Geometry
    used by one object has its transform applied on the host; geometry shared
    by several objects keeps object-space vertices and its own BVH, entered
    through an instance leaf of the top-level BVH (render/object.cpp:800-858,
    bvh/bvh.cpp:323-520)."""

    mesh: Mesh
    tfm: np.ndarray  # (3, 4) object to world
    object_color: tuple | None = None  # None: the mesh's
    pass_index: int | None = None
    object_random: float | None = None
    holdout: bool | None = None  # None: the mesh's
    particle: dict | None = None  # None: the mesh's


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
    # Light::samples (KernelLight.samples, light_select_num_samples): light
    # samples per shading point when all lights are sampled (decoupled volumes)
    samples: int = 1
    # the light's shader (Light::shader; None: the shared default emission
    # shader of strength 1, color and strength then go to KernelLight.strength)
    shader: "Closure | None" = None


@dataclass
class Camera:
    """render/camera.cpp sockets (subset): type perspective | orthographic |
    panorama; panorama_type equirectangular | fisheye_equidistant |
    fisheye_equisolid | mirrorball; depth of field (aperture size, blades,
    rotation, ratio, focal distance)."""
    eye: tuple = (0.0, 0.0, -5.0)
    target: tuple = (0.0, 0.0, 0.0)
    up: tuple = (0.0, 1.0, 0.0)
    fov: float = math.radians(40.0)  # full vertical-or-horizontal fov as in Cycles
    nearclip: float = 1e-5
    farclip: float = 1e5
    type: str = "perspective"
    ortho_scale: float = 1.0  # orthographic: the auto viewplane scaled by this (Blender's ortho_scale / 2)
    panorama_type: str = "equirectangular"
    fisheye_fov: float = math.pi
    fisheye_lens: float = 10.5
    sensorwidth: float = 36.0  # mm, in the units of fisheye_lens (Blender sync passes both in mm)
    sensorheight: float = 24.0
    latitude_min: float = -math.pi / 2
    latitude_max: float = math.pi / 2
    longitude_min: float = -math.pi
    longitude_max: float = math.pi
    aperturesize: float = 0.0
    focaldistance: float = 10.0
    blades: int = 0
    bladesrotation: float = 0.0
    aperture_ratio: float = 1.0
    # camera-to-world (4x4, Camera::matrix) instead of eye / target / up
    matrix: np.ndarray | None = None


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
    instances: list = field(default_factory=list)
    caustics_reflective: bool = True
    caustics_refractive: bool = True
    name: str = "scene"
    # world importance sampling (Blender world "Sampling Method"): a background
    # light is added when the world shader varies over directions
    # (light.cpp:210-243 test_enabled_lights); map_resolution 0 = automatic
    world_mis: bool = True
    world_map_resolution: int = 0
    # adaptive sampling (Film use_adaptive_sampling): the adaptive aux buffer and
    # sample count passes after the combined pass (blender_sync.cpp:684-689);
    # threshold / min samples 0 = automatic (integrator.cpp:186-207)
    adaptive_sampling: bool = False
    adaptive_threshold: float = 0.0
    adaptive_min_samples: int = 0
    # hair (SceneParams hair_shape / hair_subdivisions, render/scene.h:173-210):
    # curves render as "ribbon" or "thick"; curve_subdivisions = 1 << hair_subdivisions
    hairs: list = field(default_factory=list)
    hair_shape: str = "ribbon"
    hair_subdivisions: int = 3
    # world "Volume" output (a volume closure tree, e.g. a homogeneous fog)
    world_volume: "Closure | None" = None
    # Film exposure (film.cpp:363; applied by film convert)
    exposure: float = 1.0
    # decoupled volume ray marching (the CPU device's KernelIntegrator, see
    # compile_scene); False: distance sampling as GPU devices integrate
    volume_decoupled: bool = False
    # Integrator "Sampling" method (integrator.cpp:83, KernelIntegrator.branched):
    # "path" or "branched_path", with the branched sample counts per closure
    # kind and the all-lights switches (integrator.cpp:164-181; Blender's
    # defaults)
    integrator: str = "path"
    diffuse_samples: int = 1
    glossy_samples: int = 1
    transmission_samples: int = 1
    mesh_light_samples: int = 1
    sample_all_lights_direct: bool = True
    sample_all_lights_indirect: bool = True
    # AOV passes of the view layer (BlenderSync::sync_render_passes,
    # Pass::add(PASS_AOV_COLOR / PASS_AOV_VALUE, name)): (name, "color" | "value")
    aovs: list = field(default_factory=list)
    # data and light passes of the view layer (film.cpp pass_type_enum names):
    # any of "depth", "normal", "uv", "object_id", "material_id" and the light
    # passes "mist", "emission", "background", "shadow", "diffuse_direct",
    # "diffuse_indirect", "diffuse_color" (and glossy_*, transmission_*),
    # "volume_direct", "volume_indirect"
    passes: list = field(default_factory=list)
    # mist pass (Film mist_start / mist_depth / mist_falloff, film.cpp:374-376)
    mist_start: float = 0.0
    mist_depth: float = 100.0
    mist_falloff: float = 1.0
    # Film "Transparent" (Background::transparent, background.cpp:112): camera
    # rays that leave the scene, and holdouts, make the pixel transparent
    # (alpha = 1 - L_transparent) instead of showing the world
    film_transparent: bool = False


def _has_displacement(m) -> bool:
    return nodes.is_linked(getattr(m, "displacement", None))


def _displacement_method(m) -> str:
    method = getattr(m, "displacement_method", "true")
    if method not in ("true", "bump", "both"):
        raise ValueError(f"displacement_method {method!r}: true, bump or both")
    return method


def _has_bump(m) -> bool:
    """svm.cpp:836-837 has_bump: displacement method "bump" or "both" with both
    the surface and the displacement outputs linked."""
    return (m is not None and _has_displacement(m) and _displacement_method(m) != "true"
            and m.kind not in ("none", "background"))


def _has_bssrdf_bump(m) -> bool:
    """Shader::has_bssrdf_bump (svm.cpp:515-521, 855): a BSSRDF node whose
    Normal input is linked to anything but the Geometry node
    (SubsurfaceScatteringNode / PrincipledBsdfNode::has_bssrdf_bump,
    nodes.cpp:2960-2963, 3069-3075).  Bump displacement (the other source) is
    not expressible here: displacement is always the "true" method."""
    if m is None:
        return False
    if _has_bump(m):
        return True  # svm.cpp:855 has_bssrdf_bump = has_bump

    def bumped(v):
        return nodes.is_linked(v) and v.node.kind != "geometry"

    if m.kind == "mix":
        return _has_bssrdf_bump(m.a) or _has_bssrdf_bump(m.b)
    if m.kind == "subsurface":
        return bumped(m.normal)
    if m.kind == "principled":
        sss = m.params["subsurface"]
        has_sss = nodes.is_linked(sss) or float(sss) > 1e-5  # has_surface_bssrdf, CLOSURE_WEIGHT_CUTOFF
        return has_sss and bumped(m.params.get("normal"))
    return False


@dataclass
class DeviceScene:
    data: abi.KernelData
    arrays: dict
    width: int
    height: int
    samples: int
    info: dict = field(default_factory=dict)
    # SVM image slots (ImageManager): slot i holds textures[i] (nodes.Image)
    textures: list = field(default_factory=list)

    @property
    def pass_stride(self) -> int:
        return self.data.film.pass_stride

    def texture_info(self) -> tuple[np.ndarray, list]:
        """__texture_info for a host consumer (the reference CPU kernel, the
        host emulator): util_texture.h TextureInfo records (96 bytes) whose
        `data` are host addresses of the texel arrays; returns the array and
        the texel arrays, which must stay alive while it is bound."""
        info = np.zeros((len(self.textures), 24), dtype=np.uint32)
        keep = []
        for i, im in enumerate(self.textures):
            a = im.texel_array()
            keep.append(a)
            info[i, 0:2] = np.array([a.ctypes.data], dtype=np.uint64).view(np.uint32)
            info[i, 2] = _nodes.IMAGE_DATA_TYPES.index(im.data_type)
            info[i, 4] = _nodes.INTERPOLATIONS.index(im.interpolation)
            info[i, 5] = _nodes.EXTENSIONS.index(im.extension)
            info[i, 6], info[i, 7], info[i, 8] = im.dims()
            if im.transform_3d is not None:
                info[i, 9] = 1  # use_transform_3d; transform_3d at byte 48
                info[i, 12:24] = np.asarray(im.transform_3d, dtype=np.float32).reshape(12).view(np.uint32)
        return info.view(np.uint8).reshape(-1), keep


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


def _viewplane(width, height, cam=None):
    """Camera::compute_auto_viewplane (sensor fit AUTO; panorama: unit square)."""
    if cam is not None and cam.type == "panorama":
        return (0.0, 1.0, 0.0, 1.0)
    aspect = width / height
    s = cam.ortho_scale if cam is not None and cam.type == "orthographic" else 1.0
    if width >= height:
        return (-aspect * s, aspect * s, -1.0 * s, 1.0 * s)
    return (-1.0 * s, 1.0 * s, -1.0 / aspect * s, 1.0 / aspect * s)


def _from_viewplane(vp):
    l, r, b, t = vp
    s = np.diag([1.0 / (r - l), 1.0 / (t - b), 1.0, 1.0])
    tr = np.eye(4)
    tr[0, 3] = -l
    tr[1, 3] = -b
    return s @ tr


def _orthographic(n, f):
    """util_projection.h:204-210 projection_orthographic."""
    m = np.eye(4)
    m[2, 2] = 1.0 / (f - n)
    m[2, 3] = -n / (f - n)
    return m


def _perspective(fov, n, f):
    persp = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, f / (f - n), -f * n / (f - n)], [0, 0, 1, 0]], dtype=np.float64)
    inv_angle = 1.0 / math.tan(0.5 * fov)
    return np.diag([inv_angle, inv_angle, 1.0, 1.0]) @ persp


PANORAMA_TYPES = {"equirectangular": 0, "fisheye_equidistant": 1, "fisheye_equisolid": 2, "mirrorball": 3}
CAMERA_TYPES = {"perspective": 0, "orthographic": 1, "panorama": 2}


def compile_camera(kcam, cam: Camera, width: int, height: int):
    """Camera::update + Camera::device_update (render/camera.cpp:220-440)."""
    screentondc = _from_viewplane(_viewplane(width, height, cam))
    ndctoraster = np.diag([width, height, 1.0, 1.0])
    screentoraster = ndctoraster @ screentondc
    rastertoscreen = np.linalg.inv(screentoraster)
    if cam.type == "perspective":
        cameratoscreen = _perspective(cam.fov, cam.nearclip, cam.farclip)
    elif cam.type == "orthographic":
        cameratoscreen = _orthographic(cam.nearclip, cam.farclip)
    else:
        cameratoscreen = np.eye(4)
    screentocamera = np.linalg.inv(cameratoscreen)
    rastertocamera = screentocamera @ rastertoscreen
    if cam.matrix is not None:
        cameratoworld = np.eye(4)
        cameratoworld[:3] = np.asarray(cam.matrix, dtype=np.float64)[:3]
    else:
        cameratoworld = _look_at(cam.eye, cam.target, cam.up)
    worldtocamera = np.linalg.inv(cameratoworld)

    def persp(m, v):
        p = m @ np.array([v[0], v[1], v[2], 1.0])
        return p[:3] / p[3]

    if cam.type == "perspective":
        dx = persp(rastertocamera, (1, 0, 0)) - persp(rastertocamera, (0, 0, 0))
        dy = persp(rastertocamera, (0, 1, 0)) - persp(rastertocamera, (0, 0, 0))
    elif cam.type == "orthographic":
        dx = rastertocamera[:3, :3] @ np.array([1.0, 0.0, 0.0])
        dy = rastertocamera[:3, :3] @ np.array([0.0, 1.0, 0.0])
    else:
        dx = np.zeros(3)
        dy = np.zeros(3)
    dx = cameratoworld[:3, :3] @ dx
    dy = cameratoworld[:3, :3] @ dy

    kcam.type = CAMERA_TYPES[cam.type]
    kcam.panorama_type = PANORAMA_TYPES[cam.panorama_type]
    if cam.type == "panorama":
        # (left zero for the other types, which never read them)
        kcam.fisheye_fov = cam.fisheye_fov
        kcam.fisheye_lens = cam.fisheye_lens
        er = kcam.equirectangular_range
        f32 = np.float32
        er.x = float(f32(cam.longitude_min) - f32(cam.longitude_max))
        er.y = float(-f32(cam.longitude_min))
        er.z = float(f32(cam.latitude_min) - f32(cam.latitude_max))
        er.w = float(-f32(cam.latitude_min) + f32(math.pi / 2))
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
    kcam.aperturesize = cam.aperturesize
    kcam.blades = 0.0 if cam.blades < 3 else float(cam.blades)
    kcam.bladesrotation = cam.bladesrotation
    kcam.focaldistance = cam.focaldistance
    kcam.shuttertime = -1.0
    kcam.num_motion_steps = 0
    kcam.have_perspective_motion = 0
    kcam.nearclip = cam.nearclip
    kcam.cliplength = cam.farclip - cam.nearclip
    kcam.sensorwidth = cam.sensorwidth
    kcam.sensorheight = cam.sensorheight
    kcam.width = float(width)
    kcam.height = float(height)
    kcam.resolution = 1
    kcam.inv_aperture_ratio = 1.0 / cam.aperture_ratio
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

    # --- geometry (render/geometry.cpp device_update_mesh + mesh.cpp pack_*,
    # object.cpp apply_static_transforms, bvh/bvh.cpp pack_primitives /
    # pack_instances)
    g = _pack_geometry(scene)
    ntri = g["ntri"]
    tri_shader_idx = g["tri_shader_idx"]
    tri_smooth = g["tri_smooth"]
    nodes, leaves, root = g["nodes"], g["leaves"], g["root"]
    prim_index, prim_object, prim_type = g["prim_index"], g["prim_object"], g["prim_type"]
    prim_visibility, prim_tri_index, prim_tri_verts = g["prim_visibility"], g["prim_tri_index"], g["prim_tri_verts"]
    tri_vindex, tri_vnormal = g["tri_vindex"], g["tri_vnormal"]
    objects = g["objects"]

    # --- shaders (render/shader.cpp:462-475, 508-581 + svm.cpp); lamps share
    # one emission shader (the default light shader: emission 1.0), their
    # color and power go to KernelLight.strength
    mats = list(scene.materials)
    lamp_shader = None
    lamp_shaders = []  # per lamp: its shader index
    for lamp in scene.lamps:
        if lamp.shader is None:
            if lamp_shader is None:
                lamp_shader = len(mats)
                mats.append(Closure("emission", (1.0, 1.0, 1.0), strength=1.0))
            lamp_shaders.append(lamp_shader)
        else:
            ids = [i for i, m in enumerate(mats) if m is lamp.shader]
            if not ids:
                mats.append(lamp.shader)
                ids = [len(mats) - 1]
            lamp_shaders.append(ids[0])
    world = background(scene.world_color, scene.world_strength)
    world.volume = scene.world_volume
    svm_compiler = SVMCompiler()
    n_color = n_value = 0
    for name, kind in scene.aovs:
        if kind not in ("color", "value"):
            raise ValueError(f"AOV {name!r}: kind must be color or value")
        if name in svm_compiler.aov_slots:
            continue  # Pass::add: one pass per name and type
        svm_compiler.aov_slots[name] = (kind == "color", n_color if kind == "color" else n_value)
        n_color += kind == "color"
        n_value += kind == "value"
    svm = svm_compiler.compile(mats, world)
    n_shaders = len(mats) + 1
    kshaders = (abi.KernelShader * n_shaders)()
    any_transparent_shadow = False
    for i, m in enumerate(mats + [world]):
        flag = SD_USE_MIS
        if m.has_transparent():  # shader.cpp:527 (use_transparent_shadow defaults to true)
            flag |= SD_HAS_TRANSPARENT_SHADOW
            any_transparent_shadow = True
        const = m.constant_emission()
        if const is not None:
            flag |= SD_HAS_CONSTANT_EMISSION
            kshaders[i].constant_emission[:] = [float(c) for c in const]
        if _has_displacement(m) and _displacement_method(m) != "bump":
            flag |= SD_HAS_DISPLACEMENT  # shader.cpp:559-560 (displacement_method true)
        if _has_bump(m):
            flag |= SD_HAS_BUMP  # shader.cpp:557-558
        if _has_bssrdf_bump(m):
            flag |= SD_HAS_BSSRDF_BUMP  # shader.cpp:547-548
        if m.volume is not None:
            # shader.cpp:529-553: a volume shader has transparent shadows; one
            # without a surface only bounds its volume; heterogeneous_volume
            # (default true) with spatially varying inputs steps the volume
            flag |= SD_HAS_VOLUME | SD_HAS_TRANSPARENT_SHADOW
            any_transparent_shadow = True
            if m.kind == "none":
                flag |= SD_HAS_ONLY_VOLUME
            vsocks = [v for v, _ in m.volume.sockets()]
            if _nodes.has_spatial_varying(vsocks):
                flag |= SD_HETEROGENEOUS_VOLUME
            if _volume_attribute_dependency(m.volume):
                flag |= SD_NEED_VOLUME_ATTRIBUTES
            # shader.cpp:541-544 Shader::volume_sampling_method (Blender's
            # default is multiple importance; "distance" here unless asked)
            vs = getattr(m, "volume_sampling", "distance")
            if vs == "equiangular":
                flag |= SD_VOLUME_EQUIANGULAR
            elif vs == "multiple_importance":
                flag |= SD_VOLUME_MIS
            elif vs != "distance":
                raise ValueError(f"volume_sampling {vs!r}: distance, equiangular or multiple_importance")
        kshaders[i].flags = flag
        kshaders[i].pass_id = int(getattr(m, "pass_index", 0))
    tri_shader = tri_shader_idx.astype(np.uint32) | np.uint32(SHADER_CAST_SHADOW | SHADER_AREA_LIGHT)
    tri_shader = np.where(tri_smooth, tri_shader | np.uint32(SHADER_SMOOTH_NORMAL), tri_shader).astype(np.uint32)

    # --- objects (render/object.cpp:463-544 device_update_object_transform)
    nobj = len(objects)
    kobjects = (abi.KernelObject * max(nobj, 1))()
    object_flag = np.zeros(max(nobj, 1), dtype=np.uint32)
    object_node = np.zeros(max(nobj, 1), dtype=np.uint32)
    for i, ob in enumerate(objects):
        tfm = ob["tfm"]
        abi.set_transform(kobjects[i].tfm, tfm)
        abi.set_transform(kobjects[i].itfm, np.linalg.inv(np.vstack([tfm, [0, 0, 0, 1]]))[:3])
        kobjects[i].shadow_terminator_offset = 1.0  # 1 / (1 - 0.5 * 0)
        # object.cpp:454-461: color, pass_id, random_number
        if ob.get("color") is not None:
            kobjects[i].color[:] = [float(c) for c in ob["color"]]
        kobjects[i].pass_id = float(ob.get("pass_index") or 0)
        if ob.get("random") is not None:
            kobjects[i].random_number = float(ob["random"])
        kobjects[i].numverts = ob["numverts"]
        kobjects[i].numkeys = ob.get("numkeys", 0)
        if ob["applied"]:
            object_flag[i] = SD_OBJECT_TRANSFORM_APPLIED
        if ob.get("holdout"):
            object_flag[i] |= SD_OBJECT_HOLDOUT_MASK
        if ob.get("shadow_catcher"):
            object_flag[i] |= SD_OBJECT_SHADOW_CATCHER
        object_node[i] = np.uint32(ob["node"] & 0xFFFFFFFF)
    # particles (object.cpp:440-452, particles.cpp:57-103 device_update_particles):
    # entry 0 is the dummy every object without a particle reads; the
    # instancing objects' particles follow in object order
    kparticles = [None]
    for i, ob in enumerate(objects):
        if ob.get("particle") is not None:
            kobjects[i].particle_index = len(kparticles)
            kparticles.append(ob["particle"])

    # --- volume objects (object.cpp:678-736 device_update_flags,
    # object.cpp:270-349 compute_volume_step_size, :378-389 volume density)
    use_volumes = any(m.volume is not None for m in mats) or world.volume is not None
    object_volume_step = np.full(max(nobj, 1), FLT_MAX, dtype=np.float32)
    vol_bounds = []
    for i, ob in enumerate(objects):
        used = _object_shaders(ob, tri_shader_idx)
        vmats = [mats[k] for k in used if mats[k].volume is not None]
        if not vmats:
            continue
        object_flag[i] |= SD_OBJECT_HAS_VOLUME
        kobjects[i].surface_area = 1.0
        lo, hi = _object_bounds(ob, g)
        vol_bounds.append((i, lo, hi))
        step_rate = FLT_MAX
        for m in vmats:
            if _nodes.has_spatial_varying([v for v, _ in m.volume.sockets()]) or \
                    _volume_attribute_dependency(m.volume):
                step_rate = min(step_rate, 1.0)  # Shader::volume_step_rate default
        if step_rate != FLT_MAX:
            size = (hi - lo).astype(np.float32)
            avg = np.float32(np.float32(np.float32(size[0] + size[1]) + size[2]) * np.float32(1.0 / 3.0))
            object_volume_step[i] = np.float32(np.float32(0.1) * avg) * np.float32(step_rate)
    for i, ob in enumerate(objects):
        lo, hi = _object_bounds(ob, g)
        for j, vlo, vhi in vol_bounds:
            if j != i and np.all(lo <= vhi) and np.all(vlo <= hi):
                object_flag[i] |= SD_OBJECT_INTERSECTS_VOLUME
                break

    # --- geometry attributes (geometry.cpp:379-474 device_update_attributes
    # + :508-620 update_attribute_element_offset)
    attr_arrays = None
    # Scene::need_global_attribute (scene.cpp:341-351): a UV pass requests the
    # UV map of every geometry, after its shaders' requests
    global_reqs = [_nodes.ATTR_STD_UV] if "uv" in scene.passes else []
    if any(svm_compiler.requests) or global_reqs:
        attr_arrays = _pack_attributes(g, objects, tri_shader_idx, svm_compiler, kobjects, global_reqs)

    # --- lights (render/light.cpp:277-480, mesh lights only)
    # light.cpp:330-400: per object using emissive triangles, in object order,
    # world-space area (transform_point for instanced geometry)
    emissive = np.array([m.has_emission() for m in mats], dtype=bool)
    light_list = []
    for oi, ob in enumerate(objects):
        tris_g = np.arange(ob["tri_offset"], ob["tri_offset"] + ob["ntri"])
        for ti in tris_g[emissive[tri_shader_idx[tris_g]]]:
            light_list.append((oi, int(ti)))
    dist = (abi.KernelLightDistribution * (len(light_list) + 1))()
    totarea = f32(0.0)
    for k, (oi, ti) in enumerate(light_list):
        dist[k].totarea = float(totarea)
        dist[k].prim = ti
        dist[k].shader_flag = 0
        dist[k].object_id = oi
        p1, p2, p3 = g["tri_pos_object"][ti]
        if not objects[oi]["applied"]:
            p1, p2, p3 = (transform_point_f32(objects[oi]["tfm"], p) for p in (p1, p2, p3))
        totarea = f32(totarea + triangle_area_f32(p1, p2, p3))
    nd = len(light_list)
    trianglearea = totarea
    lamps = list(scene.lamps)
    # background light (blender_light.cpp:162-210 sync_background_light, appended
    # after the lamps), enabled only for a spatially varying world
    bg_light = scene.world_mis and _nodes.has_spatial_varying([v for v, _ in world.sockets()])
    num_lights = len(lamps) + int(bg_light)
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
        use_lamp_mis |= _pack_lamp(klights[li], lamp, lamp_shaders[li])
    if bg_light:
        li = len(lamps)
        e = dist[nd + li]
        e.totarea = float(totarea)
        e.prim = ~li
        e.shader_flag = f32bits_signed(1.0)  # lamp.pad
        e.object_id = f32bits_signed(0.0)  # lamp.size of the background light
        totarea = f32(totarea + lightarea)
        _pack_background_light(klights[li], n_shaders - 1)
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
    ki.transparent_shadows = int(any_transparent_shadow)  # shader.cpp:603
    ki.volume_max_steps = 1024
    ki.volume_step_rate = 1.0
    ki.caustics_reflective = int(scene.caustics_reflective)
    ki.caustics_refractive = int(scene.caustics_refractive)
    ki.filter_glossy = FLT_MAX if scene.filter_glossy == 0.0 else 1.0 / scene.filter_glossy
    ki.seed = native.hash_uint2(scene.seed, 0)
    ki.use_ambient_occlusion = 0
    ki.sample_clamp_direct = FLT_MAX
    ki.sample_clamp_indirect = FLT_MAX
    branched = scene.integrator == "branched_path"
    ki.branched = int(branched)
    # DeviceInfo::has_volume_decoupled (integrator.cpp:165): the CPU device's
    # decoupled ray marching, with the Integrator's "sample all lights"
    # defaults (true) that choose it for every volume segment
    # (kernel_volume_use_decoupled); GPU devices upload 0
    ki.volume_decoupled = int(scene.volume_decoupled)
    ki.diffuse_samples = scene.diffuse_samples
    ki.glossy_samples = scene.glossy_samples
    ki.transmission_samples = scene.transmission_samples
    ki.ao_samples = ki.subsurface_samples = ki.volume_samples = 1
    ki.mesh_light_samples = scene.mesh_light_samples
    ki.start_sample = 0
    if branched:
        ki.sample_all_lights_direct = int(scene.sample_all_lights_direct)
        ki.sample_all_lights_indirect = int(scene.sample_all_lights_indirect)
    else:
        # the decoupled volume cases keep the switches on, the setting under
        # which kernel_volume_use_decoupled takes every segment
        ki.sample_all_lights_direct = int(scene.volume_decoupled)
        ki.sample_all_lights_indirect = int(scene.volume_decoupled)
    ki.sampling_pattern = 0
    ki.aa_samples = scene.samples
    if scene.adaptive_min_samples == 0:
        ki.adaptive_min_samples = max(4, int(math.sqrt(scene.samples)))
    else:
        ki.adaptive_min_samples = max(4, scene.adaptive_min_samples)
    ki.adaptive_step = 4
    # GPU devices: info.has_adaptive_stop_per_sample = false (stopping runs per
    # step in its own kernel, CUDADevice::adaptive_sampling_filter)
    ki.adaptive_stop_per_sample = 0
    if scene.adaptive_threshold == 0.0:
        ki.adaptive_threshold = max(0.001, 1.0 / scene.samples)
    else:
        ki.adaptive_threshold = scene.adaptive_threshold
    ki.light_inv_rr_threshold = (1.0 / scene.light_sampling_threshold) if scene.light_sampling_threshold > 0 else 0.0
    ki.use_volumes = int(use_volumes)  # shader.cpp:601
    ki.max_closures = max([m.material_closures() for m in mats + [world]] + [1])
    # integrator.cpp:218-234: branched path tracing sizes the table for its
    # largest sample count
    max_samples = 1
    if branched:
        max_samples = max([max_samples] + [lamp.samples for lamp in scene.lamps])
        max_samples = max(max_samples, scene.diffuse_samples, scene.glossy_samples, scene.transmission_samples)
        max_samples = max(max_samples, ki.ao_samples, scene.mesh_light_samples, ki.subsurface_samples,
                          ki.volume_samples)
    total_bounces = scene.max_bounce + scene.transparent_max_bounce + 3 + VOLUME_BOUNDS_MAX + BSSRDF_MAX_BOUNCES
    dims = min(PRNG_BASE_NUM + max_samples * total_bounces * PRNG_BOUNCE_NUM, sobol.SOBOL_MAX_DIMENSIONS)
    lut = sobol.sample_pattern_lut(dims)

    # --- background (render/background.cpp:63-118)
    kb = kd.background
    kb.surface_shader = n_shaders - 1
    # background.cpp:92-97: the world's volume (get_shader_id: default flags)
    kb.volume_shader = ((n_shaders - 1) | SHADER_CAST_SHADOW | SHADER_AREA_LIGHT) if world.volume is not None else -1
    if kb.volume_shader != -1:
        kb.volume_shader = kb.volume_shader - (1 << 32) if kb.volume_shader >= (1 << 31) else kb.volume_shader
    if use_volumes:
        # volume_step_size * volume_step_rate (the reference writes it for every
        # scene; it is read only through a world volume, so scenes without
        # volumes keep 0 and their golden digests)
        kb.volume_step_size = float(np.float32(0.1) * np.float32(1.0))
    kb.transparent = 1 if scene.film_transparent else 0
    kb.transparent_roughness_squared_threshold = -1.0
    kb.ao_factor = 0.0
    kb.ao_bounces_factor = 0.0
    kb.ao_distance = FLT_MAX
    kb.use_mis = 0
    kb.portal_weight = 0.0
    kb.sun_weight = 0.0
    kb.map_weight = 0.0
    bg_map = None
    if bg_light and ki.use_direct_light:
        # light.cpp:509 map_weight (light->use_mis = sample_as_light) and
        # device_update_background (light.cpp:568-716): no environment texture or
        # sky sun -> automatic resolution 4096 x 2048
        kb.map_weight = 1.0
        kb.use_mis = 1
        res_x = scene.world_map_resolution or 4096
        res_y = res_x // 2 if scene.world_map_resolution else 2048
        kb.map_res_x, kb.map_res_y = res_x, res_y
        bg_map = (res_x, res_y)

    # --- film (render/film.cpp device_update, combined pass only)
    kf = kd.film
    kf.exposure = float(scene.exposure)
    kf.pass_flag = PASSMASK_COMBINED
    kf.light_pass_flag = 0
    kf.pass_stride = 4
    kf.use_light_pass = 0
    kf.pass_combined = 0
    kf.pass_alpha_threshold = 0.5
    kf.filter_table_offset = 0
    # shader.cpp:387 ColorSpaceManager defaults (no OCIO): Rec.709 luminance
    kf.rgb_to_y.x, kf.rgb_to_y.y, kf.rgb_to_y.z = 0.2126729, 0.7151522, 0.0721750
    if "xyz_to_rgb" in svm_compiler.features:
        # shader.cpp:384-386 (and :608-610): the XYZ -> linear Rec.709 rows.  The
        # reference host always uploads them; they are set here only for scenes
        # whose nodes read them (sky texture), which keeps the KernelData bytes
        # of every other golden case unchanged.
        kf.xyz_to_r.x, kf.xyz_to_r.y, kf.xyz_to_r.z = 3.2404542, -1.5371385, -0.4985314
        kf.xyz_to_g.x, kf.xyz_to_g.y, kf.xyz_to_g.z = -0.9692660, 1.8760108, 0.0415560
        kf.xyz_to_b.x, kf.xyz_to_b.y, kf.xyz_to_b.z = 0.0556434, -0.2040259, 1.0572252
    # display pass = combined (film.cpp:392, 419-423, 591-598)
    kf.display_pass_stride = 0
    kf.display_pass_components = 4
    kf.display_divide_pass_stride = -1
    kf.use_display_exposure = 1 if kf.exposure != 1.0 else 0
    kf.use_display_pass_alpha = 1
    # Film::device_update (film.cpp:425-625): the passes in the order
    # BlenderSync::sync_render_passes adds them (combined, the AOVs, the
    # adaptive sampling passes), stable-sorted by component count (Pass::add,
    # film.cpp:263-266: 4-float passes first), offsets in that order, the
    # stride aligned to 4 floats; pass_flag |= 1 << type.  PassType numbers
    # (kernel_types.h:354-376 without __KERNEL_DEBUG__): AOV_COLOR 11,
    # AOV_VALUE 12, ADAPTIVE_AUX_BUFFER 13, SAMPLE_COUNT 14.
    passes = [("combined", 1, 4)]
    # data passes (PassType DEPTH 2 .. MATERIAL_ID 6; components film.cpp:148-170:
    # normal and UV take 4 floats, the kernel adds 3)
    data_pass_types = {"depth": (2, 1), "normal": (3, 4), "uv": (4, 4), "object_id": (5, 1), "material_id": (6, 1)}
    # light passes (PassType MIST 32 .. VOLUME_INDIRECT 51, film.cpp:152-236)
    light_pass_types = {"mist": (32, 1), "emission": (33, 4), "background": (34, 4), "shadow": (36, 4),
                        "diffuse_direct": (38, 4), "diffuse_indirect": (39, 4), "diffuse_color": (40, 4),
                        "glossy_direct": (41, 4), "glossy_indirect": (42, 4), "glossy_color": (43, 4),
                        "transmission_direct": (44, 4), "transmission_indirect": (45, 4),
                        "transmission_color": (46, 4), "volume_direct": (50, 4), "volume_indirect": (51, 4)}
    all_types = {**data_pass_types, **light_pass_types}
    for name in set(scene.passes):
        if name not in all_types:
            raise ValueError(f"pass {name!r}: one of {sorted(all_types)}")
    for name in sorted(set(scene.passes), key=lambda n: all_types[n][0]):
        passes.append((name, *all_types[name]))
    seen = set()
    for name, kind in scene.aovs:
        if name not in seen:
            seen.add(name)
            passes.append(("aov_color", 11, 4) if kind == "color" else ("aov_value", 12, 1))
    if scene.adaptive_sampling:
        passes += [("adaptive_aux_buffer", 13, 4), ("sample_count", 14, 1)]
    passes.sort(key=lambda p: -p[2])  # stable
    stride = 0
    kf.pass_flag = 0
    kf.pass_aov_color_num = kf.pass_aov_value_num = 0
    for kind, ptype, comps in passes:
        # film.cpp:448-455: main passes in pass_flag, light passes in
        # light_pass_flag (and use_light_pass)
        if ptype <= 31:
            kf.pass_flag |= 1 << ptype
        else:
            kf.use_light_pass = 1
            kf.light_pass_flag |= 1 << (ptype % 32)
        if kind in ("diffuse_color", "glossy_color", "transmission_color"):
            kf.display_divide_pass_stride = stride  # film.cpp:596-599
        if kind == "combined":
            kf.pass_combined = stride
        elif kind == "aov_color":
            if kf.pass_aov_color_num == 0:
                kf.pass_aov_color = stride
            kf.pass_aov_color_num += 1
        elif kind == "aov_value":
            if kf.pass_aov_value_num == 0:
                kf.pass_aov_value = stride
            kf.pass_aov_value_num += 1
        elif kind in all_types:
            setattr(kf, "pass_" + kind, stride)
        elif kind == "adaptive_aux_buffer":
            kf.pass_adaptive_aux_buffer = stride
        else:
            kf.pass_sample_count = stride
        stride += comps
    kf.pass_stride = -(-stride // 4) * 4
    if kf.use_light_pass:
        # film.cpp:641-644 mist parameters
        kf.mist_start = float(f32(scene.mist_start))
        kf.mist_inv_depth = float(f32(1.0) / f32(scene.mist_depth)) if scene.mist_depth > 0 else 0.0
        kf.mist_falloff = float(f32(scene.mist_falloff))
        # light.cpp:483-491: the shadow pass scale compensates for emitting
        # triangles and background lights taking light samples
        kf.pass_shadow_scale = 0.0
        if ki.use_direct_light:
            scale = f32(1.0)
            if ki.pdf_triangles != 0.0:
                scale = f32(scale * f32(0.5))
            n_bg = int(bg_light)
            if n_bg < num_lights:
                scale = f32(scale * f32(f32(num_lights - n_bg) / f32(num_lights)))
            kf.pass_shadow_scale = float(scale)
    lookup = filter_table(scene.filter_type, scene.filter_width)
    kd.tables.beckmann_offset = 0
    if any(t in BECKMANN_CLOSURES for m in mats for t in m.closure_types()):
        # ShaderManager::device_update_common adds the Beckmann sampling table
        # (render/shader.cpp:52-135) through LookupTables::add_table, which
        # places tables at TABLE_CHUNK_SIZE (256) aligned offsets
        # (render/tables.cpp:67-103).  Only scenes that sample Beckmann
        # closures carry it here.
        lib = native.host_lib()
        n = lib.cyh_beckmann_table_size()
        table = np.zeros(n * n, dtype=np.float32)
        lib.cyh_beckmann_table(table.ctypes.data)
        offset = -(-len(lookup) // 256) * 256
        lookup = np.concatenate([lookup, np.zeros(offset - len(lookup), dtype=np.float32), table])
        kd.tables.beckmann_offset = offset

    # --- camera
    compile_camera(kd.cam, scene.camera, scene.width, scene.height)
    # camera.cpp:495-527 device_update_volume: a volume object whose bounds
    # hold the view plane (at the near clip: the eye) puts the camera inside
    kd.cam.is_inside_volume = 0
    if use_volumes:
        eye = np.asarray(scene.camera.eye, dtype=np.float32)
        for _, vlo, vhi in vol_bounds:
            if np.all(eye >= vlo - 1e-3) and np.all(eye <= vhi + 1e-3):
                kd.cam.is_inside_volume = 1

    # --- bvh
    kd.bvh.root = root
    kd.bvh.have_motion = 0
    kd.bvh.have_curves = int(g["ncurves"] > 0)  # object.cpp:553-628
    kd.bvh.bvh_layout = BVH_LAYOUT_BVH2
    kd.bvh.use_bvh_steps = 0
    # geometry.cpp:1096 scene->params.curve_subdivisions() (Embree's tessellation
    # limit); scenes without curves keep the value this builder always wrote
    kd.bvh.curve_subdivisions = min(max(1 << scene.hair_subdivisions, 1), 16) if g["ncurves"] else 4

    arrays = {
        "__bvh_nodes": nodes.astype(np.float32),
        "__bvh_leaf_nodes": leaves.astype(np.float32),
        "__prim_tri_verts": prim_tri_verts,
        "__prim_tri_index": prim_tri_index,
        "__prim_type": prim_type,
        "__prim_visibility": prim_visibility,
        "__prim_index": prim_index,
        "__prim_object": prim_object,
        "__object_node": object_node,
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
    if svm_compiler.ies_slots:
        # LightManager::device_update_ies (light.cpp:1080-1125)
        from .ies import pack_slots

        arrays["__ies"] = pack_slots(svm_compiler.ies_slots)
    if use_volumes:
        arrays["__object_volume_step"] = object_volume_step
        # geometry.cpp device_update_attributes: no attributes are packed, every
        # object's map is the ATTR_STD_NONE terminator (ATTR_PRIM_TYPES rows)
        arrays["__attributes_map"] = np.zeros((2, 4), dtype=np.uint32)
    if attr_arrays is not None:
        arrays.update(attr_arrays)
    if len(kparticles) > 1:
        arrays["__particles"] = _pack_particles(kparticles)
    if g["ncurves"]:
        # Hair::pack_curves (render/hair.cpp): keys with radius, per curve the
        # first key, key count and shader id (get_shader_id(shader, false))
        curves = np.zeros((g["ncurves"], 4), dtype=np.uint32)
        curves[:, 0] = g["curve_first"]
        curves[:, 1] = g["curve_nkeys"]
        curves[:, 2] = g["curve_shader"].astype(np.uint32) | np.uint32(SHADER_CAST_SHADOW | SHADER_AREA_LIGHT)
        arrays["__curves"] = curves.view(np.float32)
        arrays["__curve_keys"] = g["curve_keys"]
    if bg_map is not None:
        # filled at upload from the device's SHADER task (device.py upload_scene,
        # LightManager::device_update_background)
        arrays["__light_background_marginal_cdf"] = np.zeros((bg_map[1] + 1, 2), dtype=np.float32)
        arrays["__light_background_conditional_cdf"] = np.zeros(((bg_map[0] + 1) * bg_map[1], 2),
                                                                dtype=np.float32)
    info = {
        "triangles": ntri,
        "curves": g["ncurves"],
        "curve_segments": g["nsegments"],
        "objects": nobj,
        "instanced_objects": int(sum(not ob["applied"] for ob in objects)),
        "bvh_inner_nodes": nodes.shape[0] // 4,
        "bvh_leaves": leaves.shape[0],
        "light_triangles": nd,
        "lamps": num_lights,
        "shaders": n_shaders,
        "name": scene.name,
        "background_map": bg_map,
    }
    info["textures"] = len(svm_compiler.images)
    return DeviceScene(kd, arrays, scene.width, scene.height, scene.samples, info,
                       textures=list(svm_compiler.images))


def _volume_attribute_dependency(v) -> bool:
    """Shader::has_volume_attribute_dependency (svm.cpp:443-448): a principled
    volume, or an attribute-reading node, in the volume graph."""
    if v is None:
        return False
    if v.kind == "mix":
        return _volume_attribute_dependency(v.a) or _volume_attribute_dependency(v.b)
    if v.kind == "principled_volume":
        return True
    return any(n.kind in ("tex_coord", "geometry", "image_texture", "environment_texture")
               for s, _ in v.sockets() for n in _nodes.upstream(s))


_ATTR_TYPES = {"float": 0, "float2": 1, "float3": 2, "rgba": 3, "matrix": 4}  # NodeAttributeType
_ATTR_ELEMENTS = {"object": 1, "mesh": 2, "face": 3, "vertex": 4, "corner": 6, "corner_byte": 7, "curve": 8,
                  "curve_key": 9}


def _generated_coordinates(m: Mesh) -> np.ndarray:
    """ATTR_STD_GENERATED as Blender syncs it (blender/blender_mesh.cpp
    create_mesh: undeformed co * size - loc, blender_util.h:470-483
    mesh_texture_space) with the automatic texture space of the mesh's
    untransformed vertices: location the bounds' centre, size their half
    extents (a zero extent kept as 1)."""
    f32 = np.float32
    v = np.asarray(m.verts, dtype=f32).reshape(-1, 3)
    lo, hi = v.min(axis=0), v.max(axis=0)
    loc = ((lo + hi) * f32(0.5)).astype(f32)
    size = ((hi - lo) * f32(0.5)).astype(f32)
    size = np.where(size == 0, f32(1.0), size).astype(f32)
    size = (f32(0.5) / size).astype(f32)
    loc = (loc * size - f32(0.5)).astype(f32)
    return (v * size - loc).astype(f32)


def _mesh_attribute(gm: dict, key):
    """AttributeSet::find(AttributeRequest) on one mesh (render/attribute.cpp):
    (element, type, rows) of the attribute a request names, or None."""
    from . import nodes as _nodes_mod
    m = gm.get("mesh")
    if m is None:
        return None
    T = gm["t"].shape[0]
    if key == _nodes_mod.ATTR_STD_UV or key == "UVMap":
        if m.uv is None:
            return None
        return "corner", "float2", np.asarray(m.uv, dtype=np.float32).reshape(3 * T, 2)
    if key == _nodes_mod.ATTR_STD_GENERATED:
        return "vertex", "float3", _generated_coordinates(m)
    if key == _nodes_mod.ATTR_STD_GENERATED_TRANSFORM:
        if m.generated_transform is None:
            return None
        return "mesh", "matrix", np.asarray(m.generated_transform, dtype=np.float32).reshape(3, 4)
    if key == ATTR_STD_POSITION_UNDISPLACED:
        # Mesh::add_undisplaced: the verts before displacement, in the space the
        # geometry's verts are stored in (transform applied or not)
        if m.undisplaced is None:
            return "vertex", "float3", np.asarray(gm["v"], dtype=np.float32)
        u = np.asarray(m.undisplaced, dtype=np.float32).reshape(-1, 3)
        if gm.get("tfm") is not None and len(u):
            u = np.stack([transform_point_f32(gm["tfm"], p) for p in u]).astype(np.float32)
        return "vertex", "float3", u
    if key == _nodes_mod.ATTR_STD_VERTEX_NORMAL or key == "N":
        # Mesh::add_vertex_normals: the normals __tri_vnormal holds
        return "vertex", "float3", np.asarray(gm["nrm"], dtype=np.float32)
    if key in (_nodes_mod.ATTR_STD_UV_TANGENT, _nodes_mod.ATTR_STD_UV_TANGENT_SIGN, "UVMap.tangent",
               "UVMap.tangent_sign"):
        if m.uv is None:
            return None
        tan, sign = _uv_tangents(gm, np.asarray(m.uv, dtype=np.float32).reshape(T, 3, 2))
        if key in (_nodes_mod.ATTR_STD_UV_TANGENT, "UVMap.tangent"):
            return "corner", "float3", tan
        return "corner", "float", sign
    colors = dict(m.vertex_colors or {})
    if key == _nodes_mod.ATTR_STD_VERTEX_COLOR:
        if not colors:
            return None
        key = next(iter(colors))
    if not isinstance(key, str):
        return None
    if key in colors:
        c = np.asarray(colors[key], dtype=np.float64).reshape(3 * T, 4)
        b = np.clip(np.rint(c * 255.0), 0, 255).astype(np.uint32)
        return "corner_byte", "rgba", (b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16) | (b[:, 3] << 24)).astype(np.uint32)
    attrs = m.attributes or {}
    if key not in attrs:
        return None
    element, data = attrs[key]
    if element not in ("vertex", "face", "corner"):
        raise ValueError(f"attribute {key!r}: element must be vertex, face or corner, not {element!r}")
    rows = {"vertex": gm["v"].shape[0], "face": T, "corner": 3 * T}[element]
    a = np.asarray(data, dtype=np.float32)
    a = a.reshape(rows) if a.size == rows else a.reshape(rows, -1)
    kind = "float" if a.ndim == 1 else {2: "float2", 3: "float3"}.get(a.shape[1])
    if kind is None:
        raise ValueError(f"attribute {key!r}: rows of 1, 2 or 3 floats")
    return element, kind, a


def _uv_tangents(gm: dict, uv: np.ndarray):
    """Per-corner UV tangents and their bitangent sign (the data Blender's
    mikktspace pass stores as ATTR_STD_UV_TANGENT / _SIGN, mesh_tangents in
    blender/blender_mesh.cpp): the triangle's dP/du, orthogonalised against
    each corner's vertex normal; sign +1 or -1 from the dP/dv handedness."""
    f32 = np.float32
    v, t, nrm = gm["v"].astype(np.float64), gm["t"], gm["nrm"].astype(np.float64)
    p = v[t]  # (T, 3, 3)
    e1, e2 = p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]
    d1, d2 = (uv[:, 1] - uv[:, 0]).astype(np.float64), (uv[:, 2] - uv[:, 0]).astype(np.float64)
    det = d1[:, 0] * d2[:, 1] - d2[:, 0] * d1[:, 1]
    r = np.where(np.abs(det) > 1e-12, 1.0 / np.where(det == 0, 1.0, det), 0.0)[:, None]
    dpdu = (e1 * d2[:, 1:2] - e2 * d1[:, 1:2]) * r
    dpdv = (e2 * d1[:, 0:1] - e1 * d2[:, 0:1]) * r
    n = nrm[t]  # (T, 3, 3)
    tc = dpdu[:, None, :] - n * np.sum(n * dpdu[:, None, :], axis=2, keepdims=True)
    ln = np.linalg.norm(tc, axis=2, keepdims=True)
    tc = np.where(ln > 1e-12, tc / np.where(ln == 0, 1.0, ln), np.array([1.0, 0.0, 0.0]))
    sign = np.where(np.sum(np.cross(n, tc) * dpdv[:, None, :], axis=2) < 0.0, -1.0, 1.0)
    return tc.reshape(-1, 3).astype(f32), sign.reshape(-1).astype(f32)


def _pack_attributes(g: dict, objects: list, tri_shader_idx, svm_compiler, kobjects, global_reqs=()) -> dict:
    """GeometryManager::device_update_attributes (render/geometry.cpp:379-474)
    and update_attribute_element_offset (:508-620): per geometry one map row
    pair (geometry, subdivision) per attribute its shaders request, closed by
    the ATTR_STD_NONE pair; the data appended to the float / float2 / float3 /
    uchar4 arrays in geometry and request order, offsets corrected by the
    geometry's vert / prim offsets so the kernel indexes them with global
    vertex and triangle numbers.  Curves objects get an empty map."""
    geoms = g["geoms"]
    data = {"float": [], "float2": [], "float3": [], "uchar4": []}
    size = {"float": 0, "float2": 0, "float3": 0, "uchar4": 0}
    rows = []
    geom_offset = {}
    for gi, gm in enumerate(geoms):
        used = sorted(set(int(k) for k in np.unique(gm["sh"]))) if len(gm["sh"]) else []
        reqs = []
        for k in used:
            for key in svm_compiler.requests[k]:
                if key not in reqs:
                    reqs.append(key)
        for key in global_reqs:
            if key not in reqs:
                reqs.append(key)
        geom_offset[gi] = len(rows)
        for key in reqs:
            aid = svm_compiler.attribute_ids[key] if isinstance(key, str) else int(key)
            found = _mesh_attribute(gm, key)
            if found is None:
                # AttributeRequest defaults: element NONE, offset 0, TypeFloat
                rows.append((aid, 0, 0, 0))
            else:
                element, kind, a = found
                store = "uchar4" if kind == "rgba" else "float3" if kind in ("float3", "matrix") else kind
                if kind == "float3":
                    a4 = np.zeros((a.shape[0], 4), dtype=np.float32)
                    a4[:, :3] = a
                    a = a4
                offset = size[store]
                data[store].append(a)
                size[store] += a.shape[0]
                if element == "vertex":
                    offset -= gm["vert_offset"]
                elif element == "face":
                    offset -= gm["tri_offset"]
                elif element in ("corner", "corner_byte"):
                    offset -= 3 * gm["tri_offset"]
                rows.append((aid, _ATTR_ELEMENTS[element], offset & 0xFFFFFFFF, _ATTR_TYPES[kind]))
            rows.append((0, 0, 0, 0))  # no subdivision surface
        rows.extend([(0, 0, 0, 0)] * 2)
    # curves objects (Hair attributes): per-curve values indexed by the global
    # curve number (prim), per-key values by the global key number
    hair_offset = {}
    for i, ob in enumerate(objects):
        hr = ob.get("hair")
        if hr is None or not hr.attributes:
            continue
        used = sorted(set(int(k) for k in np.unique(np.asarray(hr.shader).reshape(-1))))
        reqs = []
        for k in used:
            for key in svm_compiler.requests[k]:
                if key not in reqs:
                    reqs.append(key)
        hair_offset[i] = len(rows)
        for key in reqs:
            aid = svm_compiler.attribute_ids[key] if isinstance(key, str) else int(key)
            if key not in hr.attributes:
                rows.append((aid, 0, 0, 0))
            else:
                element, a = hr.attributes[key]
                if element not in ("curve", "curve_key"):
                    raise ValueError(f"hair attribute {key!r}: element must be curve or curve_key")
                a = np.asarray(a, dtype=np.float32)
                kind = "float" if a.ndim == 1 else {2: "float2", 3: "float3"}[a.shape[1]]
                if kind == "float3":
                    a4 = np.zeros((a.shape[0], 4), dtype=np.float32)
                    a4[:, :3] = a
                    a = a4
                store = kind
                offset = size[store]
                data[store].append(a)
                size[store] += a.shape[0]
                offset -= ob["curve_offset"] if element == "curve" else ob["key_offset"]
                rows.append((aid, _ATTR_ELEMENTS[element], offset & 0xFFFFFFFF, _ATTR_TYPES[kind]))
            rows.append((0, 0, 0, 0))
        rows.extend([(0, 0, 0, 0)] * 2)
    empty = len(rows)
    rows.extend([(0, 0, 0, 0)] * 2)
    for i, ob in enumerate(objects):
        if i in hair_offset:
            kobjects[i].attribute_map_offset = hair_offset[i]
        else:
            kobjects[i].attribute_map_offset = geom_offset[ob["geom"]] if ob.get("geom") is not None else empty

    def cat(store, shape, dtype):
        if not data[store]:
            return np.zeros(shape, dtype=dtype)
        return np.concatenate(data[store]).astype(dtype)

    ntri = max(g["ntri"], 1)
    return {
        "__attributes_map": np.array(rows, dtype=np.uint32).reshape(-1, 4),
        "__attributes_float": cat("float", (1,), np.float32),
        "__attributes_float2": cat("float2", (1, 2), np.float32),
        "__attributes_float3": cat("float3", (1, 4), np.float32),
        "__attributes_uchar4": cat("uchar4", (1,), np.uint32),
        # Mesh::pack_patches (mesh.cpp): no subdivision patches, every triangle ~0
        "__tri_patch": np.full(ntri, 0xFFFFFFFF, dtype=np.uint32),
    }


def _object_shaders(ob, tri_shader_idx) -> list:
    """Material indices the object's triangles use (Mesh::used_shaders)."""
    lo, n = ob["tri_offset"], ob["ntri"]
    return sorted(set(int(k) for k in np.unique(tri_shader_idx[lo:lo + n]))) if n else []


def _object_bounds(ob, g):
    """World-space bounds of an object's triangles (Object::bounds)."""
    lo, n = ob["tri_offset"], ob["ntri"]
    if n == 0:
        return np.zeros(3, np.float32), np.zeros(3, np.float32)
    p = g["tri_pos_object"][lo:lo + n].reshape(-1, 3).astype(np.float32)
    if not ob["applied"]:
        p = np.array([transform_point_f32(ob["tfm"], q) for q in p], dtype=np.float32)
    return p.min(axis=0), p.max(axis=0)


def transform_point_f32(tfm, p) -> np.ndarray:
    """util_transform.h transform_point, float32 in the reference's order."""
    t = np.asarray(tfm, dtype=np.float32)
    p = np.asarray(p, dtype=np.float32)
    f32 = np.float32
    return np.array([f32(f32(f32(p[0] * t[r, 0]) + f32(p[1] * t[r, 1])) + f32(p[2] * t[r, 2])) + t[r, 3]
                     for r in range(3)], dtype=np.float32)


def triangle_area_f32(v1, v2, v3) -> np.float32:
    """util_math.h triangle_area: len(cross(v3 - v2, v1 - v2)) * 0.5."""
    f32 = np.float32
    a = (np.asarray(v3, dtype=np.float32) - np.asarray(v2, dtype=np.float32)).astype(np.float32)
    b = (np.asarray(v1, dtype=np.float32) - np.asarray(v2, dtype=np.float32)).astype(np.float32)
    c = np.array([f32(a[1] * b[2]) - f32(a[2] * b[1]), f32(a[2] * b[0]) - f32(a[0] * b[2]),
                  f32(a[0] * b[1]) - f32(a[1] * b[0])], dtype=np.float32)
    d = f32(f32(f32(c[0] * c[0]) + f32(c[1] * c[1])) + f32(c[2] * c[2]))
    return f32(f32(np.sqrt(d)) * f32(0.5))


def _mesh_arrays(m: Mesh, tfm=None):
    v = np.asarray(m.verts, dtype=np.float32).reshape(-1, 3)
    t = np.asarray(m.tris, dtype=np.int64).reshape(-1, 3)
    if tfm is not None:
        v = np.stack([transform_point_f32(tfm, p) for p in v]).astype(np.float32) if len(v) else v
    if m.normals is not None and tfm is None:
        nrm = np.asarray(m.normals, dtype=np.float32).reshape(-1, 3)
    else:
        nrm = _vertex_normals(v, t)
    sh = np.broadcast_to(np.asarray(m.shader, dtype=np.int64), (t.shape[0],))
    return v, t, sh, nrm


def _instance_props(inst) -> dict:
    def pick(a, b):
        return a if a is not None else b

    return dict(color=pick(inst.object_color, inst.mesh.object_color),
                pass_index=pick(inst.pass_index, inst.mesh.pass_index),
                random=pick(inst.object_random, inst.mesh.object_random),
                holdout=pick(inst.holdout, inst.mesh.holdout),
                particle=pick(inst.particle, inst.mesh.particle))


def _pack_geometry(scene: Scene) -> dict:
    """Geometry, objects and the packed BVH of a scene: the device arrays of
    GeometryManager::device_update_mesh (render/geometry.cpp:873-960) and
    BVH::pack_primitives / pack_instances (bvh/bvh.cpp:279-520)."""
    # objects: plain meshes (transform already applied by the caller), then instances
    users = {}
    for inst in scene.instances:
        users[id(inst.mesh)] = users.get(id(inst.mesh), 0) + 1
    ident = np.eye(4)[:3]
    geoms, geom_of = [], {}  # geometry records in first-use order
    objects = []
    for m in scene.meshes:
        v, t, sh, nrm = _mesh_arrays(m)
        geoms.append(dict(v=v, t=t, sh=sh, nrm=nrm, smooth=bool(m.smooth), applied=True, mesh=m))
        objects.append(dict(geom=len(geoms) - 1, tfm=ident, applied=True, color=m.object_color,
                            pass_index=m.pass_index, random=m.object_random, holdout=m.holdout,
                            particle=m.particle, shadow_catcher=m.shadow_catcher))
    for inst in scene.instances:
        tfm = np.asarray(inst.tfm, dtype=np.float64).reshape(3, 4)
        if inst.mesh.shadow_catcher:
            raise ValueError("shadow catchers are supported on meshes drawn once, not on instances")
        if users[id(inst.mesh)] == 1:
            v, t, sh, nrm = _mesh_arrays(inst.mesh, tfm.astype(np.float32))
            geoms.append(dict(v=v, t=t, sh=sh, nrm=nrm, smooth=bool(inst.mesh.smooth), applied=True, mesh=inst.mesh,
                              tfm=tfm.astype(np.float32)))
            objects.append(dict(geom=len(geoms) - 1, tfm=ident, applied=True,  # tfm reset on apply
                                **_instance_props(inst)))
            continue
        if id(inst.mesh) not in geom_of:
            v, t, sh, nrm = _mesh_arrays(inst.mesh)
            geoms.append(dict(v=v, t=t, sh=sh, nrm=nrm, smooth=bool(inst.mesh.smooth), applied=False, mesh=inst.mesh))
            geom_of[id(inst.mesh)] = len(geoms) - 1
        objects.append(dict(geom=geom_of[id(inst.mesh)], tfm=tfm, applied=False, **_instance_props(inst)))
    # hair objects: transforms applied, after the meshes (object order)
    for hr in scene.hairs:
        objects.append(dict(geom=None, hair=hr, tfm=ident, applied=True, holdout=hr.holdout))

    # global triangle / vertex arrays, geometry order (prim_offset, vert_offset)
    toff = voff = 0
    for gm in geoms:
        gm["tri_offset"], gm["vert_offset"] = toff, voff
        toff += gm["t"].shape[0]
        voff += gm["v"].shape[0]
    ntri, nvert = toff, voff
    tri_shader_idx = np.concatenate([gm["sh"] for gm in geoms]) if geoms else np.zeros(0, np.int64)
    tri_smooth = np.concatenate([np.full(gm["t"].shape[0], gm["smooth"]) for gm in geoms])
    tri_pos = np.concatenate([gm["v"][gm["t"]] for gm in geoms]).astype(np.float32)  # (T,3,3)
    tri_vindex = np.zeros((ntri, 4), dtype=np.uint32)
    tri_vindex[:, :3] = np.concatenate([gm["t"] + gm["vert_offset"] for gm in geoms]).astype(np.uint32)
    tri_vnormal = np.zeros((nvert, 4), dtype=np.float32)
    tri_vnormal[:, :3] = np.concatenate([gm["nrm"] for gm in geoms])
    for ob in objects:
        if ob["geom"] is None:
            ob["tri_offset"], ob["ntri"], ob["numverts"] = 0, 0, 0
            continue
        gm = geoms[ob["geom"]]
        ob["tri_offset"], ob["ntri"], ob["numverts"] = gm["tri_offset"], gm["t"].shape[0], gm["v"].shape[0]
    hair = _pack_hair(objects, scene.hair_shape)

    vis_obj = PATH_RAY_ALL_VISIBILITY & ~(PATH_RAY_SHADOW_OPAQUE_CATCHER | PATH_RAY_SHADOW_TRANSPARENT_CATCHER)
    # a shadow catcher is seen by every shadow ray but those of paths behind a
    # catcher (PATH_RAY_SHADOW_NON_CATCHER, kernel_shadow.h:402-404)
    vis_catcher = PATH_RAY_ALL_VISIBILITY & ~(PATH_RAY_SHADOW_OPAQUE_NON_CATCHER |
                                              PATH_RAY_SHADOW_TRANSPARENT_NON_CATCHER)
    catchers = [oi for oi, ob in enumerate(objects) if ob.get("shadow_catcher")]

    # top level: triangles of objects with applied transforms + one reference per instance
    ref_tri, ref_obj = [], []
    for oi, ob in enumerate(objects):
        if ob["applied"]:
            ref_tri.append(np.arange(ob["tri_offset"], ob["tri_offset"] + ob["ntri"]))
            ref_obj.append(np.full(ob["ntri"], oi))
        else:
            ref_tri.append(np.array([-1]))
            ref_obj.append(np.array([oi]))
    ref_tri = np.concatenate(ref_tri) if ref_tri else np.zeros(0, np.int64)
    ref_obj = np.concatenate(ref_obj) if ref_obj else np.zeros(0, np.int64)
    if hair["nseg"]:
        if catchers:
            raise ValueError("shadow catchers in a scene with curves are not supported")
        return _pack_geometry_with_curves(objects, geoms, ref_tri, ref_obj, tri_pos, ntri, nvert, tri_shader_idx,
                                          tri_smooth, tri_vindex, tri_vnormal, vis_obj, hair)
    nref = len(ref_tri)
    is_inst = ref_tri < 0
    vis = np.full(nref, vis_obj, dtype=np.uint32)
    if catchers:
        vis[np.isin(ref_obj, catchers)] = vis_catcher
    if is_inst.any():
        boxes = np.zeros((nref, 6), dtype=np.float32)
        tp = tri_pos[np.where(is_inst, 0, ref_tri)]
        boxes[:, :3] = tp.min(1)
        boxes[:, 3:] = tp.max(1)
        for k in np.nonzero(is_inst)[0]:
            ob = objects[ref_obj[k]]
            boxes[k] = _instance_bounds(geoms[ob["geom"]]["v"], ob["tfm"])
        nodes, leaves, order, root = build_bvh2_boxes(boxes, vis, is_inst.astype(np.int32))
    else:
        nodes, leaves, order, root = build_bvh2(tri_pos[ref_tri], vis)

    # pack_primitives (bvh.cpp:279-321)
    slot_tri = ref_tri[order]
    slot_inst = slot_tri < 0
    prim_index = np.where(slot_inst, -1, slot_tri).astype(np.int64)
    prim_object = ref_obj[order].astype(np.int64)
    prim_type = np.where(slot_inst, 0, PRIMITIVE_TRIANGLE).astype(np.int64)
    prim_visibility = np.where(slot_inst, 0, vis[order]).astype(np.int64)
    tri_slots = np.cumsum(~slot_inst) - 1
    prim_tri_index = np.where(slot_inst, -1, 3 * tri_slots).astype(np.int64)
    tv = [tri_pos[slot_tri[~slot_inst]].reshape(-1, 3)]
    n_tv = 3 * int((~slot_inst).sum())

    # pack_instances (bvh.cpp:323-520): each instanced geometry's own BVH
    # appended once; object_node = its root
    node_parts, leaf_parts = [nodes], [leaves]
    n_nodes, n_leaves = nodes.shape[0], leaves.shape[0]
    p_index, p_object, p_type, p_vis, p_tri = [prim_index], [prim_object], [prim_type], [prim_visibility], [prim_tri_index]
    n_prims = nref
    geom_node = {}
    for oi, ob in enumerate(objects):
        ob["node"] = 0
        if ob["applied"]:
            continue
        gi = ob["geom"]
        if gi in geom_node:
            ob["node"] = geom_node[gi]
            continue
        gm = geoms[gi]
        gpos = gm["v"][gm["t"]].astype(np.float32)
        gn, gl, go, groot = build_bvh2(gpos, np.full(gpos.shape[0], vis_obj, dtype=np.uint32))
        gn = gn.copy() if groot == 0 else gn[:0].copy()
        cz = gn[0::4].view(np.int32)  # rows of cnodes: vis0, vis1, child0, child1
        for c in (2, 3):
            col = cz[:, c]
            cz[:, c] = np.where(col >= 0, col + n_nodes, col - n_leaves)
        gn[0::4] = cz.view(np.float32)
        gl = gl.copy()
        li = gl.view(np.int32)
        li[:, 0] += n_prims
        li[:, 1] += n_prims
        gl = li.view(np.float32)
        ob["node"] = n_nodes if groot == 0 else -n_leaves - 1
        geom_node[gi] = ob["node"]
        k = gpos.shape[0]
        p_index.append(gm["tri_offset"] + go.astype(np.int64))
        p_object.append(np.zeros(k, np.int64))
        p_type.append(np.full(k, PRIMITIVE_TRIANGLE, np.int64))
        p_vis.append(np.full(k, vis_obj, np.int64))
        p_tri.append(3 * np.arange(k, dtype=np.int64) + n_tv)
        tv.append(gpos[go].reshape(-1, 3))
        n_tv += 3 * k
        node_parts.append(gn[: gn.shape[0]] if gn.shape[0] else gn)
        leaf_parts.append(gl)
        n_nodes += gn.shape[0]
        n_leaves += gl.shape[0]
        n_prims += k

    def u32(parts):
        return (np.concatenate(parts).astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)

    prim_index, prim_object, prim_type = u32(p_index), u32(p_object), u32(p_type)
    prim_visibility, prim_tri_index = u32(p_vis), u32(p_tri)
    verts_all = np.concatenate(tv) if tv else np.zeros((0, 3), np.float32)
    prim_tri_verts = np.ones((max(len(verts_all), 1), 4), dtype=np.float32)
    prim_tri_verts[: len(verts_all), :3] = verts_all
    # tri_vindex.w = prim_tri_index of the triangle's slot (geometry.cpp:900-905)
    is_tri = prim_type == PRIMITIVE_TRIANGLE
    tri_vindex[prim_index[is_tri].astype(np.int64), 3] = prim_tri_index[is_tri]
    tri_pos_object = tri_pos
    return dict(ntri=ntri, tri_shader_idx=tri_shader_idx, tri_smooth=tri_smooth, nodes=np.concatenate(node_parts),
                leaves=np.concatenate(leaf_parts), root=root, prim_index=prim_index, prim_object=prim_object,
                prim_type=prim_type, prim_visibility=prim_visibility, prim_tri_index=prim_tri_index,
                prim_tri_verts=prim_tri_verts, tri_vindex=tri_vindex, tri_vnormal=tri_vnormal, objects=objects,
                tri_pos_object=tri_pos_object, ncurves=0, nsegments=0, geoms=geoms)


def _pack_hair(objects: list, shape: str) -> dict:
    """Hair::pack_curves (render/hair.cpp) over the hair objects in object
    order, and one BVH reference per curve segment (BVHBuild::add_reference_curves,
    bvh/bvh_build.cpp): packed type PRIMITIVE_PACK_SEGMENT(type, segment),
    the segment's box and its Catmull-Rom span as 4 Bezier control points
    (the box of which contains the segment; BoundBox of Hair::Curve::bounds_grow)."""
    ptype0 = {"ribbon": PRIMITIVE_CURVE_RIBBON, "thick": PRIMITIVE_CURVE_THICK}[shape]
    keys_l, first_l, nk_l, sh_l, seg_curve, seg_index, seg_obj = [], [], [], [], [], [], []
    koff = coff = 0
    for oi, ob in enumerate(objects):
        hr = ob.get("hair")
        if hr is None:
            continue
        k = np.asarray(hr.keys, dtype=np.float32).reshape(-1, 3)
        r = np.asarray(hr.radius, dtype=np.float32).reshape(-1)
        first = np.asarray(hr.curve_first, dtype=np.int64).reshape(-1)
        nk = np.asarray(hr.curve_nkeys, dtype=np.int64).reshape(-1)
        if len(r) != len(k) or (nk < 2).any() or (first + nk > len(k)).any():
            raise ValueError("hair: curves need >= 2 keys inside the key array, one radius per key")
        keys_l.append(np.concatenate([k, r[:, None]], axis=1))
        first_l.append(first + koff)
        nk_l.append(nk)
        sh_l.append(np.broadcast_to(np.asarray(hr.shader, dtype=np.int64), first.shape))
        nseg = nk - 1
        seg_curve.append(np.repeat(np.arange(len(first)) + coff, nseg))
        seg_index.append(np.concatenate([np.arange(n) for n in nseg]) if len(nseg) else np.zeros(0, np.int64))
        seg_obj.append(np.full(int(nseg.sum()), oi))
        ob["numkeys"] = len(k)
        ob["key_offset"], ob["curve_offset"] = koff, coff
        koff += len(k)
        coff += len(first)
    if not coff:
        return dict(nseg=0, ncurves=0)
    keys = np.concatenate(keys_l).astype(np.float32)
    first = np.concatenate(first_l)
    nk = np.concatenate(nk_l)
    curve = np.concatenate(seg_curve)
    seg = np.concatenate(seg_index).astype(np.int64)
    k0 = first[curve] + seg
    k1 = k0 + 1
    ka = np.maximum(k0 - 1, first[curve])
    kb = np.minimum(k1 + 1, first[curve] + nk[curve] - 1)
    P = keys.astype(np.float64)
    cp = np.stack([P[k0], P[k0] + (P[k1] - P[ka]) / 6.0, P[k1] - (P[kb] - P[k0]) / 6.0, P[k1]], axis=1)  # (S,4,4)
    rmax = cp[:, :, 3].max(axis=1)
    lo = cp[:, :, :3].min(axis=1) - rmax[:, None]
    hi = cp[:, :, :3].max(axis=1) + rmax[:, None]
    pad = 1e-6 * np.maximum(np.abs(lo), np.abs(hi)) + 1e-7 * (hi - lo)
    boxes = np.concatenate([np.nextafter((lo - pad).astype(np.float32), -np.inf),
                            np.nextafter((hi + pad).astype(np.float32), np.inf)], axis=1).astype(np.float32)
    ptype = ((seg << PRIMITIVE_NUM_TOTAL) | ptype0).astype(np.uint32)
    return dict(nseg=len(seg), ncurves=coff, keys=keys, first=first, nkeys=nk, shader=np.concatenate(sh_l),
                seg_curve=curve, seg_obj=np.concatenate(seg_obj), ptype=ptype, boxes=boxes,
                cp=cp.astype(np.float32).reshape(-1, 16))


def _pack_geometry_with_curves(objects, geoms, ref_tri, ref_obj, tri_pos, ntri, nvert, tri_shader_idx, tri_smooth,
                               tri_vindex, tri_vnormal, vis_obj, hair):
    """The top-level BVH over triangles, instances and curve segments with
    unaligned nodes for curve-only subtrees (BVHParams.use_unaligned_nodes,
    geometry.cpp:1024-1025), and the primitive arrays (bvh.cpp:279-321:
    curves get prim_index = curve, prim_tri_index = -1)."""
    if (ref_tri < 0).any():
        raise ValueError("scenes with curves: instanced geometry is not supported by this stand-in host")
    nt = len(ref_tri)
    ns = hair["nseg"]
    kind = np.concatenate([np.zeros(nt, np.int32), np.full(ns, 2, np.int32)])
    boxes = np.zeros((nt + ns, 6), dtype=np.float32)
    tp = tri_pos[ref_tri] if nt else np.zeros((0, 3, 3), np.float32)
    boxes[:nt, :3] = tp.min(1) if nt else boxes[:0, :3]
    boxes[:nt, 3:] = tp.max(1) if nt else boxes[:0, 3:]
    boxes[nt:] = hair["boxes"]
    vis = np.full(nt + ns, vis_obj, dtype=np.uint32)
    ptype = np.concatenate([np.full(nt, PRIMITIVE_TRIANGLE, np.uint32), hair["ptype"]])
    cp = np.zeros((nt + ns, 16), dtype=np.float32)
    cp[nt:] = hair["cp"]
    lib = native.host_lib()
    counts = np.zeros(3, dtype=np.int64)
    bx, vs, kd, pt, cpc = (np.ascontiguousarray(a) for a in (boxes, vis, kind, ptype, cp))
    h = lib.hcb_build_prims(nt + ns, bx.ctypes.data, vs.ctypes.data, kd.ctypes.data, pt.ctypes.data, cpc.ctypes.data,
                            1, 8, counts.ctypes.data)
    try:
        nodes = np.zeros((max(int(counts[0]), 1), 4), dtype=np.float32)
        leaves = np.zeros((max(int(counts[1]), 1), 4), dtype=np.float32)
        order = np.zeros(nt + ns, dtype=np.int32)
        lib.hcb_pack(h, nodes.ctypes.data, leaves.ctypes.data, order.ctypes.data)
    finally:
        lib.hcb_free(h)
    nodes = nodes[: int(counts[0])] if counts[0] else nodes[:0]
    root = int(counts[2])
    is_curve = order >= nt
    tri_of = np.where(is_curve, 0, order)
    seg_of = np.where(is_curve, order - nt, 0)
    prim_index = np.where(is_curve, hair["seg_curve"][seg_of], ref_tri[tri_of]).astype(np.int64)
    prim_object = np.where(is_curve, hair["seg_obj"][seg_of], ref_obj[tri_of]).astype(np.int64)
    prim_type = ptype[order].astype(np.int64)
    prim_visibility = vis[order].astype(np.int64)
    tri_slots = np.cumsum(~is_curve) - 1
    prim_tri_index = np.where(is_curve, -1, 3 * tri_slots).astype(np.int64)
    verts_all = tri_pos[ref_tri[order[~is_curve]]].reshape(-1, 3) if nt else np.zeros((0, 3), np.float32)
    prim_tri_verts = np.ones((max(len(verts_all), 1), 4), dtype=np.float32)
    prim_tri_verts[: len(verts_all), :3] = verts_all

    def u32(a):
        return (a.astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)

    prim_index, prim_object, prim_type = u32(prim_index), u32(prim_object), u32(prim_type)
    prim_visibility, prim_tri_index = u32(prim_visibility), u32(prim_tri_index)
    is_tri = prim_type == PRIMITIVE_TRIANGLE
    tri_vindex[prim_index[is_tri].astype(np.int64), 3] = prim_tri_index[is_tri]
    for ob in objects:
        ob["node"] = 0
    return dict(ntri=ntri, tri_shader_idx=tri_shader_idx, tri_smooth=tri_smooth, nodes=nodes, leaves=leaves,
                root=root, prim_index=prim_index, prim_object=prim_object, prim_type=prim_type,
                prim_visibility=prim_visibility, prim_tri_index=prim_tri_index, prim_tri_verts=prim_tri_verts,
                tri_vindex=tri_vindex, tri_vnormal=tri_vnormal, objects=objects, tri_pos_object=tri_pos,
                ncurves=hair["ncurves"], nsegments=ns, curve_first=hair["first"].astype(np.uint32),
                curve_nkeys=hair["nkeys"].astype(np.uint32), curve_shader=hair["shader"],
                curve_keys=hair["keys"], geoms=geoms)


def _instance_bounds(v: np.ndarray, tfm) -> np.ndarray:
    """Object::compute_bounds (render/object.cpp): geometry bounds transformed
    (all 8 corners), as float32 min / max."""
    lo, hi = v.min(0), v.max(0)
    corners = np.array([[x, y, z] for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2])],
                       dtype=np.float32)
    w = np.stack([transform_point_f32(np.asarray(tfm, dtype=np.float32), c) for c in corners])
    return np.concatenate([w.min(0), w.max(0)]).astype(np.float32)


def build_bvh2_boxes(boxes: np.ndarray, visibility: np.ndarray, kind: np.ndarray, max_leaf: int = 8):
    lib = native.host_lib()
    n = boxes.shape[0]
    bx = np.ascontiguousarray(boxes, dtype=np.float32)
    vis = np.ascontiguousarray(visibility, dtype=np.uint32)
    kd = np.ascontiguousarray(kind, dtype=np.int32)
    counts = np.zeros(3, dtype=np.int64)
    h = lib.hcb_build_boxes(n, bx.ctypes.data, vis.ctypes.data, kd.ctypes.data, max_leaf, counts.ctypes.data)
    try:
        nodes = np.zeros((max(int(counts[0]), 1), 4), dtype=np.float32)
        leaves = np.zeros((max(int(counts[1]), 1), 4), dtype=np.float32)
        order = np.zeros(n, dtype=np.int32)
        lib.hcb_pack(h, nodes.ctypes.data, leaves.ctypes.data, order.ctypes.data)
    finally:
        lib.hcb_free(h)
    return nodes[: int(counts[0])] if counts[0] else nodes[:0], leaves, order, int(counts[2])


def f32bits_signed(x: float) -> int:
    return int(np.array([x], dtype=np.float32).view(np.int32)[0])


def _f3(v) -> np.ndarray:
    return np.asarray(v, dtype=np.float32)


def _safe_normalize(v: np.ndarray) -> np.ndarray:
    t = np.float32(np.sqrt(np.float32(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])))
    return (v * (np.float32(1.0) / t)).astype(np.float32) if t != 0 else v


LIGHT_TYPES = {"point": 0, "sun": 1, "background": 2, "area": 3, "spot": 4}


def _pack_lamp(kl, lamp: Lamp, shader_index: int) -> bool:
    """LightManager::device_update_points (render/light.cpp:722-907); returns
    whether the lamp turns on lamp MIS (light.cpp:419-427)."""
    f32 = np.float32
    shader_id = shader_index | SHADER_CAST_SHADOW | SHADER_AREA_LIGHT
    if not lamp.cast_shadow:
        shader_id &= ~SHADER_CAST_SHADOW
    kl.type = LIGHT_TYPES[lamp.kind]
    kl.samples = int(lamp.samples)
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


def _pack_background_light(kl, shader_index: int):
    """device_update_points for LIGHT_BACKGROUND (light.cpp:818-839): the world
    shader with MIS, no area-light flag; the world is visible to every ray
    type, so no exclusion bits; strength 1, max bounces 1024 (world default)."""
    shader_id = (shader_index | SHADER_CAST_SHADOW | SHADER_AREA_LIGHT) & ~SHADER_AREA_LIGHT
    shader_id |= SHADER_USE_MIS
    kl.type = LIGHT_TYPES["background"]
    kl.samples = 1
    kl.strength[:] = [1.0, 1.0, 1.0]
    kl.uni[:] = [0.0] * 12
    kl.shader_id = int(np.array([shader_id], dtype=np.uint32).view(np.int32)[0])
    kl.max_bounces = float(1024)
    kl.random = 0.0
    ident = np.eye(4)[:3]
    abi.set_transform(kl.tfm, ident)
    abi.set_transform(kl.itfm, ident)


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
    "__texture_info": 96,
    "__light_background_marginal_cdf": 8, "__light_background_conditional_cdf": 8,
    "__curves": 16, "__curve_keys": 16,
    "__object_volume_step": 4, "__attributes_map": 16,
    "__attributes_float": 4, "__attributes_float2": 8, "__attributes_float3": 16, "__attributes_uchar4": 4,
    "__tri_patch": 4, "__ies": 4, "__particles": 80,
}


def _pack_particles(parts: list) -> np.ndarray:
    """KernelParticle records (kernel_types.h:1551-1562, 80 bytes: index, age,
    lifetime, size, float4 rotation, location, velocity, angular_velocity) of
    ParticleSystemManager::device_update_particles (render/particles.cpp:57-103);
    entry 0 the all-zero dummy."""
    rec = np.zeros((len(parts), 20), dtype=np.float32)
    for i, p in enumerate(parts):
        if p is None:
            continue
        rec[i, 0] = np.array([int(p.get("index", 0))], dtype=np.int32).view(np.float32)[0]
        rec[i, 1] = p.get("age", 0.0)
        rec[i, 2] = p.get("lifetime", 0.0)
        rec[i, 3] = p.get("size", 0.0)
        rec[i, 4:8] = p.get("rotation", (0.0, 0.0, 0.0, 0.0))
        for k, name in enumerate(("location", "velocity", "angular_velocity")):
            rec[i, 8 + 4 * k:11 + 4 * k] = p.get(name, (0.0, 0.0, 0.0))
    return rec.view(np.uint8).reshape(-1).copy()
