"""ctypes mirror of the Cycles device-data ABI.

The struct layouts are generated from the single X-macro field list in
include/hipcycles_kernel_types.h (which restates kernel/kernel_types.h:1118-1670
of the reference), so the Python scene compiler, the HIP library and the
reference-layout checker cannot drift apart.  tests/test_abi_layout.py checks
every offset against the reference headers when oracle/_ref is built.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
_HEADER_CANDIDATES = [
    os.path.join(_HERE, "..", "include", "hipcycles_kernel_types.h"),
    os.path.join(_HERE, "include", "hipcycles_kernel_types.h"),
]


class float4(ctypes.Structure):
    _pack_ = 16
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float), ("w", ctypes.c_float)]


class uint4(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32), ("z", ctypes.c_uint32), ("w", ctypes.c_uint32)]


class Transform(ctypes.Structure):
    _fields_ = [("x", float4), ("y", float4), ("z", float4)]


class ProjectionTransform(ctypes.Structure):
    _fields_ = [("x", float4), ("y", float4), ("z", float4), ("w", float4)]


_CTYPE = {
    "int32_t": ctypes.c_int32,
    "uint32_t": ctypes.c_uint32,
    "float": ctypes.c_float,
    "hc_float4": float4,
    "hc_Transform": Transform,
    "hc_ProjectionTransform": ProjectionTransform,
}

# struct name in the reference -> X-macro list name in the header
STRUCT_MACROS = {
    "KernelCamera": "HC_KERNEL_CAMERA_FIELDS",
    "KernelFilm": "HC_KERNEL_FILM_FIELDS",
    "KernelBackground": "HC_KERNEL_BACKGROUND_FIELDS",
    "KernelIntegrator": "HC_KERNEL_INTEGRATOR_FIELDS",
    "KernelBVH": "HC_KERNEL_BVH_FIELDS",
    "KernelTables": "HC_KERNEL_TABLES_FIELDS",
    "KernelBake": "HC_KERNEL_BAKE_FIELDS",
    "KernelObject": "HC_KERNEL_OBJECT_FIELDS",
    "KernelLight": "HC_KERNEL_LIGHT_FIELDS",
    "KernelLightDistribution": "HC_KERNEL_LIGHT_DISTRIBUTION_FIELDS",
    "KernelShader": "HC_KERNEL_SHADER_FIELDS",
    "KernelParticle": "HC_KERNEL_PARTICLE_FIELDS",
}


def header_path() -> str:
    for p in _HEADER_CANDIDATES:
        if os.path.exists(p):
            return os.path.abspath(p)
    raise FileNotFoundError("include/hipcycles_kernel_types.h not found")


def parse_fields(text: str | None = None) -> dict[str, list[tuple[str, str, int]]]:
    """Return {reference struct name: [(ctype, field, count), ...]} from the header."""
    if text is None:
        with open(header_path()) as f:
            text = f.read()
    out = {}
    for sname, macro in STRUCT_MACROS.items():
        m = re.search(r"#define\s+%s\(X\)((?:.*\\\n)*.*)" % macro, text)
        if m is None:
            raise ValueError("field list %s missing" % macro)
        body = m.group(1)
        fields = re.findall(r"X\(\s*(\w+)\s*,\s*(\w+)\s*,\s*(\d+)\s*\)", body)
        out[sname] = [(t, n, int(c)) for t, n, c in fields]
    return out


_ALIGN16 = {"hc_float4", "hc_Transform", "hc_ProjectionTransform"}


def _make_struct(name: str, fields: list[tuple[str, str, int]]):
    """Lay the fields out like the C compiler does for the aligned(16) vector types.

    ctypes cannot over-align a member, so 16-byte-aligned members get explicit
    padding in front of them; every device struct is a multiple of 16 bytes
    (static_assert_align in kernel_types.h)."""
    cfields = []
    off = 0
    npad = 0
    for t, n, c in fields:
        ct = _CTYPE[t]
        if t in _ALIGN16 and off % 16:
            pad = 16 - off % 16
            cfields.append(("_pad%d" % npad, ctypes.c_byte * pad))
            npad += 1
            off += pad
        ft = ct * c if c > 1 else ct
        cfields.append((n, ft))
        off += ctypes.sizeof(ft)
    if off % 16:
        cfields.append(("_tailpad", ctypes.c_byte * (16 - off % 16)))
    return type(name, (ctypes.Structure,), {"_fields_": cfields})


_FIELDS = parse_fields()
KernelCamera = _make_struct("KernelCamera", _FIELDS["KernelCamera"])
KernelFilm = _make_struct("KernelFilm", _FIELDS["KernelFilm"])
KernelBackground = _make_struct("KernelBackground", _FIELDS["KernelBackground"])
KernelIntegrator = _make_struct("KernelIntegrator", _FIELDS["KernelIntegrator"])
KernelBVH = _make_struct("KernelBVH", _FIELDS["KernelBVH"])
KernelTables = _make_struct("KernelTables", _FIELDS["KernelTables"])
KernelBake = _make_struct("KernelBake", _FIELDS["KernelBake"])
KernelObject = _make_struct("KernelObject", _FIELDS["KernelObject"])
KernelLight = _make_struct("KernelLight", _FIELDS["KernelLight"])
KernelLightDistribution = _make_struct("KernelLightDistribution", _FIELDS["KernelLightDistribution"])
KernelShader = _make_struct("KernelShader", _FIELDS["KernelShader"])
KernelParticle = _make_struct("KernelParticle", _FIELDS["KernelParticle"])


class KernelData(ctypes.Structure):
    _fields_ = [
        ("cam", KernelCamera),
        ("film", KernelFilm),
        ("background", KernelBackground),
        ("integrator", KernelIntegrator),
        ("bvh", KernelBVH),
        ("tables", KernelTables),
        ("bake", KernelBake),
    ]


STRUCTS = {
    "KernelData": KernelData,
    "KernelCamera": KernelCamera,
    "KernelFilm": KernelFilm,
    "KernelBackground": KernelBackground,
    "KernelIntegrator": KernelIntegrator,
    "KernelBVH": KernelBVH,
    "KernelTables": KernelTables,
    "KernelBake": KernelBake,
    "KernelObject": KernelObject,
    "KernelLight": KernelLight,
    "KernelLightDistribution": KernelLightDistribution,
    "KernelShader": KernelShader,
    "KernelParticle": KernelParticle,
}

SIZEOF_KERNEL_DATA = 1584
assert ctypes.sizeof(KernelData) == SIZEOF_KERNEL_DATA, ctypes.sizeof(KernelData)


def to_bytes(obj) -> bytes:
    return ctypes.string_at(ctypes.addressof(obj), ctypes.sizeof(obj))


def array_bytes(records) -> bytes:
    return b"".join(to_bytes(r) for r in records)


def set_transform(t: Transform, rows) -> None:
    """rows: 3x4 (Transform) or 4x4 (ProjectionTransform) nested sequences."""
    for name, row in zip(("x", "y", "z", "w"), rows):
        v = getattr(t, name)
        v.x, v.y, v.z, v.w = (float(a) for a in row)
