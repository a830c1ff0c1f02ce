"""Loaders for the in-tree native libraries.

- libhipcycles.so       : the HIP device (kernels + C ABI of include/hipcycles.h)
- libhipcycles_host.so  : host-only helpers (BVH2 builder/packer stand-in)

Both are built in-tree by __graft_entry__.build() / tools/build.py.  A missing
device library is a hard error: there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# HIPCY_DEVICE_LIB selects an alternative in-tree build (tuning variants made
# by `python -m raytracingproject_amd.build --variant NAME -D...`)
DEVICE_LIB = os.environ.get("HIPCY_DEVICE_LIB") or os.path.join(_HERE, "libhipcycles.so")
HOST_LIB = os.path.join(_HERE, "libhipcycles_host.so")
ABI_VERSION = 6  # HIPCY_ABI_VERSION in include/hipcycles.h


def device_lib_path() -> str:
    return DEVICE_LIB

_host = None
_dev = None


class NativeLibraryMissing(RuntimeError):
    pass


def host_lib():
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB):
            raise NativeLibraryMissing(f"{HOST_LIB} not built; run python __graft_entry__.py build")
        lib = ctypes.CDLL(HOST_LIB)
        lib.hcb_build.restype = ctypes.c_void_p
        lib.hcb_build.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        lib.hcb_build_boxes.restype = ctypes.c_void_p
        lib.hcb_build_boxes.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_void_p]
        lib.hcb_build_prims.restype = ctypes.c_void_p
        lib.hcb_build_prims.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p]
        lib.hcb_pack.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.hcb_free.argtypes = [ctypes.c_void_p]
        lib.hcb_background_cdf.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]
        lib.cyh_beckmann_table.argtypes = [ctypes.c_void_p]
        lib.cyh_beckmann_table_size.restype = ctypes.c_int
        _host = lib
    return _host


class WorkTile(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_int32), ("y", ctypes.c_int32), ("w", ctypes.c_int32), ("h", ctypes.c_int32),
        ("start_sample", ctypes.c_int32), ("num_samples", ctypes.c_int32),
        ("offset", ctypes.c_int32), ("stride", ctypes.c_int32), ("buffer", ctypes.c_uint64),
    ]


# hipcy_tile_feed callbacks: acquire(user, tile*, tag*) -> int, release(user, tile*, tag), cancelled(user) -> int
FEED_ACQUIRE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(WorkTile), ctypes.POINTER(ctypes.c_uint64))
FEED_RELEASE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(WorkTile), ctypes.c_uint64)
FEED_CANCELLED = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


class TileFeed(ctypes.Structure):
    _fields_ = [
        ("user", ctypes.c_void_p), ("acquire", FEED_ACQUIRE), ("release", FEED_RELEASE),
        ("cancelled", FEED_CANCELLED), ("hold", ctypes.c_uint64),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("closest_rays", ctypes.c_uint64), ("shadow_rays", ctypes.c_uint64),
        ("inner_nodes", ctypes.c_uint64), ("leaves", ctypes.c_uint64), ("triangles", ctypes.c_uint64),
        ("iterations", ctypes.c_uint64), ("intersect_ms", ctypes.c_double), ("shade_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double), ("closest_ms", ctypes.c_double), ("closest_launches", ctypes.c_uint64),
        ("closest_nodes", ctypes.c_uint64), ("closest_leaves", ctypes.c_uint64), ("closest_tris", ctypes.c_uint64),
        ("bvh_width", ctypes.c_int32), ("bvh_depth", ctypes.c_int32), ("bvh_bytes", ctypes.c_uint64),
        ("tie_rays", ctypes.c_uint64),
        ("closest_lane_iters", ctypes.c_uint64), ("closest_wave_iters", ctypes.c_uint64),
        ("shadow_nodes", ctypes.c_uint64), ("shadow_tris", ctypes.c_uint64),
        ("shadow_lane_iters", ctypes.c_uint64), ("shadow_wave_iters", ctypes.c_uint64),
        ("shadow_ms", ctypes.c_double), ("shadow_launches", ctypes.c_uint64),
    ]


# exported symbols of include/hipcycles.h (checked by tests/test_native_build.py)
DEVICE_SYMBOLS = {
    "hipcy_abi_version": (ctypes.c_int, []),
    "hipcy_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "hipcy_device_info": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]),
    "hipcy_create": (ctypes.c_void_p, [ctypes.c_int]),
    "hipcy_destroy": (None, [ctypes.c_void_p]),
    "hipcy_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "hipcy_global_error": (ctypes.c_char_p, []),
    "hipcy_mem_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]),
    "hipcy_mem_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "hipcy_mem_copy_to": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]),
    "hipcy_mem_copy_from": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t]),
    "hipcy_mem_zero": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t]),
    "hipcy_const_copy_to": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t]),
    "hipcy_bind_global": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_size_t]),
    "hipcy_tex_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]),
    "hipcy_tex_alloc_3d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t]),
    "hipcy_tex_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hipcy_load_kernels": (ctypes.c_int, [ctypes.c_void_p]),
    "hipcy_get_bvh_layout_mask": (ctypes.c_uint32, [ctypes.c_void_p]),
    "hipcy_path_trace": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(WorkTile)]),
    "hipcy_path_trace_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(WorkTile), ctypes.c_int]),
    "hipcy_path_trace_tiles": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(WorkTile), ctypes.c_int]),
    "hipcy_render_feed": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TileFeed)]),
    "hipcy_set_stream_hold": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "hipcy_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "hipcy_get_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Stats)]),
    "hipcy_set_profiling": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hipcy_set_bvh_width": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hipcy_set_curve_layout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hipcy_set_ray_sort": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hipcy_set_traversal_budget": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "hipcy_set_traversal_refill": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "hipcy_set_tail": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "hipcy_set_shadow_sort": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hipcy_set_bvh_leaf_merge": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hipcy_set_slots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]),
    "hipcy_intersect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]),
    "hipcy_film_convert": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int]),
    "hipcy_shader_eval": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "hipcy_camera_rays": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
}


def device_lib():
    global _dev
    if _dev is None:
        if not os.path.exists(DEVICE_LIB):
            raise NativeLibraryMissing(
                f"{DEVICE_LIB} not built (the HIP device library is required; no CPU fallback)"
            )
        lib = ctypes.CDLL(DEVICE_LIB)
        for name, (res, args) in DEVICE_SYMBOLS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.hipcy_abi_version() != ABI_VERSION:
            raise NativeLibraryMissing(f"{DEVICE_LIB}: ABI {lib.hipcy_abi_version()} != {ABI_VERSION}; rebuild")
        _dev = lib
    return _dev


def hash_uint2(kx: int, ky: int) -> int:
    """util/util_hash.h:83-93 (host side, for KernelIntegrator.seed); returned as
    the int32 the seed field holds."""
    M = 0xFFFFFFFF

    def rot(x, k):
        return ((x << k) | (x >> (32 - k))) & M

    a = b = c = (0xDEADBEEF + (2 << 2) + 13) & M
    b = (b + ky) & M
    a = (a + kx) & M
    c ^= b; c = (c - rot(b, 14)) & M
    a ^= c; a = (a - rot(c, 11)) & M
    b ^= a; b = (b - rot(a, 25)) & M
    c ^= b; c = (c - rot(b, 16)) & M
    a ^= c; a = (a - rot(c, 4)) & M
    b ^= a; b = (b - rot(a, 14)) & M
    c ^= b; c = (c - rot(b, 24)) & M
    return c if c < 2**31 else c - 2**32


def background_cdf(pixels, res_x: int, res_y: int):
    """Marginal ((res_y + 1) x 2) and conditional ((res_x + 1) * res_y x 2)
    float32 CDFs of a (res_y, res_x, 4) background map
    (csrc/host/light_background.cpp, render/light.cpp:530-716)."""
    import numpy as np

    px = np.ascontiguousarray(pixels, dtype=np.float32)
    if px.shape != (res_y, res_x, 4):
        raise ValueError(f"background map must be ({res_y}, {res_x}, 4), got {px.shape}")
    marg = np.zeros((res_y + 1, 2), dtype=np.float32)
    cond = np.zeros(((res_x + 1) * res_y, 2), dtype=np.float32)
    host_lib().hcb_background_cdf(px.ctypes.data, res_x, res_y, marg.ctypes.data, cond.ctypes.data)
    return marg, cond
