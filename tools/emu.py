"""Drive tools/_build/libhost_emu.so (host build of the device code) — debugging aid."""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(variant="libhost_emu.so"):
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", variant))
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.emu_render.argtypes = [vp, ci, vp, vp, vp, vp] + [ci] * 9
    return lib


def render(ds, lib=None, samples=None, start_sample=0, tile=None):
    lib = lib or load()
    samples = ds.samples if samples is None else samples
    x, y, w, h = tile if tile is not None else (0, 0, ds.width, ds.height)
    names = list(ds.arrays)
    arrs = [np.ascontiguousarray(ds.arrays[n]) for n in names]
    c_names = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
    c_ptrs = (ctypes.c_void_p * len(names))(*[a.ctypes.data for a in arrs])
    data = (ctypes.c_char * ctypes.sizeof(ds.data)).from_buffer_copy(bytes(ds.data))
    buf = np.zeros((h, w, ds.pass_stride), dtype=np.float32)
    err = lib.emu_render(ctypes.addressof(data), len(names), c_names, c_ptrs, None, buf.ctypes.data,
                         x, y, w, h, start_sample, samples, -(x + y * w), w, ds.pass_stride)
    if err:
        raise RuntimeError("emulator device error %x" % err)
    return buf


def background_inputs(width, height):
    """LightManager's map inputs (light.cpp:49-59): uint4 per pixel, u/v float bits."""
    u = ((np.arange(width, dtype=np.float32) + np.float32(0.5)) / np.float32(width)).astype(np.float32)
    v = ((np.arange(height, dtype=np.float32) + np.float32(0.5)) / np.float32(height)).astype(np.float32)
    inp = np.zeros((height, width, 4), dtype=np.uint32)
    inp[..., 0] = u.view(np.uint32)[None, :]
    inp[..., 1] = v.view(np.uint32)[:, None]
    return inp


def background(ds, width, height, num_samples=1, lib=None):
    lib = lib or load()
    names = list(ds.arrays)
    arrs = [np.ascontiguousarray(ds.arrays[n]) for n in names]
    c_names = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
    c_ptrs = (ctypes.c_void_p * len(names))(*[a.ctypes.data for a in arrs])
    data = (ctypes.c_char * ctypes.sizeof(ds.data)).from_buffer_copy(bytes(ds.data))
    inp = background_inputs(width, height)
    out = np.zeros((height, width, 4), dtype=np.float32)
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.emu_background.argtypes = [vp, ci, vp, vp, vp, ci, ci, vp]
    err = lib.emu_background(ctypes.addressof(data), len(names), c_names, c_ptrs, inp.ctypes.data,
                             width * height, num_samples, out.ctypes.data)
    if err:
        raise RuntimeError("emulator device error %x" % err)
    return out
