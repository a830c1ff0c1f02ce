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
