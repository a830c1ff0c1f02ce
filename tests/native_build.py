"""Host (g++) builds of test-only native helpers, cached under tools/_build/.

host_emu   the HIP device's per-path code (csrc/kernel) compiled for the host,
           sample-major like the reference CPU device (tools/host_emu.cpp);
           with libm sinf/cosf (CY_HOST_LIBM_SINCOS) or with the device's own
           restatement of glibc's algorithm.
sincos     cy_sinf/cy_cosf of csrc/kernel/cy_math.h on the host.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_build")
FPFLAGS = ["-fno-trapping-math", "-fno-math-errno", "-fno-signed-zeros", "-mfpmath=sse", "-ffp-contract=off"]


def _deps():
    out = []
    for d in ("raytracingproject_amd/csrc/kernel", "include", "tools", "tests/native"):
        for root, _, files in os.walk(os.path.join(ROOT, d)):
            out += [os.path.join(root, f) for f in files if f.endswith((".h", ".cpp"))]
    return out


def build(src: str, name: str, defines=()) -> str:
    os.makedirs(OUT, exist_ok=True)
    so = os.path.join(OUT, name)
    if not os.path.exists(so) or any(os.path.getmtime(d) > os.path.getmtime(so) for d in _deps()):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", *FPFLAGS, *["-D" + d for d in defines],
               "-I" + os.path.join(ROOT, "include"), "-o", so, os.path.join(ROOT, src), "-lm"]
        subprocess.run(cmd, check=True)
    return so


def host_emu(libm_sincos: bool = True):
    if libm_sincos:
        so = build("tools/host_emu.cpp", "libhost_emu.so", ["CY_HOST_LIBM_SINCOS"])
    else:
        so = build("tools/host_emu.cpp", "libhost_emu_dsin.so")
    lib = ctypes.CDLL(so)
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.emu_render.argtypes = [vp, ci, vp, vp, vp] + [ci] * 9
    return lib


def sincos():
    lib = ctypes.CDLL(build("tests/native/sincos_check.cpp", "libsincos_check.so"))
    vp = ctypes.c_void_p
    lib.sincos_eval.argtypes = [vp, ctypes.c_long, vp, vp, vp, vp]
    return lib
