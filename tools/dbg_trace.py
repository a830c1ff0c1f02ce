"""Debugging aid: the shading stage's trace of one path (pixel X, Y, sample S;
the CY_DBG_* points of cy_integrator.h) from the device and from the host
emulation, so that the first differing line names the operation.

    python tools/dbg_trace.py host CASE X Y S [WIDTH]  > host.txt
    python tools/dbg_trace.py gpu  CASE X Y S [WIDTH]  > gpu.txt
    python tools/dbg_trace.py diff host.txt gpu.txt

`host` builds the emulator with -DCY_DBG_X/Y/S (and libm sinf/cosf, as the
parity tests do); `gpu` loads raytracingproject_amd/libhipcycles-dbg.so, built
with the same defines:

    python -m raytracingproject_amd.build --variant dbg --only mc1_tex,mc2_tex,mc4_tex,mc8_tex \\
        -DCY_DBG_X=23 -DCY_DBG_Y=7 -DCY_DBG_S=4
"""
from __future__ import annotations

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
if len(sys.argv) > 1 and sys.argv[1] == "gpu":
    # before any import of raytracingproject_amd.native reads it
    os.environ.setdefault("HIPCY_DEVICE_LIB", os.path.join(ROOT, "raytracingproject_amd", "libhipcycles-dbg.so"))


def main():
    mode = sys.argv[1]
    if mode == "diff":
        a = open(sys.argv[2]).read().splitlines()
        b = open(sys.argv[3]).read().splitlines()
        a = [l for l in a if not l.startswith("#")]
        b = [l for l in b if not l.startswith("#")]
        for i, (x, y) in enumerate(zip(a, b)):
            mark = "  " if x == y else "!!"
            print(f"{mark} {x:<48} {y}")
            if x != y:
                print(f"first difference at line {i}")
                break
        else:
            print(f"no difference in {min(len(a), len(b))} lines ({len(a)} host, {len(b)} gpu)")
        return
    name, x, y, s = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    width = int(sys.argv[6]) if len(sys.argv) > 6 else 2
    from parity_cases import compile_case, load_golden, with_background_golden

    ds = with_background_golden(compile_case(name), load_golden(name))
    if mode == "host":
        import native_build as nb

        so = nb.build("tools/host_emu.cpp", f"libhost_emu_dbg_{x}_{y}_{s}.so",
                      ["CY_HOST_LIBM_SINCOS", f"CY_DBG_X={x}", f"CY_DBG_Y={y}", f"CY_DBG_S={s}"])
        lib = nb.host_emu()  # argtypes of the regular build apply to the debug one
        dbg = ctypes.CDLL(so)
        for fn in ("emu_render", "emu_intersect", "emu_bvhw_build", "emu_set_object_root", "emu_set_width",
                   "emu_set_instancing"):
            getattr(dbg, fn).argtypes = getattr(lib, fn).argtypes
            getattr(dbg, fn).restype = getattr(lib, fn).restype
        es = nb.EmuScene(dbg, ds, width)
        print(f"# host emulation {name} pixel ({x},{y}) sample {s} W={width}", flush=True)
        es.render(tile=(x, y, 1, 1), start_sample=s, samples=1)
        ctypes.CDLL(None).fflush(None)
        return
    import torch

    torch.zeros(1, device="cuda")  # the HIP runtime comes up through torch first, as in bench.py
    from raytracingproject_amd.device import HIPDevice

    dev = HIPDevice(0)
    dev.set_bvh_width(width)
    dev.upload_scene(ds)
    print(f"# device {name} pixel ({x},{y}) sample {s} W={width}", flush=True)
    if os.environ.get("DBG_FULL_FRAME"):
        dev.render()  # the whole frame: the traced path is one of them
    else:
        dev.render(samples=1, start_sample=s, tile=(x, y, 1, 1))
    torch.cuda.synchronize()
    dev.close()
    ctypes.CDLL(None).fflush(None)


if __name__ == "__main__":
    main()
