"""GPU measurement aid: where the CLS stand-in's shading time goes.

    python tools/cls_probe.py [WIDTH HEIGHT SAMPLES]

Renders the classroom stand-in (default 960x540 at 64 spp) as is and with one
feature class swapped out at a time -- the subsurface materials replaced by
diffuse ones of their colour, the Principled wood by a diffuse, the 60 ceiling
lights merged into 6 -- and prints the per-kernel milliseconds of each render
(hipcy_stats), one JSON line per variant.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raytracingproject_amd import scene as sc  # noqa: E402
from raytracingproject_amd import scenes  # noqa: E402
from raytracingproject_amd.device import HIPDevice  # noqa: E402


def variant(kind, w, h, s):
    scn = scenes.classroom_standin(w, h, s)
    if kind in ("no_sss", "diffuse_all"):
        for i in (6, 7, 8):
            scn.materials[i] = sc.diffuse((0.8, 0.55, 0.45))
    if kind in ("no_principled", "diffuse_all"):
        scn.materials[2] = sc.diffuse((0.5, 0.33, 0.2))
    if kind == "few_lights":
        scn.lamps = scn.lamps[::10]
    return scn


def main():
    w, h, s = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (960, 540, 64)
    dev = HIPDevice(0)
    try:
        for kind in ("base", "no_sss", "no_principled", "few_lights", "diffuse_all"):
            ds = sc.compile_scene(variant(kind, w, h, s))
            dev.upload_scene(ds)
            dev.render()  # warm-up (kernel load, BVH widening)
            t = time.perf_counter()
            dev.render()
            ms = 1e3 * (time.perf_counter() - t)
            st = dev.stats()
            keys = ("closest_ms", "shade_ms", "shadow_ms", "closest_rays", "shadow_rays", "lamps")
            out = {"variant": kind, "frame_ms": round(ms, 1), "msamples_s": round(w * h * s / ms / 1e3, 2)}
            out.update({k: (round(st[k], 2) if isinstance(st.get(k), float) else st.get(k)) for k in keys[:5]})
            print(json.dumps(out), flush=True)
    finally:
        dev.close()


if __name__ == "__main__":
    main()
