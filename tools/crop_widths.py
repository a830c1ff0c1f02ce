"""Measurement / debugging aid: render a crop of a config at BVH widths 2 and
4 (and 8) on cuda:0 and report each film's checksum and how many values differ
from the width-2 film (the BVH2 traversal in the reference's order).

    python tools/crop_widths.py junkshop_standin 1664 832 512 256 [samples]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from raytracingproject_amd import scene as sc
    from raytracingproject_amd import scenes
    from raytracingproject_amd.device import HIPDevice

    name = sys.argv[1]
    x, y, w, h = (int(v) for v in sys.argv[2:6])
    ds = sc.compile_scene(scenes.CONFIGS[name]())
    S = int(sys.argv[6]) if len(sys.argv) > 6 else ds.samples
    torch.zeros(1, device="cuda")
    dev = HIPDevice(0)
    dev.upload_scene(ds)
    films = {}
    for width in (2, 4, 8):
        dev.set_bvh_width(width)
        films[width] = dev.render(tile=(x, y, w, h), samples=S)
    base = films[2].view(np.uint32)
    for width, f in films.items():
        diff = np.argwhere(f.view(np.uint32) != base)
        print(json.dumps({"config": name, "width": width, "samples": S,
                          "checksum": float(f[..., :4].astype(np.float64).sum()),
                          "differs_from_w2": int(len(diff)), "first": diff[:4].tolist()}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
