"""GPU debugging aid: locate the pixels and samples where a parity case's HIP
film differs from the reference CPU kernel.

    python tools/dbg_mismatch.py CASE [WIDTH]

Renders CASE on cuda:0 at BVH width WIDTH (default 2), lists the differing
buffer values, then renders each differing pixel one sample at a time on the
device and in the reference kernel (oracle/_ref, test infrastructure) and prints
the first sample whose contribution differs with both values.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity_cases import compile_case, load_golden, with_background_golden  # noqa: E402

from oracle.ref import RefKernel  # noqa: E402
from raytracingproject_amd.device import HIPDevice  # noqa: E402


def main():
    name = sys.argv[1]
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ds = compile_case(name)
    g = load_golden(name)
    dev = HIPDevice(0)
    dev.set_bvh_width(width)
    dev.upload_scene(ds)
    buf = dev.render()
    ref = g["buffer"]
    diff = np.argwhere(buf.view(np.uint32) != ref.view(np.uint32))
    print(f"{name} W={width}: {len(diff)} differing values")
    pixels = sorted({(int(y), int(x)) for y, x, _ in diff})
    for y, x, c in diff[:20]:
        print(f"  pixel ({x},{y}) ch {c}: hip {buf[y, x, c]!r} ref {ref[y, x, c]!r}")
    rr = RefKernel(with_background_golden(compile_case(name), g))
    for (y, x) in pixels[:4]:
        for s in range(ds.samples):
            a = dev.render(samples=1, start_sample=s, tile=(x, y, 1, 1))
            b = rr.render(samples=1, start_sample=s, tile=(x, y, 1, 1), threads=1)
            if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
                print(f"  pixel ({x},{y}) sample {s}: hip {a.ravel().tolist()} ref {b.ravel().tolist()}")
                break
        else:
            print(f"  pixel ({x},{y}): single-sample renders agree (difference is in the sum order)")
    rr.close()
    dev.close()


if __name__ == "__main__":
    main()
