"""Generate the golden parity fixtures from the REFERENCE Cycles CPU kernel.

    python tests/golden/make_golden.py

Requires oracle/_ref/libcycles_ref.so (built from /root/reference by
oracle/Makefile `ref`, in the development container only).  For every case in
tests/parity_cases.py it stores, in tests/golden/<case>.npz:
  digest    sha256 of the compiled scene (KernelData + arrays): the inputs
  buffer    reference render buffer (combined pass, all samples)
  rays / hit_f / hit_i / shadow_i   reference scene_intersect results
  cam_xys / cam_out                 reference kernel_path_trace_setup rays
  rng_q / rng_out                   reference path_rng_1D values
The fixtures are data (inputs + expected outputs); no reference source is kept.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle.ref import RefKernel  # noqa: E402
from parity_cases import CASES, camera_queries, compile_case, golden_path, make_rays, scene_digest  # noqa: E402


def main():
    for name in CASES:
        ds = compile_case(name)
        rk = RefKernel(ds)
        buf = rk.render(threads=os.cpu_count())
        rays = make_rays(ds, 4096)
        hit_f, hit_i = rk.intersect(rays)
        shadow = rays.copy()
        shadow[:, 7] = np.full(len(rays), (1 << 7) | (1 << 8) | (1 << 9) | (1 << 10), dtype=np.uint32).view(np.float32)
        sh_f, sh_i = rk.intersect(shadow)
        xys = camera_queries(ds, 1024)
        cam = rk.camera_rays(xys)
        rng = np.random.default_rng(3)
        q = np.zeros((2048, 4), dtype=np.uint32)
        q[:, 0] = rng.integers(0, 2**32, 2048, dtype=np.uint64).astype(np.uint32)
        q[:, 1] = rng.integers(0, 4096, 2048)
        q[:, 2] = ds.samples
        q[:, 3] = rng.integers(0, 150, 2048)
        rng_out = rk.rng_1d(q)
        np.savez_compressed(
            golden_path(name),
            digest=np.array(scene_digest(ds)),
            buffer=buf,
            rays=rays,
            hit_f=hit_f,
            hit_i=hit_i,
            shadow_rays=shadow,
            shadow_i=sh_i,
            cam_xys=xys,
            cam_out=cam,
            rng_q=q,
            rng_out=rng_out,
            samples=np.array(ds.samples),
        )
        print(name, "hits", int(hit_i[:, 0].sum()), "/", len(rays), "buffer mean", float(buf[..., :3].mean()))


if __name__ == "__main__":
    main()
