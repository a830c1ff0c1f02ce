"""Render one full frame of a parity_cases.FULL_DIGEST_CASES config on the GPU
and save the float32 buffer (gpurun_out/frame_<name>.npz), for diagnosing a
full-frame digest mismatch against reference crops on the CPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity_cases import FULL_DIGEST_CASES, buffer_sha256  # noqa: E402
from raytracingproject_amd import scene as sc  # noqa: E402
from raytracingproject_amd.device import HIPDevice  # noqa: E402

name = sys.argv[1]
width = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ds = sc.compile_scene(FULL_DIGEST_CASES[name]())
dev = HIPDevice(0)
dev.upload_scene(ds)
dev.set_bvh_width(width)
buf = dev.render()
dev.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"frame_{name}_w{width}.npz"), buffer=buf)
print(name, width, buffer_sha256(buf))
