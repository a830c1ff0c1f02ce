"""Per-kernel instruction mix of the device library's gfx950 ISA.

    python tools/isa_stats.py [filter-substring ...]

Compiles csrc/device/hipcycles.hip (and k_shade.hip) to assembly with the
build flags and prints, per kernel: VGPRs, scratch bytes, and the static
count of scratch loads/stores (spills), global loads/stores and LDS ops.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "raytracingproject_amd", "csrc", "device", f) for f in ("hipcycles.hip", "k_shade.hip")]


def compile_asm(src: str, out: str, extra=()) -> str:
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-rdc", "-std=c++17",
           "-I" + os.path.join(ROOT, "include"), "--offload-device-only", "-S", src, "-o", out, "-w", *extra]
    subprocess.run(cmd, check=True)
    return open(out).read()


def kernels(asm: str):
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end", asm, re.S | re.M):
        name, body = m.group(1), m.group(2)
        meta = {}
        for key in ("num_vgpr", "private_seg_size"):
            mm = re.search(re.escape(name) + r"\." + key + r", (\d+)", asm)
            meta[key] = int(mm.group(1)) if mm else -1
        yield name, body, meta


def main(filters):
    extra = [a for a in filters if a.startswith("-D")]
    filters = [a for a in filters if not a.startswith("-D")]
    for src in SRC:
        ex = extra + (["-DCY_MAX_CLOSURE=2", "-DCY_SHADE_VARIANT=mc2", "-DCY_SVM_TEX=0"] if "k_shade" in src else [])
        asm = compile_asm(src, "/tmp/_isa_stats.s", ex)
        for name, body, meta in kernels(asm):
            dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip().split("(")[0]
            if filters and not any(f in dem for f in filters):
                continue
            cnt = lambda p: len(re.findall(p, body))  # noqa: E731
            n_ds = cnt(r"\bds_")
            print(f"{dem:45s} vgpr {meta['num_vgpr']:3d} scratch {meta['private_seg_size']:5d}  "
                  f"spill st {cnt(r'scratch_store'):4d} ld {cnt(r'scratch_load'):4d}  "
                  f"global ld {cnt(r'global_load'):4d} st {cnt(r'global_store'):3d}  "
                  f"flat {cnt(r'flat_'):4d}  ds {n_ds:4d}  instrs {body.count(chr(10)):6d}")


if __name__ == "__main__":
    main(sys.argv[1:])
