"""Per-kernel VGPRs / scratch / LDS of a compiled device object (.o with an
offload bundle) without recompiling: unbundles the gfx950 code object and
reads its AMDGPU metadata notes.

    python tools/kres_obj.py build/device/default/hipcycles.o [name-filter ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "k.co")
        fb = os.path.join(d, "fb.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "-type=o", "-targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"-input={fb}", f"-output={co}", "-unbundle"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    out = []
    for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        get = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
        if name:
            out.append((name.group(1), get("vgpr_count"), get("private_segment_fixed_size"),
                        get("group_segment_fixed_size"), get("sgpr_count")))
    return out


if __name__ == "__main__":
    obj, filt = sys.argv[1], sys.argv[2:]
    names = {}
    for n, v, p, g, s in kernels(obj):
        dn = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
        dn = re.sub(r"\(CyGlobals.*\)", "", dn)
        if filt and not any(f in dn for f in filt):
            continue
        print(f"{dn:70s} vgpr {v:>4} scratch {p:>6} lds {g:>6} sgpr {s}")
