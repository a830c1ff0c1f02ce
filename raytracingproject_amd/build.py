"""In-tree build of the native libraries (no cmake; plain hipcc / g++ / make).

    python -m raytracingproject_amd.build [--no-ref]

Products (git-ignored, but they travel to the GPU box with the snapshot):
  raytracingproject_amd/libhipcycles.so       HIP device for gfx950
  raytracingproject_amd/libhipcycles_host.so  host BVH2 builder
Test infrastructure (oracle/, never imported by the product):
  oracle/_build/libcy_oracle.so               plain-C restatement
  oracle/_ref/libcycles_ref.so                reference CPU kernel (only when
                                              /root/reference is present)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# Parity-critical flags: no contraction, IEEE div/sqrt (see cy_math.h header).
HIP_FLAGS = [
    "-O3",
    "--offload-arch=gfx950",
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-rdc",
    "-fPIC",
    "-shared",
    "-std=c++17",
    "-Wno-unused-result",
    "-Wno-unused-value",
]


def _run(cmd, **kw):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, **kw)


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _sources(*dirs, exts=(".h", ".hip", ".cpp")):
    out = []
    for d in dirs:
        for root, _, files in os.walk(d):
            out += [os.path.join(root, f) for f in files if f.endswith(exts)]
    return out


def kernel_source_digest():
    """sha256 over the device sources: ties a committed profile to the code it measured."""
    import hashlib

    h = hashlib.sha256()
    deps = _sources(os.path.join(HERE, "csrc", "kernel"), os.path.join(HERE, "csrc", "device"),
                    os.path.join(REPO, "include"))
    for path in sorted(deps, key=lambda p: os.path.relpath(p, REPO)):
        h.update(os.path.relpath(path, REPO).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


SHADE_VARIANTS = (1, 2, 4, 8)  # closure-array sizes of the shade kernel (csrc/device/k_shade.h)
LARGE_SHADE_VARIANTS = (16, 64)  # texture / volume builds only (extended closure set)
EXT_SHADE_VARIANTS = (8, 64)  # integrator-extras builds (catchers, branched, light passes)


def build_device(force=False, variant=None, defines=(), traversal_only=False, only=None):
    """The HIP device library: hipcycles.hip plus k_shade.hip compiled once per
    closure-array size.  A named variant (tuning builds with extra -D defines)
    goes to libhipcycles-<variant>.so next to the default one; with
    traversal_only the variant recompiles hipcycles.hip alone and links the
    default build's shading objects; `only` (object names such as "mc2_tex" or
    "hipcycles") recompiles just those and links the rest from the default
    build (debugging builds, tools/dbg_trace.py)."""
    dev_dir = os.path.join(HERE, "csrc", "device")
    src = os.path.join(dev_dir, "hipcycles.hip")
    out = os.path.join(HERE, f"libhipcycles-{variant}.so" if variant else "libhipcycles.so")
    deps = _sources(os.path.join(HERE, "csrc", "kernel"), dev_dir, os.path.join(HERE, "csrc", "host"),
                    os.path.join(REPO, "include"))
    if not (force or variant or _stale(out, deps)):
        return out
    inc = "-I" + os.path.join(REPO, "include")
    dflags = ["-D" + d for d in defines]
    objdir = os.path.join(REPO, "build", "device", variant or "default")
    os.makedirs(objdir, exist_ok=True)
    from concurrent.futures import ThreadPoolExecutor

    cflags = [f for f in HIP_FLAGS if f != "-shared"]
    default_dir = os.path.join(REPO, "build", "device", "default")
    jobs, shade_objs = [], []
    if only is not None and "hipcycles" not in only:
        shade_objs.append(os.path.join(default_dir, "hipcycles.o"))
    else:
        jobs.append(([HIPCC, *cflags, *dflags, inc, "-c", "-o", os.path.join(objdir, "hipcycles.o"), src],
                     os.path.join(objdir, "hipcycles.o")))
    for mc in SHADE_VARIANTS + LARGE_SHADE_VARIANTS:
        # plain (closure nodes only), _tex (texture nodes, extended closures),
        # _vol (_tex with volumes)
        # _ext (_tex with the integrator extras: shadow catchers, branched path
        # tracing, light passes) and _vext (_vol with the volume extras:
        # decoupled ray marching, camera inside a volume, SSS in volume
        # scenes); 8 and 64 closures only
        # (the _vol variants -- volumes without the extras -- are not built: on
        # the GPU they rendered volume scenes wrong; every
        # volume scene takes _vext)
        kinds = ("", "_tex") if mc in SHADE_VARIANTS else ("_tex",)
        if mc in EXT_SHADE_VARIANTS:
            kinds += ("_ext", "_vext")
        for kind in kinds:
            name = f"mc{mc}{kind}"
            if traversal_only or (only is not None and name not in only):
                shade_objs.append(os.path.join(default_dir, f"k_shade_{name}.o"))
                continue
            obj = os.path.join(objdir, f"k_shade_{name}.o")
            # plain variants: the fused tail with lane pairs (CY_TAIL_PAIRS,
            # k_shade.hip; N = 8 shard 12.95 -> 12.55 ms, profiles/r06/tail/)
            pairs = ["-DCY_TAIL_PAIRS=1"] if kind == "" else []
            jobs.append(([HIPCC, *cflags, *dflags, *pairs, f"-DCY_MAX_CLOSURE={mc}", f"-DCY_SHADE_VARIANT={name}",
                          f"-DCY_SVM_TEX={0 if kind == '' else 1}",
                          f"-DCY_VOLUME={1 if kind in ('_vol', '_vext') else 0}",
                          f"-DCY_VOLUME_EXT={1 if kind == '_vext' else 0}",
                          f"-DCY_INTEGRATOR_EXT={1 if kind == '_ext' else 0}", inc,
                          "-c", "-o", obj, os.path.join(dev_dir, "k_shade.hip")], obj))
    # per-object staleness: the traversal file and the shading kernels share
    # the kernel headers but not each other's source
    shade_src = os.path.join(dev_dir, "k_shade.hip")
    def own_deps(obj):
        other = shade_src if obj.endswith("hipcycles.o") else src
        return [d for d in deps if d != other]

    jobs_run = jobs if (force or variant) else [j for j in jobs if _stale(j[1], own_deps(j[1]))]
    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs_run), os.cpu_count() or 1))) as ex:
        list(ex.map(lambda j: _run(j[0]), jobs_run))
    _run([HIPCC, "--offload-arch=gfx950", "-fno-gpu-rdc", "-shared", "-fPIC", "-o", out, *[j[1] for j in jobs],
          *shade_objs])
    return out


def build_host(force=False):
    srcs = [os.path.join(HERE, "csrc", "host", f) for f in ("bvh2_build.cpp", "light_background.cpp", "lookup_tables.cpp")]
    out = os.path.join(HERE, "libhipcycles_host.so")
    if force or _stale(out, srcs):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-o", out, *srcs])
    return out


def build_oracle(ref=True):
    oracle = os.path.join(REPO, "oracle")
    _run(["make", "-C", oracle, "oracle", "-j4"])
    if ref and os.path.isdir("/root/reference/blender/intern/cycles"):
        _run(["make", "-C", oracle, "ref", "ref-avx2", "sky", "ies", "-j4"])
        # the Device plugin linked with the reference host's device layer
        # (tests/test_plugin_harness.py; needs libhipcycles.so)
        _run(["bash", os.path.join(REPO, "tools", "plugin_harness.sh")])


def build_all(ref=True, force=False):
    build_host(force)
    if shutil.which(HIPCC) or os.path.exists(HIPCC):
        build_device(force)
    else:
        raise RuntimeError("hipcc not found: the HIP device library cannot be built")
    build_oracle(ref)


if __name__ == "__main__":
    if "--variant" in sys.argv:
        name = sys.argv[sys.argv.index("--variant") + 1]
        only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
        build_device(variant=name, defines=[a[2:] for a in sys.argv if a.startswith("-D")],
                     traversal_only="--traversal-only" in sys.argv, only=only)
    else:
        build_all(ref="--no-ref" not in sys.argv, force="--force" in sys.argv)
