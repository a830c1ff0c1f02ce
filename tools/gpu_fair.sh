#!/bin/bash
# fairness of two plugin devices on one queue at several holds (one GPU)
cd "${GRAFT_REPO_ROOT:-.}"
python - <<'PY'
import os, sys, subprocess, tempfile
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from parity_cases import FULL_DIGEST_CASES
from raytracingproject_amd import scene as sc
from test_plugin_harness import write_scene_dir, HARNESS
ds = sc.compile_scene(FULL_DIGEST_CASES["bmw"]())
d = tempfile.mkdtemp()
write_scene_dir(ds, d)
for hold in ["8388608", "16777216", "33554432"]:
    env = dict(os.environ, CYCLES_HIPCY_STREAM_HOLD=hold)
    r = subprocess.run([HARNESS, d, "1280", "720", "128", "64", str(ds.pass_stride), d + "/f.bin", "2"],
                       capture_output=True, text=True, timeout=300, env=env)
    print("hold", hold, r.returncode, [l for l in r.stdout.splitlines() if "device " in l and "tiles" in l], flush=True)
PY
