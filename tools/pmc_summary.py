"""Reduce the rocprofv3 outputs of tools/gpu_prof.sh into profiles/.

    python tools/pmc_summary.py r01

Reads gpurun_out/{trace,pmc_*}_<tag>/ and writes
  profiles/rocprof_<tag>_kernel_stats.csv   (the --kernel-trace --stats summary)
  profiles/pmc_<tag>.csv                    (per-kernel mean of every counter)
  profiles/pmc_summary.json                 (what bench.py reads for `traffic`)

HBM bytes follow MI355X_MICROARCH.md §HBM/rocprofv3: FETCH_SIZE (KiB) is
TCC_EA0_RDREQ x 64 B while every request moves a 128-B line, so the read
bytes are 2 x FETCH_SIZE; WRITE_SIZE is taken as is.  The summary records
the source-tree digest it was measured on, so bench.py ignores it once the
kernels change.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raytracingproject_amd.build import kernel_source_digest  # noqa: E402


def kernel_means(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main(tag):
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(out, f"trace_{tag}", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"rocprof_{tag}_kernel_stats.csv"))
    durations = {}
    for r in csv.DictReader(open(stats)):
        name = r["Name"].split("(")[0].replace("void ", "")
        durations[name] = float(r["AverageNs"]) / 1e6

    means = collections.defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(out, f"pmc_*_{tag}"))):
        for k, cs in kernel_means(os.path.join(d, "run_counter_collection.csv")).items():
            means[k].update(cs)
    counters = sorted({c for cs in means.values() for c in cs})
    with open(os.path.join(prof, f"pmc_{tag}.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel"] + counters)
        for k in sorted(means):
            w.writerow([k] + [round(means[k].get(c, float("nan")), 1) for c in counters])

    summary = {"tag": tag, "source_digest": kernel_source_digest(), "unit": "bytes per launch",
               "method": "reads = 2 x FETCH_SIZE(KiB) x 1024 (gfx950 128-B lines tallied at 64 B), "
                         "writes = WRITE_SIZE(KiB) x 1024"}
    for k, cs in means.items():
        if "FETCH_SIZE" not in cs or "rocclr" in k:
            continue
        rd = 2.0 * cs["FETCH_SIZE"] * 1024.0
        wr = cs.get("WRITE_SIZE", 0.0) * 1024.0
        ent = {"hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": rd + wr}
        if "TCC_HIT_sum" in cs:
            ent["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"], 1.0)
        if "SQ_WAVE_CYCLES" in cs:
            ent["wait_any_frac"] = cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"]
            ent["active_frac"] = cs["SQ_ACTIVE_INST_ANY"] / cs["SQ_WAVE_CYCLES"]
        for dk, ms in durations.items():
            if dk == k:
                ent["rocprof_avg_ms"] = ms
        summary[k] = ent
    # bench.py's name for the dominant kernel: the instance without counters
    # (k_intersect_closest<false, W>) of the BVH width that was profiled
    for k in sorted(summary):
        if k.startswith("k_intersect_closest<false"):
            summary["k_intersect_closest"] = dict(summary[k], instance=k)
    with open(os.path.join(prof, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary.get("k_intersect_closest", {}), indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
