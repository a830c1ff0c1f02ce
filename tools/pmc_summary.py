"""Reduce the rocprofv3 outputs of tools/gpu_prof.sh into profiles/.

    python tools/pmc_summary.py r02

Reads gpurun_out/{trace,trace_frame,pmc_*}_<tag>/ and writes
  profiles/<tag>/rocprof_kernel_stats.csv        (--kernel-trace --stats of the bench run)
  profiles/<tag>/rocprof_frame_kernel_stats.csv  (the same for the instrumented frame alone)
  profiles/<tag>/pmc_counters.csv                (per-dispatch counters of the instrumented frame)
  profiles/<tag>/pmc.csv                         (per-kernel sum / dispatches of every counter)
  profiles/pmc_summary.json                      (what bench.py reads for `traffic`)

Normalisation (the unit of bench.py's roofline.bytes_per_launch): every PMC
pass runs `bench.py --profile-frame`, i.e. ONE instrumented frame whose
kernels run on a single lane (no overlap) — the same frame bench.py divides
its algorithmic bytes by.  A counter per launch is its SUM over all dispatches
of one kernel instance in that run divided by the number of those dispatches;
the instance and dispatch count are recorded.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) is TCC_EA0_RDREQ
x 64 B while every request moves a 128-B line, so read bytes = 2 x FETCH_SIZE;
WRITE_SIZE is taken as is.  The summary records the source-tree digest it was
measured on, so bench.py ignores it once the kernels change.
"""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raytracingproject_amd.build import kernel_source_digest  # noqa: E402


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").strip()


def kernel_sums(path, rows_out=None):
    """{kernel: {counter: sum over dispatches}}, {kernel: dispatch ids}."""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        if rows_out is not None:
            rows_out.append((k, r["Dispatch_Id"], r["Counter_Name"], r["Counter_Value"]))
    return acc, disp


def stats_avg_ms(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[short(r["Name"])] = (float(r["AverageNs"]) / 1e6, int(r["Calls"]))
    return out


def main(tag):
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles", tag)
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(out, f"trace_{tag}", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, "rocprof_kernel_stats.csv"))
    fstats = os.path.join(out, f"trace_frame_{tag}", "run_kernel_stats.csv")
    frame_ms = {}
    if os.path.exists(fstats):
        shutil.copy(fstats, os.path.join(prof, "rocprof_frame_kernel_stats.csv"))
        frame_ms = stats_avg_ms(fstats)

    sums = collections.defaultdict(dict)
    ndisp = {}
    rows = []
    for name in sorted(os.listdir(out)):
        if not (name.startswith("pmc_") and name.endswith("_" + tag)):
            continue
        path = os.path.join(out, name, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        acc, disp = kernel_sums(path, rows)
        for k, cs in acc.items():
            sums[k].update(cs)
            n = len(disp[k])
            if k in ndisp and ndisp[k] != n:
                raise SystemExit(f"{k}: {n} dispatches in {name}, {ndisp[k]} in another pass")
            ndisp[k] = n
    with open(os.path.join(prof, "pmc_counters.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatch_id", "counter", "value"])
        w.writerows(rows)
    counters = sorted({c for cs in sums.values() for c in cs})
    with open(os.path.join(prof, "pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches"] + counters)
        for k in sorted(sums):
            w.writerow([k, ndisp[k]] + [round(sums[k][c] / ndisp[k], 1) if c in sums[k] else "" for c in counters])

    summary = {"tag": tag, "source_digest": kernel_source_digest(), "unit": "bytes per launch",
               "normalisation": "sum over the dispatches of one kernel instance in the instrumented "
                                "frame (bench.py --profile-frame, single lane) / that dispatch count",
               "method": "reads = 2 x FETCH_SIZE(KiB) x 1024 (gfx950 128-B lines tallied at 64 B), "
                         "writes = WRITE_SIZE(KiB) x 1024"}
    for k, cs in sums.items():
        if "FETCH_SIZE" not in cs or "rocclr" in k:
            continue
        n = ndisp[k]
        rd = 2.0 * cs["FETCH_SIZE"] * 1024.0 / n
        wr = cs.get("WRITE_SIZE", 0.0) * 1024.0 / n
        ent = {"dispatches": n, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": rd + wr}
        if "TCC_HIT_sum" in cs:
            ent["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"], 1.0)
        if "SQ_WAVE_CYCLES" in cs:
            ent["wait_any_frac"] = cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"]
            ent["active_frac"] = cs["SQ_ACTIVE_INST_ANY"] / cs["SQ_WAVE_CYCLES"]
        if k in frame_ms:
            ent["rocprof_avg_ms"], ent["rocprof_calls"] = frame_ms[k]
        summary[k] = ent
    # bench.py's name for the dominant kernel: the instance without counters
    # (k_intersect_closest<false, W, I>); the profiled frame runs exactly one
    # and the same for the opaque-shadow traversal (BASELINE.md's roofline
    # covers both traversal kernels)
    for base in ("k_intersect_closest", "k_intersect_shadow"):
        inst = sorted(k for k in summary if k.startswith(base + "<false"))
        if len(inst) != 1:
            raise SystemExit(f"expected one timed {base} instance, found {inst}")
        summary[base] = dict(summary[inst[0]], instance=inst[0])
    with open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary["k_intersect_closest"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
