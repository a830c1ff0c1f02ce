"""Measurement tool: per-frame GPU occupancy from a rocprofv3 kernel trace of
tools/render_modes.py.

    python tools/trace_gaps.py <run_kernel_trace.csv> [frames]

Frames are split at the render buffer's fill kernel (torch zero_) that starts
each frame.  For the last frame it prints the wall span (first to last kernel),
the union of kernel busy time (overlapping lanes counted once), the idle time
between them, and per kernel name the summed duration and launch count.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name[:70]


def main(path, nframes=None):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "FillFunctor" in r[2]]
    if not starts:
        starts = [0]
    frames = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(rows)
        frames.append(rows[s + 1:e])
    fr = frames[-1]
    t0, t1 = fr[0][0], max(r[1] for r in fr)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in fr:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = defaultdict(lambda: [0, 0])
    for s, e, n in fr:
        per[short(n)][0] += e - s
        per[short(n)][1] += 1
    print(f"frames {len(frames)}; last frame: span {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, "
          f"idle {(t1 - t0 - busy) / 1e6:.3f} ms, {len(fr)} launches")
    for n, (d, c) in sorted(per.items(), key=lambda x: -x[1][0]):
        print(f"  {d / 1e6:9.3f} ms {c:6d}  {n}")


if __name__ == "__main__":
    main(sys.argv[1])
