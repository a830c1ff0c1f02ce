"""Measurement tool: the per-lane iteration chain of one frame from a rocprofv3
kernel trace of tools/render_modes.py (where the frame's time goes when a
frame is small, e.g. shard8 = one eighth of the bench frame's rows).

    python tools/trace_iters.py <run_kernel_trace.csv>

For the last frame (split at torch's zero_ fill kernel) it lists every
traversal / shading dispatch in start order with its queue, grid size (active
paths rounded up to a block), start offset and duration, then per queue the
chain's sum of kernel time and the gaps between its kernels, and a histogram
of dispatch sizes against the time they took.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:48]


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            name = r["Kernel_Name"]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         "FillFunctor" if "FillFunctor" in name else short(name), q, g))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "FillFunctor" in r[2]]
    fr = rows[starts[-1] + 1:] if starts else rows
    fr = [r for r in fr if "rocclr" not in r[2]]
    t0 = fr[0][0]
    t1 = max(r[1] for r in fr)
    print(f"frame span {(t1 - t0) / 1e6:.3f} ms, {len(fr)} dispatches")
    per_q = defaultdict(list)
    for s, e, n, q, g in fr:
        per_q[q].append((s, e, n, g))
    for q, ks in sorted(per_q.items()):
        busy = sum(e - s for s, e, _, _ in ks)
        gaps = sum(max(0, ks[i + 1][0] - ks[i][1]) for i in range(len(ks) - 1))
        print(f"queue {q}: {len(ks)} dispatches, kernel {busy / 1e6:.3f} ms, gaps {gaps / 1e6:.3f} ms, "
              f"first {(ks[0][0] - t0) / 1e6:.3f} last end {(ks[-1][1] - t0) / 1e6:.3f} ms")
        for s, e, n, g in ks:
            print(f"    {(s - t0) / 1e3:9.1f} us {(e - s) / 1e3:8.1f} us grid {g:10d}  {n}")
    # dispatch size classes
    hist = defaultdict(lambda: [0, 0])
    for s, e, n, q, g in fr:
        if "intersect" not in n and "shade" not in n and "shadow" not in n:
            continue
        b = 1
        while b < g:
            b *= 4
        hist[b][0] += 1
        hist[b][1] += e - s
    print("dispatch grid <= : count, summed us (traversal + shading kernels)")
    for b in sorted(hist):
        print(f"  {b:10d}: {hist[b][0]:5d} {hist[b][1] / 1e3:10.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
