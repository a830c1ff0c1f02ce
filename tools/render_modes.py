"""Measurement tool: render the bench frame in one of the device's modes, for
rocprofv3 kernel traces (tools/trace_gaps.py reads them back).

    python tools/render_modes.py frame|stream|shardN [--frames 3] [--lanes-note]

frame   the whole frame as one RenderTile (bench.py's headline step, no D2H)
stream  the frame's 64x64 RenderTiles fed to hipcy_render_feed, one frame buffer
shardN  rank 0's rows of an N-way interleaved row split (bench.py --gpus N)
Each frame is bracketed by hipDeviceSynchronize; prints one JSON line with
the wall time of every frame.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse

    import torch

    from raytracingproject_amd import scene as sc
    from raytracingproject_amd import scenes
    from raytracingproject_amd.device import HIPDevice
    from raytracingproject_amd.shard import RowShard

    p = argparse.ArgumentParser()
    p.add_argument("mode")
    p.add_argument("--frames", type=int, default=3)
    p.add_argument("--config", default="bmw27_standin")
    p.add_argument("--slots", type=int, default=0)
    p.add_argument("--tail", type=int, default=-1, help="hipcy_set_tail (-1: device default)")
    p.add_argument("--shadow-sort", type=int, default=0, help="hipcy_set_shadow_sort (0, 3, 5)")
    p.add_argument("--ray-sort", type=int, default=-1, help="hipcy_set_ray_sort (-1 automatic, 0, 3, 5, 8)")
    a = p.parse_args()
    ds = sc.compile_scene(scenes.CONFIGS[a.config]())
    dev = HIPDevice(0)
    dev.set_slots(a.slots)
    if a.tail >= 0:
        dev.set_tail(a.tail)
    dev.set_shadow_sort(a.shadow_sort)
    dev.set_ray_sort(a.ray_sort)
    dev.upload_scene(ds)
    dev.load_kernels()
    W, H, S, PS = ds.width, ds.height, ds.samples, ds.pass_stride
    shard = RowShard(0, int(a.mode[5:]), W, H) if a.mode.startswith("shard") else RowShard(0, 1, W, H)
    buf = torch.zeros((shard.rows, W, PS), dtype=torch.float32, device="cuda")

    class _Buf:
        ptr = buf.data_ptr()

    tiles = [(x, y, min(64, W - x), min(64, H - y)) for y in range(0, H, 64) for x in range(0, W, 64)]

    def frame():
        buf.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if a.mode == "stream":
            nxt = [0]

            def acquire():
                k = nxt[0]
                if k >= len(tiles):
                    return None
                nxt[0] += 1
                return tiles[k], 0, S, buf.data_ptr(), 0, W, k

            dev.render_feed(acquire, lambda k, t: None)
        else:
            dev.render_tile(_Buf, shard.tile(), 0, S, shard.offset, shard.stride, y_step=shard.y_step)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    times = [frame() for _ in range(a.frames)]
    st = dev.stats()
    print(json.dumps({"mode": a.mode, "tail": a.tail, "shadow_sort": a.shadow_sort, "ray_sort": a.ray_sort, "frame_ms": [round(1e3 * t, 3) for t in times],
                      "samples": shard.rows * W * S, "iterations": int(st["iterations"])}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
