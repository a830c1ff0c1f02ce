"""Benchmark: Msamples/s of the Cycles path-tracing hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config bmw27_standin]

One step = one full frame of the configured workload (BMW27 stand-in,
1280x720, 128 spp, BASELINE.json configs[1]) rendered by the HIP device from
camera rays to the render buffer, with the scene already resident in HBM.
With N ranks (torch.distributed.run, one process per GPU) the frame's rows are
interleaved across ranks (rank r renders rows r, r+N, ...): total work per step
is fixed, so scaling is "strong".  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_summary.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", default="bmw27_standin")
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--samples", type=int, default=None)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--save", default=None, help="write the rank-0 film as PNG")
    p.add_argument("--bvh-width", type=int, default=4, choices=(2, 4, 8),
                   help="4 (default) / 8: device-widened wide BVH; 2: the bound BVH2 as is")
    p.add_argument("--leaf-merge", type=int, default=0, help="wide BVH: merge subtrees of <= N prims")
    p.add_argument("--slots", type=int, default=0, help="path slots in flight (0: device default)")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (RCCL, one GPU per rank); gloo rehearses N ranks on fewer GPUs")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    device_index = local_rank
    if args.dist_backend == "gloo":
        device_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(device_index)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(backend=args.dist_backend, init_method="env://")

    from raytracingproject_amd import scene as sc
    from raytracingproject_amd import scenes
    from raytracingproject_amd.device import HIPDevice

    kw = {}
    if args.width:
        kw["width"] = args.width
    if args.height:
        kw["height"] = args.height
    if args.samples:
        kw["samples"] = args.samples
    scene = scenes.CONFIGS[args.config](**kw)
    t0 = time.time()
    ds = sc.compile_scene(scene)
    t_compile = time.time() - t0
    dev = HIPDevice(device_index)
    dev.set_bvh_width(args.bvh_width)
    dev.set_bvh_leaf_merge(args.leaf_merge)
    dev.set_slots(args.slots)
    t0 = time.time()
    dev.upload_scene(ds)
    dev.load_kernels()  # validates the scene and widens the BVH (scene preparation)
    t_upload = time.time() - t0

    from raytracingproject_amd.shard import RowShard

    W, H, S = ds.width, ds.height, ds.samples
    shard = RowShard(rank, world, W, H)
    rows = shard.rows
    buf = dev.mem_alloc(W * rows * ds.pass_stride * 4)

    def step():
        buf.zero()
        dev.render_tile(buf, shard.tile(), 0, S, shard.offset, shard.stride, y_step=shard.y_step)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    total_samples = W * H * S * args.steps
    value = total_samples / elapsed / 1e6

    # Roofline of the dominant kernel (one extra instrumented frame, outside the
    # timed region): HIP-event durations of every launch + traversal counters.
    dev.set_profiling(1)
    step()
    timing = dev.stats()
    dev.set_profiling(2)
    step()
    counts = dev.stats()
    dev.set_profiling(0)
    kernels = {
        "k_intersect_closest": timing["closest_ms"],
        "k_shade": timing["shade_ms"],
        "k_intersect_shadow": timing["intersect_ms"] - timing["closest_ms"],
    }
    launches = max(int(timing["closest_launches"]), 1)
    # algorithmic bytes of closest-hit traversal: 52 B per
    # triangle test (prim_tri_index + 3 verts) plus, for the BVH2, 64 B per
    # inner node and 16 B per leaf; for a W-wide BVH 32*W B per node (bounds,
    # children and the leaf ranges inline, no separate leaf fetch)
    width = int(counts["bvh_width"])
    if width > 2:
        closest_bytes = 32 * width * counts["closest_nodes"] + 52 * counts["closest_tris"]
    else:
        closest_bytes = 64 * counts["closest_nodes"] + 16 * counts["closest_leaves"] + 52 * counts["closest_tris"]
    bytes_per_launch = closest_bytes / launches
    avg_ms = timing["closest_ms"] / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    if os.path.exists(PMC_FILE):
        with open(PMC_FILE) as f:
            pmc = json.load(f)
        from raytracingproject_amd.build import kernel_source_digest

        if pmc.get("source_digest") == kernel_source_digest():
            traffic = pmc.get("k_intersect_closest", {}).get("hbm_bytes_per_launch")
    roofline = {
        "bound": "hbm",
        "kernel": "k_intersect_closest",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "bytes_per_launch": bytes_per_launch,
        "avg_launch_ms": avg_ms,
        "launches_per_frame": launches,
        "bvh_width": int(counts["bvh_width"]),
        "bvh_bytes": int(counts["bvh_bytes"]),
        "nodes_per_ray": counts["closest_nodes"] / max(counts["closest_rays"], 1),
        "tris_per_ray": counts["closest_tris"] / max(counts["closest_rays"], 1),
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(ds, args.cpu_seconds)

    if args.save and rank == 0:
        from raytracingproject_amd import imageio

        part = np.zeros((rows, W, ds.pass_stride), dtype=np.float32)
        step()
        buf.copy_from_device(part)
        imageio.write_png(args.save, imageio.film_readout(part, S)[..., :3])

    if rank == 0:
        out = {
            "metric": "Msamples/sec on BMW27 @1280x720, 128 spp",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural BMW27 stand-in scene, SURVEY.md §8(d))",
            "config": {
                "workload": f"{args.config} {W}x{H} {S} spp, one frame per step",
                "triangles": ds.info["triangles"],
                "parallelism": f"rows interleaved over {world} GPU(s)",
                "wavefront_iterations_per_frame": int(timing["iterations"]),
                "scene_compile_s": round(t_compile, 2),
                "scene_upload_s": round(t_upload, 3),
            },
            "kernel_ms_per_frame": {k: round(v, 3) for k, v in kernels.items()},
            "rays_per_frame": {"closest": counts["closest_rays"], "shadow": counts["shadow_rays"]},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    buf.free()
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(ds, seconds):
    """Reference Cycles CPU kernel (oracle/_ref, compiled from the reference
    sources) on a bounded sample of the same frame: all pixels at a reduced
    sample count, on the host cores this process may use."""
    try:
        from oracle.ref import RefKernel, ref_available
    except Exception:
        return None
    if not ref_available():
        return None
    threads = min(16, os.cpu_count() or 1)
    try:
        threads = min(threads, len(os.sched_getaffinity(0)))
    except Exception:
        pass
    rk = RefKernel(ds)
    t0 = time.perf_counter()
    rk.render(samples=1, threads=threads)
    t1 = time.perf_counter() - t0
    spp = int(max(1, min(ds.samples, seconds / max(t1, 1e-3))))
    t0 = time.perf_counter()
    rk.render(samples=spp, start_sample=1, threads=threads)
    dt = time.perf_counter() - t0
    rk.close()
    return {
        "value": round(ds.width * ds.height * spp / dt / 1e6, 4),
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "reference",
        "sample": f"{ds.width}x{ds.height} at {spp} spp (samples 1..{spp}) of the same scene, {dt:.1f} s",
    }


if __name__ == "__main__":
    main()
