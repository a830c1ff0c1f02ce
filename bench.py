"""Benchmark: Msamples/s of the Cycles path-tracing hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config bmw27_standin]

One step = one full frame of the configured workload (BMW27 stand-in,
1280x720, 128 spp, BASELINE.json configs[1]) rendered by the HIP device from
camera rays to the film on the host: the render buffer is zeroed, every sample
is path traced, and the finished film is copied to host memory (with N ranks:
gathered to rank 0 over RCCL first), as BASELINE.md's render time ("until the
last tile's buffer is on the host") requires.  The scene is resident in HBM
before the timed region (scene compile / upload / BVH widening are reported
separately).

With --gpus N > 1 and no torch.distributed environment, bench.py starts N ranks
itself (torch.distributed.run, one process per GPU) before touching any GPU.
Rank r renders image rows r, r+N, r+2N, ... (raytracingproject_amd/shard.py):
total work per step is fixed, so scaling is "strong".  Rank 0 prints one JSON
line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_summary.json")


def parse(argv=None):
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
    p.add_argument("--ray-sort", type=int, default=-1, choices=(-1, 0, 3, 5, 8),
                   help="bin the closest queue by ray direction per bounce: 0 off, 3 octant, 5 octant x axis; "
                        "8: bin the shading queue by the hit's shader; -1 (default): the device's automatic "
                        "choice (8 for scenes on the extended shading kernel, else 0)")
    p.add_argument("--refill", type=int, nargs=2, default=(0, 16), metavar=("ROUNDS", "MIN_IDLE"),
                   help="lane refill of the closest-hit traversal (0 = off)")
    p.add_argument("--trav-budget", type=int, nargs=2, default=(0, 0), metavar=("FIRST", "SECOND"),
                   help="iteration budget of the wide traversal kernels (continuation launches); 0 0 disables")
    p.add_argument("--leaf-merge", type=int, default=0, help="wide BVH: merge subtrees of <= N prims")
    p.add_argument("--slots", type=int, default=0, help="path slots in flight (0: device default)")
    p.add_argument("--shadow-sort", type=int, default=0, choices=(0, 3, 5),
                   help="opaque-shadow queue sort by direction (hipcy_set_shadow_sort)")
    p.add_argument("--tail", type=int, default=-1,
                   help="fused tail threshold in live paths per lane (hipcy_set_tail; -1: device default, 0: off)")
    p.add_argument("--tile", type=int, default=64,
                   help="tile-mode leg: render one extra frame as TxT RenderTiles through the plugin path "
                        "(0 disables)")
    p.add_argument("--tile-batch", type=int, default=0,
                   help="tile-mode leg: 0 streams the tiles into one running wavefront (hipcy_render_feed, the "
                        "plugin's path); N > 0 renders N acquired tiles per device pass")
    p.add_argument("--stream-hold", type=int, default=0,
                   help="tile stream: pixel-samples the device may hold (0: device default)")
    p.add_argument("--render", default="frame", choices=("frame", "stream"),
                   help="frame: the whole frame as one RenderTile (headline); stream: the frame's --tile RenderTiles "
                        "fed to hipcy_render_feed (1 GPU; for profiling the plugin's path)")
    p.add_argument("--stream-hold-sweep", default="33554432",
                   help="comma-separated extra holds for more tile-stream legs (default: 2^25, the share the "
                        "plugin gives each of several devices on one queue)")
    p.add_argument("--profile-shard", type=int, default=1,
                   help="profiling only (N=1): the timed frame is rank 0's rows of an N-way row split")
    p.add_argument("--scaling-proxy", default="2,4,8",
                   help="single-GPU proxy of strong scaling (rank 0, N=1 only): for each N, rank 0's rows of an "
                        "N-way row split rendered alone and timed; empty disables")
    p.add_argument("--profile-frame", action="store_true",
                   help="only render the instrumented single-lane frame (for rocprofv3 PMC passes)")
    p.add_argument("--other-configs", default="bmw27_production,barbershop_standin,classroom_standin,junkshop_standin@1664x832+512x256",
                   help="BASELINE.json's other configs, one frame each after the headline measurement (rank 0, "
                        "N=1): name or name@XxY+WxH for a full-spp crop; empty disables")
    p.add_argument("--other-profile", action="store_true",
                   help="per-stage (closest / shade / shadow) times of each --other-configs frame")
    p.add_argument("--shard", default="auto", choices=("auto", "rows", "tiles"),
                   help="multi-GPU split: interleaved rows, or whole tiles per rank (auto: tiles for "
                        "adaptive-sampling scenes, whose filters run per RenderTile)")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (RCCL, one GPU per rank); gloo rehearses N ranks on fewer GPUs")
    return p.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """Start N ranks (one process per GPU) and return the launcher's exit code.
    Runs before anything in this process touches a GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
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
    from raytracingproject_amd.shard import RowShard, TileShard, assemble_tiles

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
    dev.set_ray_sort(args.ray_sort)
    dev.set_shadow_sort(args.shadow_sort)
    dev.set_traversal_budget(*args.trav_budget)
    dev.set_traversal_refill(*args.refill)
    dev.set_slots(args.slots)
    if args.tail >= 0:
        dev.set_tail(args.tail)
    t0 = time.time()
    dev.upload_scene(ds)
    dev.load_kernels()  # validates the scene and widens the BVH (scene preparation)
    t_upload = time.time() - t0

    W, H, S, PS = ds.width, ds.height, ds.samples, ds.pass_stride
    shard = RowShard(rank, world, W, H)
    rows_pad = -(-H // world)  # every rank's buffer has the same size for the gather
    if args.profile_shard > 1 and world == 1:
        shard = RowShard(0, args.profile_shard, W, H)
        rows_pad = shard.rows
    use_tiles = args.shard == "tiles" or (args.shard == "auto" and world > 1 and
                                           bool(ds.data.film.pass_adaptive_aux_buffer))
    if use_tiles:
        # whole tiles per rank, full-frame buffers (shard.TileShard)
        tile_size = args.tile if args.tile > 0 else 64
        tshards = [TileShard(r, world, W, H, tile_size) for r in range(world)]
        rows_pad = H
    cuda = torch.device("cuda", device_index)
    # render buffer: a torch allocation handed to the device as a raw pointer
    # (RenderTile.buffer), so the gather can run over RCCL without a copy
    local = torch.zeros((rows_pad, W, PS), dtype=torch.float32, device=cuda)
    gather_gpu = args.dist_backend == "nccl"
    if world > 1:
        gathered = torch.empty((world, rows_pad, W, PS), dtype=torch.float32,
                               device=cuda if gather_gpu else "cpu")
    film_host = torch.empty((H, W, PS), dtype=torch.float32, pin_memory=True) if rank == 0 else None

    class _Buf:  # the DeviceBuffer interface render_tile needs
        ptr = local.data_ptr()

    stream_tiles = [(x, y, min(args.tile or 64, W - x), min(args.tile or 64, H - y))
                    for y in range(0, H, args.tile or 64) for x in range(0, W, args.tile or 64)]

    def render_frame():
        local.zero_()
        torch.cuda.current_stream().synchronize()
        if args.render == "stream":
            # the frame's RenderTiles streamed into one wavefront (the plugin's path)
            nxt = [0]

            def acquire():
                k = nxt[0]
                if k >= len(stream_tiles):
                    return None
                nxt[0] += 1
                return stream_tiles[k], 0, S, _Buf.ptr, 0, W, k

            dev.render_feed(acquire, lambda k, t: None, hold=args.stream_hold)
        elif use_tiles:
            ts = tshards[rank]
            dev.render_tiles([(t, _Buf.ptr, ts.offset, ts.stride) for t in ts.tiles()], 0, S)
        else:
            dev.render_tile(_Buf, shard.tile(), 0, S, shard.offset, shard.stride, y_step=shard.y_step)

    def film_to_host():
        """Finished film to rank 0's host memory (gather of the row-interleaved parts)."""
        if world == 1:
            film_host[:rows_pad].copy_(local[:H])
            return
        if use_tiles:
            dist.all_gather_into_tensor(gathered.view(-1), (local if gather_gpu else local.cpu()).view(-1))
            if rank == 0:
                parts = [gathered[r].cpu().numpy() for r in range(world)]
                film_host.copy_(torch.from_numpy(assemble_tiles(parts, tshards)))
            return
        if gather_gpu:
            dist.all_gather_into_tensor(gathered.view(-1), local.view(-1))
            if rank == 0:
                full = gathered.transpose(0, 1).reshape(rows_pad * world, W, PS)[:H]
                film_host.copy_(full)
        else:
            dist.all_gather_into_tensor(gathered.view(-1), local.cpu().view(-1))
            if rank == 0:
                film_host.copy_(gathered.transpose(0, 1).reshape(rows_pad * world, W, PS)[:H])

    def step():
        render_frame()
        film_to_host()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    if args.profile_frame:
        dev.set_profiling(1)
        render_frame()
        torch.cuda.synchronize()
        st = dev.stats()
        if rank == 0:
            print(json.dumps({"profile_frame": True, "closest_ms": st["closest_ms"],
                              "closest_launches": st["closest_launches"]}), flush=True)
        dev.close()
        if dist is not None:
            dist.destroy_process_group()
        return

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
        t = torch.tensor([elapsed], dtype=torch.float64, device=cuda if gather_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    total_samples = W * (shard.rows if (args.profile_shard > 1 and world == 1) else H) * S * args.steps
    value = total_samples / elapsed / 1e6
    film = film_host.numpy().copy() if rank == 0 else None

    # Roofline of the dominant kernel (extra instrumented frames, outside the
    # timed region): HIP-event durations of every launch on a single lane (no
    # overlap), then the traversal counters.
    dev.set_profiling(1)
    render_frame()
    timing = dev.stats()
    dev.set_profiling(2)
    render_frame()
    counts = dev.stats()
    dev.set_profiling(0)
    kernels = {
        "k_intersect_closest": timing["closest_ms"],
        "k_shade": timing["shade_ms"],
        "k_intersect_shadow": timing["shadow_ms"],
    }
    roofline = traversal_roofline(timing, counts)

    tile_leg = None
    if args.tile > 0 and world == 1:
        # the plugin's behaviour (integration/device_hip.cpp: the session's tiles
        # streamed into one running wavefront, at most `hold` pixel-samples held)
        # and, for comparison, one tile per device pass
        tile_leg = [tile_mode(dev, ds, args.tile, args.tile_batch, args.stream_hold, film)]
        if args.tile_batch == 0:
            # the same stream with the tiles in one frame buffer, released without a copy:
            # the device side of the stream alone (no per-tile D2H in Python callbacks)
            tile_leg.append(tile_mode(dev, ds, args.tile, 0, args.stream_hold, film, frame_buffer=True))
        for extra in (args.stream_hold_sweep or "").split(","):
            if extra:
                tile_leg.append(tile_mode(dev, ds, args.tile, 0, int(extra), film))
        if args.tile_batch != 1:
            tile_leg.append(tile_mode(dev, ds, args.tile, 1, 0, film))

    proxy = None
    if world == 1 and args.scaling_proxy:
        proxy = scaling_proxy(dev, ds, [int(n) for n in args.scaling_proxy.split(",") if n], value)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(ds, args.cpu_seconds)

    others = None
    if rank == 0 and world == 1 and args.other_configs:
        del local
        dev.close()
        local, dev = None, None
        others = [other_config(spec, device_index, args) for spec in args.other_configs.split(",") if spec]

    if args.save and rank == 0:
        from raytracingproject_amd import imageio

        imageio.write_png(args.save, imageio.film_readout(film, S)[..., :3])

    if rank == 0:
        rays = counts["closest_rays"] + counts["shadow_rays"]
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
                "workload": f"{args.config} {W}x{H} {S} spp, one frame per step, film copied to host",
                "triangles": ds.info["triangles"],
                "parallelism": (f"{tile_size}x{tile_size} tiles dealt over {world} GPU(s)" if use_tiles
                                else f"rows interleaved over {world} GPU(s)"),
                "wavefront_iterations_per_frame": int(timing["iterations"]),
                "ray_sort": args.ray_sort,
                "shadow_sort": args.shadow_sort,
                "traversal_budget": list(args.trav_budget),
                "traversal_refill": list(args.refill),
                "scene_compile_s": round(t_compile, 2),
                "scene_upload_s": round(t_upload, 3),
            },
            "kernel_ms_per_frame": {k: round(v, 3) for k, v in kernels.items()},
            "rays_per_frame": {"closest": counts["closest_rays"], "shadow": counts["shadow_rays"],
                               "near_tie_retraced": counts["tie_rays"]},
            "mrays_per_s": round(rays * world * args.steps / elapsed / 1e6, 1),
            "film_checksum": float(np.float64(film[..., :4].sum())) if film is not None else None,
            "roofline": roofline,
            "tile_mode": tile_leg,
            "scaling_proxy": proxy,
            "other_configs": others,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    del local
    if dev is not None:
        dev.close()
    if dist is not None:
        dist.destroy_process_group()


def traversal_bytes(width, nodes, leaves, tris):
    """Algorithmic bytes of traversal: 52 B per triangle test
    (prim_tri_index + 3 verts) plus, for the BVH2, 64 B per inner node and 16 B
    per leaf; for a W-wide BVH 32*W B per node (bounds, children and the leaf
    ranges inline, no separate leaf fetch)."""
    if width > 2:
        return 32 * width * nodes + 52 * tris
    return 64 * nodes + 16 * leaves + 52 * tris


def traversal_roofline(timing, counts):
    """HBM roofline of the traversal kernels as BASELINE.md defines it: the
    algorithmic bytes of every closest-hit and shadow ray of the instrumented
    frame over the summed HIP-event time of both traversal kernels (each launch
    timed alone on one lane).  Per-kernel figures beside it; the shadow kernel's
    time also holds its finish / refill work."""
    width = int(counts["bvh_width"])
    launches = max(int(timing["closest_launches"]), 1)
    c_bytes = traversal_bytes(width, counts["closest_nodes"], counts["closest_leaves"], counts["closest_tris"])
    s_bytes = traversal_bytes(width, counts["shadow_nodes"], counts["leaves"] - counts["closest_leaves"],
                              counts["shadow_tris"])
    c_ms, s_ms = timing["closest_ms"], timing["shadow_ms"]

    def gbs(b, ms):
        return b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0

    def util(lane, wave):
        return round(lane / (64.0 * wave), 4) if wave else None

    achieved = gbs(c_bytes + s_bytes, c_ms + s_ms)
    traffic, pmc_note = None, None
    if os.path.exists(PMC_FILE):
        with open(PMC_FILE) as f:
            pmc = json.load(f)
        from raytracingproject_amd.build import kernel_source_digest

        if pmc.get("source_digest") == kernel_source_digest():
            ents = [pmc.get(k, {}) for k in ("k_intersect_closest", "k_intersect_shadow")]
            if all(e.get("hbm_bytes_per_launch") is not None for e in ents):
                traffic = sum(e["hbm_bytes_per_launch"] for e in ents)
            pmc_note = {k: {f: pmc.get(k, {}).get(f) for f in ("instance", "dispatches", "rocprof_avg_ms", "l2_hit_rate",
                                                            "hbm_read_bytes_per_launch", "hbm_write_bytes_per_launch",
                                                            "hbm_bytes_per_launch")}
                        for k in ("k_intersect_closest", "k_intersect_shadow")}
        else:
            pmc_note = "profiles/pmc_summary.json was measured on other kernel sources"
    return {
        "bound": "hbm",
        "kernel": "BVH traversal: k_intersect_closest + k_intersect_shadow (one launch of each per wavefront iteration)",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_source": pmc_note,
        "bytes_per_launch": (c_bytes + s_bytes) / launches,
        "avg_launch_ms": (c_ms + s_ms) / launches,
        "launches_per_frame": launches,
        "bvh_width": width,
        "bvh_bytes": int(counts["bvh_bytes"]),
        "per_kernel": {
            "k_intersect_closest": {
                "bytes_per_launch": c_bytes / launches, "avg_launch_ms": c_ms / launches,
                "achieved": round(gbs(c_bytes, c_ms), 2), "frac": round(gbs(c_bytes, c_ms) / HBM_PEAK_GBS, 4),
                "nodes_per_ray": counts["closest_nodes"] / max(counts["closest_rays"], 1),
                "tris_per_ray": counts["closest_tris"] / max(counts["closest_rays"], 1),
                "lane_utilisation": util(counts["closest_lane_iters"], counts["closest_wave_iters"]),
                "iters_per_wave": counts["closest_wave_iters"] / max(counts["closest_rays"] / 64.0, 1),
            },
            "k_intersect_shadow": {
                "bytes_per_launch": s_bytes / launches, "avg_launch_ms": s_ms / launches,
                "achieved": round(gbs(s_bytes, s_ms), 2), "frac": round(gbs(s_bytes, s_ms) / HBM_PEAK_GBS, 4),
                "nodes_per_ray": counts["shadow_nodes"] / max(counts["shadow_rays"], 1),
                "tris_per_ray": counts["shadow_tris"] / max(counts["shadow_rays"], 1),
                "lane_utilisation": util(counts["shadow_lane_iters"], counts["shadow_wave_iters"]),
            },
        },
    }


def tile_mode(dev, ds, tile, batch, hold=0, film=None, frame_buffer=False):
    """One frame rendered the way a Cycles Session drives a device: the frame
    split into tile x tile RenderTiles (session.h:84 default 64) acquired in
    row order, each rendered over all its samples into its own buffer
    (background mode) and copied to the host when the device releases it.
    batch 0: the tiles are streamed into one running wavefront that never holds
    more than `hold` pixel-samples (hipcy_render_feed, what the plugin does);
    batch N: N acquired tiles per device pass.  Reported beside the whole-frame
    number (with whether the tiles reassemble to its film bit for bit); not
    the headline value.  frame_buffer: every tile renders into one frame
    buffer at its offset (a Session's single RenderBuffers) and its release
    does nothing; the film is copied once at the end."""
    import torch

    W, H, S, PS = ds.width, ds.height, ds.samples, ds.pass_stride
    tiles = [(x, y, min(tile, W - x), min(tile, H - y)) for y in range(0, H, tile) for x in range(0, W, tile)]
    if frame_buffer:
        fbuf = torch.zeros((H, W, PS), dtype=torch.float32, device="cuda")
        fhost = torch.empty((H, W, PS), dtype=torch.float32, pin_memory=True)

        def fb_frame():
            fbuf.zero_()
            torch.cuda.current_stream().synchronize()
            nxt = [0]

            def acquire():
                k = nxt[0]
                if k >= len(tiles):
                    return None
                nxt[0] += 1
                return tiles[k], 0, S, fbuf.data_ptr(), 0, W, k

            dev.render_feed(acquire, lambda k, t: None, hold=hold)
            fhost.copy_(fbuf)

        fb_frame()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fb_frame()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res = {"tile": tile, "tiles": len(tiles), "mode": "stream into one frame buffer, film copied once",
               "value": round(W * H * S / dt / 1e6, 3), "unit": "Msamples/s", "ms_per_frame": round(1e3 * dt, 3),
               "hold_pixel_samples": hold or "device default: the slot pool in flight plus as much in reserve",
               "wavefront_iterations": int(dev.stats()["iterations"])}
        if film is not None:
            res["film_bit_exact_vs_whole_frame"] = bool(np.array_equal(fhost.numpy().view(np.uint32),
                                                                       film.view(np.uint32)))
        del fbuf, fhost
        return res
    bufs = [torch.zeros((t[3], t[2], PS), dtype=torch.float32, device="cuda") for t in tiles]
    # each released tile goes to pinned host memory on a copy stream, without
    # blocking the device's render thread (Session::release_tile's buffer copy)
    host = [torch.empty((t[3], t[2], PS), dtype=torch.float32, pin_memory=True) for t in tiles]
    copy_stream = torch.cuda.Stream()
    batch = max(batch, 0)

    def frame():
        for b in bufs:
            b.zero_()
        torch.cuda.current_stream().synchronize()
        if batch == 0:
            nxt = [0]

            def acquire():
                k = nxt[0]
                if k >= len(tiles):
                    return None
                nxt[0] += 1
                t = tiles[k]
                return t, 0, S, bufs[k].data_ptr(), -(t[0] + t[1] * t[2]), t[2], k

            def release(k, _):
                with torch.cuda.stream(copy_stream):
                    host[k].copy_(bufs[k], non_blocking=True)

            dev.render_feed(acquire, release, hold=hold)
        else:
            for i in range(0, len(tiles), batch):
                group = [(t, b.data_ptr(), -(t[0] + t[1] * t[2]), t[2]) for t, b in zip(tiles[i:i + batch],
                                                                                        bufs[i:i + batch])]
                dev.render_tiles(group, 0, S)
                with torch.cuda.stream(copy_stream):
                    for k in range(i, min(i + batch, len(tiles))):
                        host[k].copy_(bufs[k], non_blocking=True)
        copy_stream.synchronize()

    frame()  # warm (pools and records are sized on first use)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frame()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"tile": tile, "tiles": len(tiles), "mode": "stream" if batch == 0 else f"{batch} tile(s) per pass",
           "value": round(W * H * S / dt / 1e6, 3), "unit": "Msamples/s", "ms_per_frame": round(1e3 * dt, 3)}
    if batch == 0:
        res["hold_pixel_samples"] = hold or "device default: the slot pool in flight plus as much in reserve"
        st = dev.stats()
        res["wavefront_iterations"] = int(st["iterations"])
    if film is not None:
        full = np.zeros((H, W, PS), dtype=np.float32)
        for (x, y, w, h), b in zip(tiles, host):
            full[y:y + h, x:x + w] = b.numpy()
        res["film_bit_exact_vs_whole_frame"] = bool(np.array_equal(full.view(np.uint32), film.view(np.uint32)))
    return res


def scaling_proxy(dev, ds, ns, full_value, frames=3):
    """Per-GPU throughput at 1/N of the frame, measured on this one GPU: rank
    0's rows of an N-way interleaved row split (shard.RowShard, what
    `bench.py --gpus N` gives each rank) rendered alone, `frames` timed frames
    after a warm one, the film copied to the host as in the headline step.
    Strong scaling at N GPUs cannot exceed N x this rate / the full-frame rate
    (the ratio reported as `per_gpu_vs_full`); the rows of the other ranks cost
    the same within a few per cent (every rank gets every N-th row)."""
    import torch

    from raytracingproject_amd.shard import RowShard

    W, H, S, PS = ds.width, ds.height, ds.samples, ds.pass_stride
    out = {}
    for n in ns:
        if n < 2:
            continue
        sh = RowShard(0, n, W, H)
        buf = torch.zeros((sh.rows, W, PS), dtype=torch.float32, device="cuda")
        host = torch.empty((sh.rows, W, PS), dtype=torch.float32, pin_memory=True)

        class _Buf:
            ptr = buf.data_ptr()

        def frame():
            buf.zero_()
            dev.render_tile(_Buf, sh.tile(), 0, S, sh.offset, sh.stride, y_step=sh.y_step)
            host.copy_(buf)

        frame()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            frame()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / frames
        per_gpu = sh.rows * W * S / dt / 1e6
        out[str(n)] = {"rows": sh.rows, "ms_per_frame": round(1e3 * dt, 3), "per_gpu_value": round(per_gpu, 3),
                       "per_gpu_vs_full": round(per_gpu / full_value, 4),
                       "wavefront_iterations": int(dev.stats()["iterations"])}
        del buf, host
    return {"unit": "Msamples/s", "method": "rank 0's rows of an N-way row split on one GPU", "legs": out}


def other_config(spec, device_index, args):
    """One frame of another BASELINE.json config (its procedural stand-in,
    SURVEY.md §8(d)) on this GPU: `name` renders the whole frame at its full
    sample count, `name@XxY+WxH` the crop (x, y, w, h) at the full sample
    count (configs whose frame takes minutes).  A 1-sample frame first sizes
    the device; then one timed frame.  Failures are reported, not raised."""
    import torch

    from raytracingproject_amd import scene as sc
    from raytracingproject_amd import scenes
    from raytracingproject_amd.device import HIPDevice

    name, _, region = spec.partition("@")
    res = {"config": name}
    dev = None
    try:
        t0 = time.time()
        ds = sc.compile_scene(scenes.CONFIGS[name]())
        res["scene_compile_s"] = round(time.time() - t0, 2)
        W, H, S, PS = ds.width, ds.height, ds.samples, ds.pass_stride
        x, y, w, h = 0, 0, W, H
        if region:
            pos, _, size = region.partition("+")
            x, y = (int(v) for v in pos.split("x"))
            w, h = (int(v) for v in size.split("x"))
        dev = HIPDevice(device_index)
        dev.set_bvh_width(args.bvh_width)
        dev.set_ray_sort(args.ray_sort)
        dev.set_shadow_sort(args.shadow_sort)
        if args.tail >= 0:
            dev.set_tail(args.tail)
        dev.upload_scene(ds)
        dev.load_kernels()
        buf = torch.zeros((h, w, PS), dtype=torch.float32, device=torch.device("cuda", device_index))

        class _Buf:
            ptr = buf.data_ptr()

        dev.render_tile(_Buf, (x, y, w, h), 0, 1, -(x + y * w), w)
        torch.cuda.synchronize()
        buf.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.render_tile(_Buf, (x, y, w, h), 0, S, -(x + y * w), w)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.update({"frame": f"{W}x{H} {S} spp", "region": [x, y, w, h],
                    "value": round(w * h * S / dt / 1e6, 3), "unit": "Msamples/s", "ms": round(1e3 * dt, 1),
                    "film_checksum": float(buf[..., :4].double().sum().item())})
        if args.other_profile:
            # one more frame with per-stage HIP events (lanes serialised, so
            # the stage times add up to more than the timed frame)
            dev.set_profiling(1)
            buf.zero_()
            dev.render_tile(_Buf, (x, y, w, h), 0, S, -(x + y * w), w)
            torch.cuda.synchronize()
            st = dev.stats()
            res["stages_ms"] = {k: round(float(st[k]), 1) for k in ("closest_ms", "shade_ms", "shadow_ms", "total_ms")}
            dev.set_profiling(0)
        del buf
    except Exception as e:  # reported beside the headline, never fatal
        res["error"] = f"{type(e).__name__}: {e}"[:300]
    finally:
        if dev is not None:
            dev.close()
    return res


def cpu_baseline(ds, seconds):
    """Reference Cycles CPU kernel (oracle/_ref, compiled from the reference
    sources; the AVX2 build when the host has AVX2, as stock Blender selects it,
    device/device_cpu.cpp:76-134) on a bounded sample of the same frame: all
    pixels at a reduced sample count, on the host cores this process may use
    (the GPU box grants 16 cores per GPU)."""
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
    rk = RefKernel(ds, fast=True)
    t0 = time.perf_counter()
    rk.render(samples=1, threads=threads)
    t1 = time.perf_counter() - t0
    spp = int(max(1, min(ds.samples, seconds / max(t1, 1e-3))))
    t0 = time.perf_counter()
    rk.render(samples=spp, start_sample=1, threads=threads)
    dt = time.perf_counter() - t0
    arch = rk.arch
    rk.close()
    return {
        "value": round(ds.width * ds.height * spp / dt / 1e6, 4),
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "reference",
        "sample": f"{ds.width}x{ds.height} at {spp} spp (samples 1..{spp}) of the same scene, {dt:.1f} s, "
                  f"reference CPU kernel ({arch})",
    }


if __name__ == "__main__":
    main()
