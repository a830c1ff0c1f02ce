"""Tile-sharded multi-GPU rendering of an adaptive-sampling scene
(shard.TileShard): adaptive stopping and the x/y dilation filters run per
RenderTile, so ranks own whole tiles instead of interleaved rows.  Each
simulated rank renders its tiles in one hipcy_path_trace_tiles pass into a
full-frame buffer; the assembled frame must equal the reference CPU device's
tile-by-tile adaptive render (tests/golden/cornell_adaptive_tiles24.npz) bit
for bit, for any number of ranks."""
import numpy as np
import pytest

from parity_cases import HOST_LOOP_CASES, compile_case, load_golden, scene_digest
from raytracingproject_amd.shard import TileShard, assemble_tiles

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [1, 2, 3])
def test_adaptive_tile_shards_match_reference(world):
    from raytracingproject_amd.device import HIPDevice

    name = sorted(HOST_LOOP_CASES)[0]
    g = load_golden(f"{name}_tiles24")
    ds = compile_case(name)
    assert scene_digest(ds) == str(g["digest"])
    tile = int(g["tile"])
    dev = HIPDevice(0)
    try:
        dev.upload_scene(ds)
        parts, shards = [], []
        for rank in range(world):
            sh = TileShard(rank, world, ds.width, ds.height, tile)
            buf = dev.mem_alloc(ds.width * ds.height * ds.pass_stride * 4)
            buf.zero()
            dev.render_tiles([(t, buf, sh.offset, sh.stride) for t in sh.tiles()], 0, ds.samples)
            part = np.zeros((ds.height, ds.width, ds.pass_stride), dtype=np.float32)
            buf.copy_from_device(part)
            buf.free()
            parts.append(part)
            shards.append(sh)
        out = assemble_tiles(parts, shards)
    finally:
        dev.close()
    assert np.array_equal(out.view(np.uint32), g["buffer"].view(np.uint32))
