"""Multi-GPU partition of one frame: rows interleaved over ranks, or (for
adaptive sampling, whose stopping and dilation filters run per RenderTile)
whole tiles dealt to ranks.

The reference splits a frame into tiles that all devices pull from one
TileManager queue (render/tile.cpp:498-557, device/device_multi.cpp:689-737).
Here the split is static and finer: rank r owns image rows r, r+W, r+2W, ...
(W = world size), so every rank gets the same mix of cheap sky rows and
expensive car rows and no work queue or exchange step is needed.  Each rank
renders its rows into a compact local buffer (local row j = image row
r + j*W) through hipcy_path_trace_rows(tile, y_step=W); there is no collective
on the data path, only the optional gather of the finished film.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class RowShard:
    rank: int
    world: int
    width: int
    height: int

    @property
    def rows(self) -> int:
        return len(range(self.rank, self.height, self.world))

    @property
    def image_rows(self) -> np.ndarray:
        return np.arange(self.rank, self.height, self.world)

    def tile(self):
        """(x, y, w, h) in hipcy_work_tile terms: y is the first image row and
        h the number of rows the rank owns; rows advance by y_step = world."""
        return (0, self.rank, self.width, self.rows)

    @property
    def offset(self) -> int:
        # buffer index = offset + x + (tile.y + j) * stride = x + j * width
        return -(self.rank * self.width)

    @property
    def stride(self) -> int:
        return self.width

    @property
    def y_step(self) -> int:
        return self.world


def assemble(parts: list[np.ndarray], height: int) -> np.ndarray:
    """Interleave per-rank compact buffers (rows x width x pass_stride) back
    into the full frame."""
    world = len(parts)
    out = np.empty((height,) + parts[0].shape[1:], dtype=parts[0].dtype)
    for r, p in enumerate(parts):
        out[r::world] = p
    return out


@dataclass(frozen=True)
class TileShard:
    """Tiles of tile x tile pixels (the last row / column ragged) in row order,
    tile k owned by rank k % world: the static counterpart of the reference's
    MultiDevice tile queue (device_multi.cpp:689-737, render/tile.cpp).
    Adaptive sampling filters each RenderTile on its own
    (kernel_adaptive_sampling.h, CUDADevice::adaptive_sampling_filter), so a
    rank that owns whole tiles renders them exactly as one device would.
    Each rank renders into a full-frame buffer (offset 0, stride width); only
    its own tiles are written."""
    rank: int
    world: int
    width: int
    height: int
    tile_size: int = 64

    def all_tiles(self) -> list:
        t = self.tile_size
        return [(x, y, min(t, self.width - x), min(t, self.height - y))
                for y in range(0, self.height, t) for x in range(0, self.width, t)]

    def tiles(self) -> list:
        return self.all_tiles()[self.rank::self.world]

    @property
    def offset(self) -> int:
        return 0

    @property
    def stride(self) -> int:
        return self.width


def assemble_tiles(parts: list[np.ndarray], shards: list[TileShard]) -> np.ndarray:
    """Full-frame buffers of the ranks (each holding its own tiles) into one
    frame, copying every tile from the rank that owns it."""
    out = np.zeros_like(parts[0])
    for p, sh in zip(parts, shards):
        for x, y, w, h in sh.tiles():
            out[y:y + h, x:x + w] = p[y:y + h, x:x + w]
    return out
