"""Multi-GPU partition of one frame: rows interleaved over ranks.

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
