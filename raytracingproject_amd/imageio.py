"""Film readout and a dependency-free PNG writer.

film_readout restates RenderBuffers::get_pass_rect for the combined pass
(render/buffers.cpp:256-300): RGB divided by the sample count, alpha saturated.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np


def film_readout(buffer: np.ndarray, samples: int) -> np.ndarray:
    scale = np.float32(1.0) / np.float32(samples)
    rgba = buffer[..., :4].astype(np.float32) * scale
    rgba[..., 3] = np.clip(rgba[..., 3], 0.0, 1.0)
    return rgba


def write_png(path: str, rgb: np.ndarray, gamma: float = 2.2, flip_y: bool = True) -> None:
    img = np.clip(np.nan_to_num(rgb[..., :3]), 0.0, 1.0) ** (1.0 / gamma)
    if flip_y:
        img = img[::-1]
    a = (img * 255.0 + 0.5).astype(np.uint8)
    h, w, _ = a.shape
    raw = b"".join(b"\x00" + a[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))
