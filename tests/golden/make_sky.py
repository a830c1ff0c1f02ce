"""Sky Texture host data for the `shading_sky` parity case (tests/golden/sky.npz).

The Sky Texture node's Hosek-Wilkie and Nishita models are precomputed on the
host by Blender's intern/sky library (render/nodes.cpp:708-776, image_sky.cpp):
this script runs that library — compiled from its own sources by
`make -C oracle sky` into oracle/_ref/libsky_ref.so (test infrastructure) —
and stores what the host would put into the node and the sky image:

  hosek_configs (3, 9) float32, hosek_radiances (3,) float32
      SKY_arhosek_xyz_skymodelstate_alloc_init(turbidity, albedo, elevation)
      (configs[0..2][0..8], radiances[0..2] cast to float, nodes.cpp:736-742)
  nishita_bottom / nishita_top (3,) float32
      SKY_nishita_skymodel_precompute_sun
  nishita_texture (128, 512, 4) float32
      SKY_nishita_skymodel_precompute_texture over all rows with 3 channels,
      expanded to RGBA with alpha 1 as ImageManager does (image.cpp:549-557)

    python tests/golden/make_sky.py
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

# the case's parameters (tests/parity_cases.py shading_sky)
HOSEK_SUN = (0.3, 0.55, 0.78)
HOSEK_TURBIDITY, HOSEK_ALBEDO = 3.0, 0.4
NISHITA = dict(sun_elevation=np.float32(np.radians(12.0)), sun_size=np.float32(0.05), altitude=np.float32(800.0),
               air=np.float32(1.0), dust=np.float32(2.5), ozone=np.float32(1.0))


def hosek_elevation(sun_direction):
    """sky_texture_precompute_hosek: theta of the sun (clamped), elevation = pi/2 - theta, in float."""
    f = np.float32
    d = np.asarray(sun_direction, dtype=np.float32)
    theta = f(min(max(f(np.arccos(d[2])), f(0.0)), f(np.pi / 2)))
    return f(f(np.pi / 2) - theta)


def main():
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libsky_ref.so"))
    lib.SKY_arhosek_xyz_skymodelstate_alloc_init.restype = ctypes.c_void_p
    lib.SKY_arhosek_xyz_skymodelstate_alloc_init.argtypes = [ctypes.c_double] * 3
    lib.SKY_arhosekskymodelstate_free.argtypes = [ctypes.c_void_p]
    st = lib.SKY_arhosek_xyz_skymodelstate_alloc_init(HOSEK_TURBIDITY, HOSEK_ALBEDO,
                                                      float(hosek_elevation(HOSEK_SUN)))
    # SKY_ArHosekSkyModelState: configs[11][9] doubles, then radiances[11]
    raw = np.ctypeslib.as_array((ctypes.c_double * (99 + 11)).from_address(st)).copy()
    lib.SKY_arhosekskymodelstate_free(ctypes.c_void_p(st))
    configs = raw[:27].reshape(3, 9).astype(np.float32)
    radiances = raw[99:102].astype(np.float32)

    n = NISHITA
    fl = ctypes.c_float
    lib.SKY_nishita_skymodel_precompute_sun.argtypes = [fl] * 5 + [ctypes.c_void_p] * 2
    bottom = np.zeros(3, np.float32)
    top = np.zeros(3, np.float32)
    lib.SKY_nishita_skymodel_precompute_sun(n["sun_elevation"], n["sun_size"], n["altitude"], n["air"], n["dust"],
                                            bottom.ctypes.data, top.ctypes.data)
    w, h = 512, 128  # SkyLoader::load_metadata
    lib.SKY_nishita_skymodel_precompute_texture.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [fl] * 5
    px = np.zeros(w * h * 4, np.float32)
    lib.SKY_nishita_skymodel_precompute_texture(px.ctypes.data, 3, 0, h, w, h, n["sun_elevation"], n["altitude"],
                                                n["air"], n["dust"], n["ozone"])
    rgb = px[: w * h * 3].reshape(h, w, 3)
    tex = np.ones((h, w, 4), np.float32)
    tex[..., :3] = rgb
    np.savez_compressed(os.path.join(HERE, "sky.npz"), hosek_configs=configs, hosek_radiances=radiances,
                        nishita_bottom=bottom, nishita_top=top, nishita_texture=tex)
    print("sky.npz:", configs.shape, radiances, bottom, top, float(tex[..., :3].max()))


if __name__ == "__main__":
    main()
