"""Python mirror of the Cycles device plugin surface over the HIP C ABI.

``HIPDevice`` follows the method set of ccl::Device (device/device.h:288-500):
mem_alloc / mem_copy_to / mem_copy_from / mem_zero / mem_free, const_copy_to,
load_kernels, get_bvh_layout_mask, error_message, and a RENDER task over
RenderTiles (``render_tile`` = CUDADevice::render, device_cuda_impl.cpp:1853-1952).
``DeviceScene`` upload mirrors Scene::device_update's copy_to_device of every
named array (stack B of SURVEY.md §3).

Errors are sticky and raise ``DeviceError`` (Device::set_error semantics).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native
from .scene import ELEMENT_BYTES, DeviceScene


class DeviceError(RuntimeError):
    pass


class DeviceBuffer:
    """device_memory analogue: a device allocation owned by the device."""

    def __init__(self, device: "HIPDevice", nbytes: int):
        self.device = device
        self.nbytes = nbytes
        self.ptr = device._alloc(nbytes)

    def copy_to_device(self, host: np.ndarray):
        host = np.ascontiguousarray(host)
        if host.nbytes > self.nbytes:
            raise ValueError("copy_to_device overflows the allocation")
        self.device._check(self.device.lib.hipcy_mem_copy_to(self.device.h, self.ptr, host.ctypes.data, host.nbytes))

    def copy_from_device(self, out: np.ndarray) -> np.ndarray:
        if not out.flags.c_contiguous or out.nbytes > self.nbytes:
            raise ValueError("bad host buffer")
        self.device._check(self.device.lib.hipcy_mem_copy_from(self.device.h, out.ctypes.data, self.ptr, out.nbytes))
        return out

    def zero(self):
        self.device._check(self.device.lib.hipcy_mem_zero(self.device.h, self.ptr, self.nbytes))

    def free(self):
        if self.ptr:
            self.device._check(self.device.lib.hipcy_mem_free(self.device.h, self.ptr))
            self.ptr = 0


class HIPDevice:
    def __init__(self, ordinal: int = 0):
        self.lib = native.device_lib()
        self.ordinal = ordinal
        h = self.lib.hipcy_create(ordinal)
        if not h:
            raise DeviceError(self.lib.hipcy_global_error().decode())
        self.h = h
        self._arrays: dict[str, DeviceBuffer] = {}
        self.scene: DeviceScene | None = None

    # ---- Device API -------------------------------------------------------
    @staticmethod
    def available_devices() -> list[dict]:
        lib = native.device_lib()
        n = ctypes.c_int(0)
        lib.hipcy_device_count(ctypes.byref(n))
        out = []
        for i in range(n.value):
            name = ctypes.create_string_buffer(256)
            mem = ctypes.c_uint64(0)
            if lib.hipcy_device_info(i, name, 256, ctypes.byref(mem)) == 0:
                out.append({"ordinal": i, "name": name.value.decode(), "mem": mem.value, "type": "HIP"})
        return out

    def error_message(self) -> str:
        return self.lib.hipcy_error(self.h).decode()

    def _check(self, rc: int):
        if rc != 0:
            raise DeviceError(self.error_message() or "HIP device error %d" % rc)

    def _alloc(self, nbytes: int) -> int:
        p = ctypes.c_uint64(0)
        self._check(self.lib.hipcy_mem_alloc(self.h, nbytes, ctypes.byref(p)))
        return p.value

    def mem_alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def const_copy_to(self, name: str, data) -> None:
        raw = bytes(data)
        buf = (ctypes.c_char * len(raw)).from_buffer_copy(raw)
        self._check(self.lib.hipcy_const_copy_to(self.h, name.encode(), ctypes.addressof(buf), len(raw)))

    def global_alloc(self, name: str, host: np.ndarray) -> DeviceBuffer:
        """device_vector<T> GLOBAL memory: allocate, copy, bind to the kernel name."""
        host = np.ascontiguousarray(host)
        old = self._arrays.pop(name, None)
        if old is not None:
            old.free()
        buf = DeviceBuffer(self, max(host.nbytes, 16))
        buf.copy_to_device(host)
        self._check(self.lib.hipcy_bind_global(self.h, name.encode(), buf.ptr, host.nbytes))
        self._arrays[name] = buf
        return buf

    def get_bvh_layout_mask(self) -> int:
        return int(self.lib.hipcy_get_bvh_layout_mask(self.h))

    def load_kernels(self) -> None:
        self._check(self.lib.hipcy_load_kernels(self.h))

    def set_profiling(self, flags: int) -> None:
        """bit 0: HIP-event timing of every kernel launch; bit 1: traversal counters."""
        self.lib.hipcy_set_profiling(self.h, int(flags))

    def set_bvh_width(self, width: int) -> None:
        """4 (default) / 8: traverse the device-widened wide BVH; 2: the bound BVH2."""
        self._check(self.lib.hipcy_set_bvh_width(self.h, int(width)))

    def set_curve_layout(self, wide: bool) -> None:
        """Scenes with curves: False (default) traverse the bound BVH2; True
        lets ribbon-only scenes use the wide layout (oriented-box nodes)."""
        self._check(self.lib.hipcy_set_curve_layout(self.h, int(bool(wide))))

    def set_ray_sort(self, mode: int) -> None:
        """Bin the closest-hit queue by ray direction before every bounce
        iteration: 0 off, 3 octant, 5 octant x major axis; 8 sorts the shading
        queue by the hit's shader instead; -1 (the device default) picks 8
        for scenes on the extended shading kernel (hipcy_set_ray_sort)."""
        self._check(self.lib.hipcy_set_ray_sort(self.h, int(mode)))

    def set_traversal_budget(self, first: int, second: int | None = None) -> None:
        """Iteration budget of the wide traversal kernels (hipcy_set_traversal_budget):
        traversals longer than `first` iterations continue in packed continuation
        launches (then `second`, then unbounded).  0 disables."""
        second = 2 * first if second is None else second
        self._check(self.lib.hipcy_set_traversal_budget(self.h, int(first), int(second)))

    def set_traversal_refill(self, rounds: int, min_idle: int = 16) -> None:
        """Lane refill of the closest-hit traversal (hipcy_set_traversal_refill):
        persistent waves traversing `rounds` iterations at a time, refilled with
        new rays once `min_idle` lanes are idle.  0 disables."""
        self._check(self.lib.hipcy_set_traversal_refill(self.h, int(rounds), int(min_idle)))

    def set_shadow_sort(self, mode: int) -> None:
        """Shadow-queue sort by shadow ray direction (hipcy_set_shadow_sort):
        0 off (default), 3 octant, 5 octant x major axis."""
        self._check(self.lib.hipcy_set_shadow_sort(self.h, int(mode)))

    def set_tail(self, paths: int) -> None:
        """Fused tail (hipcy_set_tail): lanes with all items claimed and at most
        `paths` live paths finish them in one launch.  0 disables."""
        self._check(self.lib.hipcy_set_tail(self.h, int(paths)))

    def set_slots(self, slots: int = 0, record_bytes: int = 0) -> None:
        """Path slots in flight and the per-pass sample-record budget (0 keeps a value)."""
        self._check(self.lib.hipcy_set_slots(self.h, int(slots), int(record_bytes)))

    def set_bvh_leaf_merge(self, max_prims: int) -> None:
        """Wide BVH: merge BVH2 subtrees of <= max_prims contiguous primitives into one leaf."""
        self._check(self.lib.hipcy_set_bvh_leaf_merge(self.h, int(max_prims)))

    def stats(self) -> dict:
        st = native.Stats()
        self.lib.hipcy_get_stats(self.h, ctypes.byref(st))
        return {name: getattr(st, name) for name, _ in native.Stats._fields_}

    # ---- scene upload (Scene::device_update) -------------------------------
    def upload_scene(self, ds: DeviceScene) -> None:
        for name, arr in ds.arrays.items():
            if name not in ELEMENT_BYTES:
                raise KeyError(name)
            self.global_alloc(name, arr)
        for slot, im in enumerate(ds.textures):
            self.tex_alloc(slot, im)
        self.const_copy_to("__data", ds.data)
        self.load_kernels()
        if ds.info.get("background_map"):
            self.update_background_map(ds)
        self.scene = ds

    def tex_alloc(self, slot: int, image) -> None:
        """ImageManager::device_load_image -> Device::tex_alloc
        (device_cuda_impl.cpp:1105-1304): texels to device memory, slot's
        TextureInfo in the device's __texture_info table."""
        from . import nodes

        a = image.texel_array()
        w, h, d = image.dims()
        tfm = None
        if image.transform_3d is not None:
            t = np.ascontiguousarray(np.asarray(image.transform_3d, dtype=np.float32).reshape(12))
            tfm = t.ctypes.data
        self._check(self.lib.hipcy_tex_alloc_3d(self.h, slot, nodes.IMAGE_DATA_TYPES.index(image.data_type),
                                                nodes.INTERPOLATIONS.index(image.interpolation),
                                                nodes.EXTENSIONS.index(image.extension), w, h, d, tfm,
                                                a.ctypes.data, a.nbytes))

    def update_background_map(self, ds: DeviceScene) -> None:
        """LightManager::device_update_background (light.cpp:568-716): the world
        shader over the equirectangular map by this device's SHADER task, its
        CDFs built on the host, both CDF arrays re-bound."""
        res_x, res_y = ds.info["background_map"]
        pixels = self.background_eval(res_x, res_y, 1)
        marg, cond = native.background_cdf(pixels, res_x, res_y)
        self.global_alloc("__light_background_marginal_cdf", marg)
        self.global_alloc("__light_background_conditional_cdf", cond)
        self.background_cdfs = (marg, cond)
        self.load_kernels()

    # ---- RENDER task ------------------------------------------------------
    def render_tile(self, buffer: DeviceBuffer, tile, start_sample: int, num_samples: int,
                    offset: int, stride: int, y_step: int = 1) -> None:
        x, y, w, h = tile
        wt = native.WorkTile(x, y, w, h, start_sample, num_samples, offset, stride, buffer.ptr)
        if y_step == 1:
            self._check(self.lib.hipcy_path_trace(self.h, ctypes.byref(wt)))
        else:
            self._check(self.lib.hipcy_path_trace_rows(self.h, ctypes.byref(wt), y_step))

    def render_tiles(self, tiles, start_sample: int, num_samples: int) -> None:
        """Several RenderTiles in one device pass (hipcy_path_trace_tiles): tiles is
        a list of ((x, y, w, h), buffer_pointer, offset, stride)."""
        arr = (native.WorkTile * len(tiles))()
        for k, ((x, y, w, h), ptr, offset, stride) in enumerate(tiles):
            arr[k] = native.WorkTile(x, y, w, h, start_sample, num_samples, offset, stride,
                                     ptr if isinstance(ptr, int) else ptr.ptr)
        self._check(self.lib.hipcy_path_trace_tiles(self.h, arr, len(tiles)))

    def set_stream_hold(self, pixel_samples: int) -> None:
        """Default bound on the pixel-samples a tile stream holds (hipcy_set_stream_hold)."""
        self._check(self.lib.hipcy_set_stream_hold(self.h, int(pixel_samples)))

    def render_feed(self, acquire, release, hold: int = 0, cancelled=None) -> None:
        """The RENDER task's acquire_tile / release_tile loop over a tile stream
        (hipcy_render_feed; device_cuda_impl.cpp:2342-2391 thread_run).
        acquire() returns None or a tuple ((x, y, w, h), start_sample,
        num_samples, buffer_pointer, offset, stride[, tag]); release(tag, tile)
        is called once the tile's samples are in its buffer.  Exceptions raised
        by the callbacks end the stream's acquisition and are re-raised."""
        errors = []

        def _acquire(user, tile_p, tag_p):
            try:
                t = None if errors else acquire()
            except BaseException as e:  # noqa: BLE001 - re-raised after the stream drained
                errors.append(e)
                t = None
            if t is None:
                return 0
            (x, y, w, h), s0, ns, ptr, offset, stride = t[:6]
            tile_p[0] = native.WorkTile(x, y, w, h, s0, ns, offset, stride, ptr if isinstance(ptr, int) else ptr.ptr)
            tag_p[0] = int(t[6]) if len(t) > 6 else 0
            return 1

        def _release(user, tile_p, tag):
            t = tile_p[0]
            try:
                release(int(tag), (t.x, t.y, t.w, t.h, t.start_sample, t.num_samples))
            except BaseException as e:  # noqa: BLE001
                errors.append(e)

        def _cancelled(user):
            return 1 if (errors or (cancelled is not None and cancelled())) else 0

        feed = native.TileFeed(None, native.FEED_ACQUIRE(_acquire), native.FEED_RELEASE(_release),
                               native.FEED_CANCELLED(_cancelled), int(hold))
        rc = self.lib.hipcy_render_feed(self.h, ctypes.byref(feed))
        if errors:
            raise errors[0]
        self._check(rc)

    def render(self, samples: int | None = None, start_sample: int = 0, tile=None) -> np.ndarray:
        """Render (a tile of) the uploaded scene; returns the float render buffer
        [h, w, pass_stride] of the tile (buffer offset/stride as CPUDevice)."""
        ds = self.scene
        samples = ds.samples if samples is None else samples
        x, y, w, h = tile if tile is not None else (0, 0, ds.width, ds.height)
        nbytes = w * h * ds.pass_stride * 4
        buf = self.mem_alloc(nbytes)
        try:
            buf.zero()
            self.render_tile(buf, (x, y, w, h), start_sample, samples, -(x + y * w), w)
            out = np.zeros((h, w, ds.pass_stride), dtype=np.float32)
            buf.copy_from_device(out)
        finally:
            buf.free()
        return out

    # ---- SHADER task -------------------------------------------------------
    SHADER_EVAL_BACKGROUND = 1  # kernel_types.h:204
    SHADER_EVAL_DISPLACE = 0  # kernel_types.h:203

    def background_eval(self, width: int, height: int, num_samples: int = 1) -> np.ndarray:
        """World colour over a (width x height) equirectangular map, the SHADER
        task LightManager runs for the background importance map
        (light.cpp:38-85 shade_background_pixels -> CUDADevice::shader,
        device_cuda_impl.cpp:2019-2093).  Returns float32 [height, width, 4]
        (rgb accumulated num_samples times, w = 0)."""
        u = ((np.arange(width, dtype=np.float32) + np.float32(0.5)) / np.float32(width)).astype(np.float32)
        v = ((np.arange(height, dtype=np.float32) + np.float32(0.5)) / np.float32(height)).astype(np.float32)
        inp = np.zeros((height, width, 4), dtype=np.uint32)
        inp[..., 0] = u.view(np.uint32)[None, :]
        inp[..., 1] = v.view(np.uint32)[:, None]
        out = np.zeros((height, width, 4), dtype=np.float32)
        d_i = self.mem_alloc(inp.nbytes)
        d_o = self.mem_alloc(out.nbytes)
        try:
            d_i.copy_to_device(inp)
            d_o.copy_to_device(out)
            self._check(self.lib.hipcy_shader_eval(self.h, self.SHADER_EVAL_BACKGROUND, d_i.ptr, d_o.ptr, 0,
                                                   width * height, 0, num_samples))
            d_o.copy_from_device(out)
        finally:
            d_i.free()
            d_o.free()
        return out

    def displace_eval(self, inp: np.ndarray) -> np.ndarray:
        """SHADER_EVAL_DISPLACE (MeshManager::displace, mesh_displace.cpp ->
        CUDADevice::shader): inp uint32 [N, 4] = (object, prim, u bits, v bits);
        returns float32 [N, 4], the object-space displacement (w = 0)."""
        inp = np.ascontiguousarray(inp, dtype=np.uint32).reshape(-1, 4)
        out = np.zeros((len(inp), 4), dtype=np.float32)
        if len(inp) == 0:
            return out
        d_i = self.mem_alloc(inp.nbytes)
        d_o = self.mem_alloc(out.nbytes)
        try:
            d_i.copy_to_device(inp)
            d_o.copy_to_device(out)
            self._check(self.lib.hipcy_shader_eval(self.h, self.SHADER_EVAL_DISPLACE, d_i.ptr, d_o.ptr, 0,
                                                   len(inp), 0, 1))
            d_o.copy_from_device(out)
        finally:
            d_i.free()
            d_o.free()
        return out

    # ---- FILM_CONVERT task ------------------------------------------------
    def film_convert(self, buffer: np.ndarray, sample_scale: float, half: bool = False,
                     tile=None) -> np.ndarray:
        """Convert a full-frame float render buffer [H, W, pass_stride] to display
        pixels like CUDADevice::film_convert (device_cuda_impl.cpp:1954-2017):
        uint8 sRGB [H, W, 4], or half bit patterns as uint16 [H, W, 4]."""
        buffer = np.ascontiguousarray(buffer, dtype=np.float32)
        H, W = buffer.shape[:2]
        x, y, w, h = tile if tile is not None else (0, 0, W, H)
        out = np.zeros((H, W, 4), dtype=np.uint16 if half else np.uint8)
        d_b = self.mem_alloc(buffer.nbytes)
        d_o = self.mem_alloc(out.nbytes)
        try:
            d_b.copy_to_device(buffer)
            d_o.copy_to_device(out)
            self._check(self.lib.hipcy_film_convert(self.h, d_b.ptr, 0 if half else d_o.ptr, d_o.ptr if half else 0,
                                                    float(sample_scale), x, y, w, h, 0, W))
            d_o.copy_from_device(out)
        finally:
            d_b.free()
            d_o.free()
        return out

    # ---- test entry points ------------------------------------------------
    def intersect(self, rays: np.ndarray, any_hit: bool = False):
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        n = rays.shape[0]
        d_rays = self.mem_alloc(rays.nbytes)
        d_f = self.mem_alloc(n * 12)
        d_i = self.mem_alloc(n * 16)
        try:
            d_rays.copy_to_device(rays)
            self._check(self.lib.hipcy_intersect(self.h, d_rays.ptr, d_f.ptr, d_i.ptr, n, int(any_hit)))
            of = d_f.copy_from_device(np.zeros((n, 3), dtype=np.float32))
            oi = d_i.copy_from_device(np.zeros((n, 4), dtype=np.int32))
        finally:
            for b in (d_rays, d_f, d_i):
                b.free()
        return of, oi

    def camera_rays(self, xys: np.ndarray) -> np.ndarray:
        xys = np.ascontiguousarray(xys, dtype=np.int32)
        n = xys.shape[0]
        d_x = self.mem_alloc(xys.nbytes)
        d_o = self.mem_alloc(n * 32)
        try:
            d_x.copy_to_device(xys)
            self._check(self.lib.hipcy_camera_rays(self.h, d_x.ptr, d_o.ptr, n))
            out = d_o.copy_from_device(np.zeros((n, 8), dtype=np.float32))
        finally:
            d_x.free()
            d_o.free()
        return out

    def close(self):
        if getattr(self, "h", None):
            for b in self._arrays.values():
                b.ptr = 0  # freed by hipcy_destroy
            self.lib.hipcy_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
