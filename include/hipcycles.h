/*
 * hipcycles.h — C ABI of the MI355X (gfx950) Cycles path-tracing device.
 *
 * This is the drop-in boundary: a Cycles `Device` subclass (see
 * integration/device_hip.cpp and INTEGRATION.md) forwards the reference device
 * plugin calls to these entry points.  Plain pointers, sizes and 64-bit device
 * handles only.  Every call returns 0 on success and a negative value on error;
 * the first error is sticky and readable with hipcy_error(), mirroring
 * Device::set_error / error_message (device/device.h:341-348).
 *
 * Reference interface each entry point replaces (blender/intern/cycles/...):
 *   hipcy_device_count / hipcy_device_info   device/device_cuda.cpp:90 device_cuda_info,
 *                                            device/device.cpp:475-550 available_devices
 *   hipcy_create / hipcy_destroy             device/device.cpp:367-418 Device::create,
 *                                            device/cuda/device_cuda_impl.cpp (CUDADevice ctor/dtor)
 *   hipcy_error                              device/device.h:341-348 error_message
 *   hipcy_mem_alloc / _free / _copy_to /
 *   _copy_from / _zero                       device/device.h:484-488 mem_alloc/mem_copy_to/
 *                                            mem_copy_from/mem_zero/mem_free
 *   hipcy_const_copy_to                      device/device.h:366 const_copy_to("__data", ..)
 *                                            (called from render/scene.cpp:307)
 *   hipcy_bind_global                        device_cuda_impl.cpp:1088-1096 global_alloc ->
 *                                            const_copy_to(mem.name, &ptr, 8) for the arrays of
 *                                            kernel/kernel_textures.h:21-87
 *   hipcy_load_kernels                       device/device.h:375 load_kernels(DeviceRequestedFeatures)
 *   hipcy_path_trace                         device_cuda_impl.cpp:1853-1952 CUDADevice::render
 *                                            (one RenderTile, samples [start, start+num))
 *   hipcy_path_trace_tiles                   device_cuda_impl.cpp:2342-2391 the RENDER task's
 *                                            acquire_tile loop, several tiles per device pass
 *   hipcy_render_feed / hipcy_set_stream_hold device_cuda_impl.cpp:2342-2391 the RENDER task's
 *                                            acquire_tile / release_tile loop (device_task.h:157-160
 *                                            callbacks; render/tile.cpp:498-557 next_tile shared by
 *                                            the devices of device/device_multi.cpp:689-737)
 *   hipcy_synchronize                        device_cuda_impl.cpp:1933 cuCtxSynchronize
 *   hipcy_get_bvh_layout_mask                device/device.h:353 get_bvh_layout_mask
 *   hipcy_set_bvh_width / _leaf_merge        (device options) traverse the bound BVH2 as is, or
 *                                            the 4/8-wide BVH the device widens it into, like
 *                                            BVH::pack_nodes/widen_children_nodes bvh/bvh.cpp:149-176
 *   hipcy_shader_eval                        device_cuda_impl.cpp:2019-2093 CUDADevice::shader
 *                                            (DeviceTask SHADER: SHADER_EVAL_BACKGROUND,
 *                                            kernel_bake.h:474-510, light.cpp:38-85;
 *                                            SHADER_EVAL_DISPLACE, kernel_bake.h:446-472,
 *                                            mesh_displace.cpp)
 *   hipcy_tex_alloc / hipcy_tex_free         device_cuda_impl.cpp:1105-1304 CUDADevice::tex_alloc /
 *                                            tex_free + load_texture_info (device_texture of
 *                                            render/image.cpp device_load_image; the SVM image
 *                                            slot indexes __texture_info, kernel_textures.h:84)
 *   hipcy_film_convert                       device_cuda_impl.cpp:1954-2017 CUDADevice::film_convert
 *                                            (DeviceTask FILM_CONVERT; kernel/kernel_film.h)
 *   hipcy_intersect / hipcy_camera_rays      test entry points (scene_intersect, bvh/bvh.h:154;
 *                                            kernel_path_trace_setup, kernel_path_common.h:21)
 */
#ifndef HIPCYCLES_H
#define HIPCYCLES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HIPCY_ABI_VERSION 6

typedef struct hipcy_device hipcy_device;

/* RenderTile slice handed to the device (kernel_types.h:1690-1700 WorkTile). */
typedef struct hipcy_work_tile {
  int32_t x, y, w, h;
  int32_t start_sample;
  int32_t num_samples;
  int32_t offset;
  int32_t stride;
  uint64_t buffer; /* device pointer to w*h*pass_stride floats (render buffer) */
} hipcy_work_tile;

/* Traversal statistics of the last hipcy_path_trace (for the HBM roofline). */
typedef struct hipcy_stats {
  uint64_t closest_rays;
  uint64_t shadow_rays;
  uint64_t inner_nodes; /* BVH2 inner nodes visited, both ray kinds */
  uint64_t leaves;
  uint64_t triangles;   /* ray-triangle tests */
  uint64_t iterations;  /* wavefront iterations */
  double intersect_ms;  /* summed HIP-event time of the traversal kernels */
  double shade_ms;
  double total_ms;      /* first launch to last completion of the tile */
  double closest_ms;    /* closest-hit traversal kernel only */
  uint64_t closest_launches;
  uint64_t closest_nodes; /* closest-hit traversal only (the roofline kernel) */
  uint64_t closest_leaves;
  uint64_t closest_tris;
  int32_t bvh_width;      /* 2: BVH2 as bound; 4/8: device-widened wide BVH */
  int32_t bvh_depth;      /* levels of the wide BVH (0 for BVH2) */
  uint64_t bvh_bytes;     /* bytes of the traversed node array */
  uint64_t tie_rays;      /* closest rays re-traced in the reference's order (near-ties) */
  /* traversal loop iterations (nodes + leaves visited): summed over lanes, and
   * the per-wave maximum summed over waves (lane utilisation = lane / (64 wave)) */
  uint64_t closest_lane_iters;
  uint64_t closest_wave_iters;
  uint64_t shadow_nodes;  /* opaque shadow traversal only */
  uint64_t shadow_tris;
  uint64_t shadow_lane_iters;
  uint64_t shadow_wave_iters;
  double shadow_ms;       /* shadow kernel (traversal + finish / refill) */
  uint64_t shadow_launches;
} hipcy_stats;

int hipcy_abi_version(void);
int hipcy_device_count(int *count);
int hipcy_device_info(int ordinal, char *name, size_t name_len, uint64_t *total_mem);

hipcy_device *hipcy_create(int ordinal);
void hipcy_destroy(hipcy_device *dev);
const char *hipcy_error(const hipcy_device *dev); /* "" when no error */
const char *hipcy_global_error(void);             /* errors of hipcy_create */

int hipcy_mem_alloc(hipcy_device *dev, size_t bytes, uint64_t *device_pointer);
int hipcy_mem_free(hipcy_device *dev, uint64_t device_pointer);
int hipcy_mem_copy_to(hipcy_device *dev, uint64_t dst, const void *src, size_t bytes);
int hipcy_mem_copy_from(hipcy_device *dev, void *dst, uint64_t src, size_t bytes);
int hipcy_mem_zero(hipcy_device *dev, uint64_t device_pointer, size_t bytes);

int hipcy_const_copy_to(hipcy_device *dev, const char *name, const void *host, size_t size);
int hipcy_bind_global(hipcy_device *dev, const char *name, uint64_t device_pointer, size_t bytes);
/* Image textures: a 2D image of width x height texels of ImageDataType
 * data_type (util_texture.h: 0 float4, 1 byte4, 2 half4, 3 float, 4 byte,
 * 5 half, 6 ushort4, 7 ushort) with interpolation (0 linear, 1 closest,
 * 2 cubic, 3 smart) and extension (0 repeat, 1 extend, 2 clip) in SVM image
 * slot `slot`.  The pixels are copied to device memory owned by the device;
 * the device keeps the TextureInfo table and binds it as __texture_info.
 * bytes must equal width * height * the texel size.  Re-allocating a slot
 * replaces it; hipcy_tex_free releases it. */
int hipcy_tex_alloc(hipcy_device *dev, int slot, int data_type, int interpolation, int extension, int width,
                    int height, const void *pixels, size_t bytes);
/* 3D textures (TextureInfo depth > 1; the Point Density node's voxel grid,
 * kernel_tex_image_interp_3d): texels x-fastest, then y, then z;
 * transform_3d (12 floats, rows x, y, z) or NULL sets
 * TextureInfo::use_transform_3d / transform_3d (ImageManager, image.cpp). */
int hipcy_tex_alloc_3d(hipcy_device *dev, int slot, int data_type, int interpolation, int extension, int width,
                       int height, int depth, const float *transform_3d, const void *pixels, size_t bytes);
int hipcy_tex_free(hipcy_device *dev, int slot);

/* Validate that the scene uploaded so far only uses features the HIP kernels
 * implement and prepare it (widen the BVH); returns 0 or a negative code with a
 * readable hipcy_error().  hipcy_path_trace calls it too. */
int hipcy_load_kernels(hipcy_device *dev);
uint32_t hipcy_get_bvh_layout_mask(const hipcy_device *dev); /* BVH_LAYOUT_BVH2 = 1 */
/* Traversal structure: 4 (default) or 8 widens the bound BVH2 into the
 * device's 4- or 8-wide BVH before the next path_trace/intersect; 2 traverses
 * the BVH2 exactly as bound (bit-identical visiting order to the reference). */
int hipcy_set_bvh_width(hipcy_device *dev, int width);
/* Scenes with curves: 0 (default) traverses the bound BVH2 at every width
 * (measured faster on hair-heavy scenes: the JNK stand-in's crop 16.6 against
 * 15.2 Msamples/s); 1 lets ribbon-only scenes use the W-wide layout too, with
 * the BVH2's unaligned nodes kept as oriented two-child nodes (bit-exact to the
 * reference like every width; thick curves keep the BVH2 either way). */
int hipcy_set_curve_layout(hipcy_device *dev, int wide);
/* Wide BVH only: BVH2 subtrees holding at most max_prims (0..15) primitives in
 * one contiguous range become a single leaf child (0 = keep BVH2 leaves). */
int hipcy_set_bvh_leaf_merge(hipcy_device *dev, int max_prims);
/* Path slots kept in flight (default 2^27, ~28 GB) and the byte budget of the
 * per-sample record buffer of one pass (default 4 GiB; a tile whose samples do
 * not fit is rendered in several sample passes).  0 keeps a value. */
int hipcy_set_slots(hipcy_device *dev, uint64_t slots, uint64_t record_bytes);
/* Wavefront ray sorting (north_star; the reference's precedent is the split
 * kernel's kernel/split/kernel_shader_sort.h): before every bounce iteration
 * the closest-hit queue is binned by a key of the ray direction, so the rays
 * of a wave descend the same BVH subtrees.  mode 0 = off, 3 = octant of D
 * (8 bins), 5 = octant x major axis (24 of 32 bins).  Mode 8 sorts the
 * shading queue instead, between the closest-hit and shading launches, by the
 * shader of each path's hit (kernel_shader_sort.h's key), so a shading wave
 * runs one material's SVM program.  -1 (the default) picks mode 8 for scenes
 * that run the extended shading kernel (texture / Principled / BSSRDF nodes)
 * without curves, else 0.  Results never depend on the order (every path is a
 * function of its work item alone). */
int hipcy_set_ray_sort(hipcy_device *dev, int mode);
/* Iteration budget of the wide-BVH traversal kernels (compaction at traversal
 * granularity): a closest-hit or shadow traversal that has run `first` loop
 * iterations is suspended and continued by a densely packed continuation
 * launch, which suspends again after `second` iterations into a last launch
 * without a budget.  Results are bit-identical; 0, 0 disables (scenes with
 * instances always run without a budget). */
int hipcy_set_traversal_budget(hipcy_device *dev, int first, int second);
/* Lane refill of the closest-hit traversal (non-instanced wide BVH without
 * curves): persistent waves whose lanes traverse `rounds` iterations at a time
 * and, once `min_idle` lanes of a wave have finished their rays, take the next
 * rays of the queue.  Results are bit-identical; rounds 0 disables. */
int hipcy_set_traversal_refill(hipcy_device *dev, int rounds, int min_idle);
/* Fused tail: once every work item of a lane is claimed and at most `paths` of
 * its paths are live (default 2^17), one launch runs each of them to its end
 * (closest hit, shading and shadow per bounce in one kernel) instead of one
 * closest -> shade -> shadow iteration per bounce.  Plain shading variants,
 * triangle scenes with opaque shadows; results are bit-identical; 0 disables. */
int hipcy_set_tail(hipcy_device *dev, uint64_t paths);
/* Shadow-queue sort: the opaque-shadow queue binned before its traversal
 * launch by the shadow ray's direction, as hipcy_set_ray_sort mode 3 (octant)
 * or 5 (octant x major axis), so a wave's rays head for one light and share
 * the BVH nodes they open; 0 (the default) keeps the shading order.  Results
 * are bit-identical. */
int hipcy_set_shadow_sort(hipcy_device *dev, int mode);

int hipcy_path_trace(hipcy_device *dev, const hipcy_work_tile *tile);
/* Same, with the tile's rows taken every y_step image rows (y, y+y_step, ...)
 * and stored contiguously in the buffer: interleaved row sharding across GPUs. */
int hipcy_path_trace_rows(hipcy_device *dev, const hipcy_work_tile *tile, int y_step);
/* Several RenderTiles in one device pass (all with the same sample range):
 * the plugin acquires up to n tiles from the Session (DeviceTask::acquire_tile,
 * device_task.h) and renders them together, so small tiles still fill the GPU.
 * Each tile keeps its own buffer, offset and stride. */
int hipcy_path_trace_tiles(hipcy_device *dev, const hipcy_work_tile *tiles, int n_tiles);
/* Tile stream: the RENDER task's acquire_tile / release_tile loop with the
 * tiles fed to one running wavefront (hipcy_render_feed).  acquire fills
 * *tile (and an opaque tag) and returns 1, or 0 when the queue is empty;
 * release is called once for every acquired tile, from the thread that called
 * hipcy_render_feed: when every sample of the tile is in its buffer, or, if
 * the stream fails (a kernel error, an invalid or oversized tile), before
 * hipcy_render_feed returns its error -- hipcy_error() is then already set, so
 * the callback can tell an unfinished tile (CUDADevice::thread_run releases
 * every tile it acquired, device_cuda_impl.cpp:2361-2388).  cancelled (may be
 * NULL) stops the acquisition; tiles already acquired are finished.  hold is
 * the device's target of acquired-but-unfinished pixel-samples (0: the
 * hipcy_set_stream_hold value): tiles are acquired only while the unclaimed
 * work is below it.  It is approximate: tiles are taken whole (or in sample
 * chunks of a quarter of the record ring), and a tile stays held until its
 * last path ends, so a device may hold up to about twice `hold` (more with
 * holds of a few tiles).  Devices sharing one queue each take tiles only as
 * fast as they finish them. */
typedef struct hipcy_tile_feed {
  void *user;
  int (*acquire)(void *user, hipcy_work_tile *tile, uint64_t *tag);
  void (*release)(void *user, const hipcy_work_tile *tile, uint64_t tag);
  int (*cancelled)(void *user);
  uint64_t hold;
} hipcy_tile_feed;
int hipcy_render_feed(hipcy_device *dev, const hipcy_tile_feed *feed);
/* Default hold of tile streams, in pixel-samples (initially 0: twice the slot
 * pool of hipcy_set_slots, i.e. every slot in flight and as much in reserve,
 * what a device alone on the queue wants).  0 keeps the value. */
int hipcy_set_stream_hold(hipcy_device *dev, uint64_t pixel_samples);
int hipcy_synchronize(hipcy_device *dev);
int hipcy_get_stats(const hipcy_device *dev, hipcy_stats *out);
/* flags: bit 0 = per-kernel HIP-event timings (kernels then run on one stream,
 * without overlap, so each launch is timed alone), bit 1 = traversal counters. */
int hipcy_set_profiling(hipcy_device *dev, int flags);

/* DeviceTask SHADER: input uint4 per element, output float4 per element
 * accumulated (+=) num_samples times over [shader_x, shader_x + shader_w).
 * SHADER_EVAL_BACKGROUND: input (u, v float bits) of the world map, output the
 * background radiance (kernel_bake.h:474-510).  SHADER_EVAL_DISPLACE: input
 * (object, prim, u float bits, v float bits) of a mesh vertex, output the
 * object-space displacement of the shader's displacement program
 * (kernel_bake.h:446-472; MeshManager::displace, render/mesh_displace.cpp). */
#define HIPCY_SHADER_EVAL_DISPLACE 0   /* kernel_types.h:203 */
#define HIPCY_SHADER_EVAL_BACKGROUND 1 /* kernel_types.h:204 */
int hipcy_shader_eval(hipcy_device *dev, int eval_type, uint64_t input, uint64_t output, int shader_x,
                      int shader_w, int offset, int num_samples);
/* FILM_CONVERT task: the display pass (KernelFilm.display_pass_*) of pixels
 * (x..x+w-1, y..y+h-1) of `buffer` (pass_stride floats per pixel) is converted
 * to sRGB uchar4 into rgba_byte, or (rgba_byte == 0) to 4 halfs into rgba_half,
 * at pixel index offset + x + y*stride of either; sample_scale = 1 / samples
 * rendered (the reference passes 1/(task.sample+1)).  Halfs follow the CPU
 * device's truncating conversion (util_half.h:80-118). */
int hipcy_film_convert(hipcy_device *dev, uint64_t buffer, uint64_t rgba_byte, uint64_t rgba_half,
                       float sample_scale, int x, int y, int w, int h, int offset, int stride);

/* rays: n x 8 floats (P.xyz, D.xyz, t, visibility bits) in device memory;
 * out_f: n x 3 (t, u, v); out_i: n x 4 (hit, prim, object, type).
 * any_hit != 0 runs the opaque-shadow traversal. */
int hipcy_intersect(hipcy_device *dev, uint64_t rays, uint64_t out_f, uint64_t out_i, int n, int any_hit);
/* xys: n x 3 ints (x, y, sample); out: n x 8 floats (P.xyz, D.xyz, t, rng_hash bits). */
int hipcy_camera_rays(hipcy_device *dev, uint64_t xys, uint64_t out, int n);

#ifdef __cplusplus
}
#endif

#endif /* HIPCYCLES_H */
