/*
 * hipcycles_kernel_types.h — the Cycles device-data ABI as seen by the HIP device.
 *
 * These are the structs the unchanged Cycles host uploads through
 * Device::const_copy_to("__data", ...) and Device::mem_copy_to(<named array>):
 * KernelData (blender/intern/cycles/kernel/kernel_types.h:1447-1455) and the
 * per-element records of the named arrays in kernel/kernel_textures.h:21-87.
 * The layout must match the reference byte for byte; every field is listed once
 * in an X-macro so that the struct definitions, the Python ctypes mirror
 * (raytracingproject_amd/abi.py) and the offset checker run against the
 * reference headers (oracle/ref_harness.cpp, tests/test_abi_layout.py) all
 * derive from this single list.
 *
 * Field order follows kernel_types.h:1118-1572 (KernelCamera ... KernelBake),
 * 1575-1670 (KernelObject, KernelLight, KernelLightDistribution, KernelShader),
 * 1551-1562 (KernelParticle),
 * util/util_transform.h:31 (Transform) and util/util_projection.h:26.
 *
 * Plain C, no HIP or torch types: included by host C/C++, by HIP device code
 * and parsed by Python.
 */
#ifndef HIPCYCLES_KERNEL_TYPES_H
#define HIPCYCLES_KERNEL_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hc_float2 { float x, y; } hc_float2;
typedef struct __attribute__((aligned(16))) hc_float4 { float x, y, z, w; } hc_float4;
typedef struct __attribute__((aligned(16))) hc_uint4 { uint32_t x, y, z, w; } hc_uint4;
typedef struct __attribute__((aligned(16))) hc_Transform { hc_float4 x, y, z; } hc_Transform;

/* util_texture.h:93-107 TextureInfo (96 bytes: Transform is 16-byte aligned
 * on the reference CPU build).  One per SVM image slot in __texture_info;
 * `data` is the image's device address (a host pointer on the CPU device). */
typedef struct __attribute__((aligned(16))) hc_TextureInfo {
  uint64_t data;
  uint32_t data_type, cl_buffer, interpolation, extension;
  uint32_t width, height, depth, use_transform_3d;
  hc_Transform transform_3d;
} hc_TextureInfo;
typedef struct __attribute__((aligned(16))) hc_ProjectionTransform { hc_float4 x, y, z, w; } hc_ProjectionTransform;

/* X(type, name, count) — count > 1 declares an array. */

#define HC_KERNEL_CAMERA_FIELDS(X) \
  X(int32_t, type, 1) \
  X(int32_t, panorama_type, 1) \
  X(float, fisheye_fov, 1) \
  X(float, fisheye_lens, 1) \
  X(hc_float4, equirectangular_range, 1) \
  X(float, interocular_offset, 1) \
  X(float, convergence_distance, 1) \
  X(float, pole_merge_angle_from, 1) \
  X(float, pole_merge_angle_to, 1) \
  X(hc_Transform, cameratoworld, 1) \
  X(hc_ProjectionTransform, rastertocamera, 1) \
  X(hc_float4, dx, 1) \
  X(hc_float4, dy, 1) \
  X(float, aperturesize, 1) \
  X(float, blades, 1) \
  X(float, bladesrotation, 1) \
  X(float, focaldistance, 1) \
  X(float, shuttertime, 1) \
  X(int32_t, num_motion_steps, 1) \
  X(int32_t, have_perspective_motion, 1) \
  X(float, nearclip, 1) \
  X(float, cliplength, 1) \
  X(float, sensorwidth, 1) \
  X(float, sensorheight, 1) \
  X(float, width, 1) \
  X(float, height, 1) \
  X(int32_t, resolution, 1) \
  X(float, inv_aperture_ratio, 1) \
  X(int32_t, is_inside_volume, 1) \
  X(hc_ProjectionTransform, screentoworld, 1) \
  X(hc_ProjectionTransform, rastertoworld, 1) \
  X(hc_ProjectionTransform, ndctoworld, 1) \
  X(hc_ProjectionTransform, worldtoscreen, 1) \
  X(hc_ProjectionTransform, worldtoraster, 1) \
  X(hc_ProjectionTransform, worldtondc, 1) \
  X(hc_Transform, worldtocamera, 1) \
  X(hc_ProjectionTransform, perspective_pre, 1) \
  X(hc_ProjectionTransform, perspective_post, 1) \
  X(hc_Transform, motion_pass_pre, 1) \
  X(hc_Transform, motion_pass_post, 1) \
  X(int32_t, shutter_table_offset, 1) \
  X(int32_t, rolling_shutter_type, 1) \
  X(float, rolling_shutter_duration, 1) \
  X(int32_t, pad, 1)

#define HC_KERNEL_FILM_FIELDS(X) \
  X(float, exposure, 1) \
  X(int32_t, pass_flag, 1) \
  X(int32_t, light_pass_flag, 1) \
  X(int32_t, pass_stride, 1) \
  X(int32_t, use_light_pass, 1) \
  X(int32_t, pass_combined, 1) \
  X(int32_t, pass_depth, 1) \
  X(int32_t, pass_normal, 1) \
  X(int32_t, pass_motion, 1) \
  X(int32_t, pass_motion_weight, 1) \
  X(int32_t, pass_uv, 1) \
  X(int32_t, pass_object_id, 1) \
  X(int32_t, pass_material_id, 1) \
  X(int32_t, pass_diffuse_color, 1) \
  X(int32_t, pass_glossy_color, 1) \
  X(int32_t, pass_transmission_color, 1) \
  X(int32_t, pass_diffuse_indirect, 1) \
  X(int32_t, pass_glossy_indirect, 1) \
  X(int32_t, pass_transmission_indirect, 1) \
  X(int32_t, pass_volume_indirect, 1) \
  X(int32_t, pass_diffuse_direct, 1) \
  X(int32_t, pass_glossy_direct, 1) \
  X(int32_t, pass_transmission_direct, 1) \
  X(int32_t, pass_volume_direct, 1) \
  X(int32_t, pass_emission, 1) \
  X(int32_t, pass_background, 1) \
  X(int32_t, pass_ao, 1) \
  X(float, pass_alpha_threshold, 1) \
  X(int32_t, pass_shadow, 1) \
  X(float, pass_shadow_scale, 1) \
  X(int32_t, filter_table_offset, 1) \
  X(int32_t, cryptomatte_passes, 1) \
  X(int32_t, cryptomatte_depth, 1) \
  X(int32_t, pass_cryptomatte, 1) \
  X(int32_t, pass_adaptive_aux_buffer, 1) \
  X(int32_t, pass_sample_count, 1) \
  X(int32_t, pass_mist, 1) \
  X(float, mist_start, 1) \
  X(float, mist_inv_depth, 1) \
  X(float, mist_falloff, 1) \
  X(int32_t, pass_denoising_data, 1) \
  X(int32_t, pass_denoising_clean, 1) \
  X(int32_t, denoising_flags, 1) \
  X(int32_t, pass_aov_color, 1) \
  X(int32_t, pass_aov_value, 1) \
  X(int32_t, pass_aov_color_num, 1) \
  X(int32_t, pass_aov_value_num, 1) \
  X(int32_t, pad1, 1) \
  X(int32_t, pad2, 1) \
  X(int32_t, pad3, 1) \
  X(hc_float4, xyz_to_r, 1) \
  X(hc_float4, xyz_to_g, 1) \
  X(hc_float4, xyz_to_b, 1) \
  X(hc_float4, rgb_to_y, 1) \
  X(int32_t, pass_bake_primitive, 1) \
  X(int32_t, pass_bake_differential, 1) \
  X(int32_t, pad, 1) \
  X(int32_t, display_pass_stride, 1) \
  X(int32_t, display_pass_components, 1) \
  X(int32_t, display_divide_pass_stride, 1) \
  X(int32_t, use_display_exposure, 1) \
  X(int32_t, use_display_pass_alpha, 1) \
  X(int32_t, pad4, 1) \
  X(int32_t, pad5, 1) \
  X(int32_t, pad6, 1)

#define HC_KERNEL_BACKGROUND_FIELDS(X) \
  X(int32_t, surface_shader, 1) \
  X(int32_t, volume_shader, 1) \
  X(float, volume_step_size, 1) \
  X(int32_t, transparent, 1) \
  X(float, transparent_roughness_squared_threshold, 1) \
  X(float, ao_factor, 1) \
  X(float, ao_distance, 1) \
  X(float, ao_bounces_factor, 1) \
  X(float, portal_weight, 1) \
  X(int32_t, num_portals, 1) \
  X(int32_t, portal_offset, 1) \
  X(float, sun_weight, 1) \
  X(hc_float4, sun, 1) \
  X(float, map_weight, 1) \
  X(int32_t, map_res_x, 1) \
  X(int32_t, map_res_y, 1) \
  X(int32_t, use_mis, 1)

#define HC_KERNEL_INTEGRATOR_FIELDS(X) \
  X(int32_t, use_direct_light, 1) \
  X(int32_t, use_ambient_occlusion, 1) \
  X(int32_t, num_distribution, 1) \
  X(int32_t, num_all_lights, 1) \
  X(float, pdf_triangles, 1) \
  X(float, pdf_lights, 1) \
  X(float, light_inv_rr_threshold, 1) \
  X(int32_t, min_bounce, 1) \
  X(int32_t, max_bounce, 1) \
  X(int32_t, max_diffuse_bounce, 1) \
  X(int32_t, max_glossy_bounce, 1) \
  X(int32_t, max_transmission_bounce, 1) \
  X(int32_t, max_volume_bounce, 1) \
  X(int32_t, ao_bounces, 1) \
  X(int32_t, transparent_min_bounce, 1) \
  X(int32_t, transparent_max_bounce, 1) \
  X(int32_t, transparent_shadows, 1) \
  X(int32_t, caustics_reflective, 1) \
  X(int32_t, caustics_refractive, 1) \
  X(float, filter_glossy, 1) \
  X(int32_t, seed, 1) \
  X(float, sample_clamp_direct, 1) \
  X(float, sample_clamp_indirect, 1) \
  X(int32_t, branched, 1) \
  X(int32_t, volume_decoupled, 1) \
  X(int32_t, diffuse_samples, 1) \
  X(int32_t, glossy_samples, 1) \
  X(int32_t, transmission_samples, 1) \
  X(int32_t, ao_samples, 1) \
  X(int32_t, mesh_light_samples, 1) \
  X(int32_t, subsurface_samples, 1) \
  X(int32_t, sample_all_lights_direct, 1) \
  X(int32_t, sample_all_lights_indirect, 1) \
  X(int32_t, use_lamp_mis, 1) \
  X(int32_t, sampling_pattern, 1) \
  X(int32_t, aa_samples, 1) \
  X(int32_t, adaptive_min_samples, 1) \
  X(int32_t, adaptive_step, 1) \
  X(int32_t, adaptive_stop_per_sample, 1) \
  X(float, adaptive_threshold, 1) \
  X(int32_t, use_volumes, 1) \
  X(int32_t, volume_max_steps, 1) \
  X(float, volume_step_rate, 1) \
  X(int32_t, volume_samples, 1) \
  X(int32_t, start_sample, 1) \
  X(int32_t, max_closures, 1) \
  X(int32_t, pad1, 1) \
  X(int32_t, pad2, 1)

/* KernelBVH without Embree/OptiX: "int scene, pad2" (kernel_types.h:1430-1441). */
#define HC_KERNEL_BVH_FIELDS(X) \
  X(int32_t, root, 1) \
  X(int32_t, have_motion, 1) \
  X(int32_t, have_curves, 1) \
  X(int32_t, bvh_layout, 1) \
  X(int32_t, use_bvh_steps, 1) \
  X(int32_t, curve_subdivisions, 1) \
  X(int32_t, scene, 1) \
  X(int32_t, pad2, 1)

#define HC_KERNEL_TABLES_FIELDS(X) \
  X(int32_t, beckmann_offset, 1) \
  X(int32_t, pad1, 1) \
  X(int32_t, pad2, 1) \
  X(int32_t, pad3, 1)

#define HC_KERNEL_BAKE_FIELDS(X) \
  X(int32_t, object_index, 1) \
  X(int32_t, tri_offset, 1) \
  X(int32_t, type, 1) \
  X(int32_t, pass_filter, 1)

#define HC_KERNEL_OBJECT_FIELDS(X) \
  X(hc_Transform, tfm, 1) \
  X(hc_Transform, itfm, 1) \
  X(float, surface_area, 1) \
  X(float, pass_id, 1) \
  X(float, random_number, 1) \
  X(float, color, 3) \
  X(int32_t, particle_index, 1) \
  X(float, dupli_generated, 3) \
  X(float, dupli_uv, 2) \
  X(int32_t, numkeys, 1) \
  X(int32_t, numsteps, 1) \
  X(int32_t, numverts, 1) \
  X(uint32_t, patch_map_offset, 1) \
  X(uint32_t, attribute_map_offset, 1) \
  X(uint32_t, motion_offset, 1) \
  X(float, cryptomatte_object, 1) \
  X(float, cryptomatte_asset, 1) \
  X(float, shadow_terminator_offset, 1) \
  X(float, pad1, 1) \
  X(float, pad2, 1) \
  X(float, pad3, 1)

/* KernelLight: the trailing union {spot, area, distant} is 12 floats
 * (KernelAreaLight is the largest: axisu[3], invarea, axisv[3], pad1, dir[3], pad2). */
#define HC_KERNEL_LIGHT_FIELDS(X) \
  X(int32_t, type, 1) \
  X(float, co, 3) \
  X(int32_t, shader_id, 1) \
  X(int32_t, samples, 1) \
  X(float, max_bounces, 1) \
  X(float, random, 1) \
  X(float, strength, 3) \
  X(float, pad1, 1) \
  X(hc_Transform, tfm, 1) \
  X(hc_Transform, itfm, 1) \
  X(float, uni, 12)

/* KernelLightDistribution: union {mesh_light{shader_flag, object_id}, lamp{pad, size}}. */
#define HC_KERNEL_LIGHT_DISTRIBUTION_FIELDS(X) \
  X(float, totarea, 1) \
  X(int32_t, prim, 1) \
  X(int32_t, shader_flag, 1) \
  X(int32_t, object_id, 1)

#define HC_KERNEL_SHADER_FIELDS(X) \
  X(float, constant_emission, 3) \
  X(float, cryptomatte_id, 1) \
  X(int32_t, flags, 1) \
  X(int32_t, pass_id, 1) \
  X(int32_t, pad2, 1) \
  X(int32_t, pad3, 1)

/* KernelParticle (kernel_types.h:1551-1562): the Particle Info node's record */
#define HC_KERNEL_PARTICLE_FIELDS(X) \
  X(int32_t, index, 1) \
  X(float, age, 1) \
  X(float, lifetime, 1) \
  X(float, size, 1) \
  X(hc_float4, rotation, 1) \
  X(hc_float4, location, 1) \
  X(hc_float4, velocity, 1) \
  X(hc_float4, angular_velocity, 1)

#define HC_FIELD_DECL(type, name, count) type name[count];
#define HC_FIELD_DECL1(type, name, count) HC_FIELD_DECL_##count(type, name)
#define HC_FIELD_DECL_1(type, name) type name;
#define HC_FIELD_DECL_2(type, name) type name[2];
#define HC_FIELD_DECL_3(type, name) type name[3];
#define HC_FIELD_DECL_12(type, name) type name[12];

#define HC_DECLARE_STRUCT(NAME, FIELDS) \
  typedef struct __attribute__((aligned(16))) NAME { FIELDS(HC_FIELD_DECL1) } NAME;

HC_DECLARE_STRUCT(hc_KernelCamera, HC_KERNEL_CAMERA_FIELDS)
HC_DECLARE_STRUCT(hc_KernelFilm, HC_KERNEL_FILM_FIELDS)
HC_DECLARE_STRUCT(hc_KernelBackground, HC_KERNEL_BACKGROUND_FIELDS)
HC_DECLARE_STRUCT(hc_KernelIntegrator, HC_KERNEL_INTEGRATOR_FIELDS)
HC_DECLARE_STRUCT(hc_KernelBVH, HC_KERNEL_BVH_FIELDS)
HC_DECLARE_STRUCT(hc_KernelTables, HC_KERNEL_TABLES_FIELDS)
HC_DECLARE_STRUCT(hc_KernelBake, HC_KERNEL_BAKE_FIELDS)
HC_DECLARE_STRUCT(hc_KernelObject, HC_KERNEL_OBJECT_FIELDS)
HC_DECLARE_STRUCT(hc_KernelLight, HC_KERNEL_LIGHT_FIELDS)
HC_DECLARE_STRUCT(hc_KernelLightDistribution, HC_KERNEL_LIGHT_DISTRIBUTION_FIELDS)
HC_DECLARE_STRUCT(hc_KernelShader, HC_KERNEL_SHADER_FIELDS)
HC_DECLARE_STRUCT(hc_KernelParticle, HC_KERNEL_PARTICLE_FIELDS)

typedef struct __attribute__((aligned(16))) hc_KernelData {
  hc_KernelCamera cam;
  hc_KernelFilm film;
  hc_KernelBackground background;
  hc_KernelIntegrator integrator;
  hc_KernelBVH bvh;
  hc_KernelTables tables;
  hc_KernelBake bake;
} hc_KernelData;

/* Sizes measured against the reference headers. */
#define HC_SIZEOF_KERNEL_DATA 1584

#ifdef __cplusplus
}
#endif

#endif /* HIPCYCLES_KERNEL_TYPES_H */
