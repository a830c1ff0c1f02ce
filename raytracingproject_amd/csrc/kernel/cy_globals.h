/*
 * cy_globals.h — device-side view of the scene the Cycles host uploads.
 *
 * CyGlobals is the HIP analogue of the reference's KernelGlobals
 * (kernel/kernel_globals.h:131-137 for CUDA: one __constant__ pointer per named
 * array of kernel/kernel_textures.h:21-87 plus the KernelData block).  It is
 * passed by value as a kernel argument, so every pointer lives in SGPRs and every
 * KernelData field is a scalar (s_load) read.
 */
#ifndef CY_GLOBALS_H
#define CY_GLOBALS_H

#include "hipcycles_kernel_types.h"
#include "cy_math.h"

/* Names of the kernel_textures.h arrays the HIP path binds (bind_global). */
#define CY_GLOBAL_ARRAYS(X) \
  X(hc_float4, __bvh_nodes) \
  X(hc_float4, __bvh_leaf_nodes) \
  X(hc_float4, __prim_tri_verts) \
  X(uint32_t, __prim_tri_index) \
  X(uint32_t, __prim_type) \
  X(uint32_t, __prim_visibility) \
  X(uint32_t, __prim_index) \
  X(uint32_t, __prim_object) \
  X(uint32_t, __object_node) \
  X(hc_KernelObject, __objects) \
  X(uint32_t, __object_flag) \
  X(uint32_t, __tri_shader) \
  X(hc_float4, __tri_vnormal) \
  X(hc_uint4, __tri_vindex) \
  X(hc_KernelLightDistribution, __light_distribution) \
  X(hc_KernelLight, __lights) \
  X(hc_float2, __light_background_marginal_cdf) \
  X(hc_float2, __light_background_conditional_cdf) \
  X(hc_uint4, __svm_nodes) \
  X(hc_KernelShader, __shaders) \
  X(float, __lookup_table) \
  X(uint32_t, __sample_pattern_lut) \
  X(hc_TextureInfo, __texture_info) \
  X(hc_float4, __curves) \
  X(hc_float4, __curve_keys) \
  X(float, __object_volume_step) \
  X(hc_uint4, __attributes_map) \
  X(float, __attributes_float) \
  X(hc_float2, __attributes_float2) \
  X(hc_float4, __attributes_float3) \
  X(uint32_t, __attributes_uchar4) \
  X(float, __ies) \
  X(hc_KernelParticle, __particles)

typedef struct CyGlobals {
  const hc_KernelData *data;
#define CY_DECL_PTR(type, name) const type *name;
  CY_GLOBAL_ARRAYS(CY_DECL_PTR)
#undef CY_DECL_PTR
  /* device-internal W-wide BVH widened from __bvh_nodes/__bvh_leaf_nodes
   * (csrc/host/cy_bvhw_collapse.h); nullptr when traversing the BVH2 */
  const void *bvhw_nodes;
  /* per object: wide node index of the root of its own BVH (instanced
   * geometry; the W-wide counterpart of __object_node), or nullptr */
  const int *bvhw_object_root;
  /* 1 when __prim_tri_index[i] == 3 * i for every primitive (checked when the
   * BVH is widened): triangle vertices are then read without the indirection */
  int tri_index_identity;
  /* 1 when some object keeps its own transform (instanced geometry): enables
   * the instance paths of shading and light sampling (uniform branch) */
  int have_instancing;
  /* KernelBVH.have_curves: hair segments in the BVH (BVH2 traversal with
   * unaligned nodes and curve leaves; shading reads __prim_type) */
  int have_curves;
  /* 1 when a shader reads ray differentials (Bump / *_BUMP_DX / _DY nodes):
   * the paths carry dP / dD (CyPathBuffers.ray_diff) and shading points get
   * dP, dI, du, dv; otherwise they are zero */
  int use_ray_diff;
  /* wide nodes 0 .. bvhw_top-1 (the top levels, breadth first) are read from
   * the traversal kernels' LDS copy (cy_bvhw.h CY_LDS_TOP); 0 = none */
  int bvhw_top;
  /* W of the wide layout (4 or 8) when bvhw_nodes is set, else 0 */
  int bvhw_width;
} CyGlobals;

#endif /* CY_GLOBALS_H */
