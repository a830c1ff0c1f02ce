/*
 * cy_types.h — enums and register-resident records of the path integrator.
 *
 * Numeric values are those of the reference device ABI (they appear in the
 * uploaded data: shader flags in __tri_shader / __shaders, visibility bits in
 * __prim_visibility and BVH nodes, closure ids in SVM bytecode):
 *   PathRayFlag        kernel_types.h:262-334
 *   ClosureLabel       kernel_types.h:338-348
 *   ShaderFlag         kernel_types.h:540-556
 *   PrimitiveType      kernel_types.h:690-713
 *   ShaderDataFlag     kernel_types.h:832-893
 *   ShaderNodeType     svm/svm_types.h:60-162
 *   ClosureType        svm/svm_types.h:518-608
 */
#ifndef CY_TYPES_H
#define CY_TYPES_H

#include "cy_math.h"

enum {
  PATH_RAY_CAMERA = (1 << 0),
  PATH_RAY_REFLECT = (1 << 1),
  PATH_RAY_TRANSMIT = (1 << 2),
  PATH_RAY_DIFFUSE = (1 << 3),
  PATH_RAY_GLOSSY = (1 << 4),
  PATH_RAY_SINGULAR = (1 << 5),
  PATH_RAY_TRANSPARENT = (1 << 6),
  PATH_RAY_SHADOW_OPAQUE_NON_CATCHER = (1 << 7),
  PATH_RAY_SHADOW_OPAQUE_CATCHER = (1 << 8),
  PATH_RAY_SHADOW_OPAQUE = (1 << 7) | (1 << 8),
  PATH_RAY_SHADOW_TRANSPARENT_NON_CATCHER = (1 << 9),
  PATH_RAY_SHADOW_TRANSPARENT_CATCHER = (1 << 10),
  PATH_RAY_SHADOW_TRANSPARENT = (1 << 9) | (1 << 10),
  PATH_RAY_SHADOW_NON_CATCHER = (1 << 7) | (1 << 9),
  PATH_RAY_SHADOW = (1 << 7) | (1 << 8) | (1 << 9) | (1 << 10),
  PATH_RAY_VOLUME_SCATTER = (1 << 12),
  PATH_RAY_NODE_UNALIGNED = (1 << 13),
  PATH_RAY_ALL_VISIBILITY = ((1 << 14) - 1),
  PATH_RAY_MIS_SKIP = (1 << 14),
  PATH_RAY_DIFFUSE_ANCESTOR = (1 << 15),
  PATH_RAY_SINGLE_PASS_DONE = (1 << 16),
  PATH_RAY_SHADOW_CATCHER = (1 << 17),
  PATH_RAY_STORE_SHADOW_INFO = (1 << 18),
  PATH_RAY_TRANSPARENT_BACKGROUND = (1 << 19),
  PATH_RAY_TERMINATE_IMMEDIATE = (1 << 20),
  PATH_RAY_TERMINATE_AFTER_TRANSPARENT = (1 << 21),
  PATH_RAY_TERMINATE = (1 << 20) | (1 << 21),
  PATH_RAY_EMISSION = (1 << 22)
};

enum {
  LABEL_NONE = 0,
  LABEL_TRANSMIT = 1,
  LABEL_REFLECT = 2,
  LABEL_DIFFUSE = 4,
  LABEL_GLOSSY = 8,
  LABEL_SINGULAR = 16,
  LABEL_TRANSPARENT = 32,
  LABEL_VOLUME_SCATTER = 64,
  LABEL_TRANSMIT_TRANSPARENT = 128
};

#define SHADER_SMOOTH_NORMAL (1u << 31)
#define SHADER_CAST_SHADOW (1u << 30)
#define SHADER_AREA_LIGHT (1u << 29)
#define SHADER_USE_MIS (1u << 28)
#define SHADER_EXCLUDE_DIFFUSE (1u << 27)
#define SHADER_EXCLUDE_GLOSSY (1u << 26)
#define SHADER_EXCLUDE_TRANSMIT (1u << 25)
#define SHADER_EXCLUDE_CAMERA (1u << 24)
#define SHADER_EXCLUDE_SCATTER (1u << 23)
#define SHADER_EXCLUDE_ANY \
  (SHADER_EXCLUDE_DIFFUSE | SHADER_EXCLUDE_GLOSSY | SHADER_EXCLUDE_TRANSMIT | \
   SHADER_EXCLUDE_CAMERA | SHADER_EXCLUDE_SCATTER)
#define SHADER_MASK (~(SHADER_SMOOTH_NORMAL | SHADER_CAST_SHADOW | SHADER_AREA_LIGHT | \
                       SHADER_USE_MIS | SHADER_EXCLUDE_ANY))

#define PRIMITIVE_TRIANGLE (1 << 0)
#define PRIMITIVE_MOTION_TRIANGLE (1 << 1)
#define PRIMITIVE_ALL_TRIANGLE (PRIMITIVE_TRIANGLE | PRIMITIVE_MOTION_TRIANGLE)
#define PRIMITIVE_ALL_CURVE ((1 << 2) | (1 << 3) | (1 << 4) | (1 << 5))
#define PRIMITIVE_ALL (PRIMITIVE_ALL_TRIANGLE | PRIMITIVE_ALL_CURVE)

#define OBJECT_NONE (~0)
#define PRIM_NONE (~0)
#define LAMP_NONE (~0)
#define SHADER_NONE (~0)

enum {
  SD_BACKFACING = (1 << 0),
  SD_EMISSION = (1 << 1),
  SD_BSDF = (1 << 2),
  SD_BSDF_HAS_EVAL = (1 << 3),
  SD_BSSRDF = (1 << 4),
  SD_HOLDOUT = (1 << 5),
  SD_EXTINCTION = (1 << 6),
  SD_SCATTER = (1 << 7),
  SD_TRANSPARENT = (1 << 9),
  SD_BSDF_NEEDS_LCG = (1 << 10),
  SD_USE_MIS = (1 << 16),
  SD_HAS_TRANSPARENT_SHADOW = (1 << 17),
  SD_HAS_VOLUME = (1 << 18),
  SD_HAS_ONLY_VOLUME = (1 << 19),
  SD_HETEROGENEOUS_VOLUME = (1 << 20),
  SD_HAS_BSSRDF_BUMP = (1 << 21),
  SD_VOLUME_EQUIANGULAR = (1 << 22),
  SD_VOLUME_MIS = (1 << 23),
  SD_VOLUME_CUBIC = (1 << 24),
  SD_HAS_BUMP = (1 << 25),
  SD_HAS_DISPLACEMENT = (1 << 26),
  SD_HAS_CONSTANT_EMISSION = (1 << 27),
  SD_NEED_VOLUME_ATTRIBUTES = (1 << 28),
  SD_CLOSURE_FLAGS = (SD_EMISSION | SD_BSDF | SD_BSDF_HAS_EVAL | SD_BSSRDF | SD_HOLDOUT | SD_EXTINCTION |
                      SD_SCATTER | SD_BSDF_NEEDS_LCG), /* kernel_types.h:869-870 (no SD_TRANSPARENT) */
  SD_SHADER_FLAGS = (SD_USE_MIS | SD_HAS_TRANSPARENT_SHADOW | SD_HAS_VOLUME | SD_HAS_ONLY_VOLUME |
                     SD_HETEROGENEOUS_VOLUME | SD_HAS_BSSRDF_BUMP | SD_VOLUME_EQUIANGULAR | SD_VOLUME_MIS |
                     SD_VOLUME_CUBIC | SD_HAS_BUMP | SD_HAS_DISPLACEMENT | SD_HAS_CONSTANT_EMISSION |
                     SD_NEED_VOLUME_ATTRIBUTES)
};

enum {
  SD_OBJECT_HOLDOUT_MASK = (1 << 0),
  SD_OBJECT_MOTION = (1 << 1),
  SD_OBJECT_TRANSFORM_APPLIED = (1 << 2),
  SD_OBJECT_NEGATIVE_SCALE_APPLIED = (1 << 3),
  SD_OBJECT_HAS_VOLUME = (1 << 4),
  SD_OBJECT_INTERSECTS_VOLUME = (1 << 5),
  SD_OBJECT_HAS_VERTEX_MOTION = (1 << 6),
  SD_OBJECT_SHADOW_CATCHER = (1 << 7),
  SD_OBJECT_HAS_VOLUME_ATTRIBUTES = (1 << 8),
  SD_OBJECT_FLAGS = (SD_OBJECT_HOLDOUT_MASK | SD_OBJECT_MOTION | SD_OBJECT_TRANSFORM_APPLIED |
                     SD_OBJECT_NEGATIVE_SCALE_APPLIED | SD_OBJECT_HAS_VOLUME | SD_OBJECT_INTERSECTS_VOLUME |
                     SD_OBJECT_SHADOW_CATCHER | SD_OBJECT_HAS_VOLUME_ATTRIBUTES)
};

/* NodeNormalMapSpace (svm_types.h:455-461) */
enum {
  NODE_NORMAL_MAP_TANGENT = 0,
  NODE_NORMAL_MAP_OBJECT = 1,
  NODE_NORMAL_MAP_WORLD = 2,
};

/* ShaderNodeType (svm_types.h:60-162) — the subset the HIP interpreter runs. */
enum {
  NODE_END = 0,
  NODE_SHADER_JUMP = 1,
  NODE_SET_DISPLACEMENT = 20,
  NODE_DISPLACEMENT = 21,
  NODE_VECTOR_DISPLACEMENT = 22,
  NODE_CLOSURE_BSDF = 2,
  NODE_CLOSURE_EMISSION = 3,
  NODE_CLOSURE_BACKGROUND = 4,
  NODE_CLOSURE_SET_WEIGHT = 5,
  NODE_CLOSURE_WEIGHT = 6,
  NODE_EMISSION_WEIGHT = 7,
  NODE_MIX_CLOSURE = 8,
  NODE_JUMP_IF_ZERO = 9,
  NODE_JUMP_IF_ONE = 10,
  NODE_VALUE_F = 14,
  NODE_VALUE_V = 15,
  NODE_TEX_IMAGE = 23,
  NODE_TEX_IMAGE_BOX = 24,
  NODE_TEX_ENVIRONMENT = 55,
  NODE_FRESNEL = 38,
  NODE_LAYER_WEIGHT = 39,
  NODE_CLOSURE_VOLUME = 40,
  NODE_PRINCIPLED_VOLUME = 41
};

#define NODE_LAYER_WEIGHT_FRESNEL 0

/* ClosureType (svm_types.h:518-584). */
enum {
  CLOSURE_NONE_ID = 0,
  CLOSURE_BSDF_ID = 1,
  CLOSURE_BSDF_DIFFUSE_ID = 2,
  CLOSURE_BSDF_OREN_NAYAR_ID = 3,
  CLOSURE_BSDF_PRINCIPLED_DIFFUSE_ID = 5,
  CLOSURE_BSDF_PRINCIPLED_SHEEN_ID = 6,
  CLOSURE_BSDF_DIFFUSE_TOON_ID = 7,
  CLOSURE_BSDF_TRANSLUCENT_ID = 8,
  CLOSURE_BSDF_REFLECTION_ID = 9,
  CLOSURE_BSDF_MICROFACET_GGX_ID = 10,
  CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID = 11,
  CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID = 12,
  CLOSURE_BSDF_MICROFACET_BECKMANN_ID = 13,
  CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID = 14,
  CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID = 15,
  CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID = 16,
  CLOSURE_BSDF_ASHIKHMIN_VELVET_ID = 17,
  CLOSURE_BSDF_GLOSSY_TOON_ID = 20,
  CLOSURE_BSDF_HAIR_REFLECTION_ID = 21,
  CLOSURE_BSDF_REFRACTION_ID = 22,
  CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID = 23,
  CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID = 24,
  CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID = 25,
  CLOSURE_BSDF_MICROFACET_BECKMANN_GLASS_ID = 26,
  CLOSURE_BSDF_MICROFACET_GGX_GLASS_ID = 27,
  CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID = 28,
  CLOSURE_BSDF_SHARP_GLASS_ID = 29,
  CLOSURE_BSDF_HAIR_PRINCIPLED_ID = 30,
  CLOSURE_BSDF_HAIR_TRANSMISSION_ID = 31,
  CLOSURE_BSDF_BSSRDF_ID = 32,
  CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID = 33,
  CLOSURE_BSDF_TRANSPARENT_ID = 34,
  CLOSURE_BSSRDF_CUBIC_ID = 35,
  CLOSURE_BSSRDF_GAUSSIAN_ID = 36,
  CLOSURE_BSSRDF_PRINCIPLED_ID = 37,
  CLOSURE_BSSRDF_BURLEY_ID = 38,
  CLOSURE_BSSRDF_RANDOM_WALK_ID = 39,
  CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID = 40,
  CLOSURE_HOLDOUT_ID = 41,
  CLOSURE_VOLUME_ID = 42,
  CLOSURE_VOLUME_ABSORPTION_ID = 43,
  CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID = 44,
  CLOSURE_BSDF_PRINCIPLED_ID = 45,
  NBUILTIN_CLOSURES = 46
};

#define CLOSURE_IS_BSDF(type) ((type) <= CLOSURE_BSDF_TRANSPARENT_ID)
#define CLOSURE_IS_BSDF_DIFFUSE(type) \
  ((type) >= CLOSURE_BSDF_DIFFUSE_ID && (type) <= CLOSURE_BSDF_TRANSLUCENT_ID)
#define CLOSURE_IS_BSDF_OR_BSSRDF(type) ((type) <= 40)
#define CLOSURE_IS_BSDF_SINGULAR(type) \
  ((type) == CLOSURE_BSDF_REFLECTION_ID || (type) == CLOSURE_BSDF_REFRACTION_ID || \
   (type) == CLOSURE_BSDF_TRANSPARENT_ID)
#define CLOSURE_IS_BSDF_MICROFACET(type) \
  (((type) >= CLOSURE_BSDF_MICROFACET_GGX_ID && (type) <= CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID) || \
   ((type) >= CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID && \
    (type) <= CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID) || \
   ((type) == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID))
#define CLOSURE_IS_HOLDOUT(type) ((type) == CLOSURE_HOLDOUT_ID)
#define CLOSURE_IS_BSSRDF(type) ((type) >= CLOSURE_BSSRDF_CUBIC_ID && (type) <= CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID)
#define CLOSURE_IS_VOLUME(type) ((type) >= CLOSURE_VOLUME_ID && (type) <= CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID)
#define CLOSURE_IS_PHASE(type) ((type) == CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID)
#define CLOSURE_IS_DISK_BSSRDF(type) ((type) >= CLOSURE_BSSRDF_CUBIC_ID && (type) <= CLOSURE_BSSRDF_BURLEY_ID)
#define BSSRDF_MIN_RADIUS 1e-8f   /* kernel_types.h:49-51 */
#define BSSRDF_MAX_BOUNCES 256
#define BSSRDF_MAX_HITS 4 /* kernel_types.h:50 */
#define VOLUME_BOUNDS_MAX 1024    /* kernel_types.h:54 */

#define CLOSURE_WEIGHT_CUTOFF 1e-5f
#define SVM_STACK_INVALID 255

/* PathTraceDimension (kernel_types.h:232-256). */
enum {
  PRNG_FILTER_U = 0,
  PRNG_FILTER_V = 1,
  PRNG_LENS_U = 2,
  PRNG_BASE_NUM = 10,
  PRNG_BSDF_U = 0,
  PRNG_BSDF_V = 1,
  PRNG_LIGHT_U = 2,
  PRNG_LIGHT_V = 3,
  PRNG_LIGHT_TERMINATE = 4,
  PRNG_TERMINATE = 5,
  PRNG_PHASE_CHANNEL = 6,
  PRNG_SCATTER_DISTANCE = 7,
  PRNG_BOUNCE_NUM = 8
};

#define FILTER_TABLE_SIZE 1024
#define SOBOL_SKIP 64
#define BVH_STACK_SIZE 192
#define ENTRYPOINT_SENTINEL 0x76543210

/* Device error codes (written to the error word; first error wins). */
enum {
  CY_ERR_NONE = 0,
  CY_ERR_SVM_NODE = 1,        /* unsupported SVM node type */
  CY_ERR_CLOSURE = 2,         /* unsupported closure type */
  CY_ERR_SVM_STACK = 3,       /* SVM stack offset beyond the HIP stack */
  CY_ERR_BVH_STACK = 4,       /* traversal stack overflow */
  CY_ERR_PRIMITIVE = 5,       /* unsupported primitive (curve / motion) */
  CY_ERR_FEATURE = 6          /* unsupported scene feature reached at run time */
};

#ifndef CY_MAX_CLOSURE
#  define CY_MAX_CLOSURE 8 /* per-kernel closure array (k_shade.hip builds 1, 2, 4, 8) */
#endif
#define CY_SVM_STACK 32
/* Near-tie window of the wide BVH's exact closest hit (cy_bvhw.h), and the
 * bit k_intersect_closest sets in a stored primitive index whose ray the
 * shading stage re-traces in the reference's order (cy_integrator.h). */
#define CY_TIE_EPS (1.0f / 1048576.0f)
#define CY_PRIM_TIE (1 << 30)
/* 1: the SVM interpreter includes the texture / converter / input nodes
 * (cy_svm_nodes.h) and non-constant world shaders; the shading kernel is also
 * built with 0 for scenes that use neither (hipcy_load_kernels picks). */
#ifndef CY_SVM_TEX
#  define CY_SVM_TEX 1
#endif
/* threads per workgroup of every wavefront kernel, and LDS-resident traversal
 * stack depth (CY_LDS_STACK * CY_BLOCK * 4 B = 32 KiB per workgroup) */
#define CY_BLOCK 256
/* decoupled volume segments (cy_volume_decoupled.h): at most this many steps,
 * each CyVolumeStep in CY_DECOUPLED_STEP_BYTES of the slot's record */
#ifndef CY_DECOUPLED_STEPS
#  define CY_DECOUPLED_STEPS 1024
#endif
#define CY_DECOUPLED_STEP_BYTES 64
#define CY_LDS_STACK 32

/* LDS-qualified pointers: per-thread stacks and closure arrays carved out of a
 * __shared__ array are addressed through these so the compiler emits ds_*
 * instructions (a generic pointer would become flat_* accesses, which wait on
 * the vector-memory counter too).  Plain pointers on the host. */
#if defined(__HIP_DEVICE_COMPILE__)
#  define CY_LDS __attribute__((address_space(3)))
#else
#  define CY_LDS
#endif
typedef struct __attribute__((aligned(8))) CyStackEntry {
  int node;
  float t;
} CyStackEntry;

typedef struct CyRay {
  cfloat3 P;
  cfloat3 D;
  float t;
} CyRay;

/* ray differentials (kernel_types.h differential3 / differential) */
typedef struct CyDiff3 {
  cfloat3 dx, dy;
} CyDiff3;
typedef struct CyDiff {
  float dx, dy;
} CyDiff;

typedef struct CyIsect {
  float t, u, v;
  int prim;
  int object;
  int type;
} CyIsect;

/* One closure record.  CY_CLOSURE_EXT selects the closure set compiled in:
 * 1 (default) every closure of cy_closures.h, 15 dwords per record; 0 the
 * basic set the bench scene uses (diffuse, isotropic GGX, sharp reflection /
 * refraction / glass, transparent), 11 dwords, built into the shade kernels
 * without texture nodes (k_shade.hip) so their LDS and register budget stay
 * what they were before the extended closures existed.  Per-type use of the
 * parameter slots is listed at the top of cy_closures.h. */
#ifndef CY_CLOSURE_EXT
#  define CY_CLOSURE_EXT 1
#endif
typedef struct CyClosure {
  cfloat3 weight;
  int type;
  float sample_weight;
  cfloat3 N;
  float alpha_x, alpha_y, ior;
#if CY_CLOSURE_EXT
  cfloat3 T;  /* tangent of anisotropic microfacets */
  int extra;  /* MicrofacetExtra slot in the closure array, -1 for none */
#endif
} CyClosure;

typedef struct CySD {
  cfloat3 P, N, Ng, I;
  int shader;
  int flag;
  int object_flag;
  int prim;
  int type;
  float u, v;
  int object;
  int lamp; /* the light of a PRIMITIVE_LAMP shading point (read only then) */
  float ray_length;
  int num_closure;
  int num_closure_left;
  cfloat3 svm_closure_weight;
  cfloat3 closure_emission_background;
  cfloat3 closure_transparent_extinction;
#ifdef CY_DBG_X
  bool dbg = false; /* debugging builds: the traced path's shading point */
#endif
  /* working memory of the shade stage (CyShadeMem): CY_MAX_CLOSURE closures
   * and the SVM stack, element i at svm_stack[i * svm_stride] */
  CyClosure *closure;
  float *svm_stack;
  int svm_stride;
  int svm_fast;     /* entries [0, svm_fast) at svm_stack[i * svm_stride] */
  float *svm_spill; /* entries [svm_fast, CY_SVM_STACK) at svm_spill[i - svm_fast] */
#if CY_CLOSURE_EXT
  /* sd->lcg_state of closures with SD_BSDF_NEEDS_LCG (multiscatter GGX): set
   * after shader evaluation, stepped by every evaluation and sample of such a
   * closure; mutable because evaluation otherwise reads the shading point
   * only (the reference passes ShaderData by non-const pointer for it) */
  mutable uint lcg_state;
  /* surface derivatives (__DPDU__): hair closures, the Tangent node fallback */
  cfloat3 dPdu, dPdv;
  /* ray differentials at the shading point (__RAY_DIFFERENTIALS__): the Bump
   * node and the *_BUMP_DX / _DY nodes; zero unless CyGlobals.use_ray_diff */
  CyDiff3 dP, dI;
  CyDiff du, dv;
#endif
} CySD;

/* Where a shading thread keeps its closures and SVM stack.  The device kernel
 * points them into LDS (per-thread strided columns) with the deep end of the
 * stack in private memory; the host uses private arrays. */
typedef struct CyShadeMem {
  CyClosure *closure;
  float *svm_stack;
  int svm_stride;
  int svm_fast;
  float *svm_spill;
} CyShadeMem;

typedef struct CyPathState {
  int flag;
  uint rng_hash;
  int rng_offset;
  int sample;
  int num_samples;
  int bounce;
  int diffuse_bounce;
  int glossy_bounce;
  int transmission_bounce;
  int transparent_bounce;
  float min_ray_pdf;
  float ray_pdf;
  float ray_t;
  int volume_bounce;        /* volume scenes only (cy_volume.h) */
  int volume_bounds_bounce;
#ifdef CY_DBG_X
  bool dbg; /* debugging builds: this path is the traced one (CY_DBG_*) */
#endif
} CyPathState;

/* Debugging builds (-DCY_DBG_X=x -DCY_DBG_Y=y -DCY_DBG_S=sample): the shading
 * stage prints the bit patterns of its intermediate values for one path, on
 * the device (printf) and in the host emulation alike, so that the first
 * differing line names the operation (tools/dbg_trace.py). */
#ifdef CY_DBG_X
#  define CY_DBGF(st, ...) \
    do { \
      if ((st)->dbg) { \
        printf(__VA_ARGS__); \
      } \
    } while (0)
#  define CY_DBG3(st, tag, v) \
    CY_DBGF(st, "%s %08x %08x %08x\n", tag, __builtin_bit_cast(unsigned, (v).x), \
            __builtin_bit_cast(unsigned, (v).y), __builtin_bit_cast(unsigned, (v).z))
#  define CY_DBG1(st, tag, f) CY_DBGF(st, "%s %08x\n", tag, __builtin_bit_cast(unsigned, (float)(f)))
#else
#  define CY_DBGF(st, ...) \
    do { \
    } while (0)
#  define CY_DBG3(st, tag, v) CY_DBGF(st)
#  define CY_DBG1(st, tag, f) CY_DBGF(st)
#endif

#endif /* CY_TYPES_H */
