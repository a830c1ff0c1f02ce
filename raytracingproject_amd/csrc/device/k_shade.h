/*
 * k_shade.h — launchers of the shade kernel, compiled once per closure-array
 * size (k_shade.hip with CY_MAX_CLOSURE = 1, 2, 4, 8; 16 and 64 for the
 * texture / volume builds).  A scene's
 * KernelIntegrator.max_closures (render/integrator.cpp) picks the smallest
 * variant that holds its shaders' closures, so the per-path closure array
 * stays small enough to live in registers instead of scratch.  Each size is
 * built twice: plain (CY_SVM_TEX=0: closure nodes only, constant world) and
 * "_tex" with the texture / converter / input nodes and node worlds; the
 * plain kernels keep the register allocation of scenes that need no nodes.
 * Scenes with volumes use a third build, "_vol" (CY_VOLUME=1: the "_tex"
 * kernel with the volume stack, segment integration and phase closures).
 */
#ifndef K_SHADE_H
#define K_SHADE_H

#include <hip/hip_runtime.h>

#include "../kernel/cy_integrator.h"

#define CY_SHADE_LAUNCHER_ARGS \
  dim3 grid, dim3 block, hipStream_t stream, const CyGlobals &kg, const CyPathBuffers &b, const CyTile &tile, \
      int cam_n, int slot_base, const int *queue_in, const uint *count_in, int *queue_out, uint *count_out, int *shadow_queue, \
      uint *shadow_count, uint *err

void cy_launch_shade_mc1(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc2(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc4(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc8(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc1_tex(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc2_tex(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc4_tex(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc8_tex(CY_SHADE_LAUNCHER_ARGS);
/* large closure arrays (mixed Principled BSDFs and the like; the reference
 * CPU kernel's MAX_CLOSURE is 64): extended closure set only, in private
 * memory */
void cy_launch_shade_mc16_tex(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc64_tex(CY_SHADE_LAUNCHER_ARGS);
/* the integrator extras (shadow catchers, branched path tracing, light passes;
 * cy_integrator.h CY_CATCHER) on the extended closure set */
void cy_launch_shade_mc8_ext(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc64_ext(CY_SHADE_LAUNCHER_ARGS);
/* the volume extras (decoupled ray marching, camera inside a volume, SSS in
 * volume scenes; cy_integrator.h CY_VOLUME_EXT) */
void cy_launch_shade_mc8_vext(CY_SHADE_LAUNCHER_ARGS);
void cy_launch_shade_mc64_vext(CY_SHADE_LAUNCHER_ARGS);
#define CY_DEVICE_MAX_CLOSURE 64

/* the fused tail kernel (k_shade.hip k_tail_*), plain variants only */
/* lanes of a pass (slot-pool quarters on their own streams, hipcycles.hip) */
#define CY_LANES 4

/* grid.x = blocks for every waiting path; the launcher clamps it to the lane's
 * share of the resident blocks (the tail kernel is persistent), and counts[2]
 * is the kernel's take-next counter (zeroed with counts[0..1]) */
#define CY_TAIL_LAUNCHER_ARGS \
  int W, bool inst, dim3 grid, dim3 block, hipStream_t stream, const CyGlobals &kg, const CyPathBuffers &b, \
      const CyTile &tile, const int *queue_in, const uint *count_in, uint *counts, uint *err
void cy_launch_tail_mc1(CY_TAIL_LAUNCHER_ARGS);
void cy_launch_tail_mc2(CY_TAIL_LAUNCHER_ARGS);
void cy_launch_tail_mc4(CY_TAIL_LAUNCHER_ARGS);
void cy_launch_tail_mc8(CY_TAIL_LAUNCHER_ARGS);

/* false when the scene's shading variant has no tail kernel (texture nodes,
 * volumes, more than 8 closures) */
static inline bool cy_launch_tail(int max_closures, bool tex_nodes, bool volumes, CY_TAIL_LAUNCHER_ARGS)
{
  if (tex_nodes || volumes || max_closures > 8) {
    return false;
  }
  auto fn = max_closures <= 1 ? cy_launch_tail_mc1 :
            max_closures <= 2 ? cy_launch_tail_mc2 :
            max_closures <= 4 ? cy_launch_tail_mc4 :
                                cy_launch_tail_mc8;
  fn(W, inst, grid, block, stream, kg, b, tile, queue_in, count_in, counts, err);
  return true;
}

static inline void cy_launch_shade(int max_closures, bool tex_nodes, bool volumes, bool ext, bool vext,
                                   CY_SHADE_LAUNCHER_ARGS)
{
  /* volume scenes always run _vext (the host sets vext with volumes) */
  (void)volumes;
  auto fn = ext ? (max_closures <= 8 ? cy_launch_shade_mc8_ext : cy_launch_shade_mc64_ext) :
            vext ? (max_closures <= 8 ? cy_launch_shade_mc8_vext : cy_launch_shade_mc64_vext) :
            max_closures > 8 ? (max_closures <= 16 ? cy_launch_shade_mc16_tex : cy_launch_shade_mc64_tex) :
            tex_nodes ? (max_closures <= 1 ? cy_launch_shade_mc1_tex :
                         max_closures <= 2 ? cy_launch_shade_mc2_tex :
                         max_closures <= 4 ? cy_launch_shade_mc4_tex :
                                             cy_launch_shade_mc8_tex) :
                        (max_closures <= 1 ? cy_launch_shade_mc1 :
                         max_closures <= 2 ? cy_launch_shade_mc2 :
                         max_closures <= 4 ? cy_launch_shade_mc4 :
                                             cy_launch_shade_mc8);
  fn(grid, block, stream, kg, b, tile, cam_n, slot_base, queue_in, count_in, queue_out, count_out, shadow_queue, shadow_count, err);
}

#endif
