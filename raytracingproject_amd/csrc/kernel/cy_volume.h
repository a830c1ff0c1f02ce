/*
 * cy_volume.h — volumes in the shading and shadow stages.
 *
 * The reference integrates volumes in one of two ways, chosen by
 * KernelIntegrator.volume_decoupled: the CPU device records every ray-marching
 * step and samples the segment afterwards (decoupled), GPU devices
 * (device_cuda.cpp: info.has_volume_decoupled = false) integrate with
 * distance sampling while stepping.  The HIP device is a GPU device: its host
 * uploads volume_decoupled = 0 and the CPU kernel, given the same KernelData,
 * runs the same distance-sampling branch (kernel_path.h:230-247), which is what
 * the parity tests compare.  Restated here in the reference's arithmetic:
 *   kernel_volume_stack_init (camera outside volumes)  kernel_volume.h:1165-1190
 *   kernel_volume_stack_enter_exit                     kernel_volume.h:1293-1334
 *   kernel_volume_clean_stack                          kernel_volume.h:1408-1420
 *   shader_setup_from_volume                           kernel_shader.h:444-487
 *   shader_merge_closures                              kernel_shader.h:493-520
 *   shader_eval_volume                                 kernel_shader.h:1250-1308
 *   volume_shader_extinction_sample / _sample          kernel_volume.h:40-93
 *   volume_stack_step_size                             kernel_volume.h:110-143
 *   kernel_volume_step_init                            kernel_volume.h:176-192
 *   kernel_volume_shadow (+ homogeneous/heterogeneous) kernel_volume.h:199-294
 *   kernel_volume_distance_sample, emission_integrate  kernel_volume.h:343-399
 *   kernel_volume_integrate (+ homogeneous/
 *     heterogeneous_distance)                          kernel_volume.h:439-711
 *   Henyey-Greenstein phase eval / sample              closure/volume.h:36-165
 *   shader_volume_phase_eval / _sample                 kernel_shader.h:1118-1220
 *   kernel_path_volume_bounce                          kernel_path_volume.h:63-128
 * The path-level flow (where the segment is integrated, direct light from a
 * scatter point, the stack updates at volume boundaries, shadow segments) is in
 * cy_integrator.h.  Volume attributes (voxel grids) are not packed by the host,
 * so find_attribute never finds one and the principled volume's density and
 * colour come from its sockets alone.
 *
 * shader_eval_volume, volume_shadow and volume_integrate are out-of-line
 * calls (CY_NOINLINE): each runs the SVM interpreter, and a shading or shadow
 * kernel reaches them from several places.
 *
 * The volume stack of a path lives in HBM next to the other slot records
 * (CyPathBuffers.vol_stack, CY_VOLUME_STACK entries per slot); the device
 * refuses scenes whose volume objects could overflow it.
 */
#ifndef CY_VOLUME_H
#define CY_VOLUME_H

#if CY_CLOSURE_EXT

#define CY_VOLUME_STACK 16 /* entries incl. the terminator (reference VOLUME_STACK_SIZE 32) */

typedef struct CyVolumeEntry {
  int object;
  int shader;
} CyVolumeEntry;

typedef struct CyVolumeStack {
  CyVolumeEntry e[CY_VOLUME_STACK];
} CyVolumeStack;

enum { VOLUME_PATH_SCATTERED = 0, VOLUME_PATH_ATTENUATED = 1, VOLUME_PATH_MISSED = 2 };

typedef struct CyVolumeCoeff {
  cfloat3 sigma_t, sigma_s, emission;
} CyVolumeCoeff;

/* kernel_volume_stack_init with kernel_data.cam.is_inside_volume == 0 (the
 * device refuses a camera inside a volume): only the world volume. */
CY_FN void volume_stack_init(const CyGlobals *kg, CyVolumeStack *stack)
{
  if (KD->background.volume_shader != SHADER_NONE) {
    stack->e[0].shader = KD->background.volume_shader;
    stack->e[0].object = PRIM_NONE;
    stack->e[1].shader = SHADER_NONE;
    stack->e[1].object = 0;
  }
  else {
    stack->e[0].shader = SHADER_NONE;
    stack->e[0].object = 0;
  }
}

/* kernel_volume_stack_enter_exit for a surface with these flag / object /
 * shader: a backfacing hit leaves the object's volume, a front hit enters it. */
CY_FN void volume_stack_enter_exit(int sd_flag, int sd_object, int sd_shader, CyVolumeStack *stack)
{
  if (!(sd_flag & SD_HAS_VOLUME)) {
    return;
  }
  if (sd_flag & SD_BACKFACING) {
    for (int i = 0; stack->e[i].shader != SHADER_NONE; i++) {
      if (stack->e[i].object == sd_object) {
        do {
          stack->e[i] = stack->e[i + 1];
          i++;
        } while (stack->e[i].shader != SHADER_NONE);
        return;
      }
    }
  }
  else {
    int i;
    for (i = 0; stack->e[i].shader != SHADER_NONE; i++) {
      if (stack->e[i].object == sd_object) {
        return;
      }
    }
    if (i >= CY_VOLUME_STACK - 1) {
      return;
    }
    stack->e[i].shader = sd_shader;
    stack->e[i].object = sd_object;
    stack->e[i + 1].shader = SHADER_NONE;
  }
}

/* The volume objects' surfaces along a ray: scene_intersect_volume_all with
 * 2 * VOLUME_STACK_SIZE records (kernel_volume.h:1198-1199, 1366-1367),
 * sorted by distance as qsort with intersections_compare does it
 * (kernel_volume.h:1206, 1371; glibc's merge sort keeps equal distances in
 * recording order). */
#define CY_VOLUME_ALL_HITS 64
#define CY_REF_VOLUME_STACK 32 /* kernel_types.h VOLUME_STACK_SIZE */
CY_FN uint volume_all_sorted(const CyGlobals *kg, const CyRay *ray, CyIsect *hits, uint visibility, uint *err)
{
  if (!scene_intersect_valid(ray)) {
    return 0;
  }
  const uint n = kg->have_curves ?
                     bvh2_volume_all<true, 3>(kg, ray, hits, CY_VOLUME_ALL_HITS, visibility, err) :
                     bvh2_volume_all<true>(kg, ray, hits, CY_VOLUME_ALL_HITS, visibility, err);
  for (uint i = 1; i < n; i++) {
    const CyIsect h = hits[i];
    int j = (int)i - 1;
    while (j >= 0 && hits[j].t > h.t) {
      hits[j + 1] = hits[j];
      j--;
    }
    hits[j + 1] = h;
  }
  return n;
}

/* kernel_volume_stack_init (kernel_volume.h:1165-1306), __VOLUME_RECORD_ALL__
 * branch: with kernel_data.cam.is_inside_volume the camera ray, made infinite,
 * collects the volumes it leaves without having entered them; stack_sd is
 * scratch.  A stack beyond CY_VOLUME_STACK entries, or more entered volumes
 * than the reference's array holds, sets an error instead. */
CY_NOINLINE void volume_stack_init_camera(const CyGlobals *kg, CySD *stack_sd, const CyRay *ray, uint path_flag,
                                          CyVolumeStack *stack, uint *err)
{
  if (!KD->cam.is_inside_volume) {
    volume_stack_init(kg, stack);
    return;
  }
  CyRay volume_ray = *ray;
  volume_ray.t = CY_FLT_MAX;
  CyIsect hits[CY_VOLUME_ALL_HITS];
  const uint num_hits = volume_all_sorted(kg, &volume_ray, hits, path_flag & PATH_RAY_ALL_VISIBILITY, err);
  int stack_index = 0, enclosed_index = 0;
  int enclosed_volumes[CY_REF_VOLUME_STACK];
  for (uint hit = 0; hit < num_hits; hit++) {
    shader_setup_from_ray(kg, stack_sd, &hits[hit], &volume_ray);
    if (stack_sd->flag & SD_BACKFACING) {
      bool need_add = true;
      for (int i = 0; i < enclosed_index && need_add; i++) {
        if (enclosed_volumes[i] == stack_sd->object) {
          need_add = false;
        }
      }
      for (int i = 0; i < stack_index && need_add; i++) {
        if (stack->e[i].object == stack_sd->object) {
          need_add = false;
          break;
        }
      }
      if (need_add && stack_index < CY_REF_VOLUME_STACK - 1) {
        if (stack_index >= CY_VOLUME_STACK - 1) {
          cy_set_error(err, CY_ERR_FEATURE, 14); /* more nested volumes than the device's stack */
          break;
        }
        stack->e[stack_index].object = stack_sd->object;
        stack->e[stack_index].shader = stack_sd->shader;
        ++stack_index;
      }
    }
    else {
      if (enclosed_index >= CY_REF_VOLUME_STACK) {
        cy_set_error(err, CY_ERR_FEATURE, 14); /* beyond the reference's enclosed_volumes */
        break;
      }
      enclosed_volumes[enclosed_index++] = stack_sd->object;
    }
  }
  /* kernel_volume.h:1293-1305: no volume found and no world volume (a world
   * volume is not put back when the camera is found in the air) */
  if (stack_index == 0 && KD->background.volume_shader == SHADER_NONE) {
    stack->e[0].shader = KD->background.volume_shader;
    stack->e[0].object = OBJECT_NONE;
    stack->e[1].shader = SHADER_NONE;
  }
  else {
    stack->e[stack_index].shader = SHADER_NONE;
  }
}

/* kernel_volume_stack_update_for_subsurface (kernel_volume.h:1354-1375): the
 * volume surfaces between the path's previous surface point and a subsurface
 * exit point enter or leave their volumes on the exit ray's stack. */
CY_NOINLINE void volume_stack_update_for_subsurface(const CyGlobals *kg, CySD *stack_sd, const CyRay *ray,
                                                    CyVolumeStack *stack, uint *err)
{
  CyIsect hits[CY_VOLUME_ALL_HITS];
  const uint num_hits = volume_all_sorted(kg, ray, hits, PATH_RAY_ALL_VISIBILITY, err);
  for (uint hit = 0; hit < num_hits; hit++) {
    shader_setup_from_ray(kg, stack_sd, &hits[hit], ray);
    volume_stack_enter_exit(stack_sd->flag, stack_sd->object, stack_sd->shader, stack);
  }
}

/* kernel_volume_clean_stack: after a miss only the world's volume stays. */
CY_FN void volume_stack_clean(const CyGlobals *kg, CyVolumeStack *stack)
{
  if (KD->background.volume_shader != SHADER_NONE) {
    stack->e[1].shader = SHADER_NONE;
  }
  else {
    stack->e[0].shader = SHADER_NONE;
  }
}

CY_FN void shader_setup_from_volume(CySD *sd, const CyRay *ray, CyShadeMem mem)
{
  sd->closure = mem.closure;
  sd->svm_stack = mem.svm_stack;
  sd->svm_stride = mem.svm_stride;
  sd->svm_fast = mem.svm_fast;
  sd->svm_spill = mem.svm_spill;
  sd->P = ray->P;
  sd->N = neg3(ray->D);
  sd->Ng = neg3(ray->D);
  sd->I = neg3(ray->D);
  sd->shader = SHADER_NONE;
  sd->flag = 0;
  sd->object_flag = 0;
  sd->ray_length = 0.0f;
  sd->object = OBJECT_NONE;
  sd->prim = PRIM_NONE;
  sd->type = 0; /* PRIMITIVE_NONE */
  sd->u = 0.0f;
  sd->v = 0.0f;
#if CY_CLOSURE_EXT
  sd->dPdu = mk3(0.0f, 0.0f, 0.0f);
  sd->dPdv = mk3(0.0f, 0.0f, 0.0f);
  /* the reference's dP here is the segment ray's dD (kernel_shader.h:474-479),
   * read by no node a volume program runs: zero */
  sd_zero_differentials(sd);
#endif
  sd->num_closure = 0;
  sd->num_closure_left = 0;
  sd->svm_closure_weight = mk3(0.0f, 0.0f, 0.0f);
  sd->closure_emission_background = mk3(0.0f, 0.0f, 0.0f);
  sd->closure_transparent_extinction = mk3(0.0f, 0.0f, 0.0f);
}

/* shader_merge_closures: a volume holds phase closures only (bsdf_merge:
 * Henyey-Greenstein closures with equal g merge, other types never). */
CY_FN void shader_merge_volume_closures(CySD *sd)
{
  for (int i = 0; i < sd->num_closure; i++) {
    CyClosure *sci = &sd->closure[i];
    for (int j = i + 1; j < sd->num_closure; j++) {
      CyClosure *scj = &sd->closure[j];
      if (sci->type != scj->type) {
        continue;
      }
      if (!(sci->type == CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID && sci->alpha_x == scj->alpha_x)) {
        continue;
      }
      sci->weight = add3(sci->weight, scj->weight);
      sci->sample_weight += scj->sample_weight;
      const int size = sd->num_closure - (j + 1);
      for (int k = 0; k < size; k++) {
        scj[k] = scj[k + 1];
      }
      sd->num_closure--;
      j--;
    }
  }
}

/* shader_eval_volume: the closures of every volume on the stack, accumulated
 * into one array (merged after the second). */
CY_NOINLINE void shader_eval_volume(
    const CyGlobals *kg, CySD *sd, const CyPathState *state, const CyVolumeStack *stack, int path_flag, uint *err)
{
  const int max_closures = (path_flag & (PATH_RAY_TERMINATE | PATH_RAY_SHADOW | PATH_RAY_EMISSION)) ?
                               0 :
                               KD->integrator.max_closures;
  sd->num_closure = 0;
  sd->num_closure_left = (max_closures < CY_MAX_CLOSURE) ? max_closures : CY_MAX_CLOSURE; /* see shader_eval_surface */
  sd->flag = 0;
  sd->object_flag = 0;
  for (int i = 0; stack->e[i].shader != SHADER_NONE; i++) {
    sd->object = stack->e[i].object;
    sd->shader = stack->e[i].shader;
    sd->flag &= ~SD_SHADER_FLAGS;
    sd->flag |= (int)kg->__shaders[(uint)sd->shader & SHADER_MASK].flags;
    sd->object_flag &= ~SD_OBJECT_FLAGS;
    if (sd->object != OBJECT_NONE) {
      sd->object_flag |= (int)kg->__object_flag[sd->object];
    }
    svm_eval_nodes(kg, sd, state, path_flag, err, 1);
    if (i > 0) {
      shader_merge_volume_closures(sd);
    }
  }
}

/* object_volume_density (geom_object.h:325-332): KernelObject.surface_area
 * holds the density scale of volume objects (1 here, object.cpp:378-389). */
CY_FN float object_volume_density(const CyGlobals *kg, int object)
{
  return (object == OBJECT_NONE) ? 1.0f : kg->__objects[object].surface_area;
}

CY_FN float object_volume_step_size(const CyGlobals *kg, int object)
{
  return (object == OBJECT_NONE) ? KD->background.volume_step_size : kg->__object_volume_step[object];
}

CY_FN bool volume_shader_extinction_sample(const CyGlobals *kg, CySD *sd, const CyPathState *state,
                                           const CyVolumeStack *stack, cfloat3 P, cfloat3 *extinction, uint *err)
{
  sd->P = P;
  shader_eval_volume(kg, sd, state, stack, PATH_RAY_SHADOW, err);
  if (sd->flag & SD_EXTINCTION) {
    const float density = object_volume_density(kg, sd->object);
    *extinction = mul3f(sd->closure_transparent_extinction, density);
    return true;
  }
  return false;
}

CY_FN bool volume_shader_sample(const CyGlobals *kg, CySD *sd, const CyPathState *state, const CyVolumeStack *stack,
                                cfloat3 P, CyVolumeCoeff *coeff, uint *err)
{
  sd->P = P;
  shader_eval_volume(kg, sd, state, stack, state->flag, err);
  if (!(sd->flag & (SD_EXTINCTION | SD_SCATTER | SD_EMISSION))) {
    return false;
  }
  coeff->sigma_s = mk3(0.0f, 0.0f, 0.0f);
  coeff->sigma_t = (sd->flag & SD_EXTINCTION) ? sd->closure_transparent_extinction : mk3(0.0f, 0.0f, 0.0f);
  coeff->emission = (sd->flag & SD_EMISSION) ? sd->closure_emission_background : mk3(0.0f, 0.0f, 0.0f);
  if (sd->flag & SD_SCATTER) {
    for (int i = 0; i < sd->num_closure; i++) {
      const CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_VOLUME(sc->type)) {
        coeff->sigma_s = add3(coeff->sigma_s, sc->weight);
      }
    }
  }
  const float density = object_volume_density(kg, sd->object);
  coeff->sigma_s = mul3f(coeff->sigma_s, density);
  coeff->sigma_t = mul3f(coeff->sigma_t, density);
  coeff->emission = mul3f(coeff->emission, density);
  return true;
}

/* volume_stack_step_size: the smallest step of the heterogeneous volumes on
 * the stack, FLT_MAX when all are homogeneous. */
CY_FN float volume_stack_step_size(const CyGlobals *kg, const CyVolumeStack *stack)
{
  float step_size = CY_FLT_MAX;
  for (int i = 0; stack->e[i].shader != SHADER_NONE; i++) {
    const int shader_flag = (int)kg->__shaders[(uint)stack->e[i].shader & SHADER_MASK].flags;
    bool heterogeneous = false;
    if (shader_flag & SD_HETEROGENEOUS_VOLUME) {
      heterogeneous = true;
    }
    else if (shader_flag & SD_NEED_VOLUME_ATTRIBUTES) {
      const int object = stack->e[i].object;
      if (object != OBJECT_NONE && (kg->__object_flag[object] & SD_OBJECT_HAS_VOLUME_ATTRIBUTES)) {
        heterogeneous = true;
      }
    }
    if (heterogeneous) {
      float object_step_size = object_volume_step_size(kg, stack->e[i].object);
      object_step_size *= KD->integrator.volume_step_rate;
      step_size = fminf(object_step_size, step_size);
    }
  }
  return step_size;
}

/* kernel_random.h:207-219 path_state_rng_1D_hash */
CY_FN float path_state_rng_1D_hash(const CyGlobals *kg, const CyPathState *s, uint hash)
{
  return path_rng_1D(kg, cmj_hash_simple(s->rng_hash, hash), s->sample, s->rng_offset);
}

CY_FN void volume_step_init(const CyGlobals *kg, const CyPathState *state, float object_step_size, float t,
                            float *step_size, float *step_offset)
{
  const int max_steps = KD->integrator.volume_max_steps;
  float step = (object_step_size < t) ? object_step_size : t;
  if (t > max_steps * step) {
    step = t / (float)max_steps;
  }
  *step_size = step;
  *step_offset = path_state_rng_1D_hash(kg, state, 0x1e31d8a4) * step;
}

/* kernel_volume_shadow: attenuation of a segment with no surface inside it. */
CY_NOINLINE void volume_shadow(const CyGlobals *kg, CySD *sd, const CyPathState *state, const CyVolumeStack *stack,
                         const CyRay *ray, cfloat3 *throughput, CyShadeMem mem, uint *err)
{
  shader_setup_from_volume(sd, ray, mem);
  const float object_step_size = volume_stack_step_size(kg, stack);
  if (object_step_size == CY_FLT_MAX) {
    /* homogeneous: the extinction at the start holds for the whole segment */
    cfloat3 sigma_t = mk3(0.0f, 0.0f, 0.0f);
    if (volume_shader_extinction_sample(kg, sd, state, stack, ray->P, &sigma_t, err)) {
      *throughput = mul3(*throughput, volume_color_transmittance(sigma_t, ray->t));
    }
    return;
  }
  /* heterogeneous: step through, expf only every 8th step */
  cfloat3 tp = *throughput;
  const float tp_eps = 1e-6f;
  const int max_steps = KD->integrator.volume_max_steps;
  float step_offset, step_size;
  volume_step_init(kg, state, object_step_size, ray->t, &step_size, &step_offset);
  float t = 0.0f;
  cfloat3 sum = mk3(0.0f, 0.0f, 0.0f);
  for (int i = 0; i < max_steps; i++) {
    const float new_t = fminf(ray->t, (i + 1) * step_size);
    if (new_t == ray->t) {
      step_offset *= (new_t - t) / step_size;
    }
    const cfloat3 new_P = add3(ray->P, mul3f(ray->D, t + step_offset));
    cfloat3 sigma_t = mk3(0.0f, 0.0f, 0.0f);
    if (volume_shader_extinction_sample(kg, sd, state, stack, new_P, &sigma_t, err)) {
      sum = add3(sum, mul3f(neg3(sigma_t), new_t - t));
      if ((i & 0x07) == 0) {
        tp = mul3(*throughput, mk3(cy_expf(sum.x), cy_expf(sum.y), cy_expf(sum.z)));
        if (tp.x < tp_eps && tp.y < tp_eps && tp.z < tp_eps) {
          break;
        }
      }
    }
    t = new_t;
    if (t == ray->t) {
      tp = mul3(*throughput, mk3(cy_expf(sum.x), cy_expf(sum.y), cy_expf(sum.z)));
      break;
    }
  }
  *throughput = tp;
}

CY_FN float volume_distance_sample(float max_t, cfloat3 sigma_t, int channel, float xi, cfloat3 *transmittance,
                                   cfloat3 *pdf)
{
  const float sample_sigma_t = volume_channel_get(sigma_t, channel);
  const cfloat3 full_transmittance = volume_color_transmittance(sigma_t, max_t);
  const float sample_transmittance = volume_channel_get(full_transmittance, channel);
  const float sample_t = fminf(max_t, -cy_logf(1.0f - xi * (1.0f - sample_transmittance)) / sample_sigma_t);
  *transmittance = volume_color_transmittance(sigma_t, sample_t);
  *pdf = safe_divide_color(mul3(sigma_t, *transmittance), sub3(mk3(1.0f, 1.0f, 1.0f), full_transmittance));
  return sample_t;
}

CY_FN cfloat3 volume_emission_integrate(const CyVolumeCoeff *coeff, int closure_flag, cfloat3 transmittance, float t)
{
  cfloat3 emission = coeff->emission;
  if (closure_flag & SD_EXTINCTION) {
    const cfloat3 sigma_t = coeff->sigma_t;
    emission.x *= (sigma_t.x > 0.0f) ? (1.0f - transmittance.x) / sigma_t.x : t;
    emission.y *= (sigma_t.y > 0.0f) ? (1.0f - transmittance.y) / sigma_t.y : t;
    emission.z *= (sigma_t.z > 0.0f) ? (1.0f - transmittance.z) / sigma_t.z : t;
  }
  else {
    emission = mul3f(emission, t);
  }
  return emission;
}

/* path_radiance_accum_emission (kernel_accumulate.h:304-335) */
CY_FN void volume_accum_emission(const CyGlobals *kg, const CyPathState *state, cfloat3 *L, cfloat3 throughput,
                                 cfloat3 value)
{
  cfloat3 contribution = mul3(throughput, value);
  const float limit = (state->bounce - 1 > 0) ? KD->integrator.sample_clamp_indirect :
                                                KD->integrator.sample_clamp_direct;
  const float sum = fabsf(contribution.x) + fabsf(contribution.y) + fabsf(contribution.z);
  if (sum > limit) {
    contribution = mul3f(contribution, limit / sum);
  }
  *L = add3(*L, contribution);
}

/* kernel_volume_integrate_homogeneous with probalistic_scatter = true */
CY_FN int volume_integrate_homogeneous(const CyGlobals *kg, CyPathState *state, const CyRay *ray, CySD *sd,
                                       const CyVolumeStack *stack, cfloat3 *L, cfloat3 *throughput, uint *err)
{
  CyVolumeCoeff coeff;
  if (!volume_shader_sample(kg, sd, state, stack, ray->P, &coeff, err)) {
    return VOLUME_PATH_MISSED;
  }
  const int closure_flag = sd->flag;
  float t = ray->t;
  cfloat3 new_tp;
  if (closure_flag & SD_SCATTER) {
    const float rphase = path_state_rng_1D(kg, state, PRNG_PHASE_CHANNEL);
    const cfloat3 albedo = safe_divide_color(coeff.sigma_s, coeff.sigma_t);
    cfloat3 channel_pdf;
    const int channel = volume_sample_channel(albedo, *throughput, rphase, &channel_pdf);
    bool scatter = true;
    float xi = path_state_rng_1D(kg, state, PRNG_SCATTER_DISTANCE);
    {
      const float sample_sigma_t = volume_channel_get(coeff.sigma_t, channel);
      const float sample_transmittance = cy_expf(-sample_sigma_t * t);
      if (1.0f - xi >= sample_transmittance) {
        scatter = true;
        xi = 1.0f - (1.0f - xi - sample_transmittance) / (1.0f - sample_transmittance);
      }
      else {
        scatter = false;
      }
    }
    if (scatter) {
      cfloat3 pdf, transmittance;
      const float sample_t = volume_distance_sample(ray->t, coeff.sigma_t, channel, xi, &transmittance, &pdf);
      pdf = mul3(pdf, sub3(mk3(1.0f, 1.0f, 1.0f), volume_color_transmittance(coeff.sigma_t, t)));
      new_tp = div3f(mul3(mul3(*throughput, coeff.sigma_s), transmittance), dot3(channel_pdf, pdf));
      t = sample_t;
    }
    else {
      const cfloat3 transmittance = volume_color_transmittance(coeff.sigma_t, t);
      const float pdf = dot3(channel_pdf, transmittance);
      new_tp = div3f(mul3(*throughput, transmittance), pdf);
    }
  }
  else if (closure_flag & SD_EXTINCTION) {
    new_tp = mul3(*throughput, volume_color_transmittance(coeff.sigma_t, t));
  }
  else {
    new_tp = *throughput;
  }
  if (closure_flag & SD_EMISSION) {
    const cfloat3 transmittance = volume_color_transmittance(coeff.sigma_t, ray->t);
    const cfloat3 emission = volume_emission_integrate(&coeff, closure_flag, transmittance, ray->t);
    volume_accum_emission(kg, state, L, *throughput, emission);
  }
  if (closure_flag & SD_EXTINCTION) {
    *throughput = new_tp;
    if (t < ray->t) {
      sd->P = add3(ray->P, mul3f(ray->D, t));
      return VOLUME_PATH_SCATTERED;
    }
  }
  return VOLUME_PATH_ATTENUATED;
}

/* kernel_volume_integrate_heterogeneous_distance */
CY_FN int volume_integrate_heterogeneous(const CyGlobals *kg, CyPathState *state, const CyRay *ray, CySD *sd,
                                         const CyVolumeStack *stack, cfloat3 *L, cfloat3 *throughput,
                                         float object_step_size, uint *err)
{
  cfloat3 tp = *throughput;
  const float tp_eps = 1e-6f;
  const int max_steps = KD->integrator.volume_max_steps;
  float step_offset, step_size;
  volume_step_init(kg, state, object_step_size, ray->t, &step_size, &step_offset);
  float t = 0.0f;
  cfloat3 accum_transmittance = mk3(1.0f, 1.0f, 1.0f);
  float xi = path_state_rng_1D(kg, state, PRNG_SCATTER_DISTANCE);
  const float rphase = path_state_rng_1D(kg, state, PRNG_PHASE_CHANNEL);
  bool has_scatter = false;
  for (int i = 0; i < max_steps; i++) {
    float new_t = fminf(ray->t, (i + 1) * step_size);
    const float dt = new_t - t;
    if (new_t == ray->t) {
      step_offset *= (new_t - t) / step_size;
    }
    const cfloat3 new_P = add3(ray->P, mul3f(ray->D, t + step_offset));
    CyVolumeCoeff coeff;
    if (volume_shader_sample(kg, sd, state, stack, new_P, &coeff, err)) {
      const int closure_flag = sd->flag;
      cfloat3 new_tp;
      cfloat3 transmittance;
      bool scatter = false;
      if ((closure_flag & SD_SCATTER) || (has_scatter && (closure_flag & SD_EXTINCTION))) {
        has_scatter = true;
        const cfloat3 albedo = safe_divide_color(coeff.sigma_s, coeff.sigma_t);
        cfloat3 channel_pdf;
        const int channel = volume_sample_channel(albedo, tp, rphase, &channel_pdf);
        transmittance = volume_color_transmittance(coeff.sigma_t, dt);
        const float sample_transmittance = volume_channel_get(transmittance, channel);
        if (1.0f - xi >= sample_transmittance) {
          const float sample_sigma_t = volume_channel_get(coeff.sigma_t, channel);
          const float new_dt = -cy_logf(1.0f - xi) / sample_sigma_t;
          new_t = t + new_dt;
          const cfloat3 new_transmittance = volume_color_transmittance(coeff.sigma_t, new_dt);
          const cfloat3 pdf = mul3(coeff.sigma_t, new_transmittance);
          new_tp = div3f(mul3(mul3(tp, coeff.sigma_s), new_transmittance), dot3(channel_pdf, pdf));
          scatter = true;
        }
        else {
          const float pdf = dot3(channel_pdf, transmittance);
          new_tp = div3f(mul3(tp, transmittance), pdf);
          xi = 1.0f - (1.0f - xi) / sample_transmittance;
        }
      }
      else if (closure_flag & SD_EXTINCTION) {
        transmittance = volume_color_transmittance(coeff.sigma_t, dt);
        new_tp = mul3(tp, transmittance);
      }
      else {
        transmittance = mk3(0.0f, 0.0f, 0.0f);
        new_tp = tp;
      }
      if (closure_flag & SD_EMISSION) {
        const cfloat3 emission = volume_emission_integrate(&coeff, closure_flag, transmittance, dt);
        volume_accum_emission(kg, state, L, tp, emission);
      }
      if (closure_flag & SD_EXTINCTION) {
        tp = new_tp;
        if (tp.x < tp_eps && tp.y < tp_eps && tp.z < tp_eps) {
          tp = mk3(0.0f, 0.0f, 0.0f);
          break;
        }
      }
      if (scatter) {
        sd->P = add3(ray->P, mul3f(ray->D, new_t));
        *throughput = tp;
        return VOLUME_PATH_SCATTERED;
      }
      accum_transmittance = mul3(accum_transmittance, transmittance);
    }
    t = new_t;
    if (t == ray->t) {
      break;
    }
  }
  *throughput = tp;
  return VOLUME_PATH_ATTENUATED;
}

/* kernel_volume_integrate: the ray segment through the volumes on the stack */
CY_NOINLINE int volume_integrate(const CyGlobals *kg, CyPathState *state, CySD *sd, const CyVolumeStack *stack,
                           const CyRay *ray, cfloat3 *L, cfloat3 *throughput, float step_size, CyShadeMem mem,
                           uint *err)
{
  shader_setup_from_volume(sd, ray, mem);
  if (step_size != CY_FLT_MAX) {
    return volume_integrate_heterogeneous(kg, state, ray, sd, stack, L, throughput, step_size, err);
  }
  return volume_integrate_homogeneous(kg, state, ray, sd, stack, L, throughput, err);
}

/* ---- Henyey-Greenstein phase function (closure/volume.h) ---------------- */
CY_FN float single_peaked_henyey_greenstein(float cos_theta, float g)
{
  return ((1.0f - g * g) / safe_powf(1.0f + g * g - 2.0f * g * cos_theta, 1.5f)) * (CY_1_PI_F * 0.25f);
}

CY_FN cfloat3 volume_henyey_greenstein_eval_phase(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  const float g = sc->alpha_x;
  if (fabsf(g) < 1e-3f) {
    *pdf = CY_1_PI_F * 0.25f;
  }
  else {
    const float cos_theta = dot3(neg3(I), omega_in);
    *pdf = single_peaked_henyey_greenstein(cos_theta, g);
  }
  return mk3(*pdf, *pdf, *pdf);
}

CY_FN cfloat3 henyey_greenstein_sample(cfloat3 D, float g, float randu, float randv, float *pdf)
{
  float cos_theta;
  if (fabsf(g) < 1e-3f) {
    cos_theta = (1.0f - 2.0f * randu);
    *pdf = CY_1_PI_F * 0.25f;
  }
  else {
    const float k = (1.0f - g * g) / (1.0f - g + 2.0f * g * randu);
    cos_theta = (1.0f + g * g - k * k) / (2.0f * g);
    *pdf = single_peaked_henyey_greenstein(cos_theta, g);
  }
  const float sin_theta = safe_sqrtf(1.0f - cos_theta * cos_theta);
  const float phi = CY_2PI_F * randv;
  const cfloat3 dir = mk3(sin_theta * cy_cosf(phi), sin_theta * cy_sinf(phi), cos_theta);
  cfloat3 T, B;
  make_orthonormals(D, &T, &B);
  return add3(add3(mul3f(T, dir.x), mul3f(B, dir.y)), mul3f(D, dir.z));
}

/* shader_volume_phase_eval: summed phase evals, sample-weighted pdf */
CY_FN cfloat3 shader_volume_phase_eval(const CySD *sd, cfloat3 omega_in, float *pdf)
{
  cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
  float sum_pdf = 0.0f, sum_sample_weight = 0.0f;
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    if (CLOSURE_IS_PHASE(sc->type)) {
      float phase_pdf = 0.0f;
      const cfloat3 e = volume_henyey_greenstein_eval_phase(sc, sd->I, omega_in, &phase_pdf);
      if (phase_pdf != 0.0f) {
        eval = add3(eval, mul3f(e, 1.0f));
        sum_pdf += phase_pdf * sc->sample_weight;
      }
      sum_sample_weight += sc->sample_weight;
    }
  }
  *pdf = (sum_sample_weight > 0.0f) ? sum_pdf / sum_sample_weight : 0.0f;
  return eval;
}

/* shader_volume_phase_sample: one phase closure by sample weight */
CY_FN int shader_volume_phase_sample(const CySD *sd, float randu, float randv, cfloat3 *phase_eval,
                                     cfloat3 *omega_in, float *pdf)
{
  int sampled = 0;
  if (sd->num_closure > 1) {
    float sum = 0.0f;
    for (sampled = 0; sampled < sd->num_closure; sampled++) {
      if (CLOSURE_IS_PHASE(sd->closure[sampled].type)) {
        sum += sd->closure[sampled].sample_weight;
      }
    }
    const float r = randu * sum;
    float partial_sum = 0.0f;
    for (sampled = 0; sampled < sd->num_closure; sampled++) {
      const CyClosure *sc = &sd->closure[sampled];
      if (CLOSURE_IS_PHASE(sc->type)) {
        const float next_sum = partial_sum + sc->sample_weight;
        if (r <= next_sum) {
          randu = (r - partial_sum) / sc->sample_weight;
          break;
        }
        partial_sum = next_sum;
      }
    }
    if (sampled == sd->num_closure) {
      *pdf = 0.0f;
      return LABEL_NONE;
    }
  }
  const CyClosure *sc = &sd->closure[sampled];
  *pdf = 0.0f;
  int label = LABEL_NONE;
  cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
  if (sc->type == CLOSURE_VOLUME_HENYEY_GREENSTEIN_ID) {
    *omega_in = henyey_greenstein_sample(neg3(sd->I), sc->alpha_x, randu, randv, pdf);
    eval = mk3(*pdf, *pdf, *pdf);
    label = LABEL_VOLUME_SCATTER;
  }
  if (*pdf != 0.0f) {
    *phase_eval = eval;
  }
  return label;
}

#endif /* CY_CLOSURE_EXT */

#include "cy_volume_decoupled.h"

#endif /* CY_VOLUME_H */
