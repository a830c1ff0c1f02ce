/*
 * cy_volume_decoupled.h — decoupled volume ray marching, the integrator the
 * reference's CPU device runs (KernelIntegrator.volume_decoupled = 1,
 * DeviceInfo::has_volume_decoupled, integrator.cpp:165):
 *   kernel_volume_decoupled_record     kernel/kernel_volume.h:754-905
 *   kernel_volume_decoupled_scatter    kernel/kernel_volume.h:934-1128
 *   kernel_volume_equiangular_sample / _pdf, kernel_volume_distance_pdf
 *                                      kernel/kernel_volume.h:297-372
 *   volume_stack_sampling_method       kernel/kernel_volume.h:145-173
 *   kernel_volume_use_decoupled        kernel/kernel_volume.h:1133-1158
 * The segment's steps live in the slot's record in device memory
 * (CyPathBuffers.dec_steps; private memory for 1024 steps would be 60 KB of
 * scratch per lane, more than the runtime allocates for a full chip), at most
 * CY_DECOUPLED_STEPS of them (the reference mallocs volume_max_steps); a
 * segment that needs more raises CY_ERR_FEATURE 13 instead of being cut.
 * The light connection over all lights and the shade-stage driver are in
 * cy_integrator.h (volume_decoupled_path).
 */
#ifndef CY_VOLUME_DECOUPLED_H
#define CY_VOLUME_DECOUPLED_H

#if CY_CLOSURE_EXT

#ifndef CY_DECOUPLED_STEPS
#  define CY_DECOUPLED_STEPS 1024
#endif

#define SD_VOLUME_EQUIANGULAR (1 << 22) /* kernel_types.h:887 ShaderDataFlag */
#define SD_VOLUME_MIS (1 << 23)

typedef struct CyVolumeStep {
  cfloat3 sigma_s;             /* scatter coefficient */
  cfloat3 sigma_t;             /* extinction coefficient */
  cfloat3 accum_transmittance; /* accumulated transmittance including this step */
  cfloat3 cdf_distance;        /* cumulative density function for distance sampling */
  float t;                     /* distance at end of this step */
  float shade_t;               /* jittered distance where shading was done in step */
  int closure_flag;            /* shader evaluation closure flags */
} CyVolumeStep;
static_assert(sizeof(CyVolumeStep) <= CY_DECOUPLED_STEP_BYTES, "CyPathBuffers.dec_steps stride");

typedef struct CyVolumeSegment {
  CyVolumeStep *steps;
  int numsteps;
  int closure_flag;
  cfloat3 accum_emission;
  cfloat3 accum_transmittance;
  cfloat3 accum_albedo;
  int sampling_method;
} CyVolumeSegment;

/* util_math.h safe_invert_color */
CY_FN cfloat3 safe_invert_color(cfloat3 a)
{
  return mk3((a.x != 0.0f) ? 1.0f / a.x : 0.0f, (a.y != 0.0f) ? 1.0f / a.y : 0.0f, (a.z != 0.0f) ? 1.0f / a.z : 0.0f);
}

/* volume_stack_sampling_method (kernel_volume.h:145-173) */
CY_FN int volume_stack_sampling_method(const CyGlobals *kg, const CyVolumeStack *stack)
{
  if (KD->integrator.num_all_lights == 0) {
    return 0;
  }
  int method = -1;
  for (int i = 0; stack->e[i].shader != SHADER_NONE; i++) {
    const int shader_flag = (int)kg->__shaders[(uint)stack->e[i].shader & SHADER_MASK].flags;
    if (shader_flag & SD_VOLUME_MIS) {
      return SD_VOLUME_MIS;
    }
    else if (shader_flag & SD_VOLUME_EQUIANGULAR) {
      if (method == 0) {
        return SD_VOLUME_MIS;
      }
      method = SD_VOLUME_EQUIANGULAR;
    }
    else {
      if (method == SD_VOLUME_EQUIANGULAR) {
        return SD_VOLUME_MIS;
      }
      method = 0;
    }
  }
  return method;
}

/* kernel_volume_use_decoupled (kernel_volume.h:1133-1158), CPU build */
CY_FN bool volume_use_decoupled(const CyGlobals *kg, bool direct, int sampling_method)
{
  if (!KD->integrator.volume_decoupled) {
    return false;
  }
  if (sampling_method != 0) {
    return true;
  }
  return direct ? KD->integrator.sample_all_lights_direct != 0 : KD->integrator.sample_all_lights_indirect != 0;
}

/* kernel_volume_equiangular_sample (kernel_volume.h:297-317) */
CY_FN float volume_equiangular_sample(const CyRay *ray, cfloat3 light_P, float xi, float *pdf)
{
  const float t = ray->t;
  const float delta = dot3(sub3(light_P, ray->P), ray->D);
  const float D = safe_sqrtf(len_squared3(sub3(light_P, ray->P)) - delta * delta);
  if (D == 0.0f) {
    *pdf = 0.0f;
    return 0.0f;
  }
  const float theta_a = -cy_atan2f(delta, D);
  const float theta_b = cy_atan2f(t - delta, D);
  const float t_ = D * cy_tanf((xi * theta_b) + (1 - xi) * theta_a);
  if (theta_b == theta_a) {
    *pdf = 0.0f;
    return 0.0f;
  }
  *pdf = D / ((theta_b - theta_a) * (D * D + t_ * t_));
  return cmin(t, delta + t_);
}

/* kernel_volume_equiangular_pdf (kernel_volume.h:319-339) */
CY_FN float volume_equiangular_pdf(const CyRay *ray, cfloat3 light_P, float sample_t)
{
  const float delta = dot3(sub3(light_P, ray->P), ray->D);
  const float D = safe_sqrtf(len_squared3(sub3(light_P, ray->P)) - delta * delta);
  if (D == 0.0f) {
    return 0.0f;
  }
  const float t = ray->t;
  const float t_ = sample_t - delta;
  const float theta_a = -cy_atan2f(delta, D);
  const float theta_b = cy_atan2f(t - delta, D);
  if (theta_b == theta_a) {
    return 0.0f;
  }
  return D / ((theta_b - theta_a) * (D * D + t_ * t_));
}

/* kernel_volume_distance_pdf (kernel_volume.h:365-372) */
CY_FN cfloat3 volume_distance_pdf(float max_t, cfloat3 sigma_t, float sample_t)
{
  const cfloat3 full_transmittance = volume_color_transmittance(sigma_t, max_t);
  const cfloat3 transmittance = volume_color_transmittance(sigma_t, sample_t);
  return safe_divide_color(mul3(sigma_t, transmittance), sub3(mk3(1.0f, 1.0f, 1.0f), full_transmittance));
}

/* kernel_volume_decoupled_record (kernel_volume.h:754-905): the volumes'
 * coefficients along the whole segment, one jittered shading point per step
 * (one step for homogeneous volumes), with the accumulated transmittance,
 * emission and albedo and the normalised distance CDF. */
CY_FN void volume_decoupled_record(const CyGlobals *kg, const CyPathState *state, const CyRay *ray, CySD *sd,
                                   const CyVolumeStack *stack, CyVolumeSegment *segment, float object_step_size,
                                   CyVolumeStep *steps, uint *err)
{
  const float tp_eps = 1e-6f;
  int max_steps;
  float step_size, step_offset;
  if (object_step_size != CY_FLT_MAX) {
    max_steps = KD->integrator.volume_max_steps;
    volume_step_init(kg, state, object_step_size, ray->t, &step_size, &step_offset);
  }
  else {
    max_steps = 1;
    step_size = ray->t;
    step_offset = 0.0f;
  }
  segment->steps = steps;
  cfloat3 accum_emission = mk3(0.0f, 0.0f, 0.0f);
  cfloat3 accum_transmittance = mk3(1.0f, 1.0f, 1.0f);
  cfloat3 accum_albedo = mk3(0.0f, 0.0f, 0.0f);
  cfloat3 cdf_distance = mk3(0.0f, 0.0f, 0.0f);
  float t = 0.0f;
  segment->numsteps = 0;
  segment->closure_flag = 0;
  bool is_last_step_empty = false;
  int si = 0; /* steps[si]: the step being written */
  for (int i = 0; i < max_steps; i++, si++) {
    if (si >= CY_DECOUPLED_STEPS) {
      cy_set_error(err, CY_ERR_FEATURE, 13); /* segment longer than CY_DECOUPLED_STEPS steps */
      si = CY_DECOUPLED_STEPS - 1;
      break;
    }
    CyVolumeStep *step = &steps[si];
    const float new_t = cmin(ray->t, (i + 1) * step_size);
    const float dt = new_t - t;
    if (new_t == ray->t) {
      step_offset *= (new_t - t) / step_size;
    }
    const cfloat3 new_P = add3(ray->P, mul3f(ray->D, t + step_offset));
    CyVolumeCoeff coeff;
    if (volume_shader_sample(kg, sd, state, stack, new_P, &coeff, err)) {
      const int closure_flag = sd->flag;
      const cfloat3 sigma_t = coeff.sigma_t;
      if (closure_flag & SD_SCATTER) {
        accum_albedo = add3(accum_albedo, mul3f(safe_divide_color(coeff.sigma_s, sigma_t), dt));
      }
      const cfloat3 transmittance = volume_color_transmittance(sigma_t, dt);
      if (closure_flag & SD_EMISSION) {
        const cfloat3 emission = volume_emission_integrate(&coeff, closure_flag, transmittance, dt);
        accum_emission = add3(accum_emission, mul3(accum_transmittance, emission));
      }
      accum_transmittance = mul3(accum_transmittance, transmittance);
      const cfloat3 pdf_distance = mul3(mul3f(accum_transmittance, dt), coeff.sigma_s);
      cdf_distance = add3(cdf_distance, pdf_distance);
      step->sigma_t = sigma_t;
      step->sigma_s = coeff.sigma_s;
      step->closure_flag = closure_flag;
      segment->closure_flag |= closure_flag;
      is_last_step_empty = false;
      segment->numsteps++;
    }
    else {
      if (is_last_step_empty) {
        /* consecutive empty step, merge */
        si--;
        step = &steps[si];
      }
      else {
        step->sigma_t = mk3(0.0f, 0.0f, 0.0f);
        step->sigma_s = mk3(0.0f, 0.0f, 0.0f);
        step->closure_flag = 0;
        segment->numsteps++;
        is_last_step_empty = true;
      }
    }
    step->accum_transmittance = accum_transmittance;
    step->cdf_distance = cdf_distance;
    step->t = new_t;
    step->shade_t = t + step_offset;
    t = new_t;
    if (t == ray->t) {
      break;
    }
    if (accum_transmittance.x < tp_eps && accum_transmittance.y < tp_eps && accum_transmittance.z < tp_eps) {
      break;
    }
  }
  segment->accum_emission = accum_emission;
  segment->accum_transmittance = accum_transmittance;
  segment->accum_albedo = accum_albedo;
  /* normalize the distance CDF */
  const CyVolumeStep *last_step = segment->steps + segment->numsteps - 1;
  if (!is_zero3(last_step->cdf_distance)) {
    const cfloat3 inv_cdf_distance_sum = safe_invert_color(last_step->cdf_distance);
    for (int i = 0; i < segment->numsteps; i++) {
      segment->steps[i].cdf_distance = mul3(segment->steps[i].cdf_distance, inv_cdf_distance_sum);
    }
  }
}

/* kernel_volume_decoupled_scatter (kernel_volume.h:934-1128): a scatter
 * distance in the recorded segment by distance sampling of the CDF, or
 * equiangular sampling toward light_P, or MIS of both; the throughput weighted
 * accordingly, the closures set up at the chosen step (re-evaluated: the
 * shade stage's closure memory may have been reused since the record) and
 * sd->P moved there.  probalistic_scatter: scatter or pass by the segment's
 * transmittance (VOLUME_PATH_MISSED then). */
CY_FN int volume_decoupled_scatter(const CyGlobals *kg, const CyPathState *state, const CyRay *ray, CySD *sd,
                                   const CyVolumeStack *stack, cfloat3 *throughput, float rphase, float rscatter,
                                   const CyVolumeSegment *segment, const cfloat3 *light_P, bool probalistic_scatter,
                                   uint *err)
{
  cfloat3 channel_pdf;
  const int channel = volume_sample_channel(segment->accum_albedo, *throughput, rphase, &channel_pdf);
  float xi = rscatter;
  if (probalistic_scatter) {
    const float sample_transmittance = volume_channel_get(segment->accum_transmittance, channel);
    if (1.0f - xi >= sample_transmittance) {
      xi = 1.0f - (1.0f - xi - sample_transmittance) / (1.0f - sample_transmittance);
    }
    else {
      *throughput = div3f(*throughput, sample_transmittance);
      return VOLUME_PATH_MISSED;
    }
  }
  const CyVolumeStep *step;
  cfloat3 transmittance;
  float pdf, sample_t;
  float mis_weight = 1.0f;
  bool distance_sample = true;
  bool use_mis = false;
  if (segment->sampling_method && light_P) {
    if (segment->sampling_method == SD_VOLUME_MIS) {
      if (xi < 0.5f) {
        xi *= 2.0f;
      }
      else {
        xi = (xi - 0.5f) * 2.0f;
        distance_sample = false;
      }
      use_mis = true;
    }
    else {
      distance_sample = false;
    }
  }
  if (distance_sample) {
    step = segment->steps;
    float prev_t = 0.0f;
    cfloat3 step_pdf_distance = mk3(1.0f, 1.0f, 1.0f);
    if (segment->numsteps > 1) {
      float prev_cdf = 0.0f;
      float step_cdf = 1.0f;
      cfloat3 prev_cdf_distance = mk3(0.0f, 0.0f, 0.0f);
      for (int i = 0;; i++, step++) {
        step_cdf = volume_channel_get(step->cdf_distance, channel);
        if (xi < step_cdf || i == segment->numsteps - 1) {
          break;
        }
        prev_cdf = step_cdf;
        prev_t = step->t;
        prev_cdf_distance = step->cdf_distance;
      }
      xi = (xi - prev_cdf) / (step_cdf - prev_cdf);
      step_pdf_distance = sub3(step->cdf_distance, prev_cdf_distance);
    }
    const float step_t = step->t - prev_t;
    cfloat3 distance_pdf;
    sample_t = prev_t + volume_distance_sample(step_t, step->sigma_t, channel, xi, &transmittance, &distance_pdf);
    if (probalistic_scatter) {
      distance_pdf = mul3(distance_pdf, sub3(mk3(1.0f, 1.0f, 1.0f), segment->accum_transmittance));
    }
    pdf = dot3(channel_pdf, mul3(distance_pdf, step_pdf_distance));
    if (use_mis) {
      const float equi_pdf = volume_equiangular_pdf(ray, *light_P, sample_t);
      mis_weight = 2.0f * power_heuristic(pdf, equi_pdf);
    }
  }
  else {
    sample_t = volume_equiangular_sample(ray, *light_P, xi, &pdf);
    step = segment->steps;
    float prev_t = 0.0f;
    cfloat3 step_pdf_distance = mk3(1.0f, 1.0f, 1.0f);
    if (segment->numsteps > 1) {
      cfloat3 prev_cdf_distance = mk3(0.0f, 0.0f, 0.0f);
      const int numsteps = segment->numsteps;
      int high = numsteps - 1;
      int low = 0;
      int mid;
      while (low < high) {
        mid = (low + high) >> 1;
        if (sample_t < step[mid].t) {
          high = mid;
        }
        else if (sample_t >= step[mid + 1].t) {
          low = mid + 1;
        }
        else {
          prev_t = step[mid].t;
          prev_cdf_distance = step[mid].cdf_distance;
          step += mid + 1;
          break;
        }
      }
      if (low >= numsteps - 1) {
        prev_t = step[numsteps - 1].t;
        prev_cdf_distance = step[numsteps - 1].cdf_distance;
        step += numsteps - 1;
      }
      step_pdf_distance = sub3(step->cdf_distance, prev_cdf_distance);
    }
    const float step_t = step->t - prev_t;
    const float step_sample_t = sample_t - prev_t;
    transmittance = volume_color_transmittance(step->sigma_t, step_sample_t);
    if (use_mis) {
      const cfloat3 distance_pdf3 = volume_distance_pdf(step_t, step->sigma_t, step_sample_t);
      const float distance_pdf = dot3(channel_pdf, mul3(distance_pdf3, step_pdf_distance));
      mis_weight = 2.0f * power_heuristic(pdf, distance_pdf);
    }
  }
  CY_DBGF(state, "scatter dist %d mis %d steps %d\n", (int)distance_sample, (int)use_mis, segment->numsteps);
  CY_DBG3(state, "scatter t pdf mis", mk3(sample_t, pdf, mis_weight));
  if (sample_t < 0.0f || pdf == 0.0f) {
    return VOLUME_PATH_MISSED;
  }
  if (step != segment->steps) {
    transmittance = mul3(transmittance, (step - 1)->accum_transmittance);
  }
  *throughput = mul3(*throughput, mul3f(mul3(step->sigma_s, transmittance), mis_weight / pdf));
  /* the closures at the chosen step's shading point (the reference
   * re-evaluates only for several steps: one step's closures are still in its
   * ShaderData, which here may have been reused, so they are evaluated again at
   * the same point) */
  CyVolumeCoeff coeff;
  volume_shader_sample(kg, sd, state, stack, add3(ray->P, mul3f(ray->D, step->shade_t)), &coeff, err);
  sd->P = add3(ray->P, mul3f(ray->D, sample_t));
  return VOLUME_PATH_SCATTERED;
}

#endif /* CY_CLOSURE_EXT */
#endif /* CY_VOLUME_DECOUPLED_H */
