/*
 * cy_branched.h — branched path tracing (KernelIntegrator.branched) on the
 * wavefront slots, the camera segment of kernel_branched_path_integrate
 * (kernel_path_branched.h:369-500):
 *
 *   shader_merge_closures, bsdf_merge     kernel_shader.h:527-551, closure/bsdf.h:739-788
 *   connect_light_branched                kernel_path_surface.h:22-140 (all lights or one,
 *                                         the light samples traced here, path_radiance_accum_light
 *                                         and _accum_total_light, kernel_accumulate.h:402-476)
 *   branched_surface_bounce               kernel_path_surface.h:143-205
 *   branched_camera_hit                   kernel_path_branched.h:201-280 (per-closure indirect
 *                                         samples) and :470-500 (direct light, transparency)
 *
 * A camera hit's indirect samples are independent paths (kernel_path_indirect,
 * kernel_path.h:376-510) traced one after another into the same radiance: the
 * first replaces the slot's path, the others wait in the slot's branch records
 * (CyPathBuffers.br_rec, first in first out) together with the camera ray
 * carried on through the surface's transparency; each waiting path starts
 * when the one before it ends (shade_path).  An indirect path keeps its
 * branch factor (path_state_branch) beside its radiance (L.w).  Volumes,
 * BSSRDFs, ambient occlusion and shadow catchers are refused with branched
 * path tracing by hipcy_load_kernels.
 */
#ifndef CY_BRANCHED_H
#define CY_BRANCHED_H

#if CY_CLOSURE_EXT && CY_SVM_TEX

/* the MicrofacetExtra-carrying microfacet closures (svm_closure.h) */
CY_FN bool closure_has_extra(int type)
{
  return type == CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID || type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID ||
         type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID || type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID ||
         type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID ||
         type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID;
}

/* bsdf_merge (closure/bsdf.h:739-788) over CyClosure's parameter slots
 * (cy_closures.h); an extra record holds color in weight, cspec0 in N and
 * clearcoat in alpha_x */
CY_FN bool bsdf_merge(const CySD *sd, const CyClosure *a, const CyClosure *b)
{
  switch (a->type) {
    case CLOSURE_BSDF_TRANSPARENT_ID:
      return true;
    case CLOSURE_BSDF_DIFFUSE_ID:
    case CLOSURE_BSDF_BSSRDF_ID:
    case CLOSURE_BSDF_TRANSLUCENT_ID:
      return isequal3(a->N, b->N);
    case CLOSURE_BSDF_OREN_NAYAR_ID:
    case CLOSURE_BSDF_PRINCIPLED_DIFFUSE_ID:
    case CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID:
    case CLOSURE_BSDF_ASHIKHMIN_VELVET_ID:
      /* roughness / sigma in alpha_x */
      return isequal3(a->N, b->N) && a->alpha_x == b->alpha_x;
    case CLOSURE_BSDF_DIFFUSE_TOON_ID:
    case CLOSURE_BSDF_GLOSSY_TOON_ID:
      return isequal3(a->N, b->N) && a->alpha_x == b->alpha_x && a->alpha_y == b->alpha_y;
    case CLOSURE_BSDF_REFLECTION_ID:
    case CLOSURE_BSDF_REFRACTION_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID:
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID:
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID:
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID:
    case CLOSURE_BSDF_MICROFACET_BECKMANN_ID:
    case CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID:
    case CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID: {
      /* bsdf_microfacet_merge (bsdf_microfacet.h:355-368) */
      if (!(isequal3(a->N, b->N) && a->alpha_x == b->alpha_x && a->alpha_y == b->alpha_y &&
            isequal3(a->T, b->T) && a->ior == b->ior)) {
        return false;
      }
      if (!closure_has_extra(a->type)) {
        return true; /* both without extra data (the types match) */
      }
      const CyClosure *ea = &sd->closure[a->extra];
      const CyClosure *eb = &sd->closure[b->extra];
      return isequal3(ea->weight, eb->weight) && isequal3(ea->N, eb->N) && ea->alpha_x == eb->alpha_x;
    }
    default:
      return false;
  }
}

/* shader_merge_closures (kernel_shader.h:527-551): identical closures merged,
 * better when one closure at a time is sampled */
CY_FN void shader_merge_closures(CySD *sd)
{
  for (int i = 0; i < sd->num_closure; i++) {
    CyClosure *sci = &sd->closure[i];
    for (int j = i + 1; j < sd->num_closure; j++) {
      CyClosure *scj = &sd->closure[j];
      if (sci->type != scj->type) {
        continue;
      }
      if (!bsdf_merge(sd, sci, scj)) {
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

/* path_branched_rng_1D (kernel_random.h:220-233) */
CY_FN float path_branched_rng_1D(const CyGlobals *kg, uint rng_hash, const CyPathState *state, int branch,
                                 int num_branches, int dimension)
{
  return path_rng_1D(kg, rng_hash, state->sample * num_branches + branch, state->rng_offset + dimension);
}

/* direct_emission (kernel_emission.h:101-205) at a surface point: the light's
 * BSDF-weighted eval (*eval, MIS applied) and the same without the MIS weight
 * (*eval_no_mis, BsdfEval.sum_no_mis, kernel_accumulate.h:62-70); the light
 * termination (off behind a shadow catcher, kernel_emission.h:162-165);
 * *light_ray the shadow ray (t = 0: the light casts no shadow).  False: no
 * contribution. */
CY_FN bool surface_direct_emission(const CyGlobals *kg, const CySD *sd, CyLightSample *ls, const CyPathState *state,
                                   float rand_terminate, cfloat3 *eval, cfloat3 *eval_no_mis, CyRay *light_ray,
                                   CyShadeMem mem, uint *err, CyBsdfEvalLP *ev_lp = nullptr)
{
  if (ls->pdf == 0.0f) {
    return false;
  }
  cfloat3 light_eval = mk3(0.0f, 0.0f, 0.0f);
  const cfloat3 I = neg3(ls->D);
  if (shader_constant_emission_eval(kg, ls->shader, &light_eval)) {
    if ((ls->prim != PRIM_NONE) && dot3(ls->Ng, I) < 0.0f) {
      ls->Ng = neg3(ls->Ng);
    }
  }
  else if (ls->type == LIGHT_BACKGROUND) {
    light_eval = background_eval_svm(kg->data, kg->__svm_nodes, kg->__shaders, kg->__objects, kg->__texture_info,
                                     ls->D, mem, *state, PATH_RAY_EMISSION, err);
  }
  else {
    light_eval = emissive_eval_svm(kg, ls->P, ls->Ng, I, ls->shader, ls->object, ls->prim, ls->lamp, ls->u, ls->v,
                                   ls->t, mem, *state, err);
    if ((ls->prim != PRIM_NONE) && dot3(ls->Ng, I) < 0.0f) {
      ls->Ng = neg3(ls->Ng);
    }
  }
  light_eval = mul3f(light_eval, ls->eval_fac);
  if (ls->lamp != LAMP_NONE) {
    light_eval = mul3(light_eval, klight_vec(kg->__lights[ls->lamp].strength));
  }
  if (is_zero3(light_eval)) {
    return false;
  }
  cfloat3 e = mk3(0.0f, 0.0f, 0.0f); /* shader_bsdf_multi_eval accumulates */
  cfloat3 no_mis;
  if (ev_lp) {
    /* light passes: shader_bsdf_eval per component (kernel_shader.h:606-636),
     * the light's eval, the pass exclusions per component
     * (kernel_emission.h:141-153), the termination on the components' sum */
    bsdf_eval_lp_zero(ev_lp);
    float bpdf;
    shader_bsdf_multi_eval_lp(sd, ls->D, &bpdf, -1, ev_lp, 0.0f, 0.0f);
    if ((uint)ls->shader & SHADER_USE_MIS) {
      bsdf_eval_lp_mul(ev_lp, power_heuristic(ls->pdf, bpdf));
    }
    bsdf_eval_lp_mul3(ev_lp, div3f(light_eval, ls->pdf));
    const uint sh = (uint)ls->shader;
    if (sh & SHADER_EXCLUDE_ANY) {
      const cfloat3 z = mk3(0.0f, 0.0f, 0.0f);
      if (sh & SHADER_EXCLUDE_DIFFUSE) {
        ev_lp->diffuse = z;
      }
      if (sh & SHADER_EXCLUDE_GLOSSY) {
        ev_lp->glossy = z;
      }
      if (sh & SHADER_EXCLUDE_TRANSMIT) {
        ev_lp->transmission = z;
      }
      if (sh & SHADER_EXCLUDE_SCATTER) {
        ev_lp->volume = z;
      }
    }
    if (bsdf_eval_lp_is_zero(ev_lp)) {
      return false;
    }
    if (KD->integrator.light_inv_rr_threshold > 0.0f && !(state->flag & PATH_RAY_SHADOW_CATCHER)) {
      const float probability = max3f(fabs3(bsdf_eval_lp_sum(ev_lp))) * KD->integrator.light_inv_rr_threshold;
      if (probability < 1.0f) {
        if (rand_terminate >= probability) {
          return false;
        }
        bsdf_eval_lp_mul(ev_lp, 1.0f / probability);
      }
    }
    e = bsdf_eval_lp_sum(ev_lp);
    no_mis = e;
  }
  else if (KD->integrator.branched) {
    shader_bsdf_eval_branched(sd, ls->D, ls->pdf, ((uint)ls->shader & SHADER_USE_MIS) != 0, &e, &no_mis);
  }
  else {
    float bpdf;
    shader_bsdf_multi_eval(sd, ls->D, &bpdf, -1, &e, 0.0f, 0.0f);
    no_mis = e;
    if ((uint)ls->shader & SHADER_USE_MIS) {
      e = mul3f(e, power_heuristic(ls->pdf, bpdf));
    }
  }
  const cfloat3 scale = div3f(light_eval, ls->pdf);
  e = mul3(e, scale);
  no_mis = mul3(no_mis, scale);
  if (((uint)ls->shader & SHADER_EXCLUDE_ANY) && ((uint)ls->shader & SHADER_EXCLUDE_DIFFUSE)) {
    e = mk3(0.0f, 0.0f, 0.0f);
  }
  if (!ev_lp && is_zero3(e)) {
    return false;
  }
  if (!ev_lp && KD->integrator.light_inv_rr_threshold > 0.0f && !(state->flag & PATH_RAY_SHADOW_CATCHER)) {
    const float probability = max3f(fabs3(e)) * KD->integrator.light_inv_rr_threshold;
    if (probability < 1.0f) {
      if (rand_terminate >= probability) {
        return false;
      }
      e = mul3f(e, 1.0f / probability);
      no_mis = mul3f(no_mis, 1.0f / probability);
    }
  }
  if ((uint)ls->shader & SHADER_CAST_SHADOW) {
    const bool transmit = (dot3(sd->Ng, ls->D) < 0.0f);
    light_ray->P = ray_offset(sd->P, transmit ? neg3(sd->Ng) : sd->Ng);
    if (ls->t == CY_FLT_MAX) {
      light_ray->D = ls->D;
      light_ray->t = ls->t;
    }
    else {
      light_ray->D = normalize_len3(sub3(ray_offset(ls->P, ls->Ng), light_ray->P), &light_ray->t);
    }
  }
  else {
    light_ray->t = 0.0f;
  }
  *eval = e;
  *eval_no_mis = no_mis;
  return true;
}

/* kernel_branched_path_surface_connect_light (kernel_path_surface.h:22-140):
 * one light sample from the distribution, or (sample_all_lights) every
 * lamp's samples and the mesh lights' with their own sample streams; each
 * shadow ray traced here (the non-catcher visibility behind a shadow catcher,
 * kernel_shadow.h:402-404) and the light added to the radiance *L
 * (path_radiance_accum_light, kernel_accumulate.h:402-459), or to the
 * catcher's totals on a path behind a shadow catcher.  The occluders' shaders
 * are evaluated into shadow_mem, so sd's closures stay intact. */
CY_NOINLINE void connect_light_branched(const CyGlobals *kg, const CySD *sd, const CyPathState *state,
                                        cfloat3 throughput, float num_samples_adjust, bool sample_all_lights,
                                        cfloat3 *L, CyCatcher *catcher, CyShadeMem mem, uint *err,
                                        CyLightPass *lp = nullptr)
{
  if (!KD->integrator.use_direct_light) {
    return;
  }
  CyClosure shadow_closures[CY_MAX_CLOSURE];
  CyShadeMem shadow_mem = mem;
  shadow_mem.closure = shadow_closures;
  int num_lights = 1;
  if (sample_all_lights) {
    num_lights = KD->integrator.num_all_lights;
    if (KD->integrator.pdf_triangles != 0.0f) {
      num_lights += 1;
    }
  }
  const uint shadow_visibility = (state->flag & PATH_RAY_SHADOW_CATCHER) ? (uint)PATH_RAY_SHADOW_NON_CATCHER :
                                                                           (uint)PATH_RAY_SHADOW;
  for (int i = 0; i < num_lights; ++i) {
    int num_samples = 1;
    int num_all_lights = 1;
    uint lamp_rng_hash = state->rng_hash;
    bool double_pdf = false;
    bool is_mesh_light = false;
    bool is_lamp = false;
    if (sample_all_lights) {
      is_lamp = i < KD->integrator.num_all_lights;
      if (is_lamp) {
        if ((float)state->bounce > kg->__lights[i].max_bounces) {
          continue;
        }
        num_samples = (int)ceilf(num_samples_adjust * (float)kg->__lights[i].samples);
        num_all_lights = KD->integrator.num_all_lights;
        lamp_rng_hash = cmj_hash(state->rng_hash, (uint)i);
        double_pdf = KD->integrator.pdf_triangles != 0.0f;
      }
      else {
        num_samples = (int)ceilf(num_samples_adjust * (float)KD->integrator.mesh_light_samples);
        double_pdf = KD->integrator.num_all_lights != 0;
        is_mesh_light = true;
      }
    }
    const float num_samples_inv = num_samples_adjust / (float)(num_samples * num_all_lights);
    for (int j = 0; j < num_samples; j++) {
      CyRay light_ray;
      light_ray.t = 0.0f;
      bool has_emission = false;
      cfloat3 eval = mk3(0.0f, 0.0f, 0.0f), eval_no_mis = mk3(0.0f, 0.0f, 0.0f);
      CyBsdfEvalLP ev_lp;
      if (sd->flag & SD_BSDF_HAS_EVAL) {
        float light_u, light_v;
        path_branched_rng_2D(kg, lamp_rng_hash, state, j, num_samples, PRNG_LIGHT_U, &light_u, &light_v);
        const float terminate = (KD->integrator.light_inv_rr_threshold > 0.0f) ?
                                    path_branched_rng_1D(kg, lamp_rng_hash, state, j, num_samples,
                                                         PRNG_LIGHT_TERMINATE) :
                                    0.0f;
        if (is_mesh_light && double_pdf) {
          light_u = 0.5f * light_u;
        }
        CyLightSample ls;
        if (light_sample_lamp(kg, is_lamp ? i : -1, light_u, light_v, sd->P, state->bounce, &ls, err)) {
          if (double_pdf) {
            ls.pdf *= 2.0f;
          }
          has_emission = surface_direct_emission(kg, sd, &ls, state, terminate, &eval, &eval_no_mis, &light_ray,
                                                 mem, err, lp ? &ev_lp : nullptr);
          if (has_emission) {
            /* direct_emission writes is_lamp, the variable the next sample's
             * lamp choice reads (kernel_path_surface.h:98-112) */
            is_lamp = (ls.prim == PRIM_NONE && ls.type != LIGHT_BACKGROUND);
          }
        }
      }
      /* shadow_blocked (kernel_shadow.h:386-460) */
      cfloat3 shadow = mk3(1.0f, 1.0f, 1.0f);
      bool blocked = false;
      if (light_ray.t != 0.0f) {
        if (KD->integrator.transparent_shadows) {
          blocked = shadow_blocked_transparent<false>(kg, light_ray, state, shadow_mem, &shadow, err, nullptr,
                                                      kg->use_ray_diff ? &sd->dP : nullptr, CY_SREC_NONE, nullptr,
                                                      shadow_visibility);
        }
        else if (scene_intersect_valid(&light_ray)) {
          CyIsect si;
          const uint vis = shadow_visibility & (uint)PATH_RAY_SHADOW_OPAQUE;
          blocked = kg->have_curves ? bvh2_intersect<true, true, 2, CY_LDS_STACK, CY_BLOCK, 3>(
                                          kg, &light_ray, vis, &si, err, nullptr, nullptr, nullptr) :
                                      bvh2_intersect<true>(kg, &light_ray, vis, &si, err, nullptr, nullptr, nullptr);
        }
      }
      CY_DBGF(state, "branched light %d sample %d emission %d blocked %d\n", i, j, (int)has_emission, (int)blocked);
      if (has_emission) {
        const cfloat3 tp = mul3f(throughput, num_samples_inv);
        if (state->flag & PATH_RAY_STORE_SHADOW_INFO) {
          /* path_radiance_accum_light / _accum_total_light with
           * PATH_RAY_STORE_SHADOW_INFO: the catcher's totals */
          const cfloat3 light = mul3(tp, eval_no_mis);
          catcher->path_total = add3(catcher->path_total, light);
          if (!blocked) {
            catcher->path_total_shaded = add3(catcher->path_total_shaded, mul3(shadow, light));
          }
          if (state->flag & PATH_RAY_SHADOW_CATCHER) {
            continue;
          }
        }
        if (!blocked && lp) {
          /* path_radiance_accum_light with light passes (kernel_accumulate.h:425-452) */
          cfloat3 shaded_throughput = mul3(tp, shadow);
          cfloat3 full_contribution = mul3(shaded_throughput, bsdf_eval_lp_sum(&ev_lp));
          const float limit = (state->bounce > 0) ? KD->integrator.sample_clamp_indirect :
                                                    KD->integrator.sample_clamp_direct;
          const float sum = reduce_add3(fabs3(full_contribution));
          if (sum > limit) {
            const float clamp_factor = limit / sum;
            full_contribution = mul3f(full_contribution, clamp_factor);
            shaded_throughput = mul3f(shaded_throughput, clamp_factor);
          }
          if (state->bounce == 0) {
            lp->direct_diffuse = add3(lp->direct_diffuse, mul3(shaded_throughput, ev_lp.diffuse));
            lp->direct_glossy = add3(lp->direct_glossy, mul3(shaded_throughput, ev_lp.glossy));
            lp->direct_transmission = add3(lp->direct_transmission, mul3(shaded_throughput, ev_lp.transmission));
            lp->direct_volume = add3(lp->direct_volume, mul3(shaded_throughput, ev_lp.volume));
            if (is_lamp) {
              lp->shadow = add3(lp->shadow, mul3f(shadow, num_samples_inv));
            }
          }
          else {
            lp->indirect = add3(lp->indirect, full_contribution);
          }
        }
        else if (!blocked) {
          const cfloat3 contribution = mul3(mul3(tp, shadow), eval);
          *L = add3(*L, path_radiance_clamp(kg, contribution, state->bounce));
        }
      }
    }
  }
}

/* kernel_branched_path_surface_bounce (kernel_path_surface.h:143-205): closure
 * sc sampled alone (shader_bsdf_sample_closure) with the branch's random
 * numbers, the path state branched (path_state_branch); false when the
 * sample carries nothing.  *branch_factor is the branch's RR factor. */
CY_FN bool branched_surface_bounce(const CyGlobals *kg, const CySD *sd, const CyClosure *sc, int sample,
                                   int num_samples, cfloat3 *throughput, CyPathState *state, CyRay *ray,
                                   float *branch_factor, CyDiff3 *domega_in, uint *err)
{
  float bsdf_u, bsdf_v;
  path_branched_rng_2D(kg, state->rng_hash, state, sample, num_samples, PRNG_BSDF_U, &bsdf_u, &bsdf_v);
  cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
  cfloat3 omega_in = mk3(0.0f, 0.0f, 0.0f);
  float bsdf_pdf = 0.0f;
  int label;
  if (domega_in) {
    CyDiffRule rule;
    rule.kind = CY_DIFF_ZERO;
    label = bsdf_sample(kg, sd, sc, bsdf_u, bsdf_v, &eval, &omega_in, &bsdf_pdf, err, &rule);
    domega_in->dx = diff_rule_apply(rule, sd->dI.dx);
    domega_in->dy = diff_rule_apply(rule, sd->dI.dy);
  }
  else {
    label = bsdf_sample(kg, sd, sc, bsdf_u, bsdf_v, &eval, &omega_in, &bsdf_pdf, err);
  }
  if (bsdf_pdf == 0.0f) {
    return false;
  }
  eval = mul3(eval, sc->weight); /* bsdf_eval_init (shader_bsdf_sample_closure) */
  if (is_zero3(eval)) {
    return false;
  }
  /* path_radiance_bsdf_bounce (kernel_accumulate.h:240-273) */
  const float inverse_pdf = 1.0f / bsdf_pdf;
  *throughput = mul3(*throughput, mul3f(eval, inverse_pdf));
  path_state_next(kg, state, label);
  ray->P = ray_offset(sd->P, (label & LABEL_TRANSMIT) ? neg3(sd->Ng) : sd->Ng);
  ray->D = normalize3(omega_in);
  ray->t = CY_FLT_MAX;
  /* path_state_branch (kernel_path_state.h:245-255) */
  if (num_samples > 1) {
    state->sample = state->sample * num_samples + sample;
    *branch_factor *= (float)num_samples;
  }
  state->min_ray_pdf = fminf(bsdf_pdf, CY_FLT_MAX);
  state->ray_pdf = bsdf_pdf;
  state->ray_t = 0.0f;
  return true;
}

#endif /* CY_CLOSURE_EXT && CY_SVM_TEX */

#endif /* CY_BRANCHED_H */
