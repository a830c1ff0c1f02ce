/*
 * cy_subsurface.h — random-walk subsurface scattering in the shading stage.
 *
 * Restates, in the reference CPU kernel's scalar arithmetic:
 *   shader_bssrdf_pick                      kernel/kernel_shader.h:682-737
 *   scene_intersect_local, closest hit only  kernel/bvh/bvh_local.h:34-225 +
 *                                           geom/geom_triangle_intersect.h
 *                                           triangle_intersect_local (max_hits 1)
 *   subsurface_random_walk (+ remap, coefficients)
 *                                           kernel/kernel_subsurface.h:300-480
 *   henyey_greenstrein_sample (g = 0)        closure/volume.h:93-122
 *   kernel_volume_sample_channel            kernel/kernel_volume.h:402-435
 *   shader_setup_from_subsurface            kernel/kernel_shader.h:160-240
 *   triangle_refine_local                   geom/geom_triangle_intersect.h:261-318
 *   subsurface_scatter_setup_diffuse_bsdf   kernel/kernel_subsurface.h:66-107
 * Disk BSSRDFs (Subsurface Scattering node cubic / gaussian / burley, the
 * Principled BSDF's default "burley"):
 *   bssrdf profiles, bssrdf_sample / _eval / _pdf closure/bssrdf.h:34-327, 425-495
 *   subsurface_scatter_eval                 kernel/kernel_subsurface.h:26-66
 *   subsurface_scatter_disk                 kernel/kernel_subsurface.h:160-282
 *   scene_intersect_local, up to 4 hits     kernel/bvh/bvh_local.h:34-190 +
 *                                           geom/geom_triangle_intersect.h
 *                                           triangle_intersect_local (reservoir)
 *   shader_bssrdf_sum, subsurface_color_pow,
 *   subsurface_color_bump_blur              kernel/kernel_shader.h:766-795,
 *                                           kernel/kernel_subsurface.h:109-158
 * The path-level flow (kernel_path_subsurface.h:26-139: per exit point light
 * with the path's state and a bounce with rng_offset + PRNG_BOUNCE_NUM into
 * the SubsurfaceIndirectRays stack, then the indirect rays last to first) is
 * in cy_integrator.h shade_path; the stack lives in the slot's SSS records.
 */
#ifndef CY_SUBSURFACE_H
#define CY_SUBSURFACE_H

#if CY_CLOSURE_EXT

/* shader_bssrdf_pick: a BSDF or a BSSRDF by sample weight; the throughput is
 * scaled by the inverse of the picked group's probability. */
CY_FN const CyClosure *shader_bssrdf_pick(const CySD *sd, cfloat3 *throughput, float *randu)
{
  int sampled = 0;
  if (sd->num_closure > 1) {
    float sum_bsdf = 0.0f;
    float sum_bssrdf = 0.0f;
    for (int i = 0; i < sd->num_closure; i++) {
      const CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_BSDF(sc->type)) {
        sum_bsdf += sc->sample_weight;
      }
      else if (CLOSURE_IS_BSSRDF(sc->type)) {
        sum_bssrdf += sc->sample_weight;
      }
    }
    const float r = (*randu) * (sum_bsdf + sum_bssrdf);
    float partial_sum = 0.0f;
    for (int i = 0; i < sd->num_closure; i++) {
      const CyClosure *sc = &sd->closure[i];
      if (CLOSURE_IS_BSDF_OR_BSSRDF(sc->type)) {
        const float next_sum = partial_sum + sc->sample_weight;
        if (r < next_sum) {
          if (CLOSURE_IS_BSDF(sc->type)) {
            *throughput = mul3f(*throughput, (sum_bsdf + sum_bssrdf) / sum_bsdf);
            return 0;
          }
          *throughput = mul3f(*throughput, (sum_bsdf + sum_bssrdf) / sum_bssrdf);
          sampled = i;
          *randu = (r - partial_sum) / sc->sample_weight;
          break;
        }
        partial_sum = next_sum;
      }
    }
  }
  const CyClosure *sc = &sd->closure[sampled];
  return CLOSURE_IS_BSSRDF(sc->type) ? sc : 0;
}

/* scene_intersect_local with one recorded hit (no lcg state): every triangle
 * of local_object within ray->t is tested, in the reference's BVH2 order, and
 * the closest is kept (a later one at the same t replaces it); the bound is
 * never shortened.  Starts at __object_node[local_object] (the object's own
 * BVH for instances, the top level otherwise, filtered by __prim_object). */
CY_FN bool scene_intersect_local_closest(const CyGlobals *kg, const CyRay *ray, int local_object, CyIsect *hit,
                                         cfloat3 *hit_Ng, uint *err)
{
  int stack[BVH_STACK_SIZE];
  stack[0] = ENTRYPOINT_SENTINEL;
  int stack_ptr = 0;
  int node_addr = (int)kg->__object_node[local_object];
  cfloat3 P = ray->P;
  cfloat3 dir = bvh_clamp_direction(ray->D);
  cfloat3 idir = rcp3(dir);
  int object = OBJECT_NONE;
  float isect_t = ray->t;
  int num_hits = 0;
  const uint object_flag = kg->__object_flag[local_object];
  if (!(object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
    isect_t = bvh_instance_push(kg, local_object, ray, &P, &dir, &idir, isect_t);
    object = local_object;
  }
  const hc_float4 *nodes = kg->__bvh_nodes;
  do {
    do {
      while (node_addr >= 0 && node_addr != ENTRYPOINT_SENTINEL) {
        const hc_float4 cnodes = nodes[node_addr + 0];
        float c0min, c1min;
        const int traverse_mask = bvh2_node_intersect<1>(nodes, node_addr, cnodes, P, dir, idir, isect_t,
                                                           PATH_RAY_ALL_VISIBILITY, &c0min, &c1min);
        node_addr = as_int(cnodes.z);
        int node_addr_child1 = as_int(cnodes.w);
        if (traverse_mask == 3) {
          if (c1min < c0min) {
            const int tmp = node_addr;
            node_addr = node_addr_child1;
            node_addr_child1 = tmp;
          }
          if (++stack_ptr >= BVH_STACK_SIZE) {
            cy_set_error(err, CY_ERR_BVH_STACK, 2);
            return num_hits > 0;
          }
          stack[stack_ptr] = node_addr_child1;
        }
        else if (traverse_mask == 2) {
          node_addr = node_addr_child1;
        }
        else if (traverse_mask == 0) {
          node_addr = stack[stack_ptr];
          --stack_ptr;
        }
      }
      if (node_addr < 0) {
        const hc_float4 leaf = kg->__bvh_leaf_nodes[-node_addr - 1];
        int prim_addr = as_int(leaf.x);
        const int prim_addr2 = as_int(leaf.y);
        const uint type = as_uint(leaf.w);
        node_addr = stack[stack_ptr];
        --stack_ptr;
        if ((type & PRIMITIVE_ALL) == PRIMITIVE_TRIANGLE) {
          for (; prim_addr < prim_addr2; prim_addr++) {
            /* triangle_intersect_local */
            if (object == OBJECT_NONE && (int)kg->__prim_object[prim_addr] != local_object) {
              continue;
            }
            const uint tri_vindex = kg->__prim_tri_index[prim_addr];
            const cfloat3 tri_a = f4to3(kg->__prim_tri_verts[tri_vindex + 0]);
            const cfloat3 tri_b = f4to3(kg->__prim_tri_verts[tri_vindex + 1]);
            const cfloat3 tri_c = f4to3(kg->__prim_tri_verts[tri_vindex + 2]);
            float t, u, v;
            if (!ray_triangle_intersect(P, dir, isect_t, tri_a, tri_b, tri_c, &u, &v, &t)) {
              continue;
            }
            if (num_hits && t > hit->t) {
              continue;
            }
            num_hits = 1;
            hit->prim = prim_addr;
            hit->object = object;
            hit->type = PRIMITIVE_TRIANGLE;
            hit->u = u;
            hit->v = v;
            hit->t = t;
            *hit_Ng = normalize3(cross3(sub3(tri_b, tri_a), sub3(tri_c, tri_a)));
          }
        }
      }
    } while (node_addr != ENTRYPOINT_SENTINEL);
  } while (node_addr != ENTRYPOINT_SENTINEL);
  return num_hits > 0;
}

/* kernel_volume_sample_channel */
CY_FN int volume_sample_channel(cfloat3 albedo, cfloat3 throughput, float rand, cfloat3 *pdf)
{
  const cfloat3 weights = fabs3(mul3(throughput, albedo));
  const float sum_weights = weights.x + weights.y + weights.z;
  cfloat3 weights_pdf;
  if (sum_weights > 0.0f) {
    weights_pdf = div3f(weights, sum_weights);
  }
  else {
    weights_pdf = mk3(1.0f / 3.0f, 1.0f / 3.0f, 1.0f / 3.0f);
  }
  *pdf = weights_pdf;
  if (rand < weights_pdf.x) {
    return 0;
  }
  else if (rand < weights_pdf.x + weights_pdf.y) {
    return 1;
  }
  return 2;
}

CY_FN float volume_channel_get(cfloat3 value, int channel)
{
  return (channel == 0) ? value.x : ((channel == 1) ? value.y : value.z);
}

/* volume_color_transmittance: exp3(-sigma * t) */
CY_FN cfloat3 volume_color_transmittance(cfloat3 sigma, float t)
{
  const cfloat3 x = mul3f(neg3(sigma), t);
  return mk3(cy_expf(x.x), cy_expf(x.y), cy_expf(x.z));
}

/* henyey_greenstrein_sample, isotropic branch (the random walk's g = 0) */
CY_FN cfloat3 henyey_greenstein_sample_isotropic(cfloat3 D, float randu, float randv)
{
  const float cos_theta = (1.0f - 2.0f * randu);
  const float sin_theta = safe_sqrtf(1.0f - cos_theta * cos_theta);
  const float phi = CY_2PI_F * randv;
  const cfloat3 dir = mk3(sin_theta * cy_cosf(phi), sin_theta * cy_sinf(phi), cos_theta);
  cfloat3 T, B;
  make_orthonormals(D, &T, &B);
  return add3(add3(mul3f(T, dir.x), mul3f(B, dir.y)), mul3f(D, dir.z));
}

CY_FN void subsurface_random_walk_remap(float A, float d, float *sigma_t, float *sigma_s)
{
  const float a = 1.0f - cy_expf(A * (-5.09406f + A * (2.61188f - A * 4.31805f)));
  const float s = 1.9f - A + 3.5f * sqr(A - 0.8f);
  *sigma_t = 1.0f / fmaxf(d * s, 1e-16f);
  *sigma_s = *sigma_t * a;
}

/* subsurface_random_walk: into the object from a cosine-sampled direction,
 * exponential steps with hero-channel sampling, isotropic scattering and
 * Russian roulette, until the surface is hit again (true: *hit, *weight and
 * *ray hold the exit intersection, the throughput and the last step's ray). */
CY_FN bool subsurface_random_walk(const CyGlobals *kg, const CySD *sd, CyPathState *state, const CyClosure *sc,
                                  float bssrdf_u, float bssrdf_v, CyIsect *ss_hit, cfloat3 *weight, CyRay *ray,
                                  uint *err)
{
  cfloat3 D;
  float pdf;
  sample_cos_hemisphere(neg3(sd->N), bssrdf_u, bssrdf_v, &D, &pdf);
  if (dot3(neg3(sd->Ng), D) <= 0.0f) {
    return false;
  }
  /* subsurface_random_walk_coefficients */
  const cfloat3 A = bssrdf_albedo(sc);
  const cfloat3 d = bssrdf_radius(sc);
  float stx, sty, stz, ssx, ssy, ssz;
  subsurface_random_walk_remap(A.x, d.x, &stx, &ssx);
  subsurface_random_walk_remap(A.y, d.y, &sty, &ssy);
  subsurface_random_walk_remap(A.z, d.z, &stz, &ssz);
  const cfloat3 sigma_t = mk3(stx, sty, stz);
  const cfloat3 sigma_s = mk3(ssx, ssy, ssz);
  cfloat3 throughput = safe_divide_color(sc->weight, A);

  ray->P = ray_offset(sd->P, neg3(sd->Ng));
  ray->D = D;
  ray->t = CY_FLT_MAX;

  const int prev_rng_offset = state->rng_offset;
  const uint prev_rng_hash = state->rng_hash;
  state->rng_hash = cmj_hash(state->rng_hash + (uint)state->rng_offset, 0xdeadbeef);

  bool hit = false;
  for (int bounce = 0; bounce < BSSRDF_MAX_BOUNCES; bounce++) {
    state->rng_offset += PRNG_BOUNCE_NUM;
    if (bounce > 0) {
      float scatter_u, scatter_v;
      path_state_rng_2D(kg, state, PRNG_BSDF_U, &scatter_u, &scatter_v);
      ray->D = henyey_greenstein_sample_isotropic(ray->D, scatter_u, scatter_v);
    }
    const float rphase = path_state_rng_1D(kg, state, PRNG_PHASE_CHANNEL);
    const cfloat3 albedo = safe_divide_color(sigma_s, sigma_t);
    cfloat3 channel_pdf;
    const int channel = volume_sample_channel(albedo, throughput, rphase, &channel_pdf);
    const float rdist = path_state_rng_1D(kg, state, PRNG_SCATTER_DISTANCE);
    const float sample_sigma_t = volume_channel_get(sigma_t, channel);
    float t = -cy_logf(1.0f - rdist) / sample_sigma_t;
    ray->t = t;
    cfloat3 hit_Ng;
    hit = scene_intersect_local_closest(kg, ray, sd->object, ss_hit, &hit_Ng, err);
    if (hit) {
      /* world-space distance to the surface hit (object space t) */
      cfloat3 Dw = transform_direction(object_itfm(kg, sd->object), ray->D);
      Dw = mul3f(normalize3(Dw), ss_hit->t);
      Dw = transform_direction(object_tfm(kg, sd->object), Dw);
      t = len3(Dw);
    }
    ray->P = add3(ray->P, mul3f(ray->D, t));
    const cfloat3 transmittance = volume_color_transmittance(sigma_t, t);
    const float tpdf = dot3(channel_pdf, hit ? transmittance : mul3(sigma_t, transmittance));
    throughput = mul3(throughput, div3f(hit ? transmittance : mul3(sigma_s, transmittance), tpdf));
    if (hit) {
      break;
    }
    const float terminate = path_state_rng_1D(kg, state, PRNG_TERMINATE);
    const float probability = cmin(max3f(fabs3(throughput)), 1.0f);
    if (terminate >= probability) {
      break;
    }
    throughput = div3f(throughput, probability);
  }
  state->rng_offset = prev_rng_offset;
  state->rng_hash = prev_rng_hash;
  if (!hit) {
    return false;
  }
  *weight = throughput;
  return true;
}

/* triangle_refine_local: hit point of a local intersection (object space t) */
CY_FN cfloat3 triangle_refine_local(const CyGlobals *kg, const CyIsect *isect, const CyRay *ray)
{
  cfloat3 P = ray->P;
  cfloat3 D = ray->D;
  const float t = isect->t;
  if (isect->object != OBJECT_NONE) {
    const struct cy_tfm *itfm = object_itfm(kg, isect->object);
    P = transform_point(itfm, P);
    D = transform_direction(itfm, D);
    D = normalize3(D);
  }
  P = add3(P, mul3f(D, t));
  const uint tri_vindex = kg->__prim_tri_index[isect->prim];
  const hc_float4 tri_a = kg->__prim_tri_verts[tri_vindex + 0];
  const hc_float4 tri_b = kg->__prim_tri_verts[tri_vindex + 1];
  const hc_float4 tri_c = kg->__prim_tri_verts[tri_vindex + 2];
  const cfloat3 edge1 = mk3(tri_a.x - tri_c.x, tri_a.y - tri_c.y, tri_a.z - tri_c.z);
  const cfloat3 edge2 = mk3(tri_b.x - tri_c.x, tri_b.y - tri_c.y, tri_b.z - tri_c.z);
  const cfloat3 tvec = mk3(P.x - tri_c.x, P.y - tri_c.y, P.z - tri_c.z);
  const cfloat3 qvec = cross3(tvec, edge1);
  const cfloat3 pvec = cross3(D, edge2);
  const float det = dot3(edge1, pvec);
  if (det != 0.0f) {
    const float rt = dot3(edge2, qvec) / det;
    P = add3(P, mul3f(D, rt));
  }
  if (isect->object != OBJECT_NONE) {
    P = transform_point(object_tfm(kg, isect->object), P);
  }
  return P;
}

/* shader_setup_from_subsurface: the exit point on the same object; object,
 * ray length and the entry's backfacing state are kept, I = N. */
CY_FN void shader_setup_from_subsurface(const CyGlobals *kg, CySD *sd, const CyIsect *isect, const CyRay *ray)
{
  const bool backfacing = (sd->flag & SD_BACKFACING) != 0;
  sd->flag = 0;
  sd->object_flag = (int)kg->__object_flag[sd->object];
  sd->prim = (int)kg->__prim_index[isect->prim];
  sd->type = isect->type;
  sd->u = isect->u;
  sd->v = isect->v;
  const cfloat3 Ng = triangle_normal(kg, sd);
  sd->shader = (int)kg->__tri_shader[sd->prim];
  sd->P = triangle_refine_local(kg, isect, ray);
  sd->Ng = Ng;
  sd->N = Ng;
  if ((uint)sd->shader & SHADER_SMOOTH_NORMAL) {
    sd->N = triangle_smooth_normal(kg, Ng, sd->prim, sd->u, sd->v);
  }
  triangle_dPdudv(kg, sd->prim, &sd->dPdu, &sd->dPdv);
  sd->flag |= kg->__shaders[(uint)sd->shader & SHADER_MASK].flags;
  if (isect->object != OBJECT_NONE) {
    sd->N = object_normal_transform(kg, sd->object, sd->N);
    sd->Ng = object_normal_transform(kg, sd->object, sd->Ng);
    sd->dPdu = transform_direction(object_tfm(kg, sd->object), sd->dPdu);
    sd->dPdv = transform_direction(object_tfm(kg, sd->object), sd->dPdv);
  }
  if (backfacing) {
    sd->flag |= SD_BACKFACING;
    sd->Ng = neg3(sd->Ng);
    sd->N = neg3(sd->N);
    sd->dPdu = neg3(sd->dPdu);
    sd->dPdv = neg3(sd->dPdv);
  }
  sd->I = sd->N;
  if (kg->use_ray_diff) {
    /* kernel_shader.h:232-236: new du / dv from the entry's dP (dP, dI kept) */
    differential_dudv(&sd->du, &sd->dv, sd->dPdu, sd->dPdv, sd->dP, sd->Ng);
  }
}

/* subsurface_scatter_setup_diffuse_bsdf: the closures are replaced by one
 * (principled) diffuse closure carrying the scatter weight. */
CY_FN void subsurface_scatter_setup_diffuse_bsdf(const CyGlobals *kg, CySD *sd, int type, float roughness,
                                                 cfloat3 weight, cfloat3 N)
{
  sd->flag &= ~(SD_EMISSION | SD_BSDF | SD_BSDF_HAS_EVAL | SD_BSSRDF | SD_HOLDOUT | SD_EXTINCTION | SD_SCATTER |
                SD_BSDF_NEEDS_LCG);
  sd->num_closure = 0;
  sd->num_closure_left = KD->integrator.max_closures;
  CyClosure *bsdf = bsdf_alloc(sd, weight);
  if (type == CLOSURE_BSSRDF_PRINCIPLED_ID || type == CLOSURE_BSSRDF_PRINCIPLED_RANDOM_WALK_ID) {
    if (bsdf) {
      bsdf->N = N;
      bsdf->alpha_x = roughness;
      sd->flag |= SD_BSDF | SD_BSDF_HAS_EVAL; /* bsdf_principled_diffuse_setup */
      bsdf->type = CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID;
    }
  }
  else if (bsdf) {
    bsdf->N = N;
    sd->flag |= bsdf_diffuse_setup(bsdf);
    bsdf->type = CLOSURE_BSDF_BSSRDF_ID;
  }
}

/* ---------------------------------------------------------------------------
 * Disk BSSRDFs.  Closure storage (cy_path.h bssrdf_setup): radius in T,
 * sharpness in alpha_x, the channel count in alpha_y. */

#define GAUSS_TRUNCATE 12.46f
#define BURLEY_TRUNCATE 16.0f
#define BURLEY_TRUNCATE_CDF 0.9963790093708328f

CY_FN float bssrdf_channels(const CyClosure *sc)
{
  return sc->alpha_y;
}
CY_FN float bssrdf_sharpness(const CyClosure *sc)
{
  return sc->alpha_x;
}

/* bssrdf.h:47-84 */
CY_FN float bssrdf_gaussian_eval(const float radius, float r)
{
  const float v = radius * radius * (0.25f * 0.25f);
  const float Rm = sqrtf(v * GAUSS_TRUNCATE);
  if (r >= Rm) {
    return 0.0f;
  }
  return cy_expf(-r * r / (2.0f * v)) / (2.0f * CY_PI_F * v);
}
CY_FN float bssrdf_gaussian_pdf(const float radius, float r)
{
  const float area_truncated = 1.0f - cy_expf(-0.5f * GAUSS_TRUNCATE);
  return bssrdf_gaussian_eval(radius, r) * (1.0f / (area_truncated));
}
CY_FN void bssrdf_gaussian_sample(const float radius, float xi, float *r, float *h)
{
  const float v = radius * radius * (0.25f * 0.25f);
  const float Rm = sqrtf(v * GAUSS_TRUNCATE);
  const float area_truncated = 1.0f - cy_expf(-0.5f * GAUSS_TRUNCATE);
  const float r_squared = -2.0f * v * cy_logf(1.0f - xi * area_truncated);
  *r = sqrtf(r_squared);
  *h = safe_sqrtf(Rm * Rm - r_squared);
}

/* bssrdf.h:93-181 */
CY_FN float bssrdf_cubic_eval(const float radius, const float sharpness, float r)
{
  if (sharpness == 0.0f) {
    const float Rm = radius;
    if (r >= Rm) {
      return 0.0f;
    }
    const float Rm5 = (Rm * Rm) * (Rm * Rm) * Rm;
    const float f = Rm - r;
    const float num = f * f * f;
    return (10.0f * num) / (Rm5 * CY_PI_F);
  }
  float Rm = radius * (1.0f + sharpness);
  if (r >= Rm) {
    return 0.0f;
  }
  const float y = 1.0f / (1.0f + sharpness);
  float Rmy, ry, ryinv;
  if (sharpness == 1.0f) {
    Rmy = sqrtf(Rm);
    ry = sqrtf(r);
    ryinv = (ry > 0.0f) ? 1.0f / ry : 0.0f;
  }
  else {
    Rmy = cy_powf(Rm, y);
    ry = cy_powf(r, y);
    ryinv = (r > 0.0f) ? cy_powf(r, y - 1.0f) : 0.0f;
  }
  const float Rmy5 = (Rmy * Rmy) * (Rmy * Rmy) * Rmy;
  const float f = Rmy - ry;
  const float num = f * (f * f) * (y * ryinv);
  return (10.0f * num) / (Rmy5 * CY_PI_F);
}
CY_FN float bssrdf_cubic_quintic_root_find(float xi)
{
  const float tolerance = 1e-6f;
  const int max_iteration_count = 10;
  float x = 0.25f;
  for (int i = 0; i < max_iteration_count; i++) {
    float x2 = x * x;
    float x3 = x2 * x;
    float nx = (1.0f - x);
    float f = 10.0f * x2 - 20.0f * x3 + 15.0f * x2 * x2 - 4.0f * x2 * x3 - xi;
    float f_ = 20.0f * (x * nx) * (nx * nx);
    if (fabsf(f) < tolerance || f_ == 0.0f) {
      break;
    }
    x = saturate(x - f / f_);
  }
  return x;
}
CY_FN void bssrdf_cubic_sample(const float radius, const float sharpness, float xi, float *r, float *h)
{
  float Rm = radius;
  float r_ = bssrdf_cubic_quintic_root_find(xi);
  if (sharpness != 0.0f) {
    r_ = cy_powf(r_, 1.0f + sharpness);
    Rm *= (1.0f + sharpness);
  }
  r_ *= Rm;
  *r = r_;
  *h = safe_sqrtf(Rm * Rm - r_ * r_);
}

/* bssrdf.h:222-289 */
CY_FN float bssrdf_burley_eval(const float d, float r)
{
  const float Rm = BURLEY_TRUNCATE * d;
  if (r >= Rm) {
    return 0.0f;
  }
  float exp_r_3_d = cy_expf(-r / (3.0f * d));
  float exp_r_d = exp_r_3_d * exp_r_3_d * exp_r_3_d;
  return (exp_r_d + exp_r_3_d) / (4.0f * d);
}
CY_FN float bssrdf_burley_pdf(const float d, float r)
{
  return bssrdf_burley_eval(d, r) * (1.0f / BURLEY_TRUNCATE_CDF);
}
CY_FN float bssrdf_burley_root_find(float xi)
{
  const float tolerance = 1e-6f;
  const int max_iteration_count = 10;
  float r;
  if (xi <= 0.9f) {
    r = cy_expf(xi * xi * 2.4f) - 1.0f;
  }
  else {
    r = 15.0f;
  }
  for (int i = 0; i < max_iteration_count; i++) {
    float exp_r_3 = cy_expf(-r / 3.0f);
    float exp_r = exp_r_3 * exp_r_3 * exp_r_3;
    float f = 1.0f - 0.25f * exp_r - 0.75f * exp_r_3 - xi;
    float f_ = 0.25f * exp_r + 0.25f * exp_r_3;
    if (fabsf(f) < tolerance || f_ == 0.0f) {
      break;
    }
    r = r - f / f_;
    if (r < 0.0f) {
      r = 0.0f;
    }
  }
  return r;
}
CY_FN void bssrdf_burley_sample(const float d, float xi, float *r, float *h)
{
  const float Rm = BURLEY_TRUNCATE * d;
  const float r_ = bssrdf_burley_root_find(xi * BURLEY_TRUNCATE_CDF) * d;
  *r = r_;
  *h = safe_sqrtf(Rm * Rm - r_ * r_);
}

/* bssrdf.h:425-495 */
CY_FN void bssrdf_sample(const CyClosure *sc, float xi, float *r, float *h)
{
  const cfloat3 rad = bssrdf_radius(sc);
  float radius;
  xi *= bssrdf_channels(sc);
  if (xi < 1.0f) {
    radius = (rad.x > 0.0f) ? rad.x : (rad.y > 0.0f) ? rad.y : rad.z;
  }
  else if (xi < 2.0f) {
    xi -= 1.0f;
    radius = (rad.x > 0.0f) ? rad.y : rad.z;
  }
  else {
    xi -= 2.0f;
    radius = rad.z;
  }
  if (sc->type == CLOSURE_BSSRDF_CUBIC_ID) {
    bssrdf_cubic_sample(radius, bssrdf_sharpness(sc), xi, r, h);
  }
  else if (sc->type == CLOSURE_BSSRDF_GAUSSIAN_ID) {
    bssrdf_gaussian_sample(radius, xi, r, h);
  }
  else {
    bssrdf_burley_sample(radius, xi, r, h);
  }
}
CY_FN float bssrdf_channel_pdf(const CyClosure *sc, float radius, float r)
{
  if (radius == 0.0f) {
    return 0.0f;
  }
  else if (sc->type == CLOSURE_BSSRDF_CUBIC_ID) {
    return bssrdf_cubic_eval(radius, bssrdf_sharpness(sc), r); /* bssrdf_cubic_pdf */
  }
  else if (sc->type == CLOSURE_BSSRDF_GAUSSIAN_ID) {
    return bssrdf_gaussian_pdf(radius, r);
  }
  return bssrdf_burley_pdf(radius, r);
}
CY_FN cfloat3 bssrdf_eval(const CyClosure *sc, float r)
{
  const cfloat3 rad = bssrdf_radius(sc);
  return mk3(bssrdf_channel_pdf(sc, rad.x, r), bssrdf_channel_pdf(sc, rad.y, r), bssrdf_channel_pdf(sc, rad.z, r));
}
CY_FN float bssrdf_pdf(const CyClosure *sc, float r)
{
  const cfloat3 pdf = bssrdf_eval(sc, r);
  return (pdf.x + pdf.y + pdf.z) / bssrdf_channels(sc);
}

/* kernel_subsurface.h:26-66, path tracing (one BSSRDF picked: all == false) */
CY_FN cfloat3 subsurface_scatter_eval(const CySD *sd, float disk_r, float r)
{
  cfloat3 eval_sum = mk3(0.0f, 0.0f, 0.0f);
  float pdf_sum = 0.0f;
  float sample_weight_sum = 0.0f;
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    if (CLOSURE_IS_DISK_BSSRDF(sc->type)) {
      sample_weight_sum += sc->sample_weight;
    }
  }
  const float sample_weight_inv = 1.0f / sample_weight_sum;
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    if (CLOSURE_IS_DISK_BSSRDF(sc->type)) {
      const float sample_weight = sc->sample_weight * sample_weight_inv;
      const cfloat3 eval = bssrdf_eval(sc, r);
      const float pdf = bssrdf_pdf(sc, disk_r);
      eval_sum = add3(eval_sum, mul3(sc->weight, eval));
      pdf_sum += sample_weight * pdf;
    }
  }
  return (pdf_sum > 0.0f) ? div3f(eval_sum, pdf_sum) : mk3(0.0f, 0.0f, 0.0f);
}

/* LocalIntersection (kernel_types.h:1227-1232) with the scatter weights */
typedef struct CyLocalHits {
  int num_hits;
  CyIsect hits[BSSRDF_MAX_HITS];
  cfloat3 Ng[BSSRDF_MAX_HITS];
  cfloat3 weight[BSSRDF_MAX_HITS];
} CyLocalHits;

/* kernel_random.h:296-303 lcg_step_uint */
CY_FN uint lcg_step_uint(uint *rng)
{
  *rng = 1103515245u * (*rng) + 12345u;
  return *rng;
}

/* scene_intersect_local recording up to max_hits hits (bvh_local.h +
 * triangle_intersect_local with an lcg state): every triangle of local_object
 * within ray->t, in the reference's BVH2 order, kept by reservoir sampling;
 * hits at a distance already recorded are skipped; the bound never shrinks. */
CY_FN void scene_intersect_local_multi(const CyGlobals *kg, const CyRay *ray, int local_object, CyLocalHits *li,
                                       uint *lcg_state, int max_hits, uint *err)
{
  int stack[BVH_STACK_SIZE];
  stack[0] = ENTRYPOINT_SENTINEL;
  int stack_ptr = 0;
  int node_addr = (int)kg->__object_node[local_object];
  cfloat3 P = ray->P;
  cfloat3 dir = bvh_clamp_direction(ray->D);
  cfloat3 idir = rcp3(dir);
  int object = OBJECT_NONE;
  float isect_t = ray->t;
  li->num_hits = 0;
  const uint object_flag = kg->__object_flag[local_object];
  if (!(object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
    isect_t = bvh_instance_push(kg, local_object, ray, &P, &dir, &idir, isect_t);
    object = local_object;
  }
  const hc_float4 *nodes = kg->__bvh_nodes;
  do {
    do {
      while (node_addr >= 0 && node_addr != ENTRYPOINT_SENTINEL) {
        const hc_float4 cnodes = nodes[node_addr + 0];
        float c0min, c1min;
        const int traverse_mask = bvh2_node_intersect<1>(nodes, node_addr, cnodes, P, dir, idir, isect_t,
                                                           PATH_RAY_ALL_VISIBILITY, &c0min, &c1min);
        node_addr = as_int(cnodes.z);
        int node_addr_child1 = as_int(cnodes.w);
        if (traverse_mask == 3) {
          if (c1min < c0min) {
            const int tmp = node_addr;
            node_addr = node_addr_child1;
            node_addr_child1 = tmp;
          }
          if (++stack_ptr >= BVH_STACK_SIZE) {
            cy_set_error(err, CY_ERR_BVH_STACK, 2);
            return;
          }
          stack[stack_ptr] = node_addr_child1;
        }
        else if (traverse_mask == 2) {
          node_addr = node_addr_child1;
        }
        else if (traverse_mask == 0) {
          node_addr = stack[stack_ptr];
          --stack_ptr;
        }
      }
      if (node_addr < 0) {
        const hc_float4 leaf = kg->__bvh_leaf_nodes[-node_addr - 1];
        int prim_addr = as_int(leaf.x);
        const int prim_addr2 = as_int(leaf.y);
        const uint type = as_uint(leaf.w);
        node_addr = stack[stack_ptr];
        --stack_ptr;
        if ((type & PRIMITIVE_ALL) == PRIMITIVE_TRIANGLE) {
          for (; prim_addr < prim_addr2; prim_addr++) {
            /* triangle_intersect_local */
            if (object == OBJECT_NONE && (int)kg->__prim_object[prim_addr] != local_object) {
              continue;
            }
            const uint tri_vindex = kg->__prim_tri_index[prim_addr];
            const cfloat3 tri_a = f4to3(kg->__prim_tri_verts[tri_vindex + 0]);
            const cfloat3 tri_b = f4to3(kg->__prim_tri_verts[tri_vindex + 1]);
            const cfloat3 tri_c = f4to3(kg->__prim_tri_verts[tri_vindex + 2]);
            float t, u, v;
            if (!ray_triangle_intersect(P, dir, isect_t, tri_a, tri_b, tri_c, &u, &v, &t)) {
              continue;
            }
            bool seen = false;
            for (int i = (max_hits < li->num_hits ? max_hits : li->num_hits) - 1; i >= 0; --i) {
              if (li->hits[i].t == t) {
                seen = true;
                break;
              }
            }
            if (seen) {
              continue;
            }
            li->num_hits++;
            int hit;
            if (li->num_hits <= max_hits) {
              hit = li->num_hits - 1;
            }
            else {
              /* reservoir sampling */
              hit = (int)(lcg_step_uint(lcg_state) % (uint)li->num_hits);
              if (hit >= max_hits) {
                continue;
              }
            }
            CyIsect *is = &li->hits[hit];
            is->prim = prim_addr;
            is->object = object;
            is->type = PRIMITIVE_TRIANGLE;
            is->u = u;
            is->v = v;
            is->t = t;
            li->Ng[hit] = normalize3(cross3(sub3(tri_b, tri_a), sub3(tri_c, tri_a)));
          }
        }
      }
    } while (node_addr != ENTRYPOINT_SENTINEL);
  } while (node_addr != ENTRYPOINT_SENTINEL);
}

/* subsurface_scatter_disk (kernel_subsurface.h:160-282): a point on a disk
 * around the shading point along a randomly picked axis, a probe ray through
 * the object, and the hits found weighted by the profiles (MIS over the three
 * axes).  Returns the number of hits to evaluate; *ray is the probe ray. */
CY_FN int subsurface_scatter_disk(const CyGlobals *kg, CyLocalHits *li, const CySD *sd, const CyClosure *sc,
                                  uint *lcg_state, float disk_u, float disk_v, CyRay *ray, uint *err)
{
  cfloat3 disk_N, disk_T, disk_B;
  float pick_pdf_N, pick_pdf_T, pick_pdf_B;
  disk_N = sd->Ng;
  make_orthonormals(disk_N, &disk_T, &disk_B);
  if (disk_v < 0.5f) {
    pick_pdf_N = 0.5f;
    pick_pdf_T = 0.25f;
    pick_pdf_B = 0.25f;
    disk_v *= 2.0f;
  }
  else if (disk_v < 0.75f) {
    const cfloat3 tmp = disk_N;
    disk_N = disk_T;
    disk_T = tmp;
    pick_pdf_N = 0.25f;
    pick_pdf_T = 0.5f;
    pick_pdf_B = 0.25f;
    disk_v = (disk_v - 0.5f) * 4.0f;
  }
  else {
    const cfloat3 tmp = disk_N;
    disk_N = disk_B;
    disk_B = tmp;
    pick_pdf_N = 0.25f;
    pick_pdf_T = 0.25f;
    pick_pdf_B = 0.5f;
    disk_v = (disk_v - 0.75f) * 4.0f;
  }
  const float phi = CY_2PI_F * disk_v;
  float disk_height, disk_r;
  bssrdf_sample(sc, disk_u, &disk_r, &disk_height);
  const cfloat3 disk_P = add3(mul3f(disk_T, disk_r * cy_cosf(phi)), mul3f(disk_B, disk_r * cy_sinf(phi)));
  ray->P = add3(add3(sd->P, mul3f(disk_N, disk_height)), disk_P);
  ray->D = neg3(disk_N);
  ray->t = 2.0f * disk_height;
  scene_intersect_local_multi(kg, ray, sd->object, li, lcg_state, BSSRDF_MAX_HITS, err);
  const int num_eval_hits = li->num_hits < BSSRDF_MAX_HITS ? li->num_hits : BSSRDF_MAX_HITS;
  for (int hit = 0; hit < num_eval_hits; hit++) {
    if (!(sd->type & PRIMITIVE_TRIANGLE)) {
      li->weight[hit] = mk3(0.0f, 0.0f, 0.0f);
      continue;
    }
    const cfloat3 hit_P = triangle_refine_local(kg, &li->hits[hit], ray);
    cfloat3 hit_Ng = li->Ng[hit];
    if (li->hits[hit].object != OBJECT_NONE) {
      hit_Ng = object_normal_transform(kg, sd->object, hit_Ng);
    }
    const float pdf_N = pick_pdf_N * fabsf(dot3(disk_N, hit_Ng));
    const float pdf_T = pick_pdf_T * fabsf(dot3(disk_T, hit_Ng));
    const float pdf_B = pick_pdf_B * fabsf(dot3(disk_B, hit_Ng));
    float w = pdf_N / (sqr(pdf_N) + sqr(pdf_T) + sqr(pdf_B));
    if (li->num_hits > BSSRDF_MAX_HITS) {
      w *= li->num_hits / (float)BSSRDF_MAX_HITS;
    }
    const float r = len3(sub3(hit_P, sd->P));
    li->weight[hit] = mul3f(subsurface_scatter_eval(sd, disk_r, r), w);
  }
  return num_eval_hits;
}

/* shader_bssrdf_sum (kernel_shader.h:766-795) */
CY_FN cfloat3 shader_bssrdf_sum(const CySD *sd, cfloat3 *N_, float *texture_blur_)
{
  cfloat3 eval = mk3(0.0f, 0.0f, 0.0f);
  cfloat3 N = mk3(0.0f, 0.0f, 0.0f);
  float texture_blur = 0.0f, weight_sum = 0.0f;
  for (int i = 0; i < sd->num_closure; i++) {
    const CyClosure *sc = &sd->closure[i];
    if (CLOSURE_IS_BSSRDF(sc->type)) {
      const float avg_weight = fabsf(average3(sc->weight));
      N = add3(N, mul3f(sc->N, avg_weight));
      eval = add3(eval, sc->weight);
      texture_blur += bssrdf_texture_blur(sc) * avg_weight;
      weight_sum += avg_weight;
    }
  }
  if (N_) {
    *N_ = is_zero3(N) ? sd->N : normalize3(N);
  }
  if (texture_blur_) {
    *texture_blur_ = safe_divide(texture_blur, weight_sum);
  }
  return eval;
}

/* kernel_subsurface.h:111-130 */
CY_FN cfloat3 subsurface_color_pow(cfloat3 color, float exponent)
{
  color = max3v(color, mk3(0.0f, 0.0f, 0.0f)); /* max(float3) */
  if (exponent == 1.0f) {
    /* nothing to do */
  }
  else if (exponent == 0.5f) {
    color.x = sqrtf(color.x);
    color.y = sqrtf(color.y);
    color.z = sqrtf(color.z);
  }
  else {
    color.x = cy_powf(color.x, exponent);
    color.y = cy_powf(color.y, exponent);
    color.z = cy_powf(color.z, exponent);
  }
  return color;
}

/* subsurface_color_bump_blur (kernel_subsurface.h:132-158): with texture
 * blur or a bumped BSSRDF normal the shader is evaluated again at the exit
 * point; the scatter weight takes the ratio of the two points' BSSRDF colours
 * (raised to the blur) and the normal the exit point's.  The closures in sd
 * at the call are those the BSSRDF was picked from for the first exit point
 * and the previous exit point's diffuse closure for the later ones, as in the
 * reference (whose later exit points therefore see no texture blur). */
CY_FN void subsurface_color_bump_blur(const CyGlobals *kg, CySD *sd, CyPathState *state, cfloat3 *eval, cfloat3 *N,
                                      uint *err)
{
  float texture_blur;
  cfloat3 out_color = shader_bssrdf_sum(sd, 0, &texture_blur);
  const bool bump = (sd->flag & SD_HAS_BSSRDF_BUMP) != 0;
  if (bump || texture_blur > 0.0f) {
    shader_eval_surface(kg, sd, state, state->flag, err);
    cfloat3 in_color = shader_bssrdf_sum(sd, bump ? N : 0, 0);
    if (texture_blur > 0.0f) {
      out_color = subsurface_color_pow(out_color, texture_blur);
      in_color = subsurface_color_pow(in_color, texture_blur);
      *eval = mul3(*eval, safe_divide_color(in_color, out_color));
    }
  }
}

#endif /* CY_CLOSURE_EXT */
#endif /* CY_SUBSURFACE_H */
