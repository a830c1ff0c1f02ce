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
 * The path-level flow (kernel_path_subsurface.h:26-110: light at the exit
 * point with the path's state, the bounce with rng_offset + PRNG_BOUNCE_NUM)
 * is in cy_integrator.h shade_path.  A random walk leaves at one point, so the
 * SubsurfaceIndirectRays stack of the reference holds one ray and the path
 * simply continues from the exit; disk BSSRDFs (up to four exit points) are
 * rejected.
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

/* util_math.h:514 safe_divide_color */
CY_FN cfloat3 safe_divide_color(cfloat3 a, cfloat3 b)
{
  return mk3((b.x != 0.0f) ? a.x / b.x : 0.0f, (b.y != 0.0f) ? a.y / b.y : 0.0f, (b.z != 0.0f) ? a.z / b.z : 0.0f);
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
  sd->flag |= kg->__shaders[(uint)sd->shader & SHADER_MASK].flags;
  if (isect->object != OBJECT_NONE) {
    sd->N = object_normal_transform(kg, sd->object, sd->N);
    sd->Ng = object_normal_transform(kg, sd->object, sd->Ng);
  }
  if (backfacing) {
    sd->flag |= SD_BACKFACING;
    sd->Ng = neg3(sd->Ng);
    sd->N = neg3(sd->N);
  }
  sd->I = sd->N;
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

#endif /* CY_CLOSURE_EXT */
#endif /* CY_SUBSURFACE_H */
