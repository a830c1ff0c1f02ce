/*
 * cy_svm_raytrace.h — the SVM nodes that trace rays from inside a shader
 * (__SHADER_RAYTRACE__): Ambient Occlusion and Bevel.
 *   svm_ao, svm_node_ao        kernel/svm/svm_ao.h:21-104
 *   svm_bevel, svm_node_bevel  kernel/svm/svm_bevel.h:28-216
 * Declared in cy_path.h (the interpreter dispatches them) and defined here,
 * after the local traversals of cy_subsurface.h they reuse: the opaque
 * any-hit scene query for AO, the closest local query for AO "only local"
 * (the reference asks the local traversal for any hit, max_hits 0; a hit of
 * the object within the distance exists exactly when the closest one does),
 * and the reservoir-sampled multi-hit local query of the disk BSSRDFs for
 * Bevel.  A shader evaluated without a path state (the SHADER tasks' world and
 * displacement programs, whose reference counterparts run before the BVH
 * exists or without an object) returns the node's no-trace result.
 */
#ifndef CY_SVM_RAYTRACE_H
#define CY_SVM_RAYTRACE_H

#if CY_SVM_TEX && CY_CLOSURE_EXT

#define CY_NODE_AO_ONLY_LOCAL (1 << 0)
#define CY_NODE_AO_INSIDE (1 << 1)
#define CY_NODE_AO_GLOBAL_RADIUS (1 << 2)
#define CY_PRNG_BEVEL_U 6 /* kernel_types.h:256 */

/* path_branched_rng_2D (kernel_random.h:235-251) */
CY_FN void path_branched_rng_2D(const CyGlobals *kg, uint rng_hash, const CyPathState *state, int branch,
                                int num_branches, int dimension, float *fx, float *fy)
{
  path_rng_2D(kg, rng_hash, state->sample * num_branches + branch, state->rng_offset + dimension, fx, fy);
}

CY_FN float svm_ao(const CyGlobals *kg, const CySD *sd, cfloat3 N, const CyPathState *state, float max_dist,
                   int num_samples, int flags, uint *err)
{
  if (flags & CY_NODE_AO_GLOBAL_RADIUS) {
    max_dist = KD->background.ao_distance;
  }
  if (max_dist <= 0.0f || num_samples < 1 || sd->object == OBJECT_NONE || state == nullptr) {
    return 1.0f;
  }
  if (flags & CY_NODE_AO_INSIDE) {
    N = neg3(N);
  }
  cfloat3 T, B;
  make_orthonormals(N, &T, &B);
  int unoccluded = 0;
  for (int sample = 0; sample < num_samples; sample++) {
    float disk_u, disk_v;
    path_branched_rng_2D(kg, state->rng_hash, state, sample, num_samples, CY_PRNG_BEVEL_U, &disk_u, &disk_v);
    float dx, dy;
    concentric_sample_disk(disk_u, disk_v, &dx, &dy);
    const cfloat3 D = mk3(dx, dy, safe_sqrtf(1.0f - (dx * dx + dy * dy)));
    CyRay ray;
    ray.P = ray_offset(sd->P, N);
    ray.D = add3(add3(mul3f(T, D.x), mul3f(B, D.y)), mul3f(N, D.z));
    ray.t = max_dist;
    if (flags & CY_NODE_AO_ONLY_LOCAL) {
      CyIsect hit;
      cfloat3 hit_Ng;
      if (!scene_intersect_local_closest(kg, &ray, sd->object, &hit, &hit_Ng, err)) {
        unoccluded++;
      }
    }
    else {
      CyIsect isect;
      bool blocked = false;
      if (scene_intersect_valid(&ray)) {
        blocked = kg->have_curves ? bvh2_intersect<true, true, 2, CY_LDS_STACK, CY_BLOCK, 3>(
                                        kg, &ray, PATH_RAY_SHADOW_OPAQUE, &isect, err, nullptr, nullptr, nullptr) :
                                    bvh2_intersect<true>(kg, &ray, PATH_RAY_SHADOW_OPAQUE, &isect, err, nullptr,
                                                         nullptr, nullptr);
      }
      if (!blocked) {
        unoccluded++;
      }
    }
  }
  return ((float)unoccluded) / num_samples;
}

CY_FN void svm_node_ao(const CyGlobals *kg, CySD *sd, const CyPathState *state, CySvmStack stack, hc_uint4 node,
                       uint *err)
{
  uint flags, dist_offset, normal_offset, out_ao_offset;
  svm_unpack4(node.y, &flags, &dist_offset, &normal_offset, &out_ao_offset);
  uint color_offset, out_color_offset, samples;
  svm_unpack3(node.z, &color_offset, &out_color_offset, &samples);
  const float dist = svm_load_default(stack, dist_offset, node.w, err);
  const cfloat3 normal = (normal_offset != SVM_STACK_INVALID) ? svm_load3(stack, normal_offset, err) : sd->N;
  const float ao = svm_ao(kg, sd, normal, state, dist, (int)samples, (int)flags, err);
  if (out_ao_offset != SVM_STACK_INVALID) {
    svm_store(stack, out_ao_offset, ao, err);
  }
  if (out_color_offset != SVM_STACK_INVALID) {
    const cfloat3 color = svm_load3(stack, color_offset, err);
    svm_store3(stack, out_color_offset, mul3f(color, ao), err);
  }
}

/* Bevel: normals of nearby surface points of the same object, found by local
 * probe rays along the three axes of the shading frame (the cubic BSSRDF's
 * radius profile), MIS-weighted. */
CY_FN cfloat3 svm_bevel(const CyGlobals *kg, const CySD *sd, const CyPathState *state, float radius, int num_samples,
                        uint *err)
{
  if (radius <= 0.0f || num_samples < 1 || sd->object == OBJECT_NONE || state == nullptr) {
    return sd->N;
  }
  /* no bevel for blurry indirect rays */
  if (state->min_ray_pdf < 8.0f) {
    return sd->N;
  }
  uint lcg_state = lcg_init(state->rng_hash + (uint)state->rng_offset + (uint)state->sample * 0x64c6a40eu);
  cfloat3 sum_N = mk3(0.0f, 0.0f, 0.0f);
  for (int sample = 0; sample < num_samples; sample++) {
    float disk_u, disk_v;
    path_branched_rng_2D(kg, state->rng_hash, state, sample, num_samples, CY_PRNG_BEVEL_U, &disk_u, &disk_v);
    /* a random axis of the local frame and a point on the disk around it */
    cfloat3 disk_N = sd->Ng, disk_T, disk_B;
    float pick_pdf_N, pick_pdf_T, pick_pdf_B;
    make_orthonormals(disk_N, &disk_T, &disk_B);
    const float axisu = disk_u;
    if (axisu < 0.5f) {
      pick_pdf_N = 0.5f;
      pick_pdf_T = 0.25f;
      pick_pdf_B = 0.25f;
      disk_u *= 2.0f;
    }
    else if (axisu < 0.75f) {
      const cfloat3 tmp = disk_N;
      disk_N = disk_T;
      disk_T = tmp;
      pick_pdf_N = 0.25f;
      pick_pdf_T = 0.5f;
      pick_pdf_B = 0.25f;
      disk_u = (disk_u - 0.5f) * 4.0f;
    }
    else {
      const cfloat3 tmp = disk_N;
      disk_N = disk_B;
      disk_B = tmp;
      pick_pdf_N = 0.25f;
      pick_pdf_T = 0.25f;
      pick_pdf_B = 0.5f;
      disk_u = (disk_u - 0.75f) * 4.0f;
    }
    const float phi = CY_2PI_F * disk_u;
    float disk_r = disk_v;
    float disk_height;
    bssrdf_cubic_sample(radius, 0.0f, disk_r, &disk_r, &disk_height);
    const cfloat3 disk_P = add3(mul3f(disk_T, disk_r * cy_cosf(phi)), mul3f(disk_B, disk_r * cy_sinf(phi)));
    CyRay ray;
    ray.P = add3(add3(sd->P, mul3f(disk_N, disk_height)), disk_P);
    ray.D = neg3(disk_N);
    ray.t = 2.0f * disk_height;
    /* up to LOCAL_MAX_HITS hits of the same object, a random subset of all */
    CyLocalHits li;
    scene_intersect_local_multi(kg, &ray, sd->object, &li, &lcg_state, BSSRDF_MAX_HITS, err);
    const int num_eval_hits = imin(li.num_hits, BSSRDF_MAX_HITS);
    for (int hit = 0; hit < num_eval_hits; hit++) {
      /* P and Ng without a shading point setup */
      const cfloat3 hit_P = triangle_refine_local(kg, &li.hits[hit], &ray);
      cfloat3 hit_Ng = li.Ng[hit];
      const int object = (li.hits[hit].object == OBJECT_NONE) ? (int)kg->__prim_object[li.hits[hit].prim] :
                                                                  li.hits[hit].object;
      const uint object_flag = kg->__object_flag[object];
      if (object_flag & SD_OBJECT_NEGATIVE_SCALE_APPLIED) {
        hit_Ng = neg3(hit_Ng);
      }
      /* smooth normal */
      cfloat3 N = hit_Ng;
      const int prim = (int)kg->__prim_index[li.hits[hit].prim];
      const int shader = (int)kg->__tri_shader[prim];
      if ((uint)shader & SHADER_SMOOTH_NORMAL) {
        N = triangle_smooth_normal(kg, N, prim, li.hits[hit].u, li.hits[hit].v);
      }
      if (!(object_flag & SD_OBJECT_TRANSFORM_APPLIED)) {
        N = object_normal_transform(kg, sd->object, N);
        hit_Ng = object_normal_transform(kg, sd->object, hit_Ng);
      }
      /* MIS over the three axes (power heuristic; pdf_N cancels) */
      const float pdf_N = pick_pdf_N * fabsf(dot3(disk_N, hit_Ng));
      const float pdf_T = pick_pdf_T * fabsf(dot3(disk_T, hit_Ng));
      const float pdf_B = pick_pdf_B * fabsf(dot3(disk_B, hit_Ng));
      float w = pdf_N / (sqr(pdf_N) + sqr(pdf_T) + sqr(pdf_B));
      if (li.num_hits > BSSRDF_MAX_HITS) {
        w *= li.num_hits / (float)BSSRDF_MAX_HITS;
      }
      const float r = len3(sub3(hit_P, sd->P));
      const float pdf = bssrdf_cubic_eval(radius, 0.0f, r);
      const float disk_pdf = bssrdf_cubic_eval(radius, 0.0f, disk_r);
      w *= pdf / disk_pdf;
      sum_N = add3(sum_N, mul3f(N, w));
    }
  }
  const cfloat3 N = safe_normalize3(sum_N);
  return is_zero3(N) ? sd->N : (sd->flag & SD_BACKFACING) ? neg3(N) : N;
}

CY_FN void svm_node_bevel(const CyGlobals *kg, CySD *sd, const CyPathState *state, CySvmStack stack, hc_uint4 node,
                          uint *err)
{
  uint num_samples, radius_offset, normal_offset, out_offset;
  svm_unpack4(node.y, &num_samples, &radius_offset, &normal_offset, &out_offset);
  const float radius = svm_load(stack, radius_offset, err);
  cfloat3 bevel_N = svm_bevel(kg, sd, state, radius, (int)num_samples, err);
  if (normal_offset != SVM_STACK_INVALID) {
    /* keep the input normal's detail */
    const cfloat3 ref_N = svm_load3(stack, normal_offset, err);
    bevel_N = normalize3(add3(ref_N, sub3(bevel_N, sd->N)));
  }
  svm_store3(stack, out_offset, bevel_N, err);
}

#endif /* CY_SVM_TEX && CY_CLOSURE_EXT */

#endif /* CY_SVM_RAYTRACE_H */
