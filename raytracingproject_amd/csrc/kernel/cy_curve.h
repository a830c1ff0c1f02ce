/*
 * cy_curve.h — hair curve primitives: Catmull-Rom segments intersected as flat
 * ribbons or thick round curves, and the hit-point setup for shading.
 *
 * Restates kernel/geom/geom_curve_intersect.h (Cycles 2.91, itself adapted
 * from Embree's curve_intersector_sweep.h) operation for operation in the
 * scalar float arithmetic of the reference CPU kernel, so a curve hit's t, u,
 * v are the reference's bit for bit:
 *   catmull_rom_basis_eval / _derivative / _derivative2   :34-65
 *   cylinder_intersect, half_plane_intersect               :83-167
 *   curve_intersect_iterative (Newton on the sweep)        :169-258
 *   curve_intersect_recursive (thick curves)               :260-448
 *   ribbon_intersect_quad / ribbon_intersect (ribbons)     :452-618
 *   curve_intersect (segment fetch, visibility)            :620-692
 *   curve_shader_setup                                     :694-794
 * Motion curves are not implemented (rejected at load_kernels).
 *
 * The data are the host's packed hair arrays (render/hair.cpp pack_curves):
 * __curves[curve] = (first key, key count, shader, 0) as int bits,
 * __curve_keys[key] = (x, y, z, radius); a BVH primitive's __prim_type carries
 * the segment index above PRIMITIVE_NUM_TOTAL (kernel_types.h:713-717).
 */
#ifndef CY_CURVE_H
#define CY_CURVE_H

#define CY_FLT_EPSILON 1.192092896e-07f
#define CY_CURVE_NUM_BEZIER_SUBDIVISIONS 3
#define CY_CURVE_NUM_BEZIER_SUBDIVISIONS_UNSTABLE (CY_CURVE_NUM_BEZIER_SUBDIVISIONS + 1)
#define CY_CURVE_NUM_BEZIER_STEPS 2
#define CY_CURVE_NUM_JACOBIAN_ITERATIONS 5
#define CY_PRIMITIVE_CURVE_THICK (1 << 2)
#define CY_PRIMITIVE_MOTION_CURVE_THICK (1 << 3)
#define CY_PRIMITIVE_CURVE_RIBBON (1 << 4)
#define CY_PRIMITIVE_MOTION_CURVE_RIBBON (1 << 5)
#define CY_PRIMITIVE_NUM_TOTAL 6
#define CY_PRIMITIVE_UNPACK_SEGMENT(type) ((type) >> CY_PRIMITIVE_NUM_TOTAL)

/* float4 arithmetic of util_math_float4.h, scalar branch */
struct cy_c4 {
  float x, y, z, w;
};
CY_FN cy_c4 c4(float x, float y, float z, float w)
{
  cy_c4 r;
  r.x = x;
  r.y = y;
  r.z = z;
  r.w = w;
  return r;
}
CY_FN cy_c4 c4_load(const hc_float4 &a)
{
  return c4(a.x, a.y, a.z, a.w);
}
CY_FN cy_c4 c4_add(cy_c4 a, cy_c4 b)
{
  return c4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
CY_FN cy_c4 c4_sub(cy_c4 a, cy_c4 b)
{
  return c4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}
/* float4 * float and float * float4 both compute a.x * f */
CY_FN cy_c4 c4_mulf(cy_c4 a, float f)
{
  return c4(a.x * f, a.y * f, a.z * f, a.w * f);
}
CY_FN cy_c4 c4_min(cy_c4 a, cy_c4 b)
{
  return c4(cmin(a.x, b.x), cmin(a.y, b.y), cmin(a.z, b.z), cmin(a.w, b.w));
}
CY_FN cy_c4 c4_max(cy_c4 a, cy_c4 b)
{
  return c4(cmax(a.x, b.x), cmax(a.y, b.y), cmax(a.z, b.z), cmax(a.w, b.w));
}
CY_FN cy_c4 c4_fabs(cy_c4 a)
{
  return c4(fabsf(a.x), fabsf(a.y), fabsf(a.z), fabsf(a.w));
}
CY_FN cfloat3 c4_xyz(cy_c4 a)
{
  return mk3(a.x, a.y, a.z);
}
CY_FN float cmix(float a, float b, float t)
{
  return a + t * (b - a);
}

/* Catmull-Rom basis (geom_curve_intersect.h:34-65): the four weighted keys
 * summed left to right, then scaled. */
CY_FN cy_c4 catmull_rom_basis_eval(const cy_c4 curve[4], float u)
{
  const float t = u;
  const float s = 1.0f - u;
  const float n0 = -t * s * s;
  const float n1 = 2.0f + t * t * (3.0f * t - 5.0f);
  const float n2 = 2.0f + s * s * (3.0f * s - 5.0f);
  const float n3 = -s * t * t;
  const cy_c4 sum = c4_add(c4_add(c4_add(c4_mulf(curve[0], n0), c4_mulf(curve[1], n1)), c4_mulf(curve[2], n2)),
                           c4_mulf(curve[3], n3));
  return c4_mulf(sum, 0.5f);
}

CY_FN cy_c4 catmull_rom_basis_derivative(const cy_c4 curve[4], float u)
{
  const float t = u;
  const float s = 1.0f - u;
  const float n0 = -s * s + 2.0f * s * t;
  const float n1 = 2.0f * t * (3.0f * t - 5.0f) + 3.0f * t * t;
  const float n2 = 2.0f * s * (3.0f * t + 2.0f) - 3.0f * s * s;
  const float n3 = -2.0f * s * t + t * t;
  const cy_c4 sum = c4_add(c4_add(c4_add(c4_mulf(curve[0], n0), c4_mulf(curve[1], n1)), c4_mulf(curve[2], n2)),
                           c4_mulf(curve[3], n3));
  return c4_mulf(sum, 0.5f);
}

CY_FN cy_c4 catmull_rom_basis_derivative2(const cy_c4 curve[4], float u)
{
  const float t = u;
  const float n0 = -3.0f * t + 2.0f;
  const float n1 = 9.0f * t - 5.0f;
  const float n2 = -9.0f * t + 4.0f;
  const float n3 = 3.0f * t - 1.0f;
  return c4_add(c4_add(c4_add(c4_mulf(curve[0], n0), c4_mulf(curve[1], n1)), c4_mulf(curve[2], n2)),
                c4_mulf(curve[3], n3));
}

/* ---- thick curves ---- */

CY_FN cfloat3 dnormalize(cfloat3 p, cfloat3 dp)
{
  const float pp = dot3(p, p);
  const float pdp = dot3(p, dp);
  return div3f(sub3(mul3f(dp, pp), mul3f(p, pdp)), pp * sqrtf(pp));
}

CY_FN float sqr_point_to_line_distance(cfloat3 PmQ0, cfloat3 Q1mQ0)
{
  const cfloat3 N = cross3(PmQ0, Q1mQ0);
  const cfloat3 D = Q1mQ0;
  return dot3(N, N) / dot3(D, D);
}

/* cylinder_intersect (:83-153).  The hit normals it also returns are never
 * read by the recursive intersector and are not computed here. */
CY_FN bool cylinder_intersect(cfloat3 cylinder_start, cfloat3 cylinder_end, float cylinder_radius, cfloat3 ray_dir,
                              float *t_o_x, float *t_o_y, float *u0_o, float *u1_o)
{
  const float rl = 1.0f / len3(sub3(cylinder_end, cylinder_start));
  const cfloat3 P0 = cylinder_start, dP = mul3f(sub3(cylinder_end, cylinder_start), rl);
  const cfloat3 O = neg3(P0), dO = ray_dir;

  const float dOdO = dot3(dO, dO);
  const float OdO = dot3(dO, O);
  const float OO = dot3(O, O);
  const float dOz = dot3(dP, dO);
  const float Oz = dot3(dP, O);

  const float A = dOdO - sqr(dOz);
  const float B = 2.0f * (OdO - dOz * Oz);
  const float C = OO - sqr(Oz) - sqr(cylinder_radius);

  const float D = B * B - 4.0f * A * C;
  if (!(D >= 0.0f)) {
    *t_o_x = CY_FLT_MAX;
    *t_o_y = -CY_FLT_MAX;
    return false;
  }

  const float eps = 16.0f * CY_FLT_EPSILON * cmax(fabsf(dOdO), fabsf(sqr(dOz)));
  if (fabsf(A) < eps) {
    *t_o_x = -CY_FLT_MAX;
    *t_o_y = CY_FLT_MAX;
    return C <= 0.0f;
  }

  const float Q = sqrtf(D);
  const float rcp_2A = 1.0f / (2.0f * A);
  const float t0 = (-B - Q) * rcp_2A;
  const float t1 = (-B + Q) * rcp_2A;
  *u0_o = (t0 * dOz + Oz) * rl;
  *u1_o = (t1 * dOz + Oz) * rl;
  *t_o_x = t0;
  *t_o_y = t1;
  return true;
}

CY_FN void half_plane_intersect(cfloat3 P, cfloat3 N, cfloat3 ray_dir, float *lower, float *upper)
{
  const cfloat3 O = neg3(P);
  const cfloat3 D = ray_dir;
  const float ON = dot3(O, N);
  const float DN = dot3(D, N);
  const float min_rcp_input = 1e-18f;
  const bool eps = fabsf(DN) < min_rcp_input;
  const float t = -ON / DN;
  *lower = (eps || DN < 0.0f) ? -CY_FLT_MAX : t;
  *upper = (eps || DN > 0.0f) ? CY_FLT_MAX : t;
}

CY_FN bool curve_intersect_iterative(cfloat3 ray_dir, float dt, const cy_c4 curve[4], float u, float t,
                                     bool use_backfacing, CyIsect *isect)
{
  const float length_ray_dir = len3(ray_dir);

  /* Error of curve evaluations is proportional to largest coordinate.  (The
   * reference takes max(min(curve[0], curve[1]), ...) for box_max; kept.) */
  const cy_c4 box_min = c4_min(c4_min(curve[0], curve[1]), c4_min(curve[2], curve[3]));
  const cy_c4 box_max = c4_max(c4_min(curve[0], curve[1]), c4_max(curve[2], curve[3]));
  const cy_c4 box_abs = c4_max(c4_fabs(box_min), c4_fabs(box_max));
  const float P_err = 16.0f * CY_FLT_EPSILON * cmax(box_abs.x, cmax(box_abs.y, cmax(box_abs.z, box_abs.w)));
  const float radius_max = box_max.w;

  for (int i = 0; i < CY_CURVE_NUM_JACOBIAN_ITERATIONS; i++) {
    const cfloat3 Q = mul3f(ray_dir, t);
    const cfloat3 dQdt = ray_dir;
    const float Q_err = 16.0f * CY_FLT_EPSILON * length_ray_dir * t;

    const cy_c4 P4 = catmull_rom_basis_eval(curve, u);
    const cy_c4 dPdu4 = catmull_rom_basis_derivative(curve, u);

    const cfloat3 P = c4_xyz(P4);
    const cfloat3 dPdu = c4_xyz(dPdu4);
    const float radius = P4.w;
    const float dradiusdu = dPdu4.w;

    const cfloat3 ddPdu = c4_xyz(catmull_rom_basis_derivative2(curve, u));

    const cfloat3 R = sub3(Q, P);
    const float len_R = len3(R);
    const float R_err = cmax(Q_err, P_err);
    const cfloat3 dRdu = neg3(dPdu);
    const cfloat3 dRdt = dQdt;

    const cfloat3 T = normalize3(dPdu);
    const cfloat3 dTdu = dnormalize(dPdu, ddPdu);
    const float cos_err = P_err / len3(dPdu);

    const float f = dot3(R, T);
    const float f_err = len_R * P_err + R_err + cos_err * (1.0f + len_R);
    const float dfdu = dot3(dRdu, T) + dot3(R, dTdu);
    const float dfdt = dot3(dRdt, T);

    const float K = dot3(R, R) - sqr(f);
    const float dKdu = (dot3(R, dRdu) - f * dfdu);
    const float dKdt = (dot3(R, dRdt) - f * dfdt);
    const float rsqrt_K = inversesqrtf(K);

    const float g = sqrtf(K) - radius;
    const float g_err = R_err + f_err + 16.0f * CY_FLT_EPSILON * radius_max;
    const float dgdu = dKdu * rsqrt_K - dradiusdu;
    const float dgdt = dKdt * rsqrt_K;

    const float invdet = 1.0f / (dfdu * dgdt - dgdu * dfdt);
    u -= (dgdt * f - dfdt * g) * invdet;
    t -= (-dgdu * f + dfdu * g) * invdet;

    if (fabsf(f) < f_err && fabsf(g) < g_err) {
      t += dt;
      if (!(0.0f <= t && t <= isect->t)) {
        return false; /* Rejects NaNs */
      }
      if (!(u >= 0.0f && u <= 1.0f)) {
        return false; /* Rejects NaNs */
      }

      /* Backface culling. */
      const cfloat3 R2 = normalize3(sub3(Q, P));
      const cfloat3 U = add3(mul3f(R2, dradiusdu), dPdu);
      const cfloat3 V = cross3(dPdu, R2);
      const cfloat3 Ng = cross3(V, U);
      if (!use_backfacing && dot3(ray_dir, Ng) > 0.0f) {
        return false;
      }

      isect->t = t;
      isect->u = u;
      isect->v = 0.0f;
      return true;
    }
  }
  return false;
}

CY_FN bool curve_intersect_recursive(cfloat3 ray_orig, cfloat3 ray_dir, cy_c4 curve[4], CyIsect *isect)
{
  /* Move ray closer to make intersection stable. */
  const cfloat3 center = c4_xyz(c4_mulf(c4_add(c4_add(c4_add(curve[0], curve[1]), curve[2]), curve[3]), 0.25f));
  const float dt = dot3(sub3(center, ray_orig), ray_dir) / dot3(ray_dir, ray_dir);
  const cfloat3 ref = add3(ray_orig, mul3f(ray_dir, dt));
  const cy_c4 ref4 = c4(ref.x, ref.y, ref.z, 0.0f);
  curve[0] = c4_sub(curve[0], ref4);
  curve[1] = c4_sub(curve[1], ref4);
  curve[2] = c4_sub(curve[2], ref4);
  curve[3] = c4_sub(curve[3], ref4);

  const bool use_backfacing = false;
  const float step_size = 1.0f / (float)(CY_CURVE_NUM_BEZIER_STEPS);

  int depth = 0;
  float stack_u0[CY_CURVE_NUM_BEZIER_SUBDIVISIONS_UNSTABLE];
  float stack_u1[CY_CURVE_NUM_BEZIER_SUBDIVISIONS_UNSTABLE];
  int stack_i[CY_CURVE_NUM_BEZIER_SUBDIVISIONS_UNSTABLE];

  bool found = false;
  float u0 = 0.0f;
  float u1 = 1.0f;
  int i = 0;

  while (1) {
    for (; i < CY_CURVE_NUM_BEZIER_STEPS; i++) {
      const float step = i * step_size;

      /* Subdivide curve. */
      const float dscale = (u1 - u0) * (1.0f / 3.0f) * step_size;
      const float vu0 = cmix(u0, u1, step);
      const float vu1 = cmix(u0, u1, step + step_size);

      const cy_c4 P0 = catmull_rom_basis_eval(curve, vu0);
      const cy_c4 dP0du = c4_mulf(catmull_rom_basis_derivative(curve, vu0), dscale);
      const cy_c4 P3 = catmull_rom_basis_eval(curve, vu1);
      const cy_c4 dP3du = c4_mulf(catmull_rom_basis_derivative(curve, vu1), dscale);

      const cy_c4 P1 = c4_add(P0, dP0du);
      const cy_c4 P2 = c4_sub(P3, dP3du);

      /* Calculate bounding cylinders. */
      const float rr1 = sqr_point_to_line_distance(c4_xyz(dP0du), c4_xyz(c4_sub(P3, P0)));
      const float rr2 = sqr_point_to_line_distance(c4_xyz(dP3du), c4_xyz(c4_sub(P3, P0)));
      const float maxr12 = sqrtf(cmax(rr1, rr2));
      const float one_plus_ulp = 1.0f + 2.0f * CY_FLT_EPSILON;
      const float one_minus_ulp = 1.0f - 2.0f * CY_FLT_EPSILON;
      float r_outer = cmax(cmax(P0.w, P1.w), cmax(P2.w, P3.w)) + maxr12;
      float r_inner = cmin(cmin(P0.w, P1.w), cmin(P2.w, P3.w)) - maxr12;
      r_outer = one_plus_ulp * r_outer;
      r_inner = cmax(0.0f, one_minus_ulp * r_inner);
      bool valid = true;

      /* Intersect with outer cylinder. */
      float tco_x, tco_y, u_outer0 = 0.0f, u_outer1 = 0.0f;
      valid = cylinder_intersect(c4_xyz(P0), c4_xyz(P3), r_outer, ray_dir, &tco_x, &tco_y, &u_outer0, &u_outer1);
      if (!valid) {
        continue;
      }

      /* Intersect with cap-planes. */
      float tp_x = -dt, tp_y = isect->t - dt;
      tp_x = cmax(tp_x, tco_x);
      tp_y = cmin(tp_y, tco_y);
      float h_lo, h_hi;
      half_plane_intersect(c4_xyz(P0), c4_xyz(dP0du), ray_dir, &h_lo, &h_hi);
      tp_x = cmax(tp_x, h_lo);
      tp_y = cmin(tp_y, h_hi);
      half_plane_intersect(c4_xyz(P3), neg3(c4_xyz(dP3du)), ray_dir, &h_lo, &h_hi);
      tp_x = cmax(tp_x, h_lo);
      tp_y = cmin(tp_y, h_hi);
      valid = tp_x <= tp_y;
      if (!valid) {
        continue;
      }

      /* Clamp and correct u parameter. */
      u_outer0 = cclamp(u_outer0, 0.0f, 1.0f);
      u_outer1 = cclamp(u_outer1, 0.0f, 1.0f);
      u_outer0 = cmix(u0, u1, (step + u_outer0) * (1.0f / (float)(CY_CURVE_NUM_BEZIER_STEPS + 1)));
      u_outer1 = cmix(u0, u1, (step + u_outer1) * (1.0f / (float)(CY_CURVE_NUM_BEZIER_STEPS + 1)));

      /* Intersect with inner cylinder (only its hit interval is used). */
      float tci_x, tci_y, u_inner0, u_inner1;
      (void)cylinder_intersect(c4_xyz(P0), c4_xyz(P3), r_inner, ray_dir, &tci_x, &tci_y, &u_inner0, &u_inner1);

      /* The reference always subdivides to the unstable depth. */
      const bool unstable0 = true;
      const bool unstable1 = true;

      /* Subtract the inner interval from the current hit interval. */
      const float tp0_x = tp_x, tp0_y = cmin(tp_y, tci_x);
      const float tp1_x = cmax(tp_x, tci_y), tp1_y = tp_y;
      const bool valid0 = valid && (tp0_x <= tp0_y);
      const bool valid1 = valid && (tp1_x <= tp1_y);
      if (!(valid0 || valid1)) {
        continue;
      }

      /* Process one or two hits. */
      bool recurse = false;
      if (valid0) {
        const int termDepth = unstable0 ? CY_CURVE_NUM_BEZIER_SUBDIVISIONS_UNSTABLE :
                                          CY_CURVE_NUM_BEZIER_SUBDIVISIONS;
        if (depth >= termDepth) {
          found |= curve_intersect_iterative(ray_dir, dt, curve, u_outer0, tp0_x, use_backfacing, isect);
        }
        else {
          recurse = true;
        }
      }

      if (valid1 && (tp1_x + dt <= isect->t)) {
        const int termDepth = unstable1 ? CY_CURVE_NUM_BEZIER_SUBDIVISIONS_UNSTABLE :
                                          CY_CURVE_NUM_BEZIER_SUBDIVISIONS;
        if (depth >= termDepth) {
          found |= curve_intersect_iterative(ray_dir, dt, curve, u_outer1, tp1_y, use_backfacing, isect);
        }
        else {
          recurse = true;
        }
      }

      if (recurse) {
        stack_u0[depth] = u0;
        stack_u1[depth] = u1;
        stack_i[depth] = i + 1;
        depth++;

        u0 = vu0;
        u1 = vu1;
        i = -1;
      }
    }

    if (depth > 0) {
      depth--;
      u0 = stack_u0[depth];
      u1 = stack_u1[depth];
      i = stack_i[depth];
    }
    else {
      break;
    }
  }

  return found;
}

/* ---- ribbons ---- */

CY_FN bool cylinder_culling_test(float p1x, float p1y, float p2x, float p2y, float r)
{
  /* Performs culling against a cylinder. */
  const float dpx = p2x - p1x, dpy = p2y - p1y;
  const float num = dpx * p1y - dpy * p1x;
  const float den2 = (p2x - p1x) * (p2x - p1x) + (p2y - p1y) * (p2y - p1y);
  return num * num <= r * r * den2;
}

/* A quad v0 v1 v2 v3 split into triangles v0 v1 v3 and v2 v3 v1, the edge
 * v1 v2 deciding which one is tested (ray space: O = 0, D = +z). */
CY_FN bool ribbon_intersect_quad(float ray_tfar, cfloat3 quad_v0, cfloat3 quad_v1, cfloat3 quad_v2, cfloat3 quad_v3,
                                 float *u_o, float *v_o, float *t_o)
{
  const cfloat3 O = mk3(0.0f, 0.0f, 0.0f);
  const cfloat3 D = mk3(0.0f, 0.0f, 1.0f);
  const cfloat3 va = sub3(quad_v0, O);
  const cfloat3 vb = sub3(quad_v1, O);
  const cfloat3 vc = sub3(quad_v2, O);
  const cfloat3 vd = sub3(quad_v3, O);

  const cfloat3 edb = sub3(vb, vd);
  const float WW = dot3(cross3(vd, edb), D);
  const cfloat3 v0 = (WW <= 0.0f) ? va : vc;
  const cfloat3 v1 = (WW <= 0.0f) ? vb : vd;
  const cfloat3 v2 = (WW <= 0.0f) ? vd : vb;

  const cfloat3 e0 = sub3(v2, v0);
  const cfloat3 e1 = sub3(v0, v1);

  const float U = dot3(cross3(v0, e0), D);
  const float V = dot3(cross3(v1, e1), D);
  if (!(cmax(U, V) <= 0.0f)) {
    return false;
  }

  const cfloat3 Ng = cross3(e1, e0);
  const float den = dot3(Ng, D);
  const float rcpDen = 1.0f / den;

  const float t = rcpDen * dot3(v0, Ng);
  if (!(0.0f <= t && t <= ray_tfar)) {
    return false;
  }
  if (!(den != 0.0f)) {
    return false;
  }

  *t_o = t;
  *u_o = U * rcpDen;
  *v_o = V * rcpDen;
  *u_o = (WW <= 0.0f) ? *u_o : 1.0f - *u_o;
  *v_o = (WW <= 0.0f) ? *v_o : 1.0f - *v_o;
  return true;
}

CY_FN cy_c4 ribbon_to_ray_space(const cfloat3 ray_space[3], cfloat3 ray_org, cy_c4 P4)
{
  const cfloat3 P = sub3(c4_xyz(P4), ray_org);
  return c4(dot3(ray_space[0], P), dot3(ray_space[1], P), dot3(ray_space[2], P), P4.w);
}

/* ribbon_intersect (geom_curve_intersect.h:568-642) returns the hit of the
 * first subdivision step (in curve parameter order) whose quad the ray hits
 * within tfar -- not the nearest one -- so a ribbon crossed twice gives a
 * result that depends on the tfar it is tested with.  SCAN = false is the
 * reference's form (stops at that first hit).  SCAN = true (the wide BVH,
 * cy_bvhw.h) tests every step: returns the number of steps hit (capped at 2),
 * the first one's hit and the nearest distance of all of them, so the traversal can tell a
 * ribbon whose result is the same for every tfar (at most one step hit) from
 * one that needs the reference's visiting order. */
template<bool SCAN>
CY_FN int ribbon_intersect_steps(cfloat3 ray_org, cfloat3 ray_dir, int N, cy_c4 curve[4], float tfar, float *t_o,
                                 float *u_o, float *v_o, float *t_min)
{
  /* Transform control points into ray space. */
  cfloat3 ray_space[3];
  {
    const cfloat3 dx0 = mk3(0.0f, ray_dir.z, -ray_dir.y);
    const cfloat3 dx1 = mk3(-ray_dir.z, 0.0f, ray_dir.x);
    ray_space[0] = normalize3(dot3(dx0, dx0) > dot3(dx1, dx1) ? dx0 : dx1);
    ray_space[1] = normalize3(cross3(ray_dir, ray_space[0]));
    ray_space[2] = ray_dir;
  }
  curve[0] = ribbon_to_ray_space(ray_space, ray_org, curve[0]);
  curve[1] = ribbon_to_ray_space(ray_space, ray_org, curve[1]);
  curve[2] = ribbon_to_ray_space(ray_space, ray_org, curve[2]);
  curve[3] = ribbon_to_ray_space(ray_space, ray_org, curve[3]);

  const cy_c4 mx = c4_max(c4_max(c4_fabs(curve[0]), c4_fabs(curve[1])), c4_max(c4_fabs(curve[2]), c4_fabs(curve[3])));
  const float eps = 4.0f * CY_FLT_EPSILON * cmax(cmax(mx.x, mx.y), cmax(mx.z, mx.w));
  const float step_size = 1.0f / (float)N;

  /* Evaluate first point and radius scaled normal direction. */
  cy_c4 p0 = catmull_rom_basis_eval(curve, 0.0f);
  cfloat3 dp0dt = c4_xyz(catmull_rom_basis_derivative(curve, 0.0f));
  if (max3f(fabs3(dp0dt)) < eps) {
    const cy_c4 p1 = catmull_rom_basis_eval(curve, step_size);
    dp0dt = c4_xyz(c4_sub(p1, p0));
  }
  cfloat3 wn0 = mul3f(normalize3(mk3(dp0dt.y, -dp0dt.x, 0.0f)), p0.w);

  int count = 0;
  /* Evaluate the bezier curve. */
  for (int i = 0; i < N; i++) {
    const float u = i * step_size;
    const cy_c4 p1 = catmull_rom_basis_eval(curve, u + step_size);
    const bool valid = cylinder_culling_test(p0.x, p0.y, p1.x, p1.y, cmax(p0.w, p1.w));
    if (!valid) {
      /* (the reference keeps p0 / wn0 of the culled step) */
      continue;
    }

    /* Evaluate next point. */
    cfloat3 dp1dt = c4_xyz(catmull_rom_basis_derivative(curve, u + step_size));
    dp1dt = (max3f(fabs3(dp1dt)) < eps) ? c4_xyz(c4_sub(p1, p0)) : dp1dt;
    const cfloat3 wn1 = mul3f(normalize3(mk3(dp1dt.y, -dp1dt.x, 0.0f)), p1.w);

    /* Construct quad coordinates. */
    const cfloat3 lp0 = add3(c4_xyz(p0), wn0);
    const cfloat3 lp1 = add3(c4_xyz(p1), wn1);
    const cfloat3 up0 = sub3(c4_xyz(p0), wn0);
    const cfloat3 up1 = sub3(c4_xyz(p1), wn1);

    /* Intersect quad. */
    float vu, vv, vt;
    bool valid0 = ribbon_intersect_quad(tfar, lp0, lp1, up1, up0, &vu, &vv, &vt);

    if (valid0) {
      /* ignore self intersections */
      const float avoidance_factor = 2.0f;
      const float r = cmix(p0.w, p1.w, vu);
      valid0 = vt > avoidance_factor * r;

      if (valid0) {
        if (count == 0) {
          vv = 2.0f * vv - 1.0f;
          *t_o = vt;
          *u_o = u + vu * step_size;
          *v_o = vv;
          *t_min = vt;
        }
        else {
          *t_min = cmin(*t_min, vt);
        }
        count = count < 2 ? count + 1 : 2;
        if (!SCAN) {
          return count;
        }
      }
    }

    p0 = p1;
    wn0 = wn1;
  }
  return count;
}

CY_FN bool ribbon_intersect(cfloat3 ray_org, cfloat3 ray_dir, int N, cy_c4 curve[4], CyIsect *isect)
{
  float t, u, v, tmin;
  if (ribbon_intersect_steps<false>(ray_org, ray_dir, N, curve, isect->t, &t, &u, &v, &tmin)) {
    isect->t = t;
    isect->u = u;
    isect->v = v;
    return true;
  }
  return false;
}

/* The four keys of a curve segment (ka, k0, k1, kb clamped to the curve). */
CY_FN void curve_segment_keys(const CyGlobals *kg, int prim, int segment, cy_c4 curve[4])
{
  const hc_float4 v00 = kg->__curves[prim];
  const int first = as_int(v00.x);
  const int k0 = first + segment;
  const int k1 = k0 + 1;
  const int ka = imax(k0 - 1, first);
  const int kb = imin(k1 + 1, first + as_int(v00.y) - 1);
  curve[0] = c4_load(kg->__curve_keys[ka]);
  curve[1] = c4_load(kg->__curve_keys[k0]);
  curve[2] = c4_load(kg->__curve_keys[k1]);
  curve[3] = c4_load(kg->__curve_keys[kb]);
}

/* curve_intersect (:620-692), static curves: the segment of primitive slot
 * curveAddr against the ray (P, dir in the space of its BVH).  SHAPES selects
 * the intersectors compiled in (bit 0 ribbon, bit 1 thick): the thick one
 * alone sizes a traversal kernel's registers (an any-hit kernel with both
 * needs 188 VGPRs, with ribbons only 128), so kernels are instantiated for
 * the shapes a scene holds (hipcycles.hip curve_shapes). */
template<int SHAPES = 3>
CY_FN bool curve_intersect(const CyGlobals *kg, CyIsect *isect, cfloat3 P, cfloat3 dir, uint visibility, int object,
                           int curveAddr, uint type)
{
  const int segment = (int)CY_PRIMITIVE_UNPACK_SEGMENT(type);
  const int prim = (int)kg->__prim_index[curveAddr];
  cy_c4 curve[4];
  curve_segment_keys(kg, prim, segment, curve);
  if (!(kg->__prim_visibility[curveAddr] & visibility)) {
    return false;
  }
  if (type & (CY_PRIMITIVE_CURVE_RIBBON | CY_PRIMITIVE_MOTION_CURVE_RIBBON)) {
    if (!(SHAPES & 1)) {
      return false;
    }
    const int subdivisions = KD->bvh.curve_subdivisions;
    if (ribbon_intersect(P, dir, subdivisions, curve, isect)) {
      isect->prim = curveAddr;
      isect->object = object;
      isect->type = (int)type;
      return true;
    }
    return false;
  }
  if ((SHAPES & 2) && curve_intersect_recursive(P, dir, curve, isect)) {
    isect->prim = curveAddr;
    isect->object = object;
    isect->type = (int)type;
    return true;
  }
  return false;
}

/* curve_shader_setup (:694-794): hit point, shading and geometric normal,
 * u / v, dPdu / dPdv (object space here, transformed with the normals by
 * shader_setup_from_ray) and the curve's shader.  sd->prim is already
 * __prim_index[isect->prim]. */
CY_FN void curve_shader_setup(const CyGlobals *kg, CySD *sd, const CyIsect *isect, const CyRay *ray)
{
  float t = isect->t;
  cfloat3 P = ray->P;
  cfloat3 D = ray->D;
  if (isect->object != OBJECT_NONE) {
    const struct cy_tfm *tfm = object_itfm(kg, isect->object);
    P = transform_point(tfm, P);
    D = transform_direction(tfm, mul3f(D, t));
    D = normalize_len3(D, &t);
  }
  cy_c4 P_curve[4];
  curve_segment_keys(kg, sd->prim, (int)CY_PRIMITIVE_UNPACK_SEGMENT((uint)sd->type), P_curve);
  sd->u = isect->u;
  P = add3(P, mul3f(D, t));
  const cy_c4 dPdu4 = catmull_rom_basis_derivative(P_curve, isect->u);
  const cfloat3 dPdu = c4_xyz(dPdu4);
  if (sd->type & (CY_PRIMITIVE_CURVE_RIBBON | CY_PRIMITIVE_MOTION_CURVE_RIBBON)) {
    /* Rounded smooth normals for ribbons, to approximate thick curve shape. */
    const cfloat3 tangent = normalize3(dPdu);
    const cfloat3 bitangent = normalize3(cross3(tangent, neg3(D)));
    const float sine = isect->v;
    const float cosine = safe_sqrtf(1.0f - sine * sine);
    sd->N = normalize3(sub3(mul3f(bitangent, sine), mul3f(normalize3(cross3(tangent, bitangent)), cosine)));
    sd->Ng = neg3(D);
    sd->v = isect->v;
  }
  else {
    /* Thick curves: normal from the curve's centre line to the hit. */
    const cfloat3 P_inside = c4_xyz(catmull_rom_basis_eval(P_curve, isect->u));
    const cfloat3 Ng = normalize3(sub3(P, P_inside));
    sd->N = Ng;
    sd->Ng = Ng;
    sd->v = 0.0f;
  }
#if CY_CLOSURE_EXT
  sd->dPdu = dPdu;
  sd->dPdv = cross3(dPdu, sd->Ng);
#endif
  if (isect->object != OBJECT_NONE) {
    P = transform_point(object_tfm(kg, isect->object), P);
  }
  sd->P = P;
  sd->shader = as_int(kg->__curves[sd->prim].z);
}

#endif /* CY_CURVE_H */
