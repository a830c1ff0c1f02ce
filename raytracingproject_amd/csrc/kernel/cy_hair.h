/*
 * cy_hair.h — hair closures, in the reference CPU kernel's scalar arithmetic.
 *
 *   Hair BSDF node (reflection / transmission)   closure/bsdf_hair.h:38-313
 *   Principled Hair BSDF (Chiang et al. 2016)    closure/bsdf_hair_principled.h:28-527
 *
 * Closure storage (CyClosure, set up in cy_path.h svm_node_closure_bsdf):
 *   hair reflection / transmission: T tangent, alpha_x roughness1, alpha_y
 *     roughness2, ior offset;
 *   principled hair: T sigma (absorption), alpha_x v, alpha_y s, ior eta; its
 *     extra slot (PrincipledHairExtra, closure_alloc_extra) keeps geom.xyz in
 *     weight, geom.w in alpha_x, the cuticle tilt alpha in alpha_y, the
 *     primary-reflection roughness m0 in ior, and film.rgb_to_y in T (the
 *     energy weights of hair_attenuation; evaluation has no KernelGlobals).
 * libm calls go through the glibc restatements of cy_math.h (tanf, sinhf,
 * expf, logf, sinf, cosf, asinf, atan2f); fast_* are util_math_fast.h's.
 */
#ifndef CY_HAIR_H
#define CY_HAIR_H

#if CY_CLOSURE_EXT

/* util_math_fast.h:131-153 */
CY_FN float fast_cosf(float x)
{
  int q = fast_rint(x * CY_1_PI_F);
  float qf = (float)q;
  x = madd(qf, -0.78515625f * 4, x);
  x = madd(qf, -0.00024187564849853515625f * 4, x);
  x = madd(qf, -3.7747668102383613586e-08f * 4, x);
  x = madd(qf, -1.2816720341285448015e-12f * 4, x);
  x = CY_PI_2_F - (CY_PI_2_F - x);
  float s = x * x;
  float u = -2.71811842367242206819355e-07f;
  u = madd(u, s, +2.47990446951007470488548e-05f);
  u = madd(u, s, -0.00138888787478208541870117f);
  u = madd(u, s, +0.0416666641831398010253906f);
  u = madd(u, s, -0.5f);
  u = madd(u, s, +1.0f);
  if ((q & 1) != 0) {
    u = -u;
  }
  if (fabsf(u) > 1.0f) {
    u = 0.0f;
  }
  return u;
}

/* util_math_fast.h:329-356 */
CY_FN float fast_atan2f(float y, float x)
{
  const float a = fabsf(x);
  const float b = fabsf(y);
  const float k = (b == 0) ? 0.0f : ((a == b) ? 1.0f : (b > a ? a / b : b / a));
  const float s = 1.0f - (1.0f - k);
  const float t = s * s;
  float r = s * madd(0.43157974f, t, 1.0f) / madd(madd(0.05831938f, t, 0.76443945f), t, 1.0f);
  if (b > a) {
    r = CY_PI_2_F - r;
  }
  if (as_uint(x) & 0x80000000u) {
    r = CY_PI_F - r;
  }
  return copysignf(r, y);
}

CY_FN float hair_safe_asinf(float a)
{
  return cy_asinf(cclamp(a, -1.0f, 1.0f));
}

/* ---------------------------------------------------------------------------
 * Hair BSDF node */

CY_FN int bsdf_hair_setup(CyClosure *sc, int type)
{
  sc->type = type;
  sc->alpha_x = cclamp(sc->alpha_x, 0.001f, 1.0f);
  sc->alpha_y = cclamp(sc->alpha_y, 0.001f, 1.0f);
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

CY_FN cfloat3 bsdf_hair_reflection_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  const float offset = sc->ior;
  const cfloat3 Tg = sc->T;
  const float roughness1 = sc->alpha_x;
  const float roughness2 = sc->alpha_y;
  const float Iz = dot3(Tg, I);
  const cfloat3 locy = normalize3(sub3(I, mul3f(Tg, Iz)));
  const float theta_r = CY_PI_2_F - fast_acosf(Iz);
  const float omega_in_z = dot3(Tg, omega_in);
  const cfloat3 omega_in_y = normalize3(sub3(omega_in, mul3f(Tg, omega_in_z)));
  const float theta_i = CY_PI_2_F - fast_acosf(omega_in_z);
  const float cosphi_i = dot3(omega_in_y, locy);
  if (CY_PI_2_F - fabsf(theta_i) < 0.001f || cosphi_i < 0.0f) {
    *pdf = 0.0f;
    return mk3(*pdf, *pdf, *pdf);
  }
  const float roughness1_inv = 1.0f / roughness1;
  const float roughness2_inv = 1.0f / roughness2;
  float phi_i = fast_acosf(cosphi_i) * roughness2_inv;
  phi_i = fabsf(phi_i) < CY_PI_F ? phi_i : CY_PI_F;
  const float costheta_i = fast_cosf(theta_i);
  const float a_R = fast_atan2f(((CY_PI_2_F + theta_r) * 0.5f - offset) * roughness1_inv, 1.0f);
  const float b_R = fast_atan2f(((-CY_PI_2_F + theta_r) * 0.5f - offset) * roughness1_inv, 1.0f);
  const float theta_h = (theta_i + theta_r) * 0.5f;
  const float t = theta_h - offset;
  const float phi_pdf = fast_cosf(phi_i * 0.5f) * 0.25f * roughness2_inv;
  const float theta_pdf = roughness1 / (2.0f * (t * t + roughness1 * roughness1) * (a_R - b_R) * costheta_i);
  *pdf = phi_pdf * theta_pdf;
  return mk3(*pdf, *pdf, *pdf);
}

CY_FN cfloat3 bsdf_hair_transmission_eval_transmit(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  const float offset = sc->ior;
  const cfloat3 Tg = sc->T;
  const float roughness1 = sc->alpha_x;
  const float roughness2 = sc->alpha_y;
  const float Iz = dot3(Tg, I);
  const cfloat3 locy = normalize3(sub3(I, mul3f(Tg, Iz)));
  const float theta_r = CY_PI_2_F - fast_acosf(Iz);
  const float omega_in_z = dot3(Tg, omega_in);
  const cfloat3 omega_in_y = normalize3(sub3(omega_in, mul3f(Tg, omega_in_z)));
  const float theta_i = CY_PI_2_F - fast_acosf(omega_in_z);
  const float phi_i = fast_acosf(dot3(omega_in_y, locy));
  if (CY_PI_2_F - fabsf(theta_i) < 0.001f) {
    *pdf = 0.0f;
    return mk3(*pdf, *pdf, *pdf);
  }
  const float costheta_i = fast_cosf(theta_i);
  const float roughness1_inv = 1.0f / roughness1;
  const float a_TT = fast_atan2f(((CY_PI_2_F + theta_r) / 2.0f - offset) * roughness1_inv, 1.0f);
  const float b_TT = fast_atan2f(((-CY_PI_2_F + theta_r) / 2.0f - offset) * roughness1_inv, 1.0f);
  const float c_TT = 2.0f * fast_atan2f(CY_PI_2_F / roughness2, 1.0f);
  const float theta_h = (theta_i + theta_r) / 2.0f;
  const float t = theta_h - offset;
  const float phi = fabsf(phi_i);
  const float p = CY_PI_F - phi;
  const float theta_pdf = roughness1 / (2.0f * (t * t + roughness1 * roughness1) * (a_TT - b_TT) * costheta_i);
  const float phi_pdf = roughness2 / (c_TT * (p * p + roughness2 * roughness2));
  *pdf = phi_pdf * theta_pdf;
  return mk3(*pdf, *pdf, *pdf);
}

/* bsdf_hair_reflection_sample / bsdf_hair_transmission_sample */
CY_FN int bsdf_hair_sample(const CyClosure *sc, cfloat3 I, float randu, float randv, cfloat3 *eval,
                           cfloat3 *omega_in, float *pdf)
{
  const bool reflect = sc->type == CLOSURE_BSDF_HAIR_REFLECTION_ID;
  const float offset = sc->ior;
  const cfloat3 Tg = sc->T;
  const float roughness1 = sc->alpha_x;
  const float roughness2 = sc->alpha_y;
  const float Iz = dot3(Tg, I);
  const cfloat3 locy = normalize3(sub3(I, mul3f(Tg, Iz)));
  const cfloat3 locx = cross3(locy, Tg);
  const float theta_r = CY_PI_2_F - fast_acosf(Iz);
  const float roughness1_inv = 1.0f / roughness1;
  float a, b;
  if (reflect) {
    a = fast_atan2f(((CY_PI_2_F + theta_r) * 0.5f - offset) * roughness1_inv, 1.0f);
    b = fast_atan2f(((-CY_PI_2_F + theta_r) * 0.5f - offset) * roughness1_inv, 1.0f);
  }
  else {
    a = fast_atan2f(((CY_PI_2_F + theta_r) / 2.0f - offset) * roughness1_inv, 1.0f);
    b = fast_atan2f(((-CY_PI_2_F + theta_r) / 2.0f - offset) * roughness1_inv, 1.0f);
  }
  const float t = roughness1 * cy_tanf(randu * (a - b) + b);
  const float theta_h = t + offset;
  const float theta_i = 2.0f * theta_h - theta_r;
  float costheta_i, sintheta_i;
  fast_sincosf(theta_i, &sintheta_i, &costheta_i);
  float phi, phi_pdf;
  if (reflect) {
    phi = 2.0f * hair_safe_asinf(1.0f - 2.0f * randv) * roughness2;
    phi_pdf = fast_cosf(phi * 0.5f) * 0.25f / roughness2;
  }
  else {
    const float c_TT = 2.0f * fast_atan2f(CY_PI_2_F / roughness2, 1.0f);
    const float p = roughness2 * cy_tanf(c_TT * (randv - 0.5f));
    phi = p + CY_PI_F;
    phi_pdf = roughness2 / (c_TT * (p * p + roughness2 * roughness2));
  }
  const float theta_pdf = roughness1 / (2.0f * (t * t + roughness1 * roughness1) * (a - b) * costheta_i);
  float sinphi, cosphi;
  fast_sincosf(phi, &sinphi, &cosphi);
  *omega_in = add3(sub3(mul3f(locy, cosphi * costheta_i), mul3f(locx, sinphi * costheta_i)), mul3f(Tg, sintheta_i));
  *pdf = fabsf(phi_pdf * theta_pdf);
  if (CY_PI_2_F - fabsf(theta_i) < 0.001f) {
    *pdf = 0.0f;
  }
  *eval = mk3(*pdf, *pdf, *pdf);
  return reflect ? (LABEL_REFLECT | LABEL_GLOSSY) : (LABEL_TRANSMIT | LABEL_GLOSSY);
}

/* ---------------------------------------------------------------------------
 * Principled Hair BSDF */

CY_FN float cos_from_sin(float s)
{
  return safe_sqrtf(1.0f - s * s);
}

CY_FN float hair_delta_phi(int p, float gamma_o, float gamma_t)
{
  return 2.0f * (float)p * gamma_t - 2.0f * gamma_o + (float)p * CY_PI_F;
}

CY_FN float hair_wrap_angle(float a)
{
  while (a > CY_PI_F) {
    a -= CY_2PI_F;
  }
  while (a < -CY_PI_F) {
    a += CY_2PI_F;
  }
  return a;
}

CY_FN float hair_logistic(float x, float s)
{
  const float v = cy_expf(-fabsf(x) / s);
  return v / (s * sqr(1.0f + v));
}

CY_FN float hair_logistic_cdf(float x, float s)
{
  const float arg = -x / s;
  if (arg > 88.0f) {
    return 0.0f;
  }
  return 1.0f / (1.0f + cy_expf(arg));
}

/* numerical approximation of the modified Bessel function I0 */
CY_FN float bessel_I0(float x)
{
  x = sqr(x);
  float val = 1.0f + 0.25f * x;
  float pow_x_2i = sqr(x);
  uint64_t i_fac_2 = 1;
  int pow_4_i = 16;
  for (int i = 2; i < 10; i++) {
    i_fac_2 *= (uint64_t)(i * i);
    const float newval = val + pow_x_2i / (float)((uint64_t)pow_4_i * i_fac_2);
    if (val == newval) {
      return val;
    }
    val = newval;
    pow_x_2i *= x;
    pow_4_i *= 4;
  }
  return val;
}

CY_FN float log_bessel_I0(float x)
{
  if (x > 12.0f) {
    return x + 0.5f * (1.f / (8.0f * x) - 1.8378770664093454f - cy_logf(x));
  }
  return cy_logf(bessel_I0(x));
}

CY_FN float trimmed_logistic(float x, float s)
{
  const float scaling_fac = 1.0f - 2.0f * hair_logistic_cdf(-CY_PI_F, s);
  const float val = hair_logistic(x, s);
  return safe_divide(val, scaling_fac);
}

CY_FN float sample_trimmed_logistic(float u, float s)
{
  const float cdf_minuspi = hair_logistic_cdf(-CY_PI_F, s);
  const float x = -s * cy_logf(1.0f / (u * (1.0f - 2.0f * cdf_minuspi) + cdf_minuspi) - 1.0f);
  return cclamp(x, -CY_PI_F, CY_PI_F);
}

CY_FN float azimuthal_scattering(float phi, int p, float s, float gamma_o, float gamma_t)
{
  const float phi_o = hair_wrap_angle(phi - hair_delta_phi(p, gamma_o, gamma_t));
  return trimmed_logistic(phi_o, s);
}

CY_FN float longitudinal_scattering(float sin_theta_i, float cos_theta_i, float sin_theta_o, float cos_theta_o,
                                    float v)
{
  const float inv_v = 1.0f / v;
  const float cos_arg = cos_theta_i * cos_theta_o * inv_v;
  const float sin_arg = sin_theta_i * sin_theta_o * inv_v;
  if (v <= 0.1f) {
    const float i0 = log_bessel_I0(cos_arg);
    return cy_expf(i0 - sin_arg - inv_v + 0.6931f + cy_logf(0.5f * inv_v));
  }
  const float i0 = bessel_I0(cos_arg);
  return (cy_expf(-sin_arg) * i0) / (cy_sinhf(inv_v) * 2.0f * v);
}

struct CyHairF4 {
  float x, y, z, w;
};

CY_FN CyHairF4 hair_combine_with_energy(cfloat3 c, cfloat3 rgb_to_y)
{
  CyHairF4 r = {c.x, c.y, c.z, dot3(c, rgb_to_y)};
  return r;
}

/* hair_attenuation: the attenuation of each bounce from the Fresnel term and
 * the transmittance, with luminance sampling weights */
CY_FN void hair_attenuation(float f, cfloat3 T, cfloat3 rgb_to_y, CyHairF4 *Ap)
{
  Ap[0].x = Ap[0].y = Ap[0].z = Ap[0].w = f;
  cfloat3 col = mul3f(T, sqr(1.0f - f));
  Ap[1] = hair_combine_with_energy(col, rgb_to_y);
  col = mul3(col, mul3f(T, f));
  Ap[2] = hair_combine_with_energy(col, rgb_to_y);
  const cfloat3 Tf = mul3f(T, f);
  col = mul3(col, safe_divide_color(Tf, sub3(mk3(1.0f, 1.0f, 1.0f), Tf)));
  Ap[3] = hair_combine_with_energy(col, rgb_to_y);
  const float totweight = Ap[0].w + Ap[1].w + Ap[2].w + Ap[3].w;
  const float fac = safe_divide(1.0f, totweight);
  Ap[0].w *= fac;
  Ap[1].w *= fac;
  Ap[2].w *= fac;
  Ap[3].w *= fac;
}

CY_FN void hair_alpha_angles(float sin_theta_i, float cos_theta_i, float alpha, float *angles)
{
  const float sin_1alpha = cy_sinf(alpha);
  const float cos_1alpha = cos_from_sin(sin_1alpha);
  const float sin_2alpha = 2.0f * sin_1alpha * cos_1alpha;
  const float cos_2alpha = sqr(cos_1alpha) - sqr(sin_1alpha);
  const float sin_4alpha = 2.0f * sin_2alpha * cos_2alpha;
  const float cos_4alpha = sqr(cos_2alpha) - sqr(sin_2alpha);
  angles[0] = sin_theta_i * cos_2alpha + cos_theta_i * sin_2alpha;
  angles[1] = fabsf(cos_theta_i * cos_2alpha - sin_theta_i * sin_2alpha);
  angles[2] = sin_theta_i * cos_1alpha - cos_theta_i * sin_1alpha;
  angles[3] = fabsf(cos_theta_i * cos_1alpha + sin_theta_i * sin_1alpha);
  angles[4] = sin_theta_i * cos_4alpha - cos_theta_i * sin_4alpha;
  angles[5] = fabsf(cos_theta_i * cos_4alpha + sin_theta_i * sin_4alpha);
}

CY_FN float hair_pow20(float a)
{
  return sqr(sqr(sqr(sqr(a)) * a));
}
CY_FN float hair_pow22(float a)
{
  return sqr(a * sqr(sqr(sqr(a)) * a));
}

/* bsdf_principled_hair_setup (bsdf_hair_principled.h:191-229): clamps and
 * maps the roughnesses, and records the local frame's Y and the offset h
 * across the fiber in the extra slot */
CY_FN int bsdf_principled_hair_setup(const CySD *sd, CyClosure *b, CyClosure *extra)
{
  b->type = CLOSURE_BSDF_HAIR_PRINCIPLED_ID;
  float v = cclamp(b->alpha_x, 0.001f, 1.0f);
  float s = cclamp(b->alpha_y, 0.001f, 1.0f);
  float m0 = cclamp(extra->ior * v, 0.001f, 1.0f);
  v = sqr(0.726f * v + 0.812f * sqr(v) + 3.700f * hair_pow20(v));
  s = (0.265f * s + 1.194f * sqr(s) + 5.372f * hair_pow22(s)) * 0.6266570686577501f; /* M_SQRT_PI_8_F */
  m0 = sqr(0.726f * m0 + 0.812f * sqr(m0) + 3.700f * hair_pow20(m0));
  b->alpha_x = v;
  b->alpha_y = s;
  extra->ior = m0;
  const cfloat3 X = safe_normalize3(sd->dPdu);
  const cfloat3 Y = safe_normalize3(cross3(X, sd->I));
  const cfloat3 Z = safe_normalize3(cross3(X, Y));
  const float h = (sd->type & (CY_PRIMITIVE_CURVE_RIBBON | CY_PRIMITIVE_MOTION_CURVE_RIBBON)) ?
                      -sd->v :
                      dot3(cross3(sd->Ng, X), Z);
  extra->weight = Y;
  extra->alpha_x = h;
  return SD_BSDF | SD_BSDF_HAS_EVAL | SD_BSDF_NEEDS_LCG;
}

/* the four lobes (R, TT, TRT, TRRT+) of bsdf_principled_hair_eval / _sample */
CY_FN CyHairF4 hair_lobes(const CyClosure *b, const CyClosure *ex, const CyHairF4 *Ap, float sin_theta_i,
                          float cos_theta_i, float sin_theta_o, float cos_theta_o, float phi, float gamma_o,
                          float gamma_t)
{
  float angles[6];
  hair_alpha_angles(sin_theta_i, cos_theta_i, ex->alpha_y, angles);
  CyHairF4 F;
  float Mp = longitudinal_scattering(angles[0], angles[1], sin_theta_o, cos_theta_o, ex->ior);
  float Np = azimuthal_scattering(phi, 0, b->alpha_y, gamma_o, gamma_t);
  F.x = Ap[0].x * Mp * Np;
  F.y = Ap[0].y * Mp * Np;
  F.z = Ap[0].z * Mp * Np;
  F.w = Ap[0].w * Mp * Np;
  Mp = longitudinal_scattering(angles[2], angles[3], sin_theta_o, cos_theta_o, 0.25f * b->alpha_x);
  Np = azimuthal_scattering(phi, 1, b->alpha_y, gamma_o, gamma_t);
  F.x += Ap[1].x * Mp * Np;
  F.y += Ap[1].y * Mp * Np;
  F.z += Ap[1].z * Mp * Np;
  F.w += Ap[1].w * Mp * Np;
  Mp = longitudinal_scattering(angles[4], angles[5], sin_theta_o, cos_theta_o, 4.0f * b->alpha_x);
  Np = azimuthal_scattering(phi, 2, b->alpha_y, gamma_o, gamma_t);
  F.x += Ap[2].x * Mp * Np;
  F.y += Ap[2].y * Mp * Np;
  F.z += Ap[2].z * Mp * Np;
  F.w += Ap[2].w * Mp * Np;
  Mp = longitudinal_scattering(sin_theta_i, cos_theta_i, sin_theta_o, cos_theta_o, 4.0f * b->alpha_x);
  Np = 0.1591549430918953f; /* M_1_2PI_F */
  F.x += Ap[3].x * Mp * Np;
  F.y += Ap[3].y * Mp * Np;
  F.z += Ap[3].z * Mp * Np;
  F.w += Ap[3].w * Mp * Np;
  return F;
}

/* the geometry shared by evaluation and sampling */
struct CyHairFrame {
  cfloat3 X, Y, Z;
  float sin_theta_o, cos_theta_o, phi_o, gamma_o, gamma_t;
  CyHairF4 Ap[4];
};

CY_FN void hair_frame(const CySD *sd, const CyClosure *b, const CyClosure *ex, CyHairFrame *f)
{
  f->Y = ex->weight;
  f->X = safe_normalize3(sd->dPdu);
  f->Z = safe_normalize3(cross3(f->X, f->Y));
  const cfloat3 wo = mk3(dot3(sd->I, f->X), dot3(sd->I, f->Y), dot3(sd->I, f->Z));
  f->sin_theta_o = wo.x;
  f->cos_theta_o = cos_from_sin(f->sin_theta_o);
  f->phi_o = cy_atan2f(wo.z, wo.y);
  const float eta = b->ior;
  const float sin_theta_t = f->sin_theta_o / eta;
  const float cos_theta_t = cos_from_sin(sin_theta_t);
  const float sin_gamma_o = ex->alpha_x;
  const float cos_gamma_o = cos_from_sin(sin_gamma_o);
  f->gamma_o = hair_safe_asinf(sin_gamma_o);
  const float sin_gamma_t = sin_gamma_o * f->cos_theta_o / sqrtf(sqr(eta) - sqr(f->sin_theta_o));
  const float cos_gamma_t = cos_from_sin(sin_gamma_t);
  f->gamma_t = hair_safe_asinf(sin_gamma_t);
  const cfloat3 a = mul3f(neg3(b->T), 2.0f * cos_gamma_t / cos_theta_t);
  const cfloat3 T = mk3(cy_expf(a.x), cy_expf(a.y), cy_expf(a.z));
  hair_attenuation(fresnel_dielectric_cos(f->cos_theta_o * cos_gamma_o, eta), T, ex->T, f->Ap);
}

CY_FN cfloat3 bsdf_principled_hair_eval(const CySD *sd, const CyClosure *b, cfloat3 omega_in, float *pdf)
{
  const CyClosure *ex = &sd->closure[b->extra];
  CyHairFrame f;
  hair_frame(sd, b, ex, &f);
  const cfloat3 wi = mk3(dot3(omega_in, f.X), dot3(omega_in, f.Y), dot3(omega_in, f.Z));
  const float sin_theta_i = wi.x;
  const float cos_theta_i = cos_from_sin(sin_theta_i);
  const float phi_i = cy_atan2f(wi.z, wi.y);
  const float phi = phi_i - f.phi_o;
  const CyHairF4 F = hair_lobes(b, ex, f.Ap, sin_theta_i, cos_theta_i, f.sin_theta_o, f.cos_theta_o, phi, f.gamma_o,
                                f.gamma_t);
  *pdf = F.w;
  return mk3(F.x, F.y, F.z);
}

CY_FN int bsdf_principled_hair_sample(const CySD *sd, const CyClosure *b, float randu, float randv, cfloat3 *eval,
                                      cfloat3 *omega_in, float *pdf)
{
  const CyClosure *ex = &sd->closure[b->extra];
  CyHairFrame f;
  hair_frame(sd, b, ex, &f);
  float u0x = randu, u0y = randv;
  float u1x = lcg_step_float(&sd->lcg_state);
  const float u1y = lcg_step_float(&sd->lcg_state);
  int p = 0;
  for (; p < 3; p++) {
    if (u0x < f.Ap[p].w) {
      break;
    }
    u0x -= f.Ap[p].w;
  }
  float v = b->alpha_x;
  if (p == 1) {
    v *= 0.25f;
  }
  if (p >= 2) {
    v *= 4.0f;
  }
  u1x = (u1x > 1e-5f) ? u1x : 1e-5f; /* max() */
  const float fac = 1.0f + v * cy_logf(u1x + (1.0f - u1x) * cy_expf(-2.0f / v));
  float sin_theta_i = -fac * f.sin_theta_o + cos_from_sin(fac) * cy_cosf(CY_2PI_F * u1y) * f.cos_theta_o;
  float cos_theta_i = cos_from_sin(sin_theta_i);
  if (p < 3) {
    float angles[6];
    hair_alpha_angles(sin_theta_i, cos_theta_i, -ex->alpha_y, angles);
    sin_theta_i = angles[2 * p];
    cos_theta_i = angles[2 * p + 1];
  }
  float phi;
  if (p < 3) {
    phi = hair_delta_phi(p, f.gamma_o, f.gamma_t) + sample_trimmed_logistic(u0y, b->alpha_y);
  }
  else {
    phi = CY_2PI_F * u0y;
  }
  const float phi_i = f.phi_o + phi;
  const CyHairF4 F = hair_lobes(b, ex, f.Ap, sin_theta_i, cos_theta_i, f.sin_theta_o, f.cos_theta_o, phi, f.gamma_o,
                                f.gamma_t);
  *eval = mk3(F.x, F.y, F.z);
  *pdf = F.w;
  *omega_in = add3(add3(mul3f(f.X, sin_theta_i), mul3f(mul3f(f.Y, cos_theta_i), cy_cosf(phi_i))),
                   mul3f(mul3f(f.Z, cos_theta_i), cy_sinf(phi_i)));
  return LABEL_GLOSSY | ((p == 0) ? LABEL_REFLECT : LABEL_TRANSMIT);
}

/* bsdf_principled_hair_blur (Filter Glossy) */
CY_FN void bsdf_principled_hair_blur(CySD *sd, CyClosure *b, float roughness)
{
  CyClosure *ex = &sd->closure[b->extra];
  b->alpha_x = fmaxf(roughness, b->alpha_x);
  b->alpha_y = fmaxf(roughness, b->alpha_y);
  ex->ior = fmaxf(roughness, ex->ior);
}

/* bsdf_hair_principled.h:490-520 */
CY_FN float bsdf_principled_hair_albedo_roughness_scale(const float azimuthal_roughness)
{
  const float x = azimuthal_roughness;
  return (((((0.245f * x) + 5.574f) * x - 10.73f) * x + 2.532f) * x - 0.215f) * x + 5.969f;
}

CY_FN cfloat3 bsdf_principled_hair_sigma_from_reflectance(const cfloat3 color, const float azimuthal_roughness)
{
  const cfloat3 lc = mk3(cy_logf(color.x), cy_logf(color.y), cy_logf(color.z));
  const cfloat3 sigma = div3f(lc, bsdf_principled_hair_albedo_roughness_scale(azimuthal_roughness));
  return mul3(sigma, sigma);
}

CY_FN cfloat3 bsdf_principled_hair_sigma_from_concentration(const float eumelanin, const float pheomelanin)
{
  return add3(mul3f(mk3(0.506f, 0.841f, 1.653f), eumelanin), mul3f(mk3(0.343f, 0.733f, 1.924f), pheomelanin));
}

#endif /* CY_CLOSURE_EXT */
#endif /* CY_HAIR_H */
