/*
 * cy_microfacet_multi.h — multiple-scattering GGX, reflection (the Glossy /
 * Anisotropic BSDF "Multiscatter GGX" distribution and the specular layer of
 * the Principled BSDF): the single-scattering lobe evaluated analytically
 * plus a random walk over the microsurface's heights and normals, driven by
 * the shading point's LCG (sd->lcg_state, kernel_random.h lcg_*).
 *
 *   D_ggx / D_ggx_aniso, mf_sampleP22_11,
 *   mf_sample_vndf, phase functions, mf_lambda,
 *   heights, albedo / pdf approximations         closure/bsdf_microfacet_multi.h:22-318
 *   mf_eval_glossy / mf_sample_glossy            closure/bsdf_microfacet_multi_impl.h:28-274
 *                                                (MF_MULTI_GLOSSY instantiation)
 *   setups, eval_reflect, sample                 closure/bsdf_microfacet_multi.h:365-533
 *
 *   mf_sample_phase_glass / mf_eval_phase_glass,
 *   mf_ggx_transmission_albedo, mf_glass_pdf     closure/bsdf_microfacet_multi.h:138-190, 278-351
 *   mf_eval_glass / mf_sample_glass              closure/bsdf_microfacet_multi_impl.h
 *                                                (MF_MULTI_GLASS instantiation)
 *   glass setups, eval_reflect / _transmit,
 *   sample                                       closure/bsdf_microfacet_multi.h:537-731
 *
 * The glass instantiation (the Glass BSDF's multiscatter distribution and
 * the Principled BSDF's default rough transmission) evaluates the analytic
 * single-scattering transmission through beta() = expf(lgammaf(x) +
 * lgammaf(y) - lgammaf(x + y)) (util_math.h), with glibc's lgammaf restated
 * in cy_math.h (cy_lgammaf).
 *
 * Arithmetic follows the reference's scalar float3 operators (no SSE,
 * -ffp-contract=off): every product and sum in the reference's order.
 */
#ifndef CY_MICROFACET_MULTI_H
#define CY_MICROFACET_MULTI_H

/* kernel_random.h:287-292 lcg_step_float_addrspace */
CY_FN float lcg_step_float(uint *rng)
{
  *rng = 1103515245u * (*rng) + 12345u;
  return (float)*rng * (1.0f / 4294967296.0f);
}

/* kernel_random.h:171-176, 282-285 */
CY_FN uint lcg_init(uint seed)
{
  return 1103515245u * seed + 12345u;
}

/* bsdf_microfacet_multi.h:25-31 */
CY_FN float D_ggx(cfloat3 wm, float alpha)
{
  wm.z *= wm.z;
  alpha *= alpha;
  float tmp = (1.0f - wm.z) + alpha * wm.z;
  return alpha / cmax(CY_PI_F * tmp * tmp, 1e-7f);
}

/* bsdf_microfacet_multi.h:34-41 */
CY_FN float D_ggx_aniso(cfloat3 wm, float ax, float ay)
{
  float slope_x = -wm.x / ax;
  float slope_y = -wm.y / ay;
  float tmp = wm.z * wm.z + slope_x * slope_x + slope_y * slope_y;
  return 1.0f / cmax(CY_PI_F * tmp * tmp * ax * ay, 1e-7f);
}

/* bsdf_microfacet_multi.h:44-82 */
CY_FN void mf_sampleP22_11(float cosI, float randx, float randy, float *sx, float *sy)
{
  if (cosI > 0.9999f || fabsf(cosI) < 1e-6f) {
    const float r = sqrtf(randx / cmax(1.0f - randx, 1e-7f));
    const float phi = CY_2PI_F * randy;
    *sx = r * cy_cosf(phi);
    *sy = r * cy_sinf(phi);
    return;
  }
  const float sinI = safe_sqrtf(1.0f - cosI * cosI);
  const float tanI = sinI / cosI;
  const float projA = 0.5f * (cosI + 1.0f);
  if (projA < 0.0001f) {
    *sx = 0.0f;
    *sy = 0.0f;
    return;
  }
  const float A = 2.0f * randx * projA / cosI - 1.0f;
  float tmp = A * A - 1.0f;
  if (fabsf(tmp) < 1e-7f) {
    *sx = 0.0f;
    *sy = 0.0f;
    return;
  }
  tmp = 1.0f / tmp;
  const float D = safe_sqrtf(tanI * tanI * tmp * tmp - (A * A - tanI * tanI) * tmp);
  const float slopeX2 = tanI * tmp + D;
  const float slopeX = (A < 0.0f || slopeX2 > 1.0f / tanI) ? (tanI * tmp - D) : slopeX2;
  float U2;
  if (randy >= 0.5f) {
    U2 = 2.0f * (randy - 0.5f);
  }
  else {
    U2 = 2.0f * (0.5f - randy);
  }
  const float z = (U2 * (U2 * (U2 * 0.27385f - 0.73369f) + 0.46341f)) /
                  (U2 * (U2 * (U2 * 0.093073f + 0.309420f) - 1.0f) + 0.597999f);
  const float slopeY = z * sqrtf(1.0f + slopeX * slopeX);
  *sx = slopeX;
  *sy = (randy >= 0.5f) ? slopeY : -slopeY;
}

/* bsdf_microfacet_multi.h:86-100 */
CY_FN cfloat3 mf_sample_vndf(cfloat3 wi, float ax, float ay, float randx, float randy)
{
  const cfloat3 wi_11 = normalize3(mk3(ax * wi.x, ay * wi.y, wi.z));
  float s11x, s11y;
  mf_sampleP22_11(wi_11.z, randx, randy, &s11x, &s11y);
  const cfloat3 cossin_phi = safe_normalize3(mk3(wi_11.x, wi_11.y, 0.0f));
  const float slope_x = ax * (cossin_phi.x * s11x - cossin_phi.y * s11y);
  const float slope_y = ay * (cossin_phi.y * s11x + cossin_phi.x * s11y);
  return normalize3(mk3(-slope_x, -slope_y, 1.0f));
}

/* bsdf_microfacet_multi.h:105-110: -wi + 2 wm (wi . wm) */
CY_FN cfloat3 mf_sample_phase_glossy(cfloat3 wi, cfloat3 wm)
{
  return add3(neg3(wi), mul3f(mul3f(wm, 2.0f), dot3(wi, wm)));
}

/* bsdf_microfacet_multi.h:112-137 */
CY_FN float mf_eval_phase_glossy(cfloat3 w, float lambda, cfloat3 wo, float ax, float ay)
{
  if (w.z > 0.9999f) {
    return 0.0f;
  }
  const cfloat3 wh = normalize3(sub3(wo, w));
  if (wh.z < 0.0f) {
    return 0.0f;
  }
  float pArea = (w.z < -0.9999f) ? 1.0f : lambda * w.z;
  const float dotW_WH = dot3(neg3(w), wh);
  if (dotW_WH < 0.0f) {
    return 0.0f;
  }
  float phase = cmax(0.0f, dotW_WH) * 0.25f / cmax(pArea * dotW_WH, 1e-7f);
  if (ax == ay) {
    phase *= D_ggx(wh, ax);
  }
  else {
    phase *= D_ggx_aniso(wh, ax, ay);
  }
  return phase;
}

/* bsdf_microfacet_multi.h:196-210: Smith Lambda of GGX */
CY_FN float mf_lambda(cfloat3 w, float ax, float ay)
{
  if (w.z > 0.9999f) {
    return 0.0f;
  }
  else if (w.z < -0.9999f) {
    return -0.9999f;
  }
  const float inv_wz2 = 1.0f / cmax(w.z * w.z, 1e-7f);
  const float wax = w.x * ax, way = w.y * ay;
  float v = sqrtf(1.0f + (wax * wax + way * way) * inv_wz2);
  if (w.z <= 0.0f) {
    v = -v;
  }
  return 0.5f * (v - 1.0f);
}

/* bsdf_microfacet_multi.h:213-221 */
CY_FN float mf_invC1(float h)
{
  return 2.0f * saturate(h) - 1.0f;
}
CY_FN float mf_C1(float h)
{
  return saturate(0.5f * (h + 1.0f));
}

/* bsdf_microfacet_multi.h:224-231 */
CY_FN float mf_G1(cfloat3 w, float C1, float lambda)
{
  if (w.z > 0.9999f) {
    return 1.0f;
  }
  if (w.z < 1e-5f) {
    return 0.0f;
  }
  return cy_powf(C1, lambda);
}

/* bsdf_microfacet_multi.h:235-258 */
CY_FN bool mf_sample_height(cfloat3 w, float *h, float *C1, float *G1, const float *lambda, float U)
{
  if (w.z > 0.9999f) {
    return false;
  }
  if (w.z < -0.9999f) {
    *C1 *= U;
    *h = mf_invC1(*C1);
    *G1 = mf_G1(w, *C1, *lambda);
  }
  else if (fabsf(w.z) >= 0.0001f) {
    if (U > 1.0f - *G1) {
      return false;
    }
    if (*lambda >= 0.0f) {
      *C1 = 1.0f;
    }
    else {
      *C1 *= cy_powf(1.0f - U, -1.0f / *lambda);
    }
    *h = mf_invC1(*C1);
    *G1 = mf_G1(w, *C1, *lambda);
  }
  return true;
}

/* bsdf_microfacet_multi.h:266-276 */
CY_FN float mf_ggx_albedo(float r)
{
  float albedo = 0.806495f * cy_expf(-1.98712f * r * r) + 0.199531f;
  albedo -= ((((((1.76741f * r - 8.43891f) * r + 15.784f) * r - 14.398f) * r + 6.45221f) * r - 1.19722f) * r +
             0.027803f) *
                r +
            0.00568739f;
  return saturate(albedo);
}

/* bsdf_microfacet_multi.h:296-318 */
CY_FN float mf_ggx_pdf(cfloat3 wi, cfloat3 wo, float alpha)
{
  float D = D_ggx(normalize3(add3(wi, wo)), alpha);
  float lambda = mf_lambda(wi, alpha, alpha);
  float singlescatter = 0.25f * D / cmax((1.0f + lambda) * wi.z, 1e-7f);
  float multiscatter = wo.z * CY_1_PI_F;
  float albedo = mf_ggx_albedo(alpha);
  return albedo * singlescatter + (1.0f - albedo) * multiscatter;
}
CY_FN float mf_ggx_aniso_pdf(cfloat3 wi, cfloat3 wo, float ax, float ay)
{
  float D = D_ggx_aniso(normalize3(add3(wi, wo)), ax, ay);
  float lambda = mf_lambda(wi, ax, ay);
  float singlescatter = 0.25f * D / cmax((1.0f + lambda) * wi.z, 1e-7f);
  float multiscatter = wo.z * CY_1_PI_F;
  float albedo = mf_ggx_albedo(sqrtf(ax * ay));
  return albedo * singlescatter + (1.0f - albedo) * multiscatter;
}

/* bsdf_microfacet_multi_impl.h:28-182, MF_MULTI_GLOSSY */
CY_FN cfloat3 mf_eval_glossy(cfloat3 wi,
                             cfloat3 wo,
                             const bool wo_outside,
                             const cfloat3 color,
                             const float ax,
                             const float ay,
                             uint *lcg_state,
                             const float eta,
                             bool use_fresnel,
                             const cfloat3 cspec0)
{
  bool swapped = false;
  if (wo.z < wi.z) {
    swapped = true;
    cfloat3 tmp = wo;
    wo = wi;
    wi = tmp;
  }
  if (wi.z < 1e-5f || (wo.z < 1e-5f && wo_outside) || (wo.z > -1e-5f && !wo_outside)) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float lambda_r = mf_lambda(neg3(wi), ax, ay);
  float shadowing_lambda = mf_lambda(wo_outside ? wo : neg3(wo), ax, ay);

  /* single scattering, analytically */
  cfloat3 throughput = mk3(1.0f, 1.0f, 1.0f);
  const cfloat3 wh = normalize3(add3(wi, wo));
  const float G2 = 1.0f / (1.0f - (lambda_r + 1.0f) + shadowing_lambda);
  float val = G2 * 0.25f / wi.z;
  if (ax == ay) {
    val *= D_ggx(wh, ax);
  }
  else {
    val *= D_ggx_aniso(wh, ax, ay);
  }
  cfloat3 eval = mk3(val, val, val);

  float F0 = fresnel_dielectric_cos(1.0f, eta);
  if (use_fresnel) {
    throughput = interpolate_fresnel_color(wi, wh, eta, F0, cspec0);
    eval = mul3(eval, throughput);
  }

  cfloat3 wr = neg3(wi);
  float hr = 1.0f;
  float C1_r = 1.0f;
  float G1_r = 0.0f;
  const bool outside = true;

  for (int order = 0; order < 10; order++) {
    /* microfacet height, then normal */
    float height_rand = lcg_step_float(lcg_state);
    if (!mf_sample_height(wr, &hr, &C1_r, &G1_r, &lambda_r, height_rand)) {
      break;
    }
    float vndf_rand_y = lcg_step_float(lcg_state);
    float vndf_rand_x = lcg_step_float(lcg_state);
    cfloat3 wm = mf_sample_vndf(neg3(wr), ax, ay, vndf_rand_x, vndf_rand_y);

    if (order > 0) {
      /* scattering towards wo from this microfacet */
      const float p = mf_eval_phase_glossy(wr, lambda_r, wo, ax, ay);
      const cfloat3 phase = mul3(mk3(p, p, p), throughput);
      eval = add3(eval, mul3f(mul3(throughput, phase),
                              mf_G1(wo_outside ? wo : neg3(wo), mf_C1((outside == wo_outside) ? hr : -hr),
                                    shadowing_lambda)));
    }
    if (order + 1 < 10) {
      /* bounce from the microfacet */
      if (use_fresnel && order > 0) {
        throughput = mul3(throughput, interpolate_fresnel_color(neg3(wr), wm, eta, F0, cspec0));
      }
      wr = mf_sample_phase_glossy(neg3(wr), wm);
      lambda_r = mf_lambda(wr, ax, ay);
      if (!use_fresnel) {
        throughput = mul3(throughput, color);
      }
      C1_r = mf_C1(hr);
      G1_r = mf_G1(wr, C1_r, lambda_r);
    }
  }
  if (swapped) {
    eval = mul3f(eval, fabsf(wi.z / wo.z));
  }
  return eval;
}

/* bsdf_microfacet_multi_impl.h:188-274, MF_MULTI_GLOSSY */
CY_FN cfloat3 mf_sample_glossy(cfloat3 wi,
                               cfloat3 *wo,
                               const cfloat3 color,
                               const float ax,
                               const float ay,
                               uint *lcg_state,
                               const float eta,
                               bool use_fresnel,
                               const cfloat3 cspec0)
{
  cfloat3 throughput = mk3(1.0f, 1.0f, 1.0f);
  cfloat3 wr = neg3(wi);
  float lambda_r = mf_lambda(wr, ax, ay);
  float hr = 1.0f;
  float C1_r = 1.0f;
  float G1_r = 0.0f;
  const bool outside = true;

  float F0 = fresnel_dielectric_cos(1.0f, eta);
  if (use_fresnel) {
    /* normalize(wi + wr) is the zero vector normalised (NaN): the fresnel
     * term then takes its total-reflection branch, as in the reference */
    throughput = interpolate_fresnel_color(wi, normalize3(add3(wi, wr)), eta, F0, cspec0);
  }

  for (int order = 0; order < 10; order++) {
    float height_rand = lcg_step_float(lcg_state);
    if (!mf_sample_height(wr, &hr, &C1_r, &G1_r, &lambda_r, height_rand)) {
      /* the walk left the surface */
      *wo = outside ? wr : neg3(wr);
      return throughput;
    }
    float vndf_rand_y = lcg_step_float(lcg_state);
    float vndf_rand_x = lcg_step_float(lcg_state);
    cfloat3 wm = mf_sample_vndf(neg3(wr), ax, ay, vndf_rand_x, vndf_rand_y);

    /* first-bounce color is already in the mix weight */
    if (!use_fresnel && order > 0) {
      throughput = mul3(throughput, color);
    }
    if (use_fresnel) {
      cfloat3 t_color = interpolate_fresnel_color(neg3(wr), wm, eta, F0, cspec0);
      if (order == 0) {
        throughput = t_color;
      }
      else {
        throughput = mul3(throughput, t_color);
      }
    }
    wr = mf_sample_phase_glossy(neg3(wr), wm);

    lambda_r = mf_lambda(wr, ax, ay);
    G1_r = mf_G1(wr, C1_r, lambda_r);
  }
  *wo = mk3(0.0f, 0.0f, 1.0f);
  return mk3(0.0f, 0.0f, 0.0f);
}

/* bsdf_microfacet_multi.h:377-407: extra slot weight = color, N = cspec0 */
CY_FN int bsdf_microfacet_multi_ggx_common_setup(CySD *sd, CyClosure *b)
{
  CyClosure *ex = &sd->closure[b->extra];
  b->alpha_x = cclamp(b->alpha_x, 1e-4f, 1.0f);
  b->alpha_y = cclamp(b->alpha_y, 1e-4f, 1.0f);
  ex->weight = saturate3(ex->weight);
  ex->N = saturate3(ex->N);
  return SD_BSDF | SD_BSDF_HAS_EVAL | SD_BSDF_NEEDS_LCG;
}
CY_FN int bsdf_microfacet_multi_ggx_setup(CySD *sd, CyClosure *b)
{
  if (is_zero3(b->T)) {
    b->T = mk3(1.0f, 0.0f, 0.0f);
  }
  b->type = CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID;
  return bsdf_microfacet_multi_ggx_common_setup(sd, b);
}
CY_FN int bsdf_microfacet_multi_ggx_fresnel_setup(CySD *sd, CyClosure *b)
{
  if (is_zero3(b->T)) {
    b->T = mk3(1.0f, 0.0f, 0.0f);
  }
  b->type = CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID;
  bsdf_microfacet_fresnel_color(sd, b);
  return bsdf_microfacet_multi_ggx_common_setup(sd, b);
}

/* the shading frame: tangent-aligned for anisotropic roughness */
CY_FN void mf_frame(const CyClosure *b, bool is_aniso, cfloat3 *X, cfloat3 *Y)
{
  if (is_aniso) {
    make_orthonormals_tangent(b->N, b->T, X, Y);
  }
  else {
    make_orthonormals(b->N, X, Y);
  }
}

/* bsdf_microfacet_multi.h:428-467 */
CY_FN cfloat3 bsdf_microfacet_multi_ggx_eval_reflect(const CySD *sd, const CyClosure *b, cfloat3 I, cfloat3 omega_in,
                                                     float *pdf)
{
  if (b->alpha_x * b->alpha_y < 1e-7f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  const CyClosure *ex = &sd->closure[b->extra];
  const bool use_fresnel = (b->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID);
  const bool is_aniso = (b->alpha_x != b->alpha_y);
  cfloat3 X, Y;
  const cfloat3 Z = b->N;
  mf_frame(b, is_aniso, &X, &Y);
  const cfloat3 localI = mk3(dot3(I, X), dot3(I, Y), dot3(I, Z));
  const cfloat3 localO = mk3(dot3(omega_in, X), dot3(omega_in, Y), dot3(omega_in, Z));
  if (is_aniso) {
    *pdf = mf_ggx_aniso_pdf(localI, localO, b->alpha_x, b->alpha_y);
  }
  else {
    *pdf = mf_ggx_pdf(localI, localO, b->alpha_x);
  }
  return mf_eval_glossy(localI, localO, true, ex->weight, b->alpha_x, b->alpha_y, &sd->lcg_state, b->ior,
                        use_fresnel, ex->N);
}

/* bsdf_microfacet_multi.h:469-533 */
CY_FN int bsdf_microfacet_multi_ggx_sample(const CySD *sd,
                                          const CyClosure *b,
                                          cfloat3 I,
                                          cfloat3 *eval,
                                          cfloat3 *omega_in,
                                          float *pdf)
{
  const cfloat3 Z = b->N;
  if (b->alpha_x * b->alpha_y < 1e-7f) {
    *omega_in = sub3(mul3f(Z, 2.0f * dot3(Z, I)), I);
    *pdf = 1e6f;
    *eval = mk3(1e6f, 1e6f, 1e6f);
    return LABEL_REFLECT | LABEL_SINGULAR;
  }
  const CyClosure *ex = &sd->closure[b->extra];
  const bool use_fresnel = (b->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID);
  const bool is_aniso = (b->alpha_x != b->alpha_y);
  cfloat3 X, Y;
  mf_frame(b, is_aniso, &X, &Y);
  const cfloat3 localI = mk3(dot3(I, X), dot3(I, Y), dot3(I, Z));
  cfloat3 localO;
  *eval = mf_sample_glossy(localI, &localO, ex->weight, b->alpha_x, b->alpha_y, &sd->lcg_state, b->ior, use_fresnel,
                           ex->N);
  if (is_aniso) {
    *pdf = mf_ggx_aniso_pdf(localI, localO, b->alpha_x, b->alpha_y);
  }
  else {
    *pdf = mf_ggx_pdf(localI, localO, b->alpha_x);
  }
  *eval = mul3f(*eval, *pdf);
  *omega_in = add3(add3(mul3f(X, localO.x), mul3f(Y, localO.y)), mul3f(Z, localO.z));
  return LABEL_REFLECT | LABEL_GLOSSY;
}

/* ---------------------------------------------------------------------------
 * Multiscattering GGX glass */

/* bsdf_microfacet_multi.h:140-153: reflection or refraction through the
 * microfacet, by the dielectric fresnel term */
CY_FN cfloat3 mf_sample_phase_glass(cfloat3 wi, float eta, cfloat3 wm, float randV, bool *outside)
{
  const float cosI = dot3(wi, wm);
  const float f = fresnel_dielectric_cos(cosI, eta);
  if (randV < f) {
    *outside = true;
    return add3(neg3(wi), mul3f(mul3f(wm, 2.0f), cosI));
  }
  *outside = false;
  const float inv_eta = 1.0f / eta;
  const float cosT = -safe_sqrtf(1.0f - (1.0f - cosI * cosI) * inv_eta * inv_eta);
  return normalize3(sub3(mul3f(wm, cosI * inv_eta + cosT), mul3f(wi, inv_eta)));
}

/* bsdf_microfacet_multi.h:155-190 (the float3 result has three equal components) */
CY_FN float mf_eval_phase_glass(cfloat3 w, float lambda, cfloat3 wo, bool wo_outside, float alpha, float eta)
{
  if (w.z > 0.9999f) {
    return 0.0f;
  }
  const float pArea = (w.z < -0.9999f) ? 1.0f : lambda * w.z;
  float v;
  if (wo_outside) {
    const cfloat3 wh = normalize3(sub3(wo, w));
    if (wh.z < 0.0f) {
      return 0.0f;
    }
    const float dotW_WH = dot3(neg3(w), wh);
    v = fresnel_dielectric_cos(dotW_WH, eta) * cmax(0.0f, dotW_WH) * D_ggx(wh, alpha) * 0.25f / (pArea * dotW_WH);
  }
  else {
    cfloat3 wh = normalize3(sub3(mul3f(wo, eta), w));
    if (wh.z < 0.0f) {
      wh = neg3(wh);
    }
    const float dotW_WH = dot3(neg3(w), wh), dotWO_WH = dot3(wo, wh);
    if (dotW_WH < 0.0f) {
      return 0.0f;
    }
    const float temp = dotW_WH + eta * dotWO_WH;
    v = (1.0f - fresnel_dielectric_cos(dotW_WH, eta)) * cmax(0.0f, dotW_WH) * cmax(0.0f, -dotWO_WH) *
        D_ggx(wh, alpha) / (pArea * temp * temp);
  }
  return v;
}

/* bsdf_microfacet_multi.h:278-293 */
CY_FN float mf_ggx_transmission_albedo(float a, float ior)
{
  if (ior < 1.0f) {
    ior = 1.0f / ior;
  }
  a = saturate(a);
  ior = cclamp(ior, 1.0f, 3.0f);
  const float I_1 = 0.0476898f * cy_expf(-0.978352f * (ior - 0.65657f) * (ior - 0.65657f)) - 0.033756f * ior +
                    0.993261f;
  const float R_1 = (((0.116991f * a - 0.270369f) * a + 0.0501366f) * a - 0.00411511f) * a + 1.00008f;
  const float I_2 = (((-2.08704f * ior + 26.3298f) * ior - 127.906f) * ior + 292.958f) * ior - 287.946f +
                    199.803f / (ior * ior) - 101.668f / (ior * ior * ior);
  const float R_2 = ((((5.3725f * a - 24.9307f) * a + 22.7437f) * a - 3.40751f) * a + 0.0986325f) * a + 0.00493504f;
  return saturate(1.0f + I_2 * R_2 * 0.0019127f - (1.0f - I_1) * (1.0f - R_1) * 9.3205f);
}

/* bsdf_microfacet_multi.h:320-351 */
CY_FN float mf_glass_pdf(cfloat3 wi, cfloat3 wo, float alpha, float eta)
{
  const bool reflective = (wi.z * wo.z > 0.0f);
  float wh_len;
  cfloat3 wh = normalize_len3(add3(wi, reflective ? wo : mul3f(wo, eta)), &wh_len);
  if (wh.z < 0.0f) {
    wh = neg3(wh);
  }
  const cfloat3 r_wi = (wi.z < 0.0f) ? neg3(wi) : wi;
  const float lambda = mf_lambda(r_wi, alpha, alpha);
  const float D = D_ggx(wh, alpha);
  const float fresnel = fresnel_dielectric_cos(dot3(r_wi, wh), eta);
  const float multiscatter = fabsf(wo.z * CY_1_PI_F);
  if (reflective) {
    const float singlescatter = 0.25f * D / cmax((1.0f + lambda) * r_wi.z, 1e-7f);
    const float albedo = mf_ggx_albedo(alpha);
    return fresnel * (albedo * singlescatter + (1.0f - albedo) * multiscatter);
  }
  const float singlescatter = fabsf(dot3(r_wi, wh) * dot3(wo, wh) * D * eta * eta /
                                    cmax((1.0f + lambda) * r_wi.z * wh_len * wh_len, 1e-7f));
  const float albedo = mf_ggx_transmission_albedo(alpha, eta);
  return (1.0f - fresnel) * (albedo * singlescatter + (1.0f - albedo) * multiscatter);
}

/* bsdf_microfacet_multi_impl.h:28-182, MF_MULTI_GLASS (isotropic: alpha_y ==
 * alpha_x after the glass setups) */
CY_FN cfloat3 mf_eval_glass(cfloat3 wi,
                            cfloat3 wo,
                            const bool wo_outside,
                            const cfloat3 color,
                            const float alpha,
                            uint *lcg_state,
                            const float eta,
                            bool use_fresnel,
                            const cfloat3 cspec0)
{
  bool swapped = false;
  if (wi.z * wo.z < 0.0f) {
    /* transmission: the directions swap hemispheres */
    if (-wo.z < wi.z) {
      swapped = true;
      const cfloat3 tmp = neg3(wo);
      wo = neg3(wi);
      wi = tmp;
    }
  }
  else if (wo.z < wi.z) {
    swapped = true;
    const cfloat3 tmp = wo;
    wo = wi;
    wi = tmp;
  }
  if (wi.z < 1e-5f || (wo.z < 1e-5f && wo_outside) || (wo.z > -1e-5f && !wo_outside)) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float lambda_r = mf_lambda(neg3(wi), alpha, alpha);
  const float shadowing_lambda = mf_lambda(wo_outside ? wo : neg3(wo), alpha, alpha);

  /* single scattering, analytically */
  cfloat3 throughput = mk3(1.0f, 1.0f, 1.0f);
  const cfloat3 wh = normalize3(add3(wi, wo));
  const float v0 = mf_eval_phase_glass(neg3(wi), lambda_r, wo, wo_outside, alpha, eta);
  cfloat3 eval = mk3(v0, v0, v0);
  if (wo_outside) {
    eval = mul3f(eval, -lambda_r / (shadowing_lambda - lambda_r));
  }
  else {
    eval = mul3f(eval, -lambda_r * cy_beta(-lambda_r, shadowing_lambda + 1.0f));
  }

  const float F0 = fresnel_dielectric_cos(1.0f, eta);
  if (use_fresnel) {
    throughput = interpolate_fresnel_color(wi, wh, eta, F0, cspec0);
    eval = mul3(eval, throughput);
  }

  cfloat3 wr = neg3(wi);
  float hr = 1.0f;
  float C1_r = 1.0f;
  float G1_r = 0.0f;
  bool outside = true;

  for (int order = 0; order < 10; order++) {
    float height_rand = lcg_step_float(lcg_state);
    if (!mf_sample_height(wr, &hr, &C1_r, &G1_r, &lambda_r, height_rand)) {
      break;
    }
    float vndf_rand_y = lcg_step_float(lcg_state);
    float vndf_rand_x = lcg_step_float(lcg_state);
    cfloat3 wm = mf_sample_vndf(neg3(wr), alpha, alpha, vndf_rand_x, vndf_rand_y);

    if (order == 0 && use_fresnel) {
      /* with the fresnel tint the first bounce replaces the analytic term */
      const float p = outside ? mf_eval_phase_glass(wr, lambda_r, wo, wo_outside, alpha, eta) :
                                mf_eval_phase_glass(wr, lambda_r, neg3(wo), !wo_outside, alpha, 1.0f / eta);
      eval = mul3f(mul3(throughput, mk3(p, p, p)),
                   mf_G1(wo_outside ? wo : neg3(wo), mf_C1((outside == wo_outside) ? hr : -hr), shadowing_lambda));
    }
    if (order > 0) {
      const float p = outside ? mf_eval_phase_glass(wr, lambda_r, wo, wo_outside, alpha, eta) :
                                mf_eval_phase_glass(wr, lambda_r, neg3(wo), !wo_outside, alpha, 1.0f / eta);
      eval = add3(eval, mul3f(mul3(throughput, mk3(p, p, p)),
                              mf_G1(wo_outside ? wo : neg3(wo), mf_C1((outside == wo_outside) ? hr : -hr),
                                    shadowing_lambda)));
    }
    if (order + 1 < 10) {
      /* bounce from the microfacet */
      bool next_outside;
      const cfloat3 wi_prev = neg3(wr);
      const float phase_rand = lcg_step_float(lcg_state);
      wr = mf_sample_phase_glass(neg3(wr), outside ? eta : 1.0f / eta, wm, phase_rand, &next_outside);
      if (!next_outside) {
        outside = !outside;
        wr = neg3(wr);
        hr = -hr;
      }
      if (use_fresnel && !next_outside) {
        throughput = mul3(throughput, color);
      }
      else if (use_fresnel && order > 0) {
        throughput = mul3(throughput, interpolate_fresnel_color(wi_prev, wm, eta, F0, cspec0));
      }
      lambda_r = mf_lambda(wr, alpha, alpha);
      if (!use_fresnel) {
        throughput = mul3(throughput, color);
      }
      C1_r = mf_C1(hr);
      G1_r = mf_G1(wr, C1_r, lambda_r);
    }
  }
  if (swapped) {
    eval = mul3f(eval, fabsf(wi.z / wo.z));
  }
  return eval;
}

/* bsdf_microfacet_multi_impl.h:188-274, MF_MULTI_GLASS */
CY_FN cfloat3 mf_sample_glass(cfloat3 wi,
                              cfloat3 *wo,
                              const cfloat3 color,
                              const float alpha,
                              uint *lcg_state,
                              const float eta,
                              bool use_fresnel,
                              const cfloat3 cspec0)
{
  cfloat3 throughput = mk3(1.0f, 1.0f, 1.0f);
  cfloat3 wr = neg3(wi);
  float lambda_r = mf_lambda(wr, alpha, alpha);
  float hr = 1.0f;
  float C1_r = 1.0f;
  float G1_r = 0.0f;
  bool outside = true;

  const float F0 = fresnel_dielectric_cos(1.0f, eta);
  if (use_fresnel) {
    /* normalize(wi + wr) of opposite vectors: NaN, as in the reference */
    throughput = interpolate_fresnel_color(wi, normalize3(add3(wi, wr)), eta, F0, cspec0);
  }

  for (int order = 0; order < 10; order++) {
    float height_rand = lcg_step_float(lcg_state);
    if (!mf_sample_height(wr, &hr, &C1_r, &G1_r, &lambda_r, height_rand)) {
      /* the walk left the surface */
      *wo = outside ? wr : neg3(wr);
      return throughput;
    }
    float vndf_rand_y = lcg_step_float(lcg_state);
    float vndf_rand_x = lcg_step_float(lcg_state);
    cfloat3 wm = mf_sample_vndf(neg3(wr), alpha, alpha, vndf_rand_x, vndf_rand_y);

    /* first-bounce color is already in the mix weight */
    if (!use_fresnel && order > 0) {
      throughput = mul3(throughput, color);
    }
    bool next_outside;
    const cfloat3 wi_prev = neg3(wr);
    const float phase_rand = lcg_step_float(lcg_state);
    wr = mf_sample_phase_glass(neg3(wr), outside ? eta : 1.0f / eta, wm, phase_rand, &next_outside);
    if (!next_outside) {
      hr = -hr;
      wr = neg3(wr);
      outside = !outside;
    }
    if (use_fresnel) {
      if (!next_outside) {
        throughput = mul3(throughput, color);
      }
      else {
        const cfloat3 t_color = interpolate_fresnel_color(wi_prev, wm, eta, F0, cspec0);
        if (order == 0) {
          throughput = t_color;
        }
        else {
          throughput = mul3(throughput, t_color);
        }
      }
    }
    lambda_r = mf_lambda(wr, alpha, alpha);
    G1_r = mf_G1(wr, C1_r, lambda_r);
  }
  *wo = mk3(0.0f, 0.0f, 1.0f);
  return mk3(0.0f, 0.0f, 0.0f);
}

/* bsdf_microfacet_multi.h:537-564: extra slot weight = color, N = cspec0 */
CY_FN int bsdf_microfacet_multi_ggx_glass_setup(CySD *sd, CyClosure *b)
{
  CyClosure *ex = &sd->closure[b->extra];
  b->alpha_x = cclamp(b->alpha_x, 1e-4f, 1.0f);
  b->alpha_y = b->alpha_x;
  b->ior = cmax(0.0f, b->ior);
  ex->weight = saturate3(ex->weight);
  b->type = CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL | SD_BSDF_NEEDS_LCG;
}
CY_FN int bsdf_microfacet_multi_ggx_glass_fresnel_setup(CySD *sd, CyClosure *b)
{
  CyClosure *ex = &sd->closure[b->extra];
  b->alpha_x = cclamp(b->alpha_x, 1e-4f, 1.0f);
  b->alpha_y = b->alpha_x;
  b->ior = cmax(0.0f, b->ior);
  ex->weight = saturate3(ex->weight);
  ex->N = saturate3(ex->N);
  b->type = CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID;
  bsdf_microfacet_fresnel_color(sd, b);
  return SD_BSDF | SD_BSDF_HAS_EVAL | SD_BSDF_NEEDS_LCG;
}

/* bsdf_microfacet_multi.h:566-626: eval_transmit (no fresnel tint) and
 * eval_reflect */
CY_FN cfloat3 bsdf_microfacet_multi_ggx_glass_eval(const CySD *sd, const CyClosure *b, cfloat3 I, cfloat3 omega_in,
                                                   float *pdf, bool reflect)
{
  if (b->alpha_x * b->alpha_y < 1e-7f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  const CyClosure *ex = &sd->closure[b->extra];
  const bool use_fresnel = reflect && (b->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID);
  cfloat3 X, Y;
  const cfloat3 Z = b->N;
  make_orthonormals(Z, &X, &Y);
  const cfloat3 localI = mk3(dot3(I, X), dot3(I, Y), dot3(I, Z));
  const cfloat3 localO = mk3(dot3(omega_in, X), dot3(omega_in, Y), dot3(omega_in, Z));
  *pdf = mf_glass_pdf(localI, localO, b->alpha_x, b->ior);
  return mf_eval_glass(localI, localO, reflect, ex->weight, b->alpha_x, &sd->lcg_state, b->ior, use_fresnel,
                       reflect ? ex->N : ex->weight);
}

/* bsdf_microfacet_multi.h:628-731 */
CY_FN int bsdf_microfacet_multi_ggx_glass_sample(const CySD *sd,
                                                const CyClosure *b,
                                                cfloat3 I,
                                                float randu,
                                                cfloat3 *eval,
                                                cfloat3 *omega_in,
                                                float *pdf)
{
  const cfloat3 Z = b->N;
  if (b->alpha_x * b->alpha_y < 1e-7f) {
    cfloat3 R, T;
    bool inside;
    const float fresnel = fresnel_dielectric(b->ior, Z, I, &R, &T, &inside);
    *pdf = 1e6f;
    *eval = mk3(1e6f, 1e6f, 1e6f);
    if (randu < fresnel) {
      *omega_in = R;
      return LABEL_REFLECT | LABEL_SINGULAR;
    }
    *omega_in = T;
    return LABEL_TRANSMIT | LABEL_SINGULAR;
  }
  const CyClosure *ex = &sd->closure[b->extra];
  const bool use_fresnel = (b->type == CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID);
  cfloat3 X, Y;
  make_orthonormals(Z, &X, &Y);
  const cfloat3 localI = mk3(dot3(I, X), dot3(I, Y), dot3(I, Z));
  cfloat3 localO;
  *eval = mf_sample_glass(localI, &localO, ex->weight, b->alpha_x, &sd->lcg_state, b->ior, use_fresnel, ex->N);
  *pdf = mf_glass_pdf(localI, localO, b->alpha_x, b->ior);
  *eval = mul3f(*eval, *pdf);
  *omega_in = add3(add3(mul3f(X, localO.x), mul3f(Y, localO.y)), mul3f(Z, localO.z));
  if (localO.z * localI.z > 0.0f) {
    return LABEL_REFLECT | LABEL_GLOSSY;
  }
  return LABEL_TRANSMIT | LABEL_GLOSSY;
}

#endif /* CY_MICROFACET_MULTI_H */
