/*
 * cy_closures.h — the BSDF closures of the reference SVM kernel, evaluated and
 * sampled with the reference's arithmetic (bit-exact bar, see cy_math.h):
 *
 *   diffuse, translucent           closure/bsdf_diffuse.h
 *   Oren-Nayar                     closure/bsdf_oren_nayar.h
 *   diffuse / glossy toon          closure/bsdf_toon.h
 *   Ashikhmin velvet               closure/bsdf_ashikhmin_velvet.h
 *   Ashikhmin-Shirley (isotropic)  closure/bsdf_ashikhmin_shirley.h
 *   principled diffuse / sheen     closure/bsdf_principled_diffuse.h, _sheen.h
 *   sharp reflection / refraction  closure/bsdf_reflection.h, bsdf_refraction.h
 *   transparent (sample)           closure/bsdf_transparent.h
 *   GGX + Beckmann microfacets     closure/bsdf_microfacet.h: reflection and
 *                                  refraction, isotropic and anisotropic
 *                                  (tangent frame), GGX fresnel / clearcoat
 *                                  variants (extra data in a closure slot)
 *   dispatch                       closure/bsdf.h:113-705 (bsdf_sample,
 *                                  bsdf_eval, bump shadowing term)
 *
 * Beckmann sampling follows the reference CPU kernel (the oracle): slope_x
 * from the host's precomputed table (KernelTables.beckmann_offset in
 * __lookup_table, render/shader.cpp beckmann_table_build), not the GPU
 * Newton iteration the CUDA build uses (bsdf_microfacet.h:87-131).
 *
 * Parameter slots of CyClosure per closure type (the reference casts
 * ShaderClosure to per-type structs; here one 64-byte record serves all):
 *   microfacet     alpha_x, alpha_y, ior, T, extra (index of the
 *                  MicrofacetExtra slot in sd->closure, -1 for none)
 *   Oren-Nayar     alpha_x = roughness, alpha_y = a, ior = b
 *   velvet         alpha_x = sigma, alpha_y = 1 / sigma^2
 *   toon           alpha_x = size, alpha_y = smooth
 *   principled     diffuse: alpha_x = roughness; sheen: alpha_x = avg_value
 * A MicrofacetExtra slot (closure_alloc_extra, svm_closure.h) holds
 * weight = color, N = cspec0, T = fresnel_color, alpha_x = clearcoat.
 */
#ifndef CY_CLOSURES_H
#define CY_CLOSURES_H

#define CY_PI_2_F_CLOSURE CY_PI_2_F
#define CY_1_2PI_F 0.159154943091895335768f
#define CY_LN2_F 0.6931471805599453f

/* ---------------------------------------------------------------------------
 * Small helpers (util_math.h, util_math_fast.h, kernel_montecarlo.h)
 */
CY_FN float safe_divide(float a, float b)
{
  return (b != 0.0f) ? a / b : 0.0f;
}

CY_FN cfloat3 saturate3(cfloat3 a)
{
  return mk3(saturate(a.x), saturate(a.y), saturate(a.z));
}

/* kernel_montecarlo.h:50-54 */
CY_FN void make_orthonormals_tangent(cfloat3 N, cfloat3 T, cfloat3 *a, cfloat3 *b)
{
  *b = normalize3(cross3(N, T));
  *a = cross3(*b, N);
}

/* util_math.h:563-582 */
CY_FN cfloat3 rotate_around_axis(cfloat3 p, cfloat3 axis, float angle)
{
  float costheta = cy_cosf(angle);
  float sintheta = cy_sinf(angle);
  cfloat3 r;
  r.x = ((costheta + (1 - costheta) * axis.x * axis.x) * p.x) +
        (((1 - costheta) * axis.x * axis.y - axis.z * sintheta) * p.y) +
        (((1 - costheta) * axis.x * axis.z + axis.y * sintheta) * p.z);
  r.y = (((1 - costheta) * axis.x * axis.y + axis.z * sintheta) * p.x) +
        ((costheta + (1 - costheta) * axis.y * axis.y) * p.y) +
        (((1 - costheta) * axis.y * axis.z - axis.x * sintheta) * p.z);
  r.z = (((1 - costheta) * axis.x * axis.z - axis.y * sintheta) * p.x) +
        (((1 - costheta) * axis.y * axis.z + axis.x * sintheta) * p.y) +
        ((costheta + (1 - costheta) * axis.z * axis.z) * p.z);
  return r;
}

/* kernel_montecarlo.h:69-82 */
CY_FN void sample_uniform_hemisphere(cfloat3 N, float randu, float randv, cfloat3 *omega_in, float *pdf)
{
  float z = randu;
  float r = sqrtf(cmax(0.0f, 1.0f - z * z));
  float phi = CY_2PI_F * randv;
  float x = r * cy_cosf(phi);
  float y = r * cy_sinf(phi);
  cfloat3 T, B;
  make_orthonormals(N, &T, &B);
  *omega_in = add3(add3(mul3f(T, x), mul3f(B, y)), mul3f(N, z));
  *pdf = 0.5f * CY_1_PI_F;
}

/* kernel_montecarlo.h:84-99 */
CY_FN void sample_uniform_cone(cfloat3 N, float angle, float randu, float randv, cfloat3 *omega_in, float *pdf)
{
  float zMin = cy_cosf(angle);
  float z = zMin - zMin * randu + randu;
  float r = safe_sqrtf(1.0f - sqr(z));
  float phi = CY_2PI_F * randv;
  float x = r * cy_cosf(phi);
  float y = r * cy_sinf(phi);
  cfloat3 T, B;
  make_orthonormals(N, &T, &B);
  *omega_in = add3(add3(mul3f(T, x), mul3f(B, y)), mul3f(N, z));
  *pdf = CY_1_2PI_F / (1.0f - zMin);
}

/* util_math_fast.h:362-394 (madd is a * b + c, no contraction) */
CY_FN float fast_log2f(float x)
{
  x = cclamp(x, 1.17549435e-38f, CY_FLT_MAX);
  uint bits = as_uint(x);
  int exponent = (int)(bits >> 23) - 127;
  float f = as_float((bits & 0x007FFFFFu) | 0x3f800000u) - 1.0f;
  float f2 = f * f;
  float f4 = f2 * f2;
  float hi = f * -0.00931049621349f + 0.05206469089414f;
  float lo = f * 0.47868480909345f + -0.72116591947498f;
  hi = f * hi + -0.13753123777116f;
  hi = f * hi + 0.24187369696082f;
  hi = f * hi + -0.34730547155299f;
  lo = f * lo + 1.442689881667200f;
  return ((f4 * hi) + (f * lo)) + (float)exponent;
}
CY_FN float fast_logf(float x)
{
  return fast_log2f(x) * CY_LN2_F;
}

/* util_math_fast.h:579-601 (Abramowitz-Stegun 7.1.28) */
CY_FN float fast_erff(float x)
{
  const float a1 = 0.0705230784f, a2 = 0.0422820123f, a3 = 0.0092705272f;
  const float a4 = 0.0001520143f, a5 = 0.0002765672f, a6 = 0.0000430638f;
  const float a = fabsf(x);
  if (a >= 12.3f) {
    return copysignf(1.0f, x);
  }
  const float b = 1.0f - (1.0f - a);
  const float r = ((((((a6 * b + a5) * b + a4) * b + a3) * b + a2) * b + a1) * b + 1.0f);
  const float s = r * r;
  const float t = s * s;
  const float u = t * t;
  const float v = u * u;
  return copysignf(1.0f - 1.0f / v, x);
}

/* util_math_fast.h:614-648 (Giles' erfinv) */
CY_FN float fast_ierff(float x)
{
  float a = fabsf(x);
  if (a > 0.99999994f) {
    a = 0.99999994f;
  }
  float w = -fast_logf((1.0f - a) * (1.0f + a)), p;
  if (w < 5.0f) {
    w = w - 2.5f;
    p = 2.81022636e-08f;
    p = p * w + 3.43273939e-07f;
    p = p * w + -3.5233877e-06f;
    p = p * w + -4.39150654e-06f;
    p = p * w + 0.00021858087f;
    p = p * w + -0.00125372503f;
    p = p * w + -0.00417768164f;
    p = p * w + 0.246640727f;
    p = p * w + 1.50140941f;
  }
  else {
    w = sqrtf(w) - 3.0f;
    p = -0.000200214257f;
    p = p * w + 0.000100950558f;
    p = p * w + 0.00134934322f;
    p = p * w + -0.00367342844f;
    p = p * w + 0.00573950773f;
    p = p * w + -0.0076224613f;
    p = p * w + 0.00943887047f;
    p = p * w + 1.00167406f;
    p = p * w + 2.83297682f;
  }
  return p * x;
}

/* kernel_globals.h:229-244 */
CY_FN float lookup_table_read_2D(const CyGlobals *kg, float x, float y, int offset, int xsize, int ysize)
{
  y = saturate(y) * (ysize - 1);
  int index = imin((int)y, ysize - 1);
  int nindex = imin(index + 1, ysize - 1);
  float t = y - index;
  float data0 = lookup_table_read(kg, x, offset + xsize * index, xsize);
  if (t == 0.0f) {
    return data0;
  }
  float data1 = lookup_table_read(kg, x, offset + xsize * nindex, xsize);
  return (1.0f - t) * data0 + t * data1;
}

#define CY_BECKMANN_TABLE_SIZE 256

/* ---------------------------------------------------------------------------
 * Fresnel (bsdf_util.h)
 */
CY_FN float fresnel_dielectric(
    float eta, const cfloat3 N, const cfloat3 I, cfloat3 *R, cfloat3 *T, bool *is_inside)
{
  float cos = dot3(N, I), neta;
  cfloat3 Nn;
  if (cos > 0) {
    neta = 1 / eta;
    Nn = N;
    *is_inside = false;
  }
  else {
    cos = -cos;
    neta = eta;
    Nn = neg3(N);
    *is_inside = true;
  }
  *R = sub3(mul3f(Nn, (2 * cos)), I);
  float arg = 1 - (neta * neta * (1 - (cos * cos)));
  if (arg < 0) {
    *T = mk3(0.0f, 0.0f, 0.0f);
    return 1;
  }
  float dnp = cmax(sqrtf(arg), 1e-7f);
  float nK = (neta * cos) - dnp;
  *T = add3(neg3(mul3f(I, neta)), mul3f(Nn, nK));
  float cosTheta1 = cos;
  float cosTheta2 = -dot3(Nn, *T);
  float pPara = (cosTheta1 - eta * cosTheta2) / (cosTheta1 + eta * cosTheta2);
  float pPerp = (eta * cosTheta1 - cosTheta2) / (eta * cosTheta1 + cosTheta2);
  return 0.5f * (pPara * pPara + pPerp * pPerp);
}

CY_FN float fresnel_dielectric_cos(float cosi, float eta)
{
  float c = fabsf(cosi);
  float g = eta * eta - 1 + c * c;
  if (g > 0) {
    g = sqrtf(g);
    float A = (g - c) / (g + c);
    float B = (c * (g + c) - 1) / (c * (g - c) + 1);
    return 0.5f * A * A * (1 + B * B);
  }
  return 1.0f;
}

/* bsdf_util.h:139-149 */
CY_FN cfloat3 interpolate_fresnel_color(cfloat3 L, cfloat3 H, float ior, float F0, cfloat3 cspec0)
{
  float F0_norm = 1.0f / (1.0f - F0);
  float FH = (fresnel_dielectric_cos(dot3(L, H), ior) - F0) * F0_norm;
  return add3(mul3f(cspec0, (1.0f - FH)), mul3f(mk3(1.0f, 1.0f, 1.0f), FH));
}

#if CY_CLOSURE_EXT
/* closure.h closure_alloc_extra (kernel_shader.h): one closure slot taken from
 * the end of the array; returns its index or -1 (and drops the closure just
 * allocated, like the reference). */
CY_FN int closure_alloc_extra(CySD *sd)
{
  if (1 > sd->num_closure_left) {
    sd->num_closure--;
    sd->num_closure_left++;
    return -1;
  }
  sd->num_closure_left -= 1;
  return sd->num_closure + sd->num_closure_left;
}
#endif

/* ---------------------------------------------------------------------------
 * Setups (bsdf_*.h *_setup)
 */
CY_FN int bsdf_diffuse_setup(CyClosure *b)
{
  b->type = CLOSURE_BSDF_DIFFUSE_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

CY_FN int bsdf_translucent_setup(CyClosure *b)
{
  b->type = CLOSURE_BSDF_TRANSLUCENT_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

/* bsdf_oren_nayar.h:45-60: alpha_x = roughness in, a and b out */
CY_FN int bsdf_oren_nayar_setup(CyClosure *b)
{
  float sigma = b->alpha_x;
  b->type = CLOSURE_BSDF_OREN_NAYAR_ID;
  sigma = saturate(sigma);
  float div = 1.0f / (CY_PI_F + ((3.0f * CY_PI_F - 4.0f) / 6.0f) * sigma);
  b->alpha_y = 1.0f * div;
  b->ior = sigma * div;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

/* bsdf_ashikhmin_velvet.h:47-55: alpha_x = sigma */
CY_FN int bsdf_ashikhmin_velvet_setup(CyClosure *b)
{
  float sigma = fmaxf(b->alpha_x, 0.01f);
  b->alpha_y = 1.0f / (sigma * sigma);
  b->type = CLOSURE_BSDF_ASHIKHMIN_VELVET_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

/* bsdf_toon.h:47-54, 152-159: alpha_x = size, alpha_y = smooth */
CY_FN int bsdf_toon_setup(CyClosure *b, int type)
{
  b->type = type;
  b->alpha_x = saturate(b->alpha_x);
  b->alpha_y = saturate(b->alpha_y);
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

/* bsdf_microfacet.h:307-317, 370-380, 790-813 */
CY_FN int bsdf_microfacet_ggx_setup(CyClosure *b)
{
#if CY_CLOSURE_EXT
  b->extra = -1;
#endif
  b->alpha_x = saturate(b->alpha_x);
  b->alpha_y = saturate(b->alpha_y);
  b->type = CLOSURE_BSDF_MICROFACET_GGX_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}
CY_FN int bsdf_microfacet_ggx_refraction_setup(CyClosure *b)
{
#if CY_CLOSURE_EXT
  b->extra = -1;
#endif
  b->alpha_x = saturate(b->alpha_x);
  b->alpha_y = b->alpha_x;
  b->type = CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}
CY_FN int bsdf_microfacet_beckmann_setup(CyClosure *b)
{
  b->alpha_x = saturate(b->alpha_x);
  b->alpha_y = saturate(b->alpha_y);
  b->type = CLOSURE_BSDF_MICROFACET_BECKMANN_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}
CY_FN int bsdf_microfacet_beckmann_refraction_setup(CyClosure *b)
{
  b->alpha_x = saturate(b->alpha_x);
  b->alpha_y = b->alpha_x;
  b->type = CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}
/* bsdf_ashikhmin_shirley.h:37-45 */
CY_FN int bsdf_ashikhmin_shirley_setup(CyClosure *b)
{
  b->alpha_x = cclamp(b->alpha_x, 1e-4f, 1.0f);
  b->alpha_y = cclamp(b->alpha_y, 1e-4f, 1.0f);
  b->type = CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

#if CY_CLOSURE_EXT
/* bsdf_microfacet.h:277-289: the fresnel tint evaluated at the shading point
 * scales the sample weight (extra slot: N = cspec0, T = fresnel_color,
 * alpha_x = clearcoat) */
CY_FN void bsdf_microfacet_fresnel_color(CySD *sd, CyClosure *b)
{
  CyClosure *ex = &sd->closure[b->extra];
  float F0 = fresnel_dielectric_cos(1.0f, b->ior);
  ex->T = interpolate_fresnel_color(sd->I, b->N, b->ior, F0, ex->N);
  if (b->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID) {
    ex->T = mul3f(ex->T, 0.25f * ex->alpha_x);
  }
  b->sample_weight *= average3(ex->T);
}
CY_FN int bsdf_microfacet_ggx_fresnel_setup(CyClosure *b, CySD *sd)
{
  CyClosure *ex = &sd->closure[b->extra];
  ex->N = saturate3(ex->N);
  b->alpha_x = saturate(b->alpha_x);
  b->alpha_y = saturate(b->alpha_y);
  b->type = CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID;
  bsdf_microfacet_fresnel_color(sd, b);
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}
CY_FN int bsdf_microfacet_ggx_clearcoat_setup(CyClosure *b, CySD *sd)
{
  CyClosure *ex = &sd->closure[b->extra];
  ex->N = saturate3(ex->N);
  b->alpha_x = saturate(b->alpha_x);
  b->alpha_y = b->alpha_x;
  b->type = CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID;
  bsdf_microfacet_fresnel_color(sd, b);
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}
#endif

/* ---------------------------------------------------------------------------
 * Diffuse family
 */
/* cosine hemisphere: kernel_montecarlo.h:57-66 */
CY_FN void sample_cos_hemisphere(cfloat3 N, float randu, float randv, cfloat3 *omega_in, float *pdf)
{
  float phi = CY_2PI_F * randu;
  float r = sqrtf(randv);
  randu = r * cy_cosf(phi);
  randv = r * cy_sinf(phi);
  float costheta = sqrtf(cmax(1.0f - randu * randu - randv * randv, 0.0f));
  cfloat3 T, B;
  make_orthonormals(N, &T, &B);
  *omega_in = add3(add3(mul3f(T, randu), mul3f(B, randv)), mul3f(N, costheta));
  *pdf = costheta * CY_1_PI_F;
}

/* bsdf_diffuse.h:46-111 */
CY_FN cfloat3 bsdf_diffuse_eval_reflect(const CyClosure *sc, cfloat3 omega_in, float *pdf)
{
  float cos_pi = fmaxf(dot3(sc->N, omega_in), 0.0f) * CY_1_PI_F;
  *pdf = cos_pi;
  return mk3(cos_pi, cos_pi, cos_pi);
}

CY_FN int bsdf_diffuse_sample(const CyClosure *sc,
                              cfloat3 Ng,
                              float randu,
                              float randv,
                              cfloat3 *eval,
                              cfloat3 *omega_in,
                              float *pdf)
{
  sample_cos_hemisphere(sc->N, randu, randv, omega_in, pdf);
  if (dot3(Ng, *omega_in) > 0.0f) {
    *eval = mk3(*pdf, *pdf, *pdf);
  }
  else {
    *pdf = 0.0f;
  }
  return LABEL_REFLECT | LABEL_DIFFUSE;
}

/* bsdf_diffuse.h:115-175 (translucent: the lower hemisphere) */
CY_FN cfloat3 bsdf_translucent_eval_transmit(const CyClosure *sc, cfloat3 omega_in, float *pdf)
{
  float cos_pi = fmaxf(-dot3(sc->N, omega_in), 0.0f) * CY_1_PI_F;
  *pdf = cos_pi;
  return mk3(cos_pi, cos_pi, cos_pi);
}

CY_FN int bsdf_translucent_sample(const CyClosure *sc,
                                  cfloat3 Ng,
                                  float randu,
                                  float randv,
                                  cfloat3 *eval,
                                  cfloat3 *omega_in,
                                  float *pdf)
{
  sample_cos_hemisphere(neg3(sc->N), randu, randv, omega_in, pdf);
  if (dot3(Ng, *omega_in) < 0) {
    *eval = mk3(*pdf, *pdf, *pdf);
  }
  else {
    *pdf = 0;
  }
  return LABEL_TRANSMIT | LABEL_DIFFUSE;
}

/* bsdf_oren_nayar.h:32-43, 70-120 */
CY_FN cfloat3 bsdf_oren_nayar_get_intensity(const CyClosure *sc, cfloat3 n, cfloat3 v, cfloat3 l)
{
  float nl = cmax(dot3(n, l), 0.0f);
  float nv = cmax(dot3(n, v), 0.0f);
  float t = dot3(l, v) - nl * nv;
  if (t > 0.0f) {
    t /= cmax(nl, nv) + 1.17549435e-38f;
  }
  float is = nl * (sc->alpha_y + sc->ior * t);
  return mk3(is, is, is);
}

CY_FN cfloat3 bsdf_oren_nayar_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  if (dot3(sc->N, omega_in) > 0.0f) {
    *pdf = 0.5f * CY_1_PI_F;
    return bsdf_oren_nayar_get_intensity(sc, sc->N, I, omega_in);
  }
  *pdf = 0.0f;
  return mk3(0.0f, 0.0f, 0.0f);
}

CY_FN int bsdf_oren_nayar_sample(const CyClosure *sc,
                                 cfloat3 Ng,
                                 cfloat3 I,
                                 float randu,
                                 float randv,
                                 cfloat3 *eval,
                                 cfloat3 *omega_in,
                                 float *pdf)
{
  sample_uniform_hemisphere(sc->N, randu, randv, omega_in, pdf);
  if (dot3(Ng, *omega_in) > 0.0f) {
    *eval = bsdf_oren_nayar_get_intensity(sc, sc->N, I, *omega_in);
  }
  else {
    *pdf = 0.0f;
    *eval = mk3(0.0f, 0.0f, 0.0f);
  }
  return LABEL_REFLECT | LABEL_DIFFUSE;
}

/* bsdf_ashikhmin_velvet.h:65-176 */
CY_FN float bsdf_velvet_power(float m_invsigma2, float cosNO, float cosNI, float cosNH, float cosHO)
{
  float cosNHdivHO = cosNH / cosHO;
  cosNHdivHO = fmaxf(cosNHdivHO, 1e-5f);
  float fac1 = 2 * fabsf(cosNHdivHO * cosNO);
  float fac2 = 2 * fabsf(cosNHdivHO * cosNI);
  float sinNH2 = 1 - cosNH * cosNH;
  float sinNH4 = sinNH2 * sinNH2;
  float cotangent2 = (cosNH * cosNH) / sinNH2;
  float D = cy_expf(-cotangent2 * m_invsigma2) * m_invsigma2 * CY_1_PI_F / sinNH4;
  float G = cmin(1.0f, cmin(fac1, fac2));
  return 0.25f * (D * G) / cosNO;
}

CY_FN cfloat3 bsdf_ashikhmin_velvet_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  float m_invsigma2 = sc->alpha_y;
  cfloat3 N = sc->N;
  float cosNO = dot3(N, I);
  float cosNI = dot3(N, omega_in);
  if (cosNO > 0 && cosNI > 0) {
    cfloat3 H = normalize3(add3(omega_in, I));
    float cosNH = dot3(N, H);
    float cosHO = fabsf(dot3(I, H));
    if (!(fabsf(cosNH) < 1.0f - 1e-5f && cosHO > 1e-5f)) {
      return mk3(0.0f, 0.0f, 0.0f);
    }
    float out = bsdf_velvet_power(m_invsigma2, cosNO, cosNI, cosNH, cosHO);
    *pdf = 0.5f * CY_1_PI_F;
    return mk3(out, out, out);
  }
  return mk3(0.0f, 0.0f, 0.0f);
}

CY_FN int bsdf_ashikhmin_velvet_sample(const CyClosure *sc,
                                       cfloat3 Ng,
                                       cfloat3 I,
                                       float randu,
                                       float randv,
                                       cfloat3 *eval,
                                       cfloat3 *omega_in,
                                       float *pdf)
{
  float m_invsigma2 = sc->alpha_y;
  cfloat3 N = sc->N;
  sample_uniform_hemisphere(N, randu, randv, omega_in, pdf);
  if (dot3(Ng, *omega_in) > 0) {
    cfloat3 H = normalize3(add3(*omega_in, I));
    float cosNI = dot3(N, *omega_in);
    float cosNO = dot3(N, I);
    float cosNH = dot3(N, H);
    float cosHO = fabsf(dot3(I, H));
    if (fabsf(cosNO) > 1e-5f && fabsf(cosNH) < 1.0f - 1e-5f && cosHO > 1e-5f) {
      float power = bsdf_velvet_power(m_invsigma2, cosNO, cosNI, cosNH, cosHO);
      *eval = mk3(power, power, power);
    }
    else {
      *pdf = 0.0f;
    }
  }
  else {
    *pdf = 0.0f;
  }
  return LABEL_REFLECT | LABEL_DIFFUSE;
}

/* bsdf_toon.h:64-248 */
CY_FN float bsdf_toon_get_intensity(float max_angle, float smooth, float angle)
{
  float is;
  if (angle < max_angle) {
    is = 1.0f;
  }
  else if (angle < (max_angle + smooth) && smooth != 0.0f) {
    is = (1.0f - (angle - max_angle) / smooth);
  }
  else {
    is = 0.0f;
  }
  return is;
}
CY_FN float bsdf_toon_get_sample_angle(float max_angle, float smooth)
{
  return fminf(max_angle + smooth, CY_PI_2_F);
}

CY_FN cfloat3 bsdf_diffuse_toon_eval_reflect(const CyClosure *sc, cfloat3 omega_in, float *pdf)
{
  float max_angle = sc->alpha_x * CY_PI_2_F;
  float smooth = sc->alpha_y * CY_PI_2_F;
  float angle = safe_acosf(fmaxf(dot3(sc->N, omega_in), 0.0f));
  float is = bsdf_toon_get_intensity(max_angle, smooth, angle);
  if (is > 0.0f) {
    float sample_angle = bsdf_toon_get_sample_angle(max_angle, smooth);
    *pdf = 0.5f * CY_1_PI_F / (1.0f - cy_cosf(sample_angle));
    return mk3(*pdf * is, *pdf * is, *pdf * is);
  }
  return mk3(0.0f, 0.0f, 0.0f);
}

CY_FN int bsdf_diffuse_toon_sample(const CyClosure *sc,
                                   cfloat3 Ng,
                                   float randu,
                                   float randv,
                                   cfloat3 *eval,
                                   cfloat3 *omega_in,
                                   float *pdf)
{
  float max_angle = sc->alpha_x * CY_PI_2_F;
  float smooth = sc->alpha_y * CY_PI_2_F;
  float sample_angle = bsdf_toon_get_sample_angle(max_angle, smooth);
  float angle = sample_angle * randu;
  if (sample_angle > 0.0f) {
    sample_uniform_cone(sc->N, sample_angle, randu, randv, omega_in, pdf);
    if (dot3(Ng, *omega_in) > 0.0f) {
      float is = bsdf_toon_get_intensity(max_angle, smooth, angle);
      *eval = mk3(*pdf * is, *pdf * is, *pdf * is);
    }
    else {
      *pdf = 0.0f;
    }
  }
  return LABEL_REFLECT | LABEL_DIFFUSE;
}

CY_FN cfloat3 bsdf_glossy_toon_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  float max_angle = sc->alpha_x * CY_PI_2_F;
  float smooth = sc->alpha_y * CY_PI_2_F;
  float cosNI = dot3(sc->N, omega_in);
  float cosNO = dot3(sc->N, I);
  if (cosNI > 0 && cosNO > 0) {
    cfloat3 R = sub3(mul3f(sc->N, (2 * cosNO)), I);
    float cosRI = dot3(R, omega_in);
    float angle = safe_acosf(fmaxf(cosRI, 0.0f));
    float is = bsdf_toon_get_intensity(max_angle, smooth, angle);
    float sample_angle = bsdf_toon_get_sample_angle(max_angle, smooth);
    *pdf = 0.5f * CY_1_PI_F / (1.0f - cy_cosf(sample_angle));
    return mk3(*pdf * is, *pdf * is, *pdf * is);
  }
  return mk3(0.0f, 0.0f, 0.0f);
}

CY_FN int bsdf_glossy_toon_sample(const CyClosure *sc,
                                  cfloat3 Ng,
                                  cfloat3 I,
                                  float randu,
                                  float randv,
                                  cfloat3 *eval,
                                  cfloat3 *omega_in,
                                  float *pdf)
{
  float max_angle = sc->alpha_x * CY_PI_2_F;
  float smooth = sc->alpha_y * CY_PI_2_F;
  float cosNO = dot3(sc->N, I);
  if (cosNO > 0) {
    cfloat3 R = sub3(mul3f(sc->N, (2 * cosNO)), I);
    float sample_angle = bsdf_toon_get_sample_angle(max_angle, smooth);
    float angle = sample_angle * randu;
    sample_uniform_cone(R, sample_angle, randu, randv, omega_in, pdf);
    if (dot3(Ng, *omega_in) > 0.0f) {
      float cosNI = dot3(sc->N, *omega_in);
      if (cosNI > 0) {
        float is = bsdf_toon_get_intensity(max_angle, smooth, angle);
        *eval = mk3(*pdf * is, *pdf * is, *pdf * is);
      }
      else {
        *pdf = 0.0f;
      }
    }
    else {
      *pdf = 0.0f;
    }
  }
  return LABEL_GLOSSY | LABEL_REFLECT;
}

#if CY_CLOSURE_EXT
/* bsdf_util.h:129-134 */
CY_FN float schlick_fresnel(float u)
{
  float m = cclamp(1.0f - u, 0.0f, 1.0f);
  float m2 = m * m;
  return m2 * m2 * m;
}

/* bsdf_principled_diffuse.h:33-118 (alpha_x = roughness) */
CY_FN cfloat3 calculate_principled_diffuse_brdf(const CyClosure *sc, cfloat3 N, cfloat3 V, cfloat3 L, cfloat3 H,
                                                float *pdf)
{
  float NdotL = cmax(dot3(N, L), 0.0f);
  float NdotV = cmax(dot3(N, V), 0.0f);
  if (NdotL < 0 || NdotV < 0) {
    *pdf = 0.0f;
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float LdotH = dot3(L, H);
  float FL = schlick_fresnel(NdotL), FV = schlick_fresnel(NdotV);
  const float Fd90 = 0.5f + 2.0f * LdotH * LdotH * sc->alpha_x;
  float Fd = (1.0f * (1.0f - FL) + Fd90 * FL) * (1.0f * (1.0f - FV) + Fd90 * FV);
  float value = CY_1_PI_F * NdotL * Fd;
  return mk3(value, value, value);
}

CY_FN cfloat3 bsdf_principled_diffuse_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  cfloat3 N = sc->N;
  cfloat3 H = normalize3(add3(omega_in, I));
  if (dot3(N, omega_in) > 0.0f) {
    *pdf = fmaxf(dot3(N, omega_in), 0.0f) * CY_1_PI_F;
    return calculate_principled_diffuse_brdf(sc, N, I, omega_in, H, pdf);
  }
  *pdf = 0.0f;
  return mk3(0.0f, 0.0f, 0.0f);
}

CY_FN int bsdf_principled_diffuse_sample(const CyClosure *sc,
                                         cfloat3 Ng,
                                         cfloat3 I,
                                         float randu,
                                         float randv,
                                         cfloat3 *eval,
                                         cfloat3 *omega_in,
                                         float *pdf)
{
  cfloat3 N = sc->N;
  sample_cos_hemisphere(N, randu, randv, omega_in, pdf);
  if (dot3(Ng, *omega_in) > 0) {
    cfloat3 H = normalize3(add3(I, *omega_in));
    *eval = calculate_principled_diffuse_brdf(sc, N, I, *omega_in, H, pdf);
  }
  else {
    *pdf = 0.0f;
  }
  return LABEL_REFLECT | LABEL_DIFFUSE;
}

/* bsdf_principled_sheen.h:33-137 (alpha_x = avg_value) */
CY_FN float calculate_avg_principled_sheen_brdf(cfloat3 N, cfloat3 I)
{
  float NdotI = dot3(N, I);
  if (NdotI < 0.0f) {
    return 0.0f;
  }
  return schlick_fresnel(NdotI) * NdotI;
}

CY_FN cfloat3 calculate_principled_sheen_brdf(cfloat3 N, cfloat3 V, cfloat3 L, cfloat3 H, float *pdf)
{
  float NdotL = dot3(N, L);
  float NdotV = dot3(N, V);
  if (NdotL < 0 || NdotV < 0) {
    *pdf = 0.0f;
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float LdotH = dot3(L, H);
  float value = schlick_fresnel(LdotH) * NdotL;
  return mk3(value, value, value);
}

CY_FN int bsdf_principled_sheen_setup(const CySD *sd, CyClosure *b)
{
  b->type = CLOSURE_BSDF_PRINCIPLED_SHEEN_ID;
  b->alpha_x = calculate_avg_principled_sheen_brdf(b->N, sd->I);
  b->sample_weight *= b->alpha_x;
  return SD_BSDF | SD_BSDF_HAS_EVAL;
}

CY_FN cfloat3 bsdf_principled_sheen_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  cfloat3 N = sc->N;
  cfloat3 H = normalize3(add3(omega_in, I));
  if (dot3(N, omega_in) > 0.0f) {
    *pdf = fmaxf(dot3(N, omega_in), 0.0f) * CY_1_PI_F;
    return calculate_principled_sheen_brdf(N, I, omega_in, H, pdf);
  }
  *pdf = 0.0f;
  return mk3(0.0f, 0.0f, 0.0f);
}

CY_FN int bsdf_principled_sheen_sample(const CyClosure *sc,
                                       cfloat3 Ng,
                                       cfloat3 I,
                                       float randu,
                                       float randv,
                                       cfloat3 *eval,
                                       cfloat3 *omega_in,
                                       float *pdf)
{
  cfloat3 N = sc->N;
  sample_cos_hemisphere(N, randu, randv, omega_in, pdf);
  if (dot3(Ng, *omega_in) > 0) {
    cfloat3 H = normalize3(add3(I, *omega_in));
    *eval = calculate_principled_sheen_brdf(N, I, *omega_in, H, pdf);
  }
  else {
    *pdf = 0.0f;
  }
  return LABEL_REFLECT | LABEL_DIFFUSE;
}
#endif /* CY_CLOSURE_EXT: principled diffuse / sheen */

/* ---------------------------------------------------------------------------
 * Singular closures (bsdf_reflection.h:60-95, bsdf_refraction.h:62-111)
 */
CY_FN int bsdf_reflection_sample(
    const CyClosure *sc, cfloat3 Ng, cfloat3 I, cfloat3 *eval, cfloat3 *omega_in, float *pdf)
{
  cfloat3 N = sc->N;
  float cosNO = dot3(N, I);
  if (cosNO > 0) {
    *omega_in = sub3(mul3f(N, (2 * cosNO)), I);
    if (dot3(Ng, *omega_in) > 0) {
      *pdf = 1e6f;
      *eval = mk3(1e6f, 1e6f, 1e6f);
    }
  }
  return LABEL_REFLECT | LABEL_SINGULAR;
}

CY_FN int bsdf_refraction_sample(
    const CyClosure *sc, cfloat3 I, cfloat3 *eval, cfloat3 *omega_in, float *pdf)
{
  float m_eta = sc->ior;
  cfloat3 R, T;
  bool inside;
  float fresnel = fresnel_dielectric(m_eta, sc->N, I, &R, &T, &inside);
  if (!inside && fresnel != 1.0f) {
    *pdf = 1e6f;
    *eval = mk3(1e6f, 1e6f, 1e6f);
    *omega_in = T;
  }
  return LABEL_TRANSMIT | LABEL_SINGULAR;
}

/* ---------------------------------------------------------------------------
 * Microfacets (bsdf_microfacet.h)
 */
/* bsdf_microfacet.h:261-274 (fresnel / clearcoat tint of a reflection) */
CY_FN cfloat3 reflection_color(const CySD *sd, const CyClosure *sc, cfloat3 L, cfloat3 H)
{
  cfloat3 F = mk3(1.0f, 1.0f, 1.0f);
  bool use_fresnel = (sc->type == CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID ||
                      sc->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID);
#if CY_CLOSURE_EXT
  if (use_fresnel) {
    float F0 = fresnel_dielectric_cos(1.0f, sc->ior);
    F = interpolate_fresnel_color(L, H, sc->ior, F0, sd->closure[sc->extra].N);
  }
#endif
  return F;
}

/* bsdf_microfacet.h:270-277 */
CY_FN float D_GTR1(float NdotH, float alpha)
{
  if (alpha >= 1.0f) {
    return CY_1_PI_F;
  }
  float alpha2 = alpha * alpha;
  float t = 1.0f + (alpha2 - 1.0f) * NdotH * NdotH;
  return (alpha2 - 1.0f) / (CY_PI_F * cy_logf(alpha2) * t);
}

/* GGX: anisotropic D and the G1 of one direction (bsdf_microfacet.h:443-474) */
CY_FN float ggx_aniso_D(cfloat3 X, cfloat3 Y, cfloat3 Z, cfloat3 m, float alpha_x, float alpha_y, float alpha2)
{
  cfloat3 local_m = mk3(dot3(X, m), dot3(Y, m), dot3(Z, m));
  float slope_x = -local_m.x / (local_m.z * alpha_x);
  float slope_y = -local_m.y / (local_m.z * alpha_y);
  float slope_len = 1 + slope_x * slope_x + slope_y * slope_y;
  float cosThetaM = local_m.z;
  float cosThetaM2 = cosThetaM * cosThetaM;
  float cosThetaM4 = cosThetaM2 * cosThetaM2;
  return 1 / ((slope_len * slope_len) * CY_PI_F * alpha2 * cosThetaM4);
}
CY_FN float ggx_aniso_G1(cfloat3 X, cfloat3 Y, cfloat3 w, float cosNw, float alpha_x, float alpha_y)
{
  float tanTheta2 = (1 - cosNw * cosNw) / (cosNw * cosNw);
  float cosPhi = dot3(w, X);
  float sinPhi = dot3(w, Y);
  float alpha2w = (cosPhi * cosPhi) * (alpha_x * alpha_x) + (sinPhi * sinPhi) * (alpha_y * alpha_y);
  alpha2w /= cosPhi * cosPhi + sinPhi * sinPhi;
  return 2 / (1 + safe_sqrtf(1 + alpha2w * tanTheta2));
}

/* bsdf_microfacet.h:390-501 */
CY_FN cfloat3 bsdf_ggx_eval_reflect(const CySD *sd, const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  float alpha_x = sc->alpha_x;
  float alpha_y = sc->alpha_y;
  bool m_refractive = sc->type == CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID;
  cfloat3 N = sc->N;
  if (m_refractive || alpha_x * alpha_y <= 1e-7f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float cosNO = dot3(N, I);
  float cosNI = dot3(N, omega_in);
  if (cosNI > 0 && cosNO > 0) {
    cfloat3 m = normalize3(add3(omega_in, I));
    float alpha2 = alpha_x * alpha_y;
    float D, G1o, G1i;
    if (alpha_x == alpha_y) {
      float cosThetaM = dot3(N, m);
      float cosThetaM2 = cosThetaM * cosThetaM;
      float cosThetaM4 = cosThetaM2 * cosThetaM2;
      float tanThetaM2 = (1 - cosThetaM2) / cosThetaM2;
      if (sc->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID) {
        D = D_GTR1(cosThetaM, sc->alpha_x);
        alpha2 = 0.0625f;
      }
      else {
        D = alpha2 / (CY_PI_F * cosThetaM4 * (alpha2 + tanThetaM2) * (alpha2 + tanThetaM2));
      }
      G1o = 2 / (1 + safe_sqrtf(1 + alpha2 * (1 - cosNO * cosNO) / (cosNO * cosNO)));
      G1i = 2 / (1 + safe_sqrtf(1 + alpha2 * (1 - cosNI * cosNI) / (cosNI * cosNI)));
    }
#if CY_CLOSURE_EXT
    else {
      cfloat3 X, Y, Z = N;
      make_orthonormals_tangent(Z, sc->T, &X, &Y);
      D = ggx_aniso_D(X, Y, Z, m, alpha_x, alpha_y, alpha2);
      G1o = ggx_aniso_G1(X, Y, I, cosNO, alpha_x, alpha_y);
      G1i = ggx_aniso_G1(X, Y, omega_in, cosNI, alpha_x, alpha_y);
    }
#else
    else {
      return mk3(0.0f, 0.0f, 0.0f); /* anisotropic: extended closure set only */
    }
#endif
    float G = G1o * G1i;
    float common = D * 0.25f / cosNO;
    cfloat3 F = reflection_color(sd, sc, omega_in, m);
#if CY_CLOSURE_EXT
    if (sc->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID) {
      F = mul3f(F, 0.25f * sd->closure[sc->extra].alpha_x);
    }
#endif
    cfloat3 out = mul3f(mul3f(F, G), common);
    *pdf = G1o * common;
    return out;
  }
  return mk3(0.0f, 0.0f, 0.0f);
}

/* bsdf_microfacet.h:503-559 */
CY_FN cfloat3 bsdf_ggx_eval_transmit(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  float alpha_x = sc->alpha_x;
  float alpha_y = sc->alpha_y;
  float m_eta = sc->ior;
  bool m_refractive = sc->type == CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID;
  cfloat3 N = sc->N;
  if (!m_refractive || alpha_x * alpha_y <= 1e-7f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float cosNO = dot3(N, I);
  float cosNI = dot3(N, omega_in);
  if (cosNO <= 0 || cosNI >= 0) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  cfloat3 ht = neg3(add3(mul3f(omega_in, m_eta), I));
  cfloat3 Ht = normalize3(ht);
  float cosHO = dot3(Ht, I);
  float cosHI = dot3(Ht, omega_in);
  float alpha2 = alpha_x * alpha_y;
  float cosThetaM = dot3(N, Ht);
  float cosThetaM2 = cosThetaM * cosThetaM;
  float tanThetaM2 = (1 - cosThetaM2) / cosThetaM2;
  float cosThetaM4 = cosThetaM2 * cosThetaM2;
  float D = alpha2 / (CY_PI_F * cosThetaM4 * (alpha2 + tanThetaM2) * (alpha2 + tanThetaM2));
  float G1o = 2 / (1 + safe_sqrtf(1 + alpha2 * (1 - cosNO * cosNO) / (cosNO * cosNO)));
  float G1i = 2 / (1 + safe_sqrtf(1 + alpha2 * (1 - cosNI * cosNI) / (cosNI * cosNI)));
  float G = G1o * G1i;
  float Ht2 = dot3(ht, ht);
  float common = D * (m_eta * m_eta) / (cosNO * Ht2);
  float out = G * fabsf(cosHI * cosHO) * common;
  *pdf = G1o * fabsf(cosHO * cosHI) * common;
  return mk3(out, out, out);
}

/* bsdf_microfacet.h:143-253 (GGX visible-normal sampling). */
CY_FN void microfacet_ggx_sample_slopes(const float cos_theta_i,
                                        const float sin_theta_i,
                                        float randu,
                                        float randv,
                                        float *slope_x,
                                        float *slope_y,
                                        float *G1i)
{
  if (cos_theta_i >= 0.99999f) {
    const float r = sqrtf(randu / (1.0f - randu));
    const float phi = CY_2PI_F * randv;
    *slope_x = r * cy_cosf(phi);
    *slope_y = r * cy_sinf(phi);
    *G1i = 1.0f;
    return;
  }
  const float tan_theta_i = sin_theta_i / cos_theta_i;
  const float G1_inv = 0.5f * (1.0f + safe_sqrtf(1.0f + tan_theta_i * tan_theta_i));
  *G1i = 1.0f / G1_inv;
  const float A = 2.0f * randu * G1_inv - 1.0f;
  const float AA = A * A;
  const float tmp = 1.0f / (AA - 1.0f);
  const float B = tan_theta_i;
  const float BB = B * B;
  const float D = safe_sqrtf(BB * (tmp * tmp) - (AA - BB) * tmp);
  const float slope_x_1 = B * tmp - D;
  const float slope_x_2 = B * tmp + D;
  *slope_x = (A < 0.0f || slope_x_2 * tan_theta_i > 1.0f) ? slope_x_1 : slope_x_2;
  float S;
  if (randv > 0.5f) {
    S = 1.0f;
    randv = 2.0f * (randv - 0.5f);
  }
  else {
    S = -1.0f;
    randv = 2.0f * (0.5f - randv);
  }
  const float z = (randv * (randv * (randv * 0.27385f - 0.73369f) + 0.46341f)) /
                  (randv * (randv * (randv * 0.093073f + 0.309420f) - 1.000000f) + 0.597999f);
  *slope_y = S * z * safe_sqrtf(1.0f + (*slope_x) * (*slope_x));
}

#if CY_CLOSURE_EXT
/* bsdf_microfacet.h:56-130, CPU branch: slope_x from the precomputed table */
CY_FN void microfacet_beckmann_sample_slopes(const CyGlobals *kg,
                                             const float cos_theta_i,
                                             const float sin_theta_i,
                                             float randu,
                                             float randv,
                                             float *slope_x,
                                             float *slope_y,
                                             float *G1i)
{
  if (cos_theta_i >= 0.99999f) {
    const float r = sqrtf(-cy_logf(randu));
    const float phi = CY_2PI_F * randv;
    *slope_x = r * cy_cosf(phi);
    *slope_y = r * cy_sinf(phi);
    *G1i = 1.0f;
    return;
  }
  const float tan_theta_i = sin_theta_i / cos_theta_i;
  const float inv_a = tan_theta_i;
  const float cot_theta_i = 1.0f / tan_theta_i;
  const float erf_a = fast_erff(cot_theta_i);
  const float exp_a2 = cy_expf(-cot_theta_i * cot_theta_i);
  const float SQRT_PI_INV = 0.56418958354f;
  const float Lambda = 0.5f * (erf_a - 1.0f) + (0.5f * SQRT_PI_INV) * (exp_a2 * inv_a);
  const float G1 = 1.0f / (1.0f + Lambda);
  *G1i = G1;
  *slope_x = lookup_table_read_2D(kg, randu, cos_theta_i, KD->tables.beckmann_offset, CY_BECKMANN_TABLE_SIZE,
                                  CY_BECKMANN_TABLE_SIZE);
  *slope_y = fast_ierff(2.0f * randv - 1.0f);
}
#endif

/* bsdf_microfacet.h:190-252 */
CY_FN cfloat3 microfacet_sample_stretched(const CyGlobals *kg,
                                          const cfloat3 omega_i,
                                          const float alpha_x,
                                          const float alpha_y,
                                          const float randu,
                                          const float randv,
                                          bool beckmann,
                                          float *G1i)
{
  cfloat3 omega_i_ = mk3(alpha_x * omega_i.x, alpha_y * omega_i.y, omega_i.z);
  omega_i_ = normalize3(omega_i_);
  float costheta_ = 1.0f;
  float sintheta_ = 0.0f;
  float cosphi_ = 1.0f;
  float sinphi_ = 0.0f;
  if (omega_i_.z < 0.99999f) {
    costheta_ = omega_i_.z;
    sintheta_ = safe_sqrtf(1.0f - costheta_ * costheta_);
    float invlen = 1.0f / sintheta_;
    cosphi_ = omega_i_.x * invlen;
    sinphi_ = omega_i_.y * invlen;
  }
  float slope_x, slope_y;
#if CY_CLOSURE_EXT
  if (beckmann) {
    microfacet_beckmann_sample_slopes(kg, costheta_, sintheta_, randu, randv, &slope_x, &slope_y, G1i);
  }
  else
#endif
  {
    microfacet_ggx_sample_slopes(costheta_, sintheta_, randu, randv, &slope_x, &slope_y, G1i);
  }
  float tmp = cosphi_ * slope_x - sinphi_ * slope_y;
  slope_y = sinphi_ * slope_x + cosphi_ * slope_y;
  slope_x = tmp;
  slope_x = alpha_x * slope_x;
  slope_y = alpha_y * slope_y;
  return normalize3(mk3(-slope_x, -slope_y, 1.0f));
}

/* bsdf_microfacet.h:561-788 */
CY_FN int bsdf_ggx_sample(const CyGlobals *kg,
                          const CySD *sd,
                          const CyClosure *sc,
                          cfloat3 Ng,
                          cfloat3 I,
                          float randu,
                          float randv,
                          cfloat3 *eval,
                          cfloat3 *omega_in,
                          float *pdf,
                          cfloat3 *m_out = nullptr)
{
  float alpha_x = sc->alpha_x;
  float alpha_y = sc->alpha_y;
  bool m_refractive = sc->type == CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID;
  cfloat3 N = sc->N;
  int label;
  float cosNO = dot3(N, I);
  if (cosNO > 0) {
    cfloat3 X, Y, Z = N;
#if CY_CLOSURE_EXT
    if (alpha_x == alpha_y) {
      make_orthonormals(Z, &X, &Y);
    }
    else {
      make_orthonormals_tangent(Z, sc->T, &X, &Y);
    }
#else
    make_orthonormals(Z, &X, &Y);
#endif
    cfloat3 local_I = mk3(dot3(X, I), dot3(Y, I), cosNO);
    cfloat3 local_m;
    float G1o;
    local_m = microfacet_sample_stretched(kg, local_I, alpha_x, alpha_y, randu, randv, false, &G1o);
    cfloat3 m = add3(add3(mul3f(X, local_m.x), mul3f(Y, local_m.y)), mul3f(Z, local_m.z));
    if (m_out) {
      *m_out = m;
    }
    float cosThetaM = local_m.z;
    if (!m_refractive) {
      float cosMO = dot3(m, I);
      label = LABEL_REFLECT | LABEL_GLOSSY;
      if (cosMO > 0) {
        *omega_in = sub3(mul3f(m, 2 * cosMO), I);
        if (dot3(Ng, *omega_in) > 0) {
          if (alpha_x * alpha_y <= 1e-7f) {
            *pdf = 1e6f;
            *eval = mk3(1e6f, 1e6f, 1e6f);
            bool use_fresnel = (sc->type == CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID ||
                                sc->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID);
            if (use_fresnel) {
              *eval = mul3(*eval, reflection_color(sd, sc, *omega_in, m));
            }
            label = LABEL_REFLECT | LABEL_SINGULAR;
          }
          else {
            float alpha2 = alpha_x * alpha_y;
            float D, G1i;
            if (alpha_x == alpha_y) {
              float cosThetaM2 = cosThetaM * cosThetaM;
              float cosThetaM4 = cosThetaM2 * cosThetaM2;
              float tanThetaM2 = 1 / (cosThetaM2)-1;
              float cosNI = dot3(N, *omega_in);
              if (sc->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID) {
                D = D_GTR1(cosThetaM, sc->alpha_x);
                alpha2 = 0.0625f;
                G1o = 2 / (1 + safe_sqrtf(1 + alpha2 * (1 - cosNO * cosNO) / (cosNO * cosNO)));
              }
              else {
                D = alpha2 / (CY_PI_F * cosThetaM4 * (alpha2 + tanThetaM2) * (alpha2 + tanThetaM2));
              }
              G1i = 2 / (1 + safe_sqrtf(1 + alpha2 * (1 - cosNI * cosNI) / (cosNI * cosNI)));
            }
            else {
              D = ggx_aniso_D(X, Y, Z, m, alpha_x, alpha_y, alpha2);
              float cosNI = dot3(N, *omega_in);
              G1i = ggx_aniso_G1(X, Y, *omega_in, cosNI, alpha_x, alpha_y);
            }
            float common = (G1o * D) * 0.25f / cosNO;
            *pdf = common;
            cfloat3 F = reflection_color(sd, sc, *omega_in, m);
            /* G1i * common * F: scalar * scalar first, then the float3 product. */
            *eval = mul3f(F, G1i * common);
          }
#if CY_CLOSURE_EXT
          if (sc->type == CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID) {
            *eval = mul3f(*eval, 0.25f * sd->closure[sc->extra].alpha_x);
          }
#endif
        }
      }
    }
    else {
      label = LABEL_TRANSMIT | LABEL_GLOSSY;
      cfloat3 R, T;
      float m_eta = sc->ior, fresnel;
      bool inside;
      fresnel = fresnel_dielectric(m_eta, m, I, &R, &T, &inside);
      if (!inside && fresnel != 1.0f) {
        *omega_in = T;
        if (alpha_x * alpha_y <= 1e-7f || fabsf(m_eta - 1.0f) < 1e-4f) {
          *pdf = 1e6f;
          *eval = mk3(1e6f, 1e6f, 1e6f);
          label = LABEL_TRANSMIT | LABEL_SINGULAR;
        }
        else {
          float alpha2 = alpha_x * alpha_y;
          float cosThetaM2 = cosThetaM * cosThetaM;
          float cosThetaM4 = cosThetaM2 * cosThetaM2;
          float tanThetaM2 = 1 / (cosThetaM2)-1;
          float D = alpha2 / (CY_PI_F * cosThetaM4 * (alpha2 + tanThetaM2) * (alpha2 + tanThetaM2));
          float cosNI = dot3(N, *omega_in);
          float G1i = 2 / (1 + safe_sqrtf(1 + alpha2 * (1 - cosNI * cosNI) / (cosNI * cosNI)));
          float cosHI = dot3(m, *omega_in);
          float cosHO = dot3(m, I);
          float Ht2 = m_eta * cosHI + cosHO;
          Ht2 *= Ht2;
          float common = (G1o * D) * (m_eta * m_eta) / (cosNO * Ht2);
          float out = G1i * fabsf(cosHI * cosHO) * common;
          *pdf = cosHO * fabsf(cosHI) * common;
          *eval = mk3(out, out, out);
        }
      }
    }
  }
  else {
    label = (m_refractive) ? LABEL_TRANSMIT | LABEL_GLOSSY : LABEL_REFLECT | LABEL_GLOSSY;
  }
  return label;
}

#if CY_CLOSURE_EXT
/* bsdf_microfacet.h:823-852 */
CY_FN float bsdf_beckmann_G1(float alpha, float cos_n)
{
  cos_n *= cos_n;
  float invA = alpha * safe_sqrtf((1.0f - cos_n) / cos_n);
  if (invA < 0.625f) {
    return 1.0f;
  }
  float a = 1.0f / invA;
  return ((2.181f * a + 3.535f) * a) / ((2.577f * a + 2.276f) * a + 1.0f);
}
CY_FN float bsdf_beckmann_aniso_G1(float alpha_x, float alpha_y, float cos_n, float cos_phi, float sin_phi)
{
  cos_n *= cos_n;
  sin_phi *= sin_phi;
  cos_phi *= cos_phi;
  alpha_x *= alpha_x;
  alpha_y *= alpha_y;
  float alphaO2 = (cos_phi * alpha_x + sin_phi * alpha_y) / (cos_phi + sin_phi);
  float invA = safe_sqrtf(alphaO2 * (1 - cos_n) / cos_n);
  if (invA < 0.625f) {
    return 1.0f;
  }
  float a = 1.0f / invA;
  return ((2.181f * a + 3.535f) * a) / ((2.577f * a + 2.276f) * a + 1.0f);
}
CY_FN float beckmann_aniso_D(cfloat3 X, cfloat3 Y, cfloat3 Z, cfloat3 m, float alpha_x, float alpha_y, float alpha2)
{
  cfloat3 local_m = mk3(dot3(X, m), dot3(Y, m), dot3(Z, m));
  float slope_x = -local_m.x / (local_m.z * alpha_x);
  float slope_y = -local_m.y / (local_m.z * alpha_y);
  float cosThetaM = local_m.z;
  float cosThetaM2 = cosThetaM * cosThetaM;
  float cosThetaM4 = cosThetaM2 * cosThetaM2;
  return cy_expf(-slope_x * slope_x - slope_y * slope_y) / (CY_PI_F * alpha2 * cosThetaM4);
}

/* bsdf_microfacet.h:854-920 */
CY_FN cfloat3 bsdf_beckmann_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  float alpha_x = sc->alpha_x;
  float alpha_y = sc->alpha_y;
  bool m_refractive = sc->type == CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID;
  cfloat3 N = sc->N;
  if (m_refractive || alpha_x * alpha_y <= 1e-7f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float cosNO = dot3(N, I);
  float cosNI = dot3(N, omega_in);
  if (cosNO > 0 && cosNI > 0) {
    cfloat3 m = normalize3(add3(omega_in, I));
    float alpha2 = alpha_x * alpha_y;
    float D, G1o, G1i;
    if (alpha_x == alpha_y) {
      float cosThetaM = dot3(N, m);
      float cosThetaM2 = cosThetaM * cosThetaM;
      float tanThetaM2 = (1 - cosThetaM2) / cosThetaM2;
      float cosThetaM4 = cosThetaM2 * cosThetaM2;
      D = cy_expf(-tanThetaM2 / alpha2) / (CY_PI_F * alpha2 * cosThetaM4);
      G1o = bsdf_beckmann_G1(alpha_x, cosNO);
      G1i = bsdf_beckmann_G1(alpha_x, cosNI);
    }
    else {
      cfloat3 X, Y, Z = N;
      make_orthonormals_tangent(Z, sc->T, &X, &Y);
      D = beckmann_aniso_D(X, Y, Z, m, alpha_x, alpha_y, alpha2);
      G1o = bsdf_beckmann_aniso_G1(alpha_x, alpha_y, cosNO, dot3(I, X), dot3(I, Y));
      G1i = bsdf_beckmann_aniso_G1(alpha_x, alpha_y, cosNI, dot3(omega_in, X), dot3(omega_in, Y));
    }
    float G = G1o * G1i;
    float common = D * 0.25f / cosNO;
    float out = G * common;
    *pdf = G1o * common;
    return mk3(out, out, out);
  }
  return mk3(0.0f, 0.0f, 0.0f);
}

/* bsdf_microfacet.h:922-975 */
CY_FN cfloat3 bsdf_beckmann_eval_transmit(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  float alpha_x = sc->alpha_x;
  float alpha_y = sc->alpha_y;
  float m_eta = sc->ior;
  bool m_refractive = sc->type == CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID;
  cfloat3 N = sc->N;
  if (!m_refractive || alpha_x * alpha_y <= 1e-7f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  float cosNO = dot3(N, I);
  float cosNI = dot3(N, omega_in);
  if (cosNO <= 0 || cosNI >= 0) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  cfloat3 ht = neg3(add3(mul3f(omega_in, m_eta), I));
  cfloat3 Ht = normalize3(ht);
  float cosHO = dot3(Ht, I);
  float cosHI = dot3(Ht, omega_in);
  float alpha2 = alpha_x * alpha_y;
  float cosThetaM = cmin(dot3(N, Ht), 1.0f);
  float cosThetaM2 = cosThetaM * cosThetaM;
  float tanThetaM2 = (1 - cosThetaM2) / cosThetaM2;
  float cosThetaM4 = cosThetaM2 * cosThetaM2;
  float D = cy_expf(-tanThetaM2 / alpha2) / (CY_PI_F * alpha2 * cosThetaM4);
  float G1o = bsdf_beckmann_G1(alpha_x, cosNO);
  float G1i = bsdf_beckmann_G1(alpha_x, cosNI);
  float G = G1o * G1i;
  float Ht2 = dot3(ht, ht);
  float common = D * (m_eta * m_eta) / (cosNO * Ht2);
  float out = G * fabsf(cosHI * cosHO) * common;
  *pdf = G1o * fabsf(cosHO * cosHI) * common;
  return mk3(out, out, out);
}

/* bsdf_microfacet.h:988-1175.  The reference stretches by (alpha_x, alpha_x)
 * here, also for anisotropic closures; kept. */
CY_FN int bsdf_beckmann_sample(const CyGlobals *kg,
                               const CyClosure *sc,
                               cfloat3 Ng,
                               cfloat3 I,
                               float randu,
                               float randv,
                               cfloat3 *eval,
                               cfloat3 *omega_in,
                               float *pdf,
                          cfloat3 *m_out = nullptr)
{
  float alpha_x = sc->alpha_x;
  float alpha_y = sc->alpha_y;
  bool m_refractive = sc->type == CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID;
  cfloat3 N = sc->N;
  int label;
  float cosNO = dot3(N, I);
  if (cosNO > 0) {
    cfloat3 X, Y, Z = N;
    if (alpha_x == alpha_y) {
      make_orthonormals(Z, &X, &Y);
    }
    else {
      make_orthonormals_tangent(Z, sc->T, &X, &Y);
    }
    cfloat3 local_I = mk3(dot3(X, I), dot3(Y, I), cosNO);
    float G1o;
    cfloat3 local_m = microfacet_sample_stretched(kg, local_I, alpha_x, alpha_x, randu, randv, true, &G1o);
    cfloat3 m = add3(add3(mul3f(X, local_m.x), mul3f(Y, local_m.y)), mul3f(Z, local_m.z));
    if (m_out) {
      *m_out = m;
    }
    float cosThetaM = local_m.z;
    if (!m_refractive) {
      label = LABEL_REFLECT | LABEL_GLOSSY;
      float cosMO = dot3(m, I);
      if (cosMO > 0) {
        *omega_in = sub3(mul3f(m, 2 * cosMO), I);
        if (dot3(Ng, *omega_in) > 0) {
          if (alpha_x * alpha_y <= 1e-7f) {
            *pdf = 1e6f;
            *eval = mk3(1e6f, 1e6f, 1e6f);
            label = LABEL_REFLECT | LABEL_SINGULAR;
          }
          else {
            float alpha2 = alpha_x * alpha_y;
            float D, G1i;
            if (alpha_x == alpha_y) {
              float cosThetaM2 = cosThetaM * cosThetaM;
              float cosThetaM4 = cosThetaM2 * cosThetaM2;
              float tanThetaM2 = 1 / (cosThetaM2)-1;
              D = cy_expf(-tanThetaM2 / alpha2) / (CY_PI_F * alpha2 * cosThetaM4);
              float cosNI = dot3(N, *omega_in);
              G1i = bsdf_beckmann_G1(alpha_x, cosNI);
            }
            else {
              D = beckmann_aniso_D(X, Y, Z, m, alpha_x, alpha_y, alpha2);
              G1i = bsdf_beckmann_aniso_G1(alpha_x, alpha_y, dot3(*omega_in, N), dot3(*omega_in, X),
                                           dot3(*omega_in, Y));
            }
            float G = G1o * G1i;
            float common = D * 0.25f / cosNO;
            float out = G * common;
            *pdf = G1o * common;
            *eval = mk3(out, out, out);
          }
        }
      }
    }
    else {
      label = LABEL_TRANSMIT | LABEL_GLOSSY;
      cfloat3 R, T;
      float m_eta = sc->ior, fresnel;
      bool inside;
      fresnel = fresnel_dielectric(m_eta, m, I, &R, &T, &inside);
      if (!inside && fresnel != 1.0f) {
        *omega_in = T;
        if (alpha_x * alpha_y <= 1e-7f || fabsf(m_eta - 1.0f) < 1e-4f) {
          *pdf = 1e6f;
          *eval = mk3(1e6f, 1e6f, 1e6f);
          label = LABEL_TRANSMIT | LABEL_SINGULAR;
        }
        else {
          float alpha2 = alpha_x * alpha_y;
          float cosThetaM2 = cosThetaM * cosThetaM;
          float cosThetaM4 = cosThetaM2 * cosThetaM2;
          float tanThetaM2 = 1 / (cosThetaM2)-1;
          float D = cy_expf(-tanThetaM2 / alpha2) / (CY_PI_F * alpha2 * cosThetaM4);
          float cosNI = dot3(N, *omega_in);
          float G1i = bsdf_beckmann_G1(alpha_x, cosNI);
          float G = G1o * G1i;
          float cosHI = dot3(m, *omega_in);
          float cosHO = dot3(m, I);
          float Ht2 = m_eta * cosHI + cosHO;
          Ht2 *= Ht2;
          float common = D * (m_eta * m_eta) / (cosNO * Ht2);
          float out = G * fabsf(cosHI * cosHO) * common;
          *pdf = G1o * cosHO * fabsf(cosHI) * common;
          *eval = mk3(out, out, out);
        }
      }
    }
  }
  else {
    label = (m_refractive) ? LABEL_TRANSMIT | LABEL_GLOSSY : LABEL_REFLECT | LABEL_GLOSSY;
  }
  return label;
}

/* bsdf_ashikhmin_shirley.h:47-120 (isotropic; svm rejects anisotropic, whose
 * sampling needs libm tanf) */
CY_FN float bsdf_ashikhmin_shirley_roughness_to_exponent(float roughness)
{
  return 2.0f / (roughness * roughness) - 2.0f;
}

CY_FN cfloat3 bsdf_ashikhmin_shirley_eval_reflect(const CyClosure *sc, cfloat3 I, cfloat3 omega_in, float *pdf)
{
  cfloat3 N = sc->N;
  float NdotI = dot3(N, I);
  float NdotO = dot3(N, omega_in);
  float out = 0.0f;
  if (fmaxf(sc->alpha_x, sc->alpha_y) <= 1e-4f) {
    return mk3(0.0f, 0.0f, 0.0f);
  }
  if (NdotI > 0.0f && NdotO > 0.0f) {
    NdotI = fmaxf(NdotI, 1e-6f);
    NdotO = fmaxf(NdotO, 1e-6f);
    cfloat3 H = normalize3(add3(omega_in, I));
    float HdotI = fmaxf(fabsf(dot3(H, I)), 1e-6f);
    float HdotN = fmaxf(dot3(H, N), 1e-6f);
    float pump = 1.0f / fmaxf(1e-6f, (HdotI * fmaxf(NdotO, NdotI)));
    float n_x = bsdf_ashikhmin_shirley_roughness_to_exponent(sc->alpha_x);
    float n_y = bsdf_ashikhmin_shirley_roughness_to_exponent(sc->alpha_y);
    if (n_x == n_y) {
      float e = n_x;
      float lobe = cy_powf(HdotN, e);
      float norm = (n_x + 1.0f) / (8.0f * CY_PI_F);
      out = NdotO * norm * lobe * pump;
      *pdf = norm * lobe / HdotI;
    }
    else {
      cfloat3 X, Y;
      make_orthonormals_tangent(N, sc->T, &X, &Y);
      float HdotX = dot3(H, X);
      float HdotY = dot3(H, Y);
      float lobe;
      if (HdotN < 1.0f) {
        float e = (n_x * HdotX * HdotX + n_y * HdotY * HdotY) / (1.0f - HdotN * HdotN);
        lobe = cy_powf(HdotN, e);
      }
      else {
        lobe = 1.0f;
      }
      float norm = sqrtf((n_x + 1.0f) * (n_y + 1.0f)) / (8.0f * CY_PI_F);
      out = NdotO * norm * lobe * pump;
      *pdf = norm * lobe / HdotI;
    }
  }
  return mk3(out, out, out);
}

/* bsdf_ashikhmin_shirley.h:131-240, isotropic sampling */
CY_FN int bsdf_ashikhmin_shirley_sample(const CyClosure *sc,
                                        cfloat3 I,
                                        float randu,
                                        float randv,
                                        cfloat3 *eval,
                                        cfloat3 *omega_in,
                                        float *pdf,
                                        uint *err)
{
  cfloat3 N = sc->N;
  int label = LABEL_REFLECT | LABEL_GLOSSY;
  float NdotI = dot3(N, I);
  if (NdotI > 0.0f) {
    float n_x = bsdf_ashikhmin_shirley_roughness_to_exponent(sc->alpha_x);
    float n_y = bsdf_ashikhmin_shirley_roughness_to_exponent(sc->alpha_y);
    if (n_x != n_y) {
      cy_set_error(err, CY_ERR_CLOSURE, 1000 + CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID);
      return label;
    }
    cfloat3 X, Y;
    make_orthonormals(N, &X, &Y);
    float phi = CY_2PI_F * randu;
    float cos_theta = cy_powf(randv, 1.0f / (n_x + 1.0f));
    float sin_theta = sqrtf(fmaxf(0.0f, 1.0f - cos_theta * cos_theta));
    float cos_phi = cy_cosf(phi);
    float sin_phi = cy_sinf(phi);
    cfloat3 h = mk3(sin_theta * cos_phi, sin_theta * sin_phi, cos_theta);
    cfloat3 H = add3(add3(mul3f(X, h.x), mul3f(Y, h.y)), mul3f(N, h.z));
    float HdotI = dot3(H, I);
    if (HdotI < 0.0f) {
      H = neg3(H);
    }
    *omega_in = add3(neg3(I), mul3f(H, (2.0f * HdotI)));
    if (fmaxf(sc->alpha_x, sc->alpha_y) <= 1e-4f) {
      *pdf = 1e6f;
      *eval = mk3(1e6f, 1e6f, 1e6f);
      label = LABEL_REFLECT | LABEL_SINGULAR;
    }
    else {
      *eval = bsdf_ashikhmin_shirley_eval_reflect(sc, I, *omega_in, pdf);
    }
  }
  return label;
}

#endif /* CY_CLOSURE_EXT: Beckmann, Ashikhmin-Shirley */

#if CY_CLOSURE_EXT
#  include "cy_microfacet_multi.h"
#  include "cy_hair.h"
#endif

/* ---------------------------------------------------------------------------
 * Dispatch (bsdf.h)
 */
CY_FN float bsdf_get_specular_roughness_squared(const CyClosure *sc)
{
  if (CLOSURE_IS_BSDF_SINGULAR(sc->type)) {
    return 0.0f;
  }
  if (CLOSURE_IS_BSDF_MICROFACET(sc->type)) {
    return sc->alpha_x * sc->alpha_y;
  }
  return 1.0f;
}

/* bsdf.h:82-98 */
CY_FN float bump_shadowing_term(cfloat3 Ng, cfloat3 N, cfloat3 I)
{
  float g = safe_divide(dot3(Ng, I), dot3(N, I) * dot3(Ng, N));
  if (g >= 1.0f) {
    return 1.0f;
  }
  if (g < 0.0f) {
    return 0.0f;
  }
  float g2 = sqr(g);
  return -g2 * g + g2 + g;
}

#if CY_CLOSURE_EXT
/* The differentials of a sampled direction follow from the shading point's
 * dI by one of a few rules (the __RAY_DIFFERENTIALS__ lines of each closure's
 * sample function): the mirror about n (bsdf_diffuse.h:104), its negation
 * (bsdf_diffuse.h:166), -dI (bsdf_transparent.h:117), fresnel_dielectric's
 * refracted differential (bsdf_util.h:92) or zero (total internal reflection). */
enum { CY_DIFF_ZERO = 0, CY_DIFF_MIRROR, CY_DIFF_NEG_MIRROR, CY_DIFF_NEG, CY_DIFF_REFRACT };
typedef struct CyDiffRule {
  int kind;
  cfloat3 n;
  float neta, k; /* refraction: -(neta * dI) + (k * dot(dI, n)) * n */
} CyDiffRule;

CY_FN cfloat3 diff_rule_apply(const CyDiffRule &r, cfloat3 dI)
{
  switch (r.kind) {
    case CY_DIFF_MIRROR:
      return sub3(mul3f(r.n, 2 * dot3(r.n, dI)), dI);
    case CY_DIFF_NEG_MIRROR:
      return neg3(sub3(mul3f(r.n, 2 * dot3(r.n, dI)), dI));
    case CY_DIFF_NEG:
      return neg3(dI);
    case CY_DIFF_REFRACT:
      return add3(neg3(mul3f(dI, r.neta)), mul3f(r.n, r.k * dot3(dI, r.n)));
    default:
      return mk3(0.0f, 0.0f, 0.0f);
  }
}

CY_FN void diff_rule_set(CyDiffRule *r, int kind, cfloat3 n)
{
  r->kind = kind;
  r->n = n;
}

/* fresnel_dielectric's dR (reflect) or dT (bsdf_util.h:53-93) */
CY_FN void diff_rule_fresnel(CyDiffRule *r, float eta, cfloat3 N, cfloat3 I, bool reflect)
{
  float cos = dot3(N, I), neta;
  cfloat3 Nn;
  if (cos > 0) {
    neta = 1 / eta;
    Nn = N;
  }
  else {
    cos = -cos;
    neta = eta;
    Nn = neg3(N);
  }
  r->n = Nn;
  if (reflect) {
    r->kind = CY_DIFF_MIRROR;
    return;
  }
  const float arg = 1 - (neta * neta * (1 - (cos * cos)));
  if (arg < 0) {
    r->kind = CY_DIFF_ZERO;
    return;
  }
  const float dnp = cmax(sqrtf(arg), 1e-7f);
  r->kind = CY_DIFF_REFRACT;
  r->neta = neta;
  r->k = neta - neta * neta * cos / dnp;
}
#endif

/* bsdf.h:113-489.  The shadow-terminator offset (object frequency multiplier
 * > 1) is rejected at load_kernels.  With ray differentials the sampled
 * direction's rule comes out in *rule. */
CY_FN int bsdf_sample(const CyGlobals *kg,
                      const CySD *sd,
                      const CyClosure *sc,
                      float randu,
                      float randv,
                      cfloat3 *eval,
                      cfloat3 *omega_in,
                      float *pdf,
                      uint *err
#if CY_CLOSURE_EXT
                      ,
                      CyDiffRule *rule = nullptr
#endif
)
{
  int label;
  /* bsdf.h:124-126: curves sample against the closure's smooth normal */
  const cfloat3 Ng = (sd->type & PRIMITIVE_ALL_CURVE) ? sc->N : sd->Ng;
  switch (sc->type) {
    case CLOSURE_BSDF_DIFFUSE_ID:
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_BSSRDF_ID: /* the diffuse closure replacing a BSSRDF after its scatter step */
#endif
      label = bsdf_diffuse_sample(sc, Ng, randu, randv, eval, omega_in, pdf);
      break;
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_OREN_NAYAR_ID:
      label = bsdf_oren_nayar_sample(sc, Ng, sd->I, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_TRANSLUCENT_ID:
      label = bsdf_translucent_sample(sc, Ng, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_PRINCIPLED_DIFFUSE_ID:
    case CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID:
      label = bsdf_principled_diffuse_sample(sc, Ng, sd->I, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_PRINCIPLED_SHEEN_ID:
      label = bsdf_principled_sheen_sample(sc, Ng, sd->I, randu, randv, eval, omega_in, pdf);
      break;
#endif
    case CLOSURE_BSDF_REFLECTION_ID:
      label = bsdf_reflection_sample(sc, Ng, sd->I, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_REFRACTION_ID:
      label = bsdf_refraction_sample(sc, sd->I, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_TRANSPARENT_ID:
      /* bsdf_transparent.h:89-110: straight through */
      *omega_in = neg3(sd->I);
      *pdf = 1.0f;
      *eval = mk3(1.0f, 1.0f, 1.0f);
      label = LABEL_TRANSMIT | LABEL_TRANSPARENT;
      break;
    case CLOSURE_BSDF_MICROFACET_GGX_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID:
    case CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID:
#if CY_CLOSURE_EXT
      if (rule) {
        cfloat3 m = mk3(0.0f, 0.0f, 0.0f);
        label = bsdf_ggx_sample(kg, sd, sc, Ng, sd->I, randu, randv, eval, omega_in, pdf, &m);
        /* bsdf_microfacet.h:702, 720-740 */
        if (sc->type == CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID) {
          diff_rule_fresnel(rule, sc->ior, m, sd->I, false);
        }
        else {
          diff_rule_set(rule, CY_DIFF_MIRROR, m);
        }
        break;
      }
#endif
      label = bsdf_ggx_sample(kg, sd, sc, Ng, sd->I, randu, randv, eval, omega_in, pdf);
      break;
#if CY_CLOSURE_EXT
    case CLOSURE_BSDF_MICROFACET_BECKMANN_ID:
    case CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID:
      if (rule) {
        cfloat3 m = mk3(0.0f, 0.0f, 0.0f);
        label = bsdf_beckmann_sample(kg, sc, Ng, sd->I, randu, randv, eval, omega_in, pdf, &m);
        /* bsdf_microfacet.h:1093, 1111-1131 */
        if (sc->type == CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID) {
          diff_rule_fresnel(rule, sc->ior, m, sd->I, false);
        }
        else {
          diff_rule_set(rule, CY_DIFF_MIRROR, m);
        }
        break;
      }
      label = bsdf_beckmann_sample(kg, sc, Ng, sd->I, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID:
      label = bsdf_ashikhmin_shirley_sample(sc, sd->I, randu, randv, eval, omega_in, pdf, err);
      break;
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID:
      label = bsdf_microfacet_multi_ggx_sample(sd, sc, sd->I, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID:
    case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID:
      label = bsdf_microfacet_multi_ggx_glass_sample(sd, sc, sd->I, randu, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_ASHIKHMIN_VELVET_ID:
      label = bsdf_ashikhmin_velvet_sample(sc, Ng, sd->I, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_DIFFUSE_TOON_ID:
      label = bsdf_diffuse_toon_sample(sc, Ng, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_GLOSSY_TOON_ID:
      label = bsdf_glossy_toon_sample(sc, Ng, sd->I, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_HAIR_REFLECTION_ID:
    case CLOSURE_BSDF_HAIR_TRANSMISSION_ID:
      label = bsdf_hair_sample(sc, sd->I, randu, randv, eval, omega_in, pdf);
      break;
    case CLOSURE_BSDF_HAIR_PRINCIPLED_ID:
      label = bsdf_principled_hair_sample(sd, sc, randu, randv, eval, omega_in, pdf);
      break;
#endif
    case CLOSURE_NONE_ID:
      label = LABEL_NONE;
      break;
    default:
      cy_set_error(err, CY_ERR_CLOSURE, (uint)sc->type);
      label = LABEL_NONE;
      break;
  }
#if CY_CLOSURE_EXT
  if (rule) {
    switch (sc->type) {
      case CLOSURE_BSDF_DIFFUSE_ID:
      case CLOSURE_BSDF_BSSRDF_ID:
      case CLOSURE_BSDF_OREN_NAYAR_ID:
      case CLOSURE_BSDF_REFLECTION_ID:
      case CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID:
      case CLOSURE_BSDF_ASHIKHMIN_VELVET_ID:
      case CLOSURE_BSDF_DIFFUSE_TOON_ID:
      case CLOSURE_BSDF_GLOSSY_TOON_ID:
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID:
        diff_rule_set(rule, CY_DIFF_MIRROR, sc->N);
        break;
      case CLOSURE_BSDF_TRANSLUCENT_ID:
      case CLOSURE_BSDF_PRINCIPLED_DIFFUSE_ID:
      case CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID:
      case CLOSURE_BSDF_PRINCIPLED_SHEEN_ID:
        diff_rule_set(rule, CY_DIFF_NEG_MIRROR, sc->N);
        break;
      case CLOSURE_BSDF_TRANSPARENT_ID:
        rule->kind = CY_DIFF_NEG;
        break;
      case CLOSURE_BSDF_REFRACTION_ID:
        diff_rule_fresnel(rule, sc->ior, sc->N, sd->I, false);
        break;
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID:
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID:
        if (sc->alpha_x * sc->alpha_y < 1e-7f) {
          /* bsdf_microfacet_multi.h:651-690 */
          diff_rule_fresnel(rule, sc->ior, sc->N, sd->I, (label & LABEL_REFLECT) != 0);
        }
        else if (label & LABEL_REFLECT) {
          diff_rule_set(rule, CY_DIFF_MIRROR, sc->N);
        }
        else {
          /* bsdf_microfacet_multi.h:720-726: the refraction with neta = ior */
          const float ior = sc->ior;
          const float cosI = dot3(sc->N, sd->I);
          const float dnp = cmax(sqrtf(1.0f - (ior * ior * (1.0f - cosI * cosI))), 1e-7f);
          rule->kind = CY_DIFF_REFRACT;
          rule->n = sc->N;
          rule->neta = ior;
          rule->k = ior - ior * ior * cosI / dnp;
        }
        break;
      case CLOSURE_BSDF_HAIR_REFLECTION_ID:
      case CLOSURE_BSDF_HAIR_TRANSMISSION_ID: {
        /* bsdf_hair.h:231-232 */
        const float Iz = dot3(sc->T, sd->I);
        diff_rule_set(rule, CY_DIFF_MIRROR, normalize3(sub3(sd->I, mul3f(sc->T, Iz))));
        break;
      }
      case CLOSURE_BSDF_HAIR_PRINCIPLED_ID:
        /* bsdf_hair_principled.h:477-479 */
        diff_rule_set(rule, CY_DIFF_MIRROR, safe_normalize3(add3(sd->I, *omega_in)));
        break;
      case CLOSURE_BSDF_MICROFACET_GGX_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID:
      case CLOSURE_BSDF_MICROFACET_BECKMANN_ID:
      case CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID:
        break; /* set above */
      default:
        rule->kind = CY_DIFF_ZERO;
        break;
    }
  }
#endif
  if (label & LABEL_TRANSMIT) {
    float threshold_squared = KD->background.transparent_roughness_squared_threshold;
    if (threshold_squared >= 0.0f) {
      if (bsdf_get_specular_roughness_squared(sc) <= threshold_squared) {
        label |= LABEL_TRANSMIT_TRANSPARENT;
      }
    }
  }
  else if (label & LABEL_DIFFUSE) {
    if (!isequal3(sc->N, sd->N)) {
      *eval = mul3f(*eval, bump_shadowing_term(sd->N, sc->N, *omega_in));
    }
  }
  return label;
}

/* bsdf.h:495-700 */
CY_FN cfloat3 bsdf_eval(const CySD *sd, const CyClosure *sc, cfloat3 omega_in, float *pdf)
{
  cfloat3 eval;
  /* bsdf.h:506-508: curves evaluate against the smooth normal */
  const cfloat3 Ng_eval = (sd->type & PRIMITIVE_ALL_CURVE) ? sd->N : sd->Ng;
  if (dot3(Ng_eval, omega_in) >= 0.0f) {
    switch (sc->type) {
      case CLOSURE_BSDF_DIFFUSE_ID:
#if CY_CLOSURE_EXT
      case CLOSURE_BSDF_BSSRDF_ID:
#endif
        eval = bsdf_diffuse_eval_reflect(sc, omega_in, pdf);
        break;
#if CY_CLOSURE_EXT
      case CLOSURE_BSDF_OREN_NAYAR_ID:
        eval = bsdf_oren_nayar_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_PRINCIPLED_DIFFUSE_ID:
      case CLOSURE_BSDF_BSSRDF_PRINCIPLED_ID:
        eval = bsdf_principled_diffuse_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_PRINCIPLED_SHEEN_ID:
        eval = bsdf_principled_sheen_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
#endif
      case CLOSURE_BSDF_MICROFACET_GGX_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID:
        eval = bsdf_ggx_eval_reflect(sd, sc, sd->I, omega_in, pdf);
        break;
#if CY_CLOSURE_EXT
      case CLOSURE_BSDF_MICROFACET_BECKMANN_ID:
      case CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID:
        eval = bsdf_beckmann_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_ASHIKHMIN_SHIRLEY_ID:
        eval = bsdf_ashikhmin_shirley_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID:
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID:
        eval = bsdf_microfacet_multi_ggx_eval_reflect(sd, sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID:
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID:
        eval = bsdf_microfacet_multi_ggx_glass_eval(sd, sc, sd->I, omega_in, pdf, true);
        break;
      case CLOSURE_BSDF_ASHIKHMIN_VELVET_ID:
        eval = bsdf_ashikhmin_velvet_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_DIFFUSE_TOON_ID:
        eval = bsdf_diffuse_toon_eval_reflect(sc, omega_in, pdf);
        break;
      case CLOSURE_BSDF_GLOSSY_TOON_ID:
        eval = bsdf_glossy_toon_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_HAIR_PRINCIPLED_ID:
        eval = bsdf_principled_hair_eval(sd, sc, omega_in, pdf);
        break;
      case CLOSURE_BSDF_HAIR_REFLECTION_ID:
        eval = bsdf_hair_reflection_eval_reflect(sc, sd->I, omega_in, pdf);
        break;
#endif
      default: /* translucent, singular closures, NONE: zero */
        eval = mk3(0.0f, 0.0f, 0.0f);
        break;
    }
    if (CLOSURE_IS_BSDF_DIFFUSE(sc->type)) {
      if (!isequal3(sc->N, sd->N)) {
        eval = mul3f(eval, bump_shadowing_term(sd->N, sc->N, omega_in));
      }
    }
  }
  else {
    switch (sc->type) {
#if CY_CLOSURE_EXT
      case CLOSURE_BSDF_TRANSLUCENT_ID:
        eval = bsdf_translucent_eval_transmit(sc, omega_in, pdf);
        break;
#endif
      case CLOSURE_BSDF_MICROFACET_GGX_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_FRESNEL_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_CLEARCOAT_ID:
      case CLOSURE_BSDF_MICROFACET_GGX_REFRACTION_ID:
        eval = bsdf_ggx_eval_transmit(sc, sd->I, omega_in, pdf);
        break;
#if CY_CLOSURE_EXT
      case CLOSURE_BSDF_MICROFACET_BECKMANN_ID:
      case CLOSURE_BSDF_MICROFACET_BECKMANN_REFRACTION_ID:
        eval = bsdf_beckmann_eval_transmit(sc, sd->I, omega_in, pdf);
        break;
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_ID: /* bsdf_microfacet_multi.h:418-426 */
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_FRESNEL_ID:
        *pdf = 0.0f;
        eval = mk3(0.0f, 0.0f, 0.0f);
        break;
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_ID:
      case CLOSURE_BSDF_MICROFACET_MULTI_GGX_GLASS_FRESNEL_ID:
        eval = bsdf_microfacet_multi_ggx_glass_eval(sd, sc, sd->I, omega_in, pdf, false);
        break;
      case CLOSURE_BSDF_HAIR_PRINCIPLED_ID:
        eval = bsdf_principled_hair_eval(sd, sc, omega_in, pdf);
        break;
      case CLOSURE_BSDF_HAIR_TRANSMISSION_ID:
        eval = bsdf_hair_transmission_eval_transmit(sc, sd->I, omega_in, pdf);
        break;
#endif
      default:
        eval = mk3(0.0f, 0.0f, 0.0f);
        break;
    }
    if (CLOSURE_IS_BSDF_DIFFUSE(sc->type)) {
      if (!isequal3(sc->N, sd->N)) {
        eval = mul3f(eval, bump_shadowing_term(neg3(sd->N), sc->N, omega_in));
      }
    }
  }
  return eval;
}

#endif /* CY_CLOSURES_H */
