/*
 * cy_svm_nodes.h — SVM texture, converter and input nodes (kernel/svm/svm_*.h),
 * restated for the HIP device with the reference's operation order.  Included
 * by cy_path.h after the stack accessors; dispatched from svm_eval_nodes.
 *
 * Every libm call of these nodes is glibc's algorithm (cy_math.h: sinf, cosf,
 * powf, expf, logf, asinf, acosf, atanf, atan2f), so the device agrees with the
 * reference CPU kernel bit for bit (tan, sinh, cosh, tanh and expm1 too).
 */
#ifndef CY_SVM_NODES_H
#define CY_SVM_NODES_H

/* svm_types.h:64-156 node ids beyond the closure set (cy_types.h) */
enum {
  NODE_GEOMETRY = 11,
  NODE_CONVERT = 12,
  NODE_TEX_COORD = 13,
  NODE_GEOMETRY_BUMP_DX = 18,
  NODE_GEOMETRY_BUMP_DY = 19,
  NODE_ATTR_BUMP_DX = 27,
  NODE_ATTR_BUMP_DY = 28,
  NODE_VERTEX_COLOR_BUMP_DX = 29,
  NODE_VERTEX_COLOR_BUMP_DY = 30,
  NODE_TEX_COORD_BUMP_DX = 31,
  NODE_TEX_COORD_BUMP_DY = 32,
  NODE_CLOSURE_SET_NORMAL = 33,
  NODE_ENTER_BUMP_EVAL = 34,
  NODE_LEAVE_BUMP_EVAL = 35,
  NODE_TEX_VOXEL = 87,
  NODE_AOV_START = 88,
  NODE_AOV_COLOR = 89,
  NODE_AOV_VALUE = 90,
  NODE_HSV = 36,
  NODE_MATH = 42,
  NODE_VECTOR_MATH = 43,
  NODE_RGB_RAMP = 44,
  NODE_GAMMA = 45,
  NODE_BRIGHTCONTRAST = 46,
  NODE_LIGHT_PATH = 47,
  NODE_CLOSURE_HOLDOUT = 37,
  NODE_TEXTURE_MAPPING = 51,
  NODE_MAPPING = 52,
  NODE_MIN_MAX = 53,
  NODE_TEX_GRADIENT = 57,
  NODE_TEX_CHECKER = 62,
  NODE_LIGHT_FALLOFF = 66,
  NODE_INVERT = 72,
  NODE_WIREFRAME = 80,
  NODE_MIX = 73,
  NODE_SEPARATE_VECTOR = 74,
  NODE_COMBINE_VECTOR = 75,
  NODE_SEPARATE_HSV = 76,
  NODE_COMBINE_HSV = 77,
  NODE_MAP_RANGE = 83,
  NODE_CLAMP = 84,
  NODE_BEVEL = 85,
  NODE_AMBIENT_OCCLUSION = 86
};

CY_FN void svm_unpack3(uint i, uint *x, uint *y, uint *z)
{
  *x = i & 0xFF;
  *y = (i >> 8) & 0xFF;
  *z = (i >> 16) & 0xFF;
}
CY_FN void svm_unpack4(uint i, uint *x, uint *y, uint *z, uint *w)
{
  svm_unpack3(i, x, y, z);
  *w = (i >> 24) & 0xFF;
}
CY_FN float svm_load_default(CySvmStack stack, uint a, uint value, uint *err)
{
  return (a == SVM_STACK_INVALID) ? as_float(value) : svm_load(stack, a, err);
}

/* ---- util_math.h helpers ------------------------------------------------ */
CY_FN float cy_min(float a, float b)
{
  return (a < b) ? a : b;
}
CY_FN float cy_max(float a, float b)
{
  return (a > b) ? a : b;
}
CY_FN float cy_clampf(float a, float mn, float mx)
{
  return cy_min(cy_max(a, mn), mx);
}
/* safe_divide: cy_closures.h */
CY_FN float safe_modulo(float a, float b)
{
  return (b != 0.0f) ? fmodf(a, b) : 0.0f;
}
CY_FN float fractf(float x)
{
  return x - floorf(x);
}
CY_FN float wrapf(float value, float max, float min)
{
  const float range = max - min;
  return (range != 0.0f) ? value - (range * floorf((value - min) / range)) : min;
}
CY_FN float pingpongf(float a, float b)
{
  return (b != 0.0f) ? fabsf(fractf((a - b) / (b * 2.0f)) * b * 2.0f - b) : 0.0f;
}
CY_FN float smoothminf(float a, float b, float k)
{
  if (k != 0.0f) {
    const float h = fmaxf(k - fabsf(a - b), 0.0f) / k;
    return fminf(a, b) - h * h * h * k * (1.0f / 6.0f);
  }
  return fminf(a, b);
}
CY_FN float signf(float f)
{
  return (f < 0.0f) ? -1.0f : 1.0f;
}
CY_FN float compatible_signf(float f)
{
  return (f == 0.0f) ? 0.0f : signf(f);
}
CY_FN float safe_powf(float a, float b)
{
  if (a < 0.0f && b != (float)cy_ftoi(b)) {
    return 0.0f;
  }
  return cy_powf(a, b);
}
CY_FN float safe_logf(float a, float b)
{
  if (a <= 0.0f || b <= 0.0f) {
    return 0.0f;
  }
  return safe_divide(cy_logf(a), cy_logf(b));
}
CY_FN float safe_asinf(float a)
{
  return cy_asinf(cy_clampf(a, -1.0f, 1.0f));
}
CY_FN float smoothstepf_edges(float edge0, float edge1, float x)
{
  float result;
  if (x < edge0) {
    result = 0.0f;
  }
  else if (x >= edge1) {
    result = 1.0f;
  }
  else {
    const float t = (x - edge0) / (edge1 - edge0);
    result = (3.0f - 2.0f * t) * (t * t);
  }
  return result;
}
CY_FN cfloat3 safe_divide3(cfloat3 a, cfloat3 b)
{
  return mk3((b.x != 0.0f) ? a.x / b.x : 0.0f, (b.y != 0.0f) ? a.y / b.y : 0.0f,
             (b.z != 0.0f) ? a.z / b.z : 0.0f);
}
CY_FN cfloat3 floor3(cfloat3 a)
{
  return mk3(floorf(a.x), floorf(a.y), floorf(a.z));
}
CY_FN cfloat3 interp3(cfloat3 a, cfloat3 b, float t)
{
  return add3(a, mul3f(sub3(b, a), t));
}
CY_FN cfloat3 min3v(cfloat3 a, cfloat3 b)
{
  return mk3(cy_min(a.x, b.x), cy_min(a.y, b.y), cy_min(a.z, b.z));
}
CY_FN cfloat3 max3v(cfloat3 a, cfloat3 b)
{
  return mk3(cy_max(a.x, b.x), cy_max(a.y, b.y), cy_max(a.z, b.z));
}

/* ---- svm_math.h / svm_math_util.h --------------------------------------- */
CY_FN float svm_math(uint type, float a, float b, float c, uint *err)
{
  switch (type) {
    case 0: /* ADD */
      return a + b;
    case 1: /* SUBTRACT */
      return a - b;
    case 2: /* MULTIPLY */
      return a * b;
    case 3: /* DIVIDE */
      return safe_divide(a, b);
    case 4: /* SINE */
      return cy_sinf(a);
    case 5: /* COSINE */
      return cy_cosf(a);
    case 7: /* ARCSINE */
      return safe_asinf(a);
    case 8: /* ARCCOSINE */
      return safe_acosf(a);
    case 9: /* ARCTANGENT */
      return cy_atanf(a);
    case 10: /* POWER */
      return safe_powf(a, b);
    case 11: /* LOGARITHM */
      return safe_logf(a, b);
    case 12: /* MINIMUM */
      return fminf(a, b);
    case 13: /* MAXIMUM */
      return fmaxf(a, b);
    case 14: /* ROUND */
      return floorf(a + 0.5f);
    case 15: /* LESS_THAN */
      return (a < b) ? 1.0f : 0.0f;
    case 16: /* GREATER_THAN */
      return (a > b) ? 1.0f : 0.0f;
    case 17: /* MODULO */
      return safe_modulo(a, b);
    case 18: /* ABSOLUTE */
      return fabsf(a);
    case 19: /* ARCTAN2 */
      return cy_atan2f(a, b);
    case 20: /* FLOOR */
      return floorf(a);
    case 21: /* CEIL */
      return ceilf(a);
    case 22: /* FRACTION */
      return a - floorf(a);
    case 23: /* SQRT */
      return safe_sqrtf(a);
    case 24: /* INV_SQRT */
      return inversesqrtf(a);
    case 25: /* SIGN */
      return compatible_signf(a);
    case 26: /* EXPONENT */
      return cy_expf(a);
    case 27: /* RADIANS */
      return a * (CY_PI_F / 180.0f);
    case 28: /* DEGREES */
      return a * (180.0f / CY_PI_F);
    case 32: /* TRUNC */
      return a >= 0.0f ? floorf(a) : ceilf(a);
    case 33: /* SNAP */
      return floorf(safe_divide(a, b)) * b;
    case 34: /* WRAP */
      return wrapf(a, b, c);
    case 35: /* COMPARE */
      return ((a == b) || (fabsf(a - b) <= fmaxf(c, 1.192092896e-07f))) ? 1.0f : 0.0f;
    case 36: /* MULTIPLY_ADD */
      return a * b + c;
    case 37: /* PINGPONG */
      return pingpongf(a, b);
    case 38: /* SMOOTH_MIN */
      return smoothminf(a, b, c);
    case 39: /* SMOOTH_MAX */
      return -smoothminf(-a, -b, c);
    case 6: /* TANGENT */
      return cy_tanf(a);
    case 29: /* SINH */
      return cy_sinhf(a);
    case 30: /* COSH */
      return cy_coshf(a);
    case 31: /* TANH */
      return cy_tanhf(a);
    default:
      cy_set_error(err, CY_ERR_SVM_NODE, 10000 + type);
      return 0.0f;
  }
}

CY_FN void svm_vector_math(
    float *value, cfloat3 *vector, uint type, cfloat3 a, cfloat3 b, cfloat3 c, float scale, uint *err)
{
  switch (type) {
    case 0: /* ADD */
      *vector = add3(a, b);
      break;
    case 1: /* SUBTRACT */
      *vector = sub3(a, b);
      break;
    case 2: /* MULTIPLY */
      *vector = mul3(a, b);
      break;
    case 3: /* DIVIDE */
      *vector = safe_divide3(a, b);
      break;
    case 4: /* CROSS_PRODUCT */
      *vector = cross3(a, b);
      break;
    case 5: { /* PROJECT: util_math_float3.h project() */
      const float len_squared = dot3(b, b);
      *vector = (len_squared != 0.0f) ? mul3f(b, dot3(a, b) / len_squared) : mk3(0.0f, 0.0f, 0.0f);
      break;
    }
    case 6: { /* REFLECT: reflect(incident, normal) */
      const cfloat3 unit_normal = normalize3(b);
      *vector = sub3(a, mul3f(unit_normal, 2.0f * dot3(unit_normal, a)));
      break;
    }
    case 7: /* DOT_PRODUCT */
      *value = dot3(a, b);
      break;
    case 8: /* DISTANCE */
      *value = len3(sub3(a, b));
      break;
    case 9: /* LENGTH */
      *value = len3(a);
      break;
    case 10: /* SCALE */
      *vector = mul3f(a, scale);
      break;
    case 11: /* NORMALIZE */
      *vector = safe_normalize3(a);
      break;
    case 12: /* SNAP */
      *vector = mul3(floor3(safe_divide3(a, b)), b);
      break;
    case 13: /* FLOOR */
      *vector = floor3(a);
      break;
    case 14: /* CEIL */
      *vector = mk3(ceilf(a.x), ceilf(a.y), ceilf(a.z));
      break;
    case 15: /* MODULO */
      *vector = mk3(safe_modulo(a.x, b.x), safe_modulo(a.y, b.y), safe_modulo(a.z, b.z));
      break;
    case 16: /* FRACTION */
      *vector = sub3(a, floor3(a));
      break;
    case 17: /* ABSOLUTE */
      *vector = fabs3(a);
      break;
    case 18: /* MINIMUM */
      *vector = min3v(a, b);
      break;
    case 19: /* MAXIMUM */
      *vector = max3v(a, b);
      break;
    case 20: /* WRAP */
      *vector = mk3(wrapf(a.x, b.x, c.x), wrapf(a.y, b.y, c.y), wrapf(a.z, b.z, c.z));
      break;
    case 21: /* SINE */
      *vector = mk3(cy_sinf(a.x), cy_sinf(a.y), cy_sinf(a.z));
      break;
    case 22: /* COSINE */
      *vector = mk3(cy_cosf(a.x), cy_cosf(a.y), cy_cosf(a.z));
      break;
    case 23: /* TANGENT */
      *vector = mk3(cy_tanf(a.x), cy_tanf(a.y), cy_tanf(a.z));
      break;
    default:
      cy_set_error(err, CY_ERR_SVM_NODE, 11000 + type);
      *vector = mk3(0.0f, 0.0f, 0.0f);
      *value = 0.0f;
      break;
  }
}

/* svm_math.h:19-35 */
CY_FN void svm_node_math(CySvmStack stack, uint type, uint inputs, uint result, uint *err)
{
  uint a_off, b_off, c_off;
  svm_unpack3(inputs, &a_off, &b_off, &c_off);
  const float a = svm_load(stack, a_off, err);
  const float b = svm_load(stack, b_off, err);
  const float c = svm_load(stack, c_off, err);
  svm_store(stack, result, svm_math(type, a, b, c, err), err);
}

/* svm_math.h:37-72 */
CY_FN void svm_node_vector_math(
    const CyGlobals *kg, CySvmStack stack, uint type, uint inputs, uint outputs, int *offset, uint *err)
{
  uint a_off, b_off, scale_off, value_off, vector_off, unused;
  svm_unpack3(inputs, &a_off, &b_off, &scale_off);
  svm_unpack3(outputs, &value_off, &vector_off, &unused);
  const cfloat3 a = svm_load3(stack, a_off, err);
  const cfloat3 b = svm_load3(stack, b_off, err);
  cfloat3 c = mk3(0.0f, 0.0f, 0.0f);
  const float scale = svm_load(stack, scale_off, err);
  float value = 0.0f;
  cfloat3 vector = mk3(0.0f, 0.0f, 0.0f);
  if (type == 20) { /* WRAP: third operand in an extra node */
    const hc_uint4 extra = kg->__svm_nodes[*offset];
    (*offset)++;
    c = svm_load3(stack, extra.x, err);
  }
  svm_vector_math(&value, &vector, type, a, b, c, scale, err);
  if (value_off != SVM_STACK_INVALID) {
    svm_store(stack, value_off, value, err);
  }
  if (vector_off != SVM_STACK_INVALID) {
    svm_store3(stack, vector_off, vector, err);
  }
}

/* ---- colors: util_color.h rgb_to_hsv / hsv_to_rgb, svm_color_util.h ------ */
CY_FN cfloat3 rgb_to_hsv(cfloat3 rgb)
{
  float h, s;
  const float cmax_ = fmaxf(rgb.x, fmaxf(rgb.y, rgb.z));
  const float cmin_ = cy_min(rgb.x, cy_min(rgb.y, rgb.z));
  const float cdelta = cmax_ - cmin_;
  const float v = cmax_;
  if (cmax_ != 0.0f) {
    s = cdelta / cmax_;
  }
  else {
    s = 0.0f;
    h = 0.0f;
  }
  if (s != 0.0f) {
    const cfloat3 c = div3f(sub3(mk3(cmax_, cmax_, cmax_), rgb), cdelta);
    if (rgb.x == cmax_) {
      h = c.z - c.y;
    }
    else if (rgb.y == cmax_) {
      h = 2.0f + c.x - c.z;
    }
    else {
      h = 4.0f + c.y - c.x;
    }
    h /= 6.0f;
    if (h < 0.0f) {
      h += 1.0f;
    }
  }
  else {
    h = 0.0f;
  }
  return mk3(h, s, v);
}

CY_FN cfloat3 hsv_to_rgb(cfloat3 hsv)
{
  float h = hsv.x;
  const float s = hsv.y, v = hsv.z;
  if (s != 0.0f) {
    if (h == 1.0f) {
      h = 0.0f;
    }
    h *= 6.0f;
    const float i = floorf(h);
    const float f = h - i;
    const float p = v * (1.0f - s);
    const float q = v * (1.0f - (s * f));
    const float t = v * (1.0f - (s * (1.0f - f)));
    if (i == 0.0f) {
      return mk3(v, t, p);
    }
    else if (i == 1.0f) {
      return mk3(q, v, p);
    }
    else if (i == 2.0f) {
      return mk3(p, v, t);
    }
    else if (i == 3.0f) {
      return mk3(p, q, v);
    }
    else if (i == 4.0f) {
      return mk3(t, p, v);
    }
    return mk3(v, p, q);
  }
  return mk3(v, v, v);
}

CY_FN float svm_mix_overlay1(float o, float c2, float t, float tm)
{
  return (o < 0.5f) ? o * (tm + 2.0f * t * c2) : 1.0f - (tm + 2.0f * t * (1.0f - c2)) * (1.0f - o);
}
CY_FN float svm_mix_div1(float o, float c2, float t, float tm)
{
  return (c2 != 0.0f) ? tm * o + t * o / c2 : o;
}
CY_FN float svm_mix_dodge1(float o, float c2, float t)
{
  if (o != 0.0f) {
    float tmp = 1.0f - t * c2;
    if (tmp <= 0.0f) {
      return 1.0f;
    }
    else if ((tmp = o / tmp) > 1.0f) {
      return 1.0f;
    }
    return tmp;
  }
  return o;
}
CY_FN float svm_mix_burn1(float o, float c2, float t, float tm)
{
  float tmp = tm + t * c2;
  if (tmp <= 0.0f) {
    return 0.0f;
  }
  else if ((tmp = (1.0f - (1.0f - o) / tmp)) < 0.0f) {
    return 0.0f;
  }
  else if (tmp > 1.0f) {
    return 1.0f;
  }
  return tmp;
}

/* svm_color_util.h:235-285 svm_mix */
CY_FN cfloat3 svm_mix(uint type, float fac, cfloat3 c1, cfloat3 c2)
{
  const float t = saturate(fac);
  const float tm = 1.0f - t;
  const cfloat3 one = mk3(1.0f, 1.0f, 1.0f);
  switch (type) {
    case 0: /* BLEND */
      return interp3(c1, c2, t);
    case 1: /* ADD */
      return interp3(c1, add3(c1, c2), t);
    case 2: /* MUL */
      return interp3(c1, mul3(c1, c2), t);
    case 3: /* SUB */
      return interp3(c1, sub3(c1, c2), t);
    case 4: /* SCREEN */
      return sub3(one, mul3(add3(mk3(tm, tm, tm), mul3f(sub3(one, c2), t)), sub3(one, c1)));
    case 5: /* DIV */
      return mk3(svm_mix_div1(c1.x, c2.x, t, tm), svm_mix_div1(c1.y, c2.y, t, tm), svm_mix_div1(c1.z, c2.z, t, tm));
    case 6: /* DIFF */
      return interp3(c1, fabs3(sub3(c1, c2)), t);
    case 7: /* DARK */
      return interp3(c1, min3v(c1, c2), t);
    case 8: /* LIGHT */
      return interp3(c1, max3v(c1, c2), t);
    case 9: /* OVERLAY */
      return mk3(svm_mix_overlay1(c1.x, c2.x, t, tm), svm_mix_overlay1(c1.y, c2.y, t, tm),
                 svm_mix_overlay1(c1.z, c2.z, t, tm));
    case 10: /* DODGE */
      return mk3(svm_mix_dodge1(c1.x, c2.x, t), svm_mix_dodge1(c1.y, c2.y, t), svm_mix_dodge1(c1.z, c2.z, t));
    case 11: /* BURN */
      return mk3(svm_mix_burn1(c1.x, c2.x, t, tm), svm_mix_burn1(c1.y, c2.y, t, tm),
                 svm_mix_burn1(c1.z, c2.z, t, tm));
    case 12: { /* HUE */
      cfloat3 outcol = c1;
      const cfloat3 hsv2 = rgb_to_hsv(c2);
      if (hsv2.y != 0.0f) {
        cfloat3 hsv = rgb_to_hsv(outcol);
        hsv.x = hsv2.x;
        outcol = interp3(outcol, hsv_to_rgb(hsv), t);
      }
      return outcol;
    }
    case 13: { /* SAT */
      cfloat3 outcol = c1;
      cfloat3 hsv = rgb_to_hsv(outcol);
      if (hsv.y != 0.0f) {
        const cfloat3 hsv2 = rgb_to_hsv(c2);
        hsv.y = tm * hsv.y + t * hsv2.y;
        outcol = hsv_to_rgb(hsv);
      }
      return outcol;
    }
    case 14: { /* VAL */
      cfloat3 hsv = rgb_to_hsv(c1);
      const cfloat3 hsv2 = rgb_to_hsv(c2);
      hsv.z = tm * hsv.z + t * hsv2.z;
      return hsv_to_rgb(hsv);
    }
    case 15: { /* COLOR */
      cfloat3 outcol = c1;
      const cfloat3 hsv2 = rgb_to_hsv(c2);
      if (hsv2.y != 0.0f) {
        cfloat3 hsv = rgb_to_hsv(outcol);
        hsv.x = hsv2.x;
        hsv.y = hsv2.y;
        outcol = interp3(outcol, hsv_to_rgb(hsv), t);
      }
      return outcol;
    }
    case 16: { /* SOFT */
      const cfloat3 scr = sub3(one, mul3(sub3(one, c2), sub3(one, c1)));
      return add3(mul3f(c1, tm), mul3f(add3(mul3(mul3(sub3(one, c1), c2), c1), mul3(c1, scr)), t));
    }
    case 17: /* LINEAR */
      return add3(c1, mul3f(add3(mul3f(c2, 2.0f), mk3(-1.0f, -1.0f, -1.0f)), t));
    case 18: /* CLAMP */
      return mk3(saturate(c1.x), saturate(c1.y), saturate(c1.z));
  }
  return mk3(0.0f, 0.0f, 0.0f);
}

/* svm_mix.h:21-38 */
CY_FN void svm_node_mix(
    const CyGlobals *kg, CySvmStack stack, uint fac_off, uint c1_off, uint c2_off, int *offset, uint *err)
{
  const hc_uint4 node1 = kg->__svm_nodes[*offset];
  (*offset)++;
  const float fac = svm_load(stack, fac_off, err);
  const cfloat3 c1 = svm_load3(stack, c1_off, err);
  const cfloat3 c2 = svm_load3(stack, c2_off, err);
  svm_store3(stack, node1.z, svm_mix(node1.y, fac, c1, c2), err);
}

/* svm_hsv.h:21-60 */
CY_FN void svm_node_hsv(CySvmStack stack, hc_uint4 node, uint *err)
{
  uint in_color_off, fac_off, out_color_off, hue_off, sat_off, val_off;
  svm_unpack3(node.y, &in_color_off, &fac_off, &out_color_off);
  svm_unpack3(node.z, &hue_off, &sat_off, &val_off);
  const float fac = svm_load(stack, fac_off, err);
  const cfloat3 in_color = svm_load3(stack, in_color_off, err);
  const float hue = svm_load(stack, hue_off, err);
  const float sat = svm_load(stack, sat_off, err);
  const float val = svm_load(stack, val_off, err);
  cfloat3 color = rgb_to_hsv(in_color);
  color.x = fmodf(color.x + hue + 0.5f, 1.0f);
  color.y = saturate(color.y * sat);
  color.z *= val;
  color = hsv_to_rgb(color);
  color.x = fac * color.x + (1.0f - fac) * in_color.x;
  color.y = fac * color.y + (1.0f - fac) * in_color.y;
  color.z = fac * color.z + (1.0f - fac) * in_color.z;
  color.x = cy_max(color.x, 0.0f);
  color.y = cy_max(color.y, 0.0f);
  color.z = cy_max(color.z, 0.0f);
  if (out_color_off != SVM_STACK_INVALID) {
    svm_store3(stack, out_color_off, color, err);
  }
}

/* svm_gamma.h, svm_math_util.h:253-266 svm_math_gamma_color */
CY_FN void svm_node_gamma(CySvmStack stack, uint in_gamma, uint in_color, uint out_color, uint *err)
{
  cfloat3 color = svm_load3(stack, in_color, err);
  const float gamma = svm_load(stack, in_gamma, err);
  if (gamma == 0.0f) {
    color = mk3(1.0f, 1.0f, 1.0f);
  }
  else {
    if (color.x > 0.0f) {
      color.x = cy_powf(color.x, gamma);
    }
    if (color.y > 0.0f) {
      color.y = cy_powf(color.y, gamma);
    }
    if (color.z > 0.0f) {
      color.z = cy_powf(color.z, gamma);
    }
  }
  if (out_color != SVM_STACK_INVALID) {
    svm_store3(stack, out_color, color, err);
  }
}

/* svm_brightness.h, svm_color_util.h:287-297 */
CY_FN void svm_node_brightness(CySvmStack stack, uint in_color, uint out_color, uint node, uint *err)
{
  cfloat3 color = svm_load3(stack, in_color, err);
  const float brightness = svm_load(stack, node & 0xFF, err);
  const float contrast = svm_load(stack, (node >> 8) & 0xFF, err);
  const float a = 1.0f + contrast;
  const float b = brightness - contrast * 0.5f;
  color.x = cy_max(a * color.x + b, 0.0f);
  color.y = cy_max(a * color.y + b, 0.0f);
  color.z = cy_max(a * color.z + b, 0.0f);
  if (out_color != SVM_STACK_INVALID) {
    svm_store3(stack, out_color, color, err);
  }
}

/* svm_invert.h */
CY_FN float svm_invert1(float color, float factor)
{
  return factor * (1.0f - color) + (1.0f - factor) * color;
}
CY_FN void svm_node_invert(CySvmStack stack, uint in_fac, uint in_color, uint out_color, uint *err)
{
  const float factor = svm_load(stack, in_fac, err);
  cfloat3 color = svm_load3(stack, in_color, err);
  color.x = svm_invert1(color.x, factor);
  color.y = svm_invert1(color.y, factor);
  color.z = svm_invert1(color.z, factor);
  if (out_color != SVM_STACK_INVALID) {
    svm_store3(stack, out_color, color, err);
  }
}

/* svm_sepcomb_hsv.h */
CY_FN void svm_node_combine_hsv(
    const CyGlobals *kg, CySvmStack stack, uint hue_in, uint sat_in, uint val_in, int *offset, uint *err)
{
  const hc_uint4 node1 = kg->__svm_nodes[*offset];
  (*offset)++;
  const cfloat3 color = hsv_to_rgb(
      mk3(svm_load(stack, hue_in, err), svm_load(stack, sat_in, err), svm_load(stack, val_in, err)));
  if (node1.y != SVM_STACK_INVALID) {
    svm_store3(stack, node1.y, color, err);
  }
}
CY_FN void svm_node_separate_hsv(
    const CyGlobals *kg, CySvmStack stack, uint color_in, uint hue_out, uint sat_out, int *offset, uint *err)
{
  const hc_uint4 node1 = kg->__svm_nodes[*offset];
  (*offset)++;
  const cfloat3 color = rgb_to_hsv(svm_load3(stack, color_in, err));
  if (hue_out != SVM_STACK_INVALID) {
    svm_store(stack, hue_out, color.x, err);
  }
  if (sat_out != SVM_STACK_INVALID) {
    svm_store(stack, sat_out, color.y, err);
  }
  if (node1.y != SVM_STACK_INVALID) {
    svm_store(stack, node1.y, color.z, err);
  }
}

/* ---- svm_ramp.h ---------------------------------------------------------- */
CY_FN hc_float4 svm_f4(float x, float y, float z, float w)
{
  hc_float4 r;
  r.x = x;
  r.y = y;
  r.z = z;
  r.w = w;
  return r;
}
CY_FN hc_float4 svm_node_float4(const CyGlobals *kg, int offset)
{
  const hc_uint4 n = kg->__svm_nodes[offset];
  return svm_f4(as_float(n.x), as_float(n.y), as_float(n.z), as_float(n.w));
}
CY_FN hc_float4 rgb_ramp_lookup(const CyGlobals *kg, int offset, float f, bool interpolate, int table_size)
{
  f = saturate(f) * (float)(table_size - 1);
  int i = (int)f;
  i = (i < 0) ? 0 : ((i > table_size - 1) ? table_size - 1 : i);
  const float t = f - (float)i;
  hc_float4 a = svm_node_float4(kg, offset + i);
  if (interpolate && t > 0.0f) {
    const hc_float4 b = svm_node_float4(kg, offset + i + 1);
    const float u = 1.0f - t;
    a = svm_f4(u * a.x + t * b.x, u * a.y + t * b.y, u * a.z + t * b.z, u * a.w + t * b.w);
  }
  return a;
}
CY_FN void svm_node_rgb_ramp(const CyGlobals *kg, CySvmStack stack, hc_uint4 node, int *offset, uint *err)
{
  uint fac_off, color_off, alpha_off;
  svm_unpack3(node.y, &fac_off, &color_off, &alpha_off);
  const uint table_size = kg->__svm_nodes[*offset].x;
  (*offset)++;
  const float fac = svm_load(stack, fac_off, err);
  const hc_float4 color = rgb_ramp_lookup(kg, *offset, fac, node.z != 0u, (int)table_size);
  if (color_off != SVM_STACK_INVALID) {
    svm_store3(stack, color_off, mk3(color.x, color.y, color.z), err);
  }
  if (alpha_off != SVM_STACK_INVALID) {
    svm_store(stack, alpha_off, color.w, err);
  }
  *offset += (int)table_size;
}

/* ---- svm_mapping.h, util_transform.h:151-178 euler_to_transform --------- */
CY_FN cfloat3 svm_mapping(uint type, cfloat3 vector, cfloat3 location, cfloat3 rotation, cfloat3 scale)
{
  const float cx = cy_cosf(rotation.x), cy = cy_cosf(rotation.y), cz = cy_cosf(rotation.z);
  const float sx = cy_sinf(rotation.x), sy = cy_sinf(rotation.y), sz = cy_sinf(rotation.z);
  struct cy_tfm t;
  t.x.x = cy * cz;
  t.y.x = cy * sz;
  t.z.x = -sy;
  t.x.y = sy * sx * cz - cx * sz;
  t.y.y = sy * sx * sz + cx * cz;
  t.z.y = cy * sx;
  t.x.z = sy * cx * cz + sx * sz;
  t.y.z = sy * cx * sz - sx * cz;
  t.z.z = cy * cx;
  t.x.w = t.y.w = t.z.w = 0.0f;
  switch (type) {
    case 0: /* POINT */
      return add3(transform_direction(&t, mul3(vector, scale)), location);
    case 1: /* TEXTURE */
      return safe_divide3(transform_direction_transposed(&t, sub3(vector, location)), scale);
    case 2: /* VECTOR */
      return transform_direction(&t, mul3(vector, scale));
    case 3: /* NORMAL */
      return safe_normalize3(transform_direction(&t, safe_divide3(vector, scale)));
  }
  return mk3(0.0f, 0.0f, 0.0f);
}
CY_FN void svm_node_mapping(CySvmStack stack, uint type, uint inputs, uint result, uint *err)
{
  uint vec_off, loc_off, rot_off, scale_off;
  svm_unpack4(inputs, &vec_off, &loc_off, &rot_off, &scale_off);
  const cfloat3 vector = svm_load3(stack, vec_off, err);
  const cfloat3 location = svm_load3(stack, loc_off, err);
  const cfloat3 rotation = svm_load3(stack, rot_off, err);
  const cfloat3 scale = svm_load3(stack, scale_off, err);
  svm_store3(stack, result, svm_mapping(type, vector, location, rotation, scale), err);
}

/* ---- svm_checker.h, svm_gradient.h -------------------------------------- */
CY_FN float svm_checker(cfloat3 p)
{
  p.x = (p.x + 0.000001f) * 0.999999f;
  p.y = (p.y + 0.000001f) * 0.999999f;
  p.z = (p.z + 0.000001f) * 0.999999f;
  /* abs(xi) % 2 as the parity bit xi & 1: the same for every int, and defined
   * for INT_MIN (the x86 conversion of an out-of-range coordinate), where
   * abs() is undefined and the device compiler may fold it to anything */
  const int xi = cy_ftoi(floorf(p.x)) & 1;
  const int yi = cy_ftoi(floorf(p.y)) & 1;
  const int zi = cy_ftoi(floorf(p.z)) & 1;
  return ((xi == yi) == zi) ? 1.0f : 0.0f;
}
CY_FN void svm_node_tex_checker(CySvmStack stack, hc_uint4 node, uint *err)
{
  uint co_off, color1_off, color2_off, scale_off, color_off, fac_off, unused;
  svm_unpack4(node.y, &co_off, &color1_off, &color2_off, &scale_off);
  svm_unpack3(node.z, &color_off, &fac_off, &unused);
  const cfloat3 co = svm_load3(stack, co_off, err);
  const cfloat3 color1 = svm_load3(stack, color1_off, err);
  const cfloat3 color2 = svm_load3(stack, color2_off, err);
  const float scale = svm_load_default(stack, scale_off, node.w, err);
  const float f = svm_checker(mul3f(co, scale));
  if (color_off != SVM_STACK_INVALID) {
    svm_store3(stack, color_off, (f == 1.0f) ? color1 : color2, err);
  }
  if (fac_off != SVM_STACK_INVALID) {
    svm_store(stack, fac_off, f, err);
  }
}

CY_FN float svm_gradient(cfloat3 p, uint type)
{
  const float x = p.x, y = p.y, z = p.z;
  if (type == 0) { /* LINEAR */
    return x;
  }
  else if (type == 1) { /* QUADRATIC */
    const float r = fmaxf(x, 0.0f);
    return r * r;
  }
  else if (type == 2) { /* EASING */
    const float r = fminf(fmaxf(x, 0.0f), 1.0f);
    const float t = r * r;
    return (3.0f * t - 2.0f * t * r);
  }
  else if (type == 3) { /* DIAGONAL */
    return (x + y) * 0.5f;
  }
  else if (type == 4) { /* RADIAL */
    return cy_atan2f(y, x) / 6.2831853071795864f + 0.5f; /* M_2PI_F */
  }
  const float r = fmaxf(0.999999f - sqrtf(x * x + y * y + z * z), 0.0f);
  if (type == 5) { /* QUADRATIC_SPHERE */
    return r * r;
  }
  else if (type == 6) { /* SPHERICAL */
    return r;
  }
  return 0.0f;
}
CY_FN void svm_node_tex_gradient(CySvmStack stack, hc_uint4 node, uint *err)
{
  uint type, co_off, fac_off, color_off;
  svm_unpack4(node.y, &type, &co_off, &fac_off, &color_off);
  const float f = saturate(svm_gradient(svm_load3(stack, co_off, err), type));
  if (fac_off != SVM_STACK_INVALID) {
    svm_store(stack, fac_off, f, err);
  }
  if (color_off != SVM_STACK_INVALID) {
    svm_store3(stack, color_off, mk3(f, f, f), err);
  }
}

/* ---- svm_clamp.h, svm_map_range.h --------------------------------------- */
CY_FN void svm_node_clamp(
    const CyGlobals *kg, CySvmStack stack, uint value_off, uint params, uint result_off, int *offset, uint *err)
{
  uint min_off, max_off, type;
  svm_unpack3(params, &min_off, &max_off, &type);
  const hc_uint4 defaults = kg->__svm_nodes[*offset];
  (*offset)++;
  const float value = svm_load(stack, value_off, err);
  const float mn = svm_load_default(stack, min_off, defaults.x, err);
  const float mx = svm_load_default(stack, max_off, defaults.y, err);
  if (type == 1 && (mn > mx)) { /* NODE_CLAMP_RANGE */
    svm_store(stack, result_off, cy_clampf(value, mx, mn), err);
  }
  else {
    svm_store(stack, result_off, cy_clampf(value, mn, mx), err);
  }
}

CY_FN float smootherstep(float edge0, float edge1, float x)
{
  x = cy_clampf(safe_divide((x - edge0), (edge1 - edge0)), 0.0f, 1.0f);
  return x * x * x * (x * (x * 6.0f - 15.0f) + 10.0f);
}
CY_FN void svm_node_map_range(
    const CyGlobals *kg, CySvmStack stack, uint value_off, uint params, uint results, int *offset, uint *err)
{
  uint from_min_off, from_max_off, to_min_off, to_max_off, type, steps_off, result_off;
  svm_unpack4(params, &from_min_off, &from_max_off, &to_min_off, &to_max_off);
  svm_unpack3(results, &type, &steps_off, &result_off);
  const hc_uint4 defaults = kg->__svm_nodes[*offset];
  const hc_uint4 defaults2 = kg->__svm_nodes[*offset + 1];
  *offset += 2;
  const float value = svm_load(stack, value_off, err);
  const float from_min = svm_load_default(stack, from_min_off, defaults.x, err);
  const float from_max = svm_load_default(stack, from_max_off, defaults.y, err);
  const float to_min = svm_load_default(stack, to_min_off, defaults.z, err);
  const float to_max = svm_load_default(stack, to_max_off, defaults.w, err);
  const float steps = svm_load_default(stack, steps_off, defaults2.x, err);
  float result;
  if (from_max != from_min) {
    float factor = value;
    switch (type) {
      default:
      case 0: /* LINEAR */
        factor = (value - from_min) / (from_max - from_min);
        break;
      case 1: /* STEPPED */
        factor = (value - from_min) / (from_max - from_min);
        factor = (steps > 0.0f) ? floorf(factor * (steps + 1.0f)) / steps : 0.0f;
        break;
      case 2: /* SMOOTHSTEP */
        factor = (from_min > from_max) ? 1.0f - smoothstepf_edges(from_max, from_min, factor) :
                                         smoothstepf_edges(from_min, from_max, factor);
        break;
      case 3: /* SMOOTHERSTEP */
        factor = (from_min > from_max) ? 1.0f - smootherstep(from_max, from_min, factor) :
                                         smootherstep(from_min, from_max, factor);
        break;
    }
    result = to_min + factor * (to_max - to_min);
  }
  else {
    result = 0.0f;
  }
  svm_store(stack, result_off, result, err);
}

/* ---- svm_sepcomb_vector.h ------------------------------------------------ */
CY_FN void svm_node_combine_vector(CySvmStack stack, uint in_off, uint index, uint out_off, uint *err)
{
  const float v = svm_load(stack, in_off, err);
  if (out_off != SVM_STACK_INVALID) {
    svm_store(stack, out_off + index, v, err);
  }
}
CY_FN void svm_node_separate_vector(CySvmStack stack, uint in_off, uint index, uint out_off, uint *err)
{
  const cfloat3 v = svm_load3(stack, in_off, err);
  if (out_off != SVM_STACK_INVALID) {
    svm_store(stack, out_off, (index == 0) ? v.x : ((index == 1) ? v.y : v.z), err);
  }
}

/* ---- svm_convert.h ------------------------------------------------------- */
CY_FN void svm_node_convert(const CyGlobals *kg, CySvmStack stack, uint type, uint from, uint to, uint *err)
{
  /* linear_rgb_to_gray (kernel_color.h): dot with the film's rgb_to_y */
  const cfloat3 rgb_to_y = mk3(KD->film.rgb_to_y.x, KD->film.rgb_to_y.y, KD->film.rgb_to_y.z);
  switch (type) {
    case 0: { /* FV */
      const float f = svm_load(stack, from, err);
      svm_store3(stack, to, mk3(f, f, f), err);
      break;
    }
    case 1: /* FI */
      svm_store(stack, to, int_as_float(cy_ftoi(svm_load(stack, from, err))), err);
      break;
    case 2: /* CF */
      svm_store(stack, to, dot3(svm_load3(stack, from, err), rgb_to_y), err);
      break;
    case 3: /* CI */
      svm_store(stack, to, int_as_float(cy_ftoi(dot3(svm_load3(stack, from, err), rgb_to_y))), err);
      break;
    case 4: /* VF */
      svm_store(stack, to, average3(svm_load3(stack, from, err)), err);
      break;
    case 5: /* VI */
      svm_store(stack, to, int_as_float(cy_ftoi(average3(svm_load3(stack, from, err)))), err);
      break;
    case 6: /* IF */
      svm_store(stack, to, (float)as_int(svm_load(stack, from, err)), err);
      break;
    case 7: { /* IV */
      const float f = (float)as_int(svm_load(stack, from, err));
      svm_store3(stack, to, mk3(f, f, f), err);
      break;
    }
  }
}

/* ---- svm_geometry.h, svm_tex_coord.h, svm_light_path.h ----------------- */
CY_FN void svm_node_geometry(CySD *sd, CySvmStack stack, uint type, uint out_off, uint *err)
{
  cfloat3 data;
  switch (type) {
    case 0: /* P */
      data = sd->P;
      break;
    case 1: /* N */
      data = sd->N;
      break;
    case 3: /* I */
      data = sd->I;
      break;
    case 4: /* Ng */
      data = sd->Ng;
      break;
    case 5: /* uv */
      data = mk3(sd->u, sd->v, 0.0f);
      break;
    default: /* T: needs the generated-coordinate attribute */
      cy_set_error(err, CY_ERR_SVM_NODE, 12000 + type);
      data = mk3(0.0f, 0.0f, 0.0f);
      break;
  }
  svm_store3(stack, out_off, data, err);
}

CY_FN void svm_node_tex_coord(
    const CyGlobals *kg, CySD *sd, int path_flag, CySvmStack stack, hc_uint4 node, int *offset, uint *err)
{
  cfloat3 data = mk3(0.0f, 0.0f, 0.0f);
  const uint type = node.y;
  switch (type) {
    case 1: { /* OBJECT */
      data = sd->P;
      if (node.w == 0) {
        if (sd->object != OBJECT_NONE) {
          data = transform_point(object_itfm(kg, sd->object), data);
        }
      }
      else {
        struct cy_tfm tfm;
        const hc_float4 a = svm_node_float4(kg, *offset), b = svm_node_float4(kg, *offset + 1),
                        c = svm_node_float4(kg, *offset + 2);
        *offset += 3;
        tfm.x.x = a.x; tfm.x.y = a.y; tfm.x.z = a.z; tfm.x.w = a.w;
        tfm.y.x = b.x; tfm.y.y = b.y; tfm.y.z = b.z; tfm.y.w = b.w;
        tfm.z.x = c.x; tfm.z.y = c.y; tfm.z.z = c.z; tfm.z.w = c.w;
        data = transform_point(&tfm, data);
      }
      break;
    }
    case 0: /* NORMAL: object_inverse_normal_transform (geom_object.h:144-162; the CPU
             * kernel's __OBJECT_MOTION__ form: a lamp's shading point uses the lamp's
             * transform, ob_tfm = lamp_fetch_transform) */
      data = sd->N;
      if (sd->object != OBJECT_NONE) {
        data = normalize3(transform_direction_transposed(object_tfm(kg, sd->object), data));
      }
      else if (sd->type == (1 << 6) /* PRIMITIVE_LAMP */) {
        data = normalize3(transform_direction_transposed((const struct cy_tfm *)&kg->__lights[sd->lamp].tfm, data));
      }
      break;
    case 2: { /* CAMERA */
      const struct cy_tfm *w2c = (const struct cy_tfm *)&KD->cam.worldtocamera;
      if (sd->object != OBJECT_NONE) {
        data = transform_point(w2c, sd->P);
      }
      else {
        const struct cy_tfm *c2w = (const struct cy_tfm *)&KD->cam.cameratoworld;
        data = transform_point(w2c, add3(sd->P, mk3(c2w->x.w, c2w->y.w, c2w->z.w)));
      }
      break;
    }
    case 3: { /* WINDOW: camera_world_to_ndc (perspective / orthographic) */
      if (KD->cam.type == 2) {
        cy_set_error(err, CY_ERR_SVM_NODE, 13000 + type);
        break;
      }
      cfloat3 P = sd->P;
      if ((path_flag & PATH_RAY_CAMERA) && sd->object == OBJECT_NONE && KD->cam.type == 1) {
        cy_set_error(err, CY_ERR_SVM_NODE, 13100 + type); /* needs sd->ray_P */
        break;
      }
      if (sd->object == PRIM_NONE && KD->cam.type == 0) {
        const struct cy_tfm *c2w = (const struct cy_tfm *)&KD->cam.cameratoworld;
        P = add3(P, mk3(c2w->x.w, c2w->y.w, c2w->z.w));
      }
      data = transform_perspective((const struct cy_ptfm *)&KD->cam.worldtondc, P);
      data.z = 0.0f;
      break;
    }
    case 4: /* REFLECTION */
      if (sd->object != OBJECT_NONE) {
        data = sub3(mul3f(sd->N, 2.0f * dot3(sd->N, sd->I)), sd->I);
      }
      else {
        data = sd->I;
      }
      break;
    default: /* DUPLI / VOLUME generated */
      cy_set_error(err, CY_ERR_SVM_NODE, 13000 + type);
      break;
  }
  svm_store3(stack, node.z, data, err);
}

CY_FN void svm_node_light_path(
    const CySD *sd, const CyPathState *state, CySvmStack stack, uint type, uint out_off, int path_flag, uint *err)
{
  float info = 0.0f;
  switch (type) {
    case 0:
      info = (path_flag & PATH_RAY_CAMERA) ? 1.0f : 0.0f;
      break;
    case 1:
      info = (path_flag & PATH_RAY_SHADOW) ? 1.0f : 0.0f;
      break;
    case 2:
      info = (path_flag & PATH_RAY_DIFFUSE) ? 1.0f : 0.0f;
      break;
    case 3:
      info = (path_flag & PATH_RAY_GLOSSY) ? 1.0f : 0.0f;
      break;
    case 4:
      info = (path_flag & PATH_RAY_SINGULAR) ? 1.0f : 0.0f;
      break;
    case 5:
      info = (path_flag & PATH_RAY_REFLECT) ? 1.0f : 0.0f;
      break;
    case 6:
      info = (path_flag & PATH_RAY_TRANSMIT) ? 1.0f : 0.0f;
      break;
    case 7:
      info = (path_flag & PATH_RAY_VOLUME_SCATTER) ? 1.0f : 0.0f;
      break;
    case 8:
      info = (sd->flag & SD_BACKFACING) ? 1.0f : 0.0f;
      break;
    case 9:
      info = sd->ray_length;
      break;
    case 10:
      info = (float)state->bounce;
      break;
    case 11:
      info = (float)state->diffuse_bounce;
      break;
    case 12:
      info = (float)state->glossy_bounce;
      break;
    case 13:
      info = (float)state->transparent_bounce;
      break;
    case 14:
      info = (float)state->transmission_bounce;
      break;
  }
  svm_store(stack, out_off, info, err);
}

/* svm_light_path.h:78-106 */
CY_FN void svm_node_light_falloff(const CySD *sd, CySvmStack stack, hc_uint4 node, uint *err)
{
  uint strength_off, out_off, smooth_off;
  svm_unpack3(node.z, &strength_off, &smooth_off, &out_off);
  float strength = svm_load(stack, strength_off, err);
  switch (node.y) {
    case 0: /* QUADRATIC */
      break;
    case 1: /* LINEAR */
      strength *= sd->ray_length;
      break;
    case 2: /* CONSTANT */
      strength *= sd->ray_length * sd->ray_length;
      break;
  }
  const float smooth = svm_load(stack, smooth_off, err);
  if (smooth > 0.0f) {
    const float squared = sd->ray_length * sd->ray_length;
    if (isfinite(squared)) {
      strength *= squared / (smooth + squared);
    }
  }
  svm_store(stack, out_off, strength, err);
}

#endif /* CY_SVM_NODES_H */
