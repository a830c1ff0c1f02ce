/*
 * cy_svm_ies.h — the IES Texture node (kernel/svm/svm_ies.h:21-119) for the HIP
 * device: the light's candela table from `__ies` (LightManager::device_update_ies,
 * render/light.cpp:1080-1125: a slot offset table, then per slot h_num, v_num,
 * the horizontal and vertical angles in radians and h_num x v_num intensities),
 * looked up by the direction's spherical angles with cubic interpolation along
 * both axes.  Included by cy_path.h after cy_svm_image.h.
 */
#ifndef CY_SVM_IES_H
#define CY_SVM_IES_H

enum { NODE_IES = 67 };

/* util_math.h:425-438 */
CY_FN float ies_inverse_lerp(float a, float b, float x)
{
  return (x - a) / (b - a);
}
CY_FN float ies_cubic_interp(float a, float b, float c, float d, float x)
{
  return 0.5f * (((d + 3.0f * (b - c) - a) * x + (2.0f * a - 5.0f * b + 4.0f * c - d)) * x + (c - a)) * x + b;
}

/* svm_ies.h:21-40 */
CY_FN float interpolate_ies_vertical(const float *ies, int ofs, int v, int v_num, float v_frac, int h)
{
  const float a = ies[ofs + h * v_num + ((v == 0) ? 1 : v - 1)];
  const float b = ies[ofs + h * v_num + v];
  const float c = ies[ofs + h * v_num + v + 1];
  const float d = ies[ofs + h * v_num + ((v + 2 < v_num - 1) ? v + 2 : v_num - 1)];
  return ies_cubic_interp(a, b, c, d, v_frac);
}

/* svm_ies.h:42-95.  The angle searches are bounded by the table sizes (the
 * reference relies on the host's angle ranges: h from 0 to 2 pi, v from 0). */
CY_FN float kernel_ies_interp(const float *ies, int slot, float h_angle, float v_angle)
{
  int ofs = as_int(ies[slot]);
  if (ofs == -1) {
    return 100.0f;
  }
  const int h_num = as_int(ies[ofs++]);
  const int v_num = as_int(ies[ofs++]);
  if (v_angle >= ies[ofs + h_num + v_num - 1]) {
    return 0.0f;
  }
  int h_i, v_i;
  for (h_i = 0; h_i + 2 < h_num && ies[ofs + h_i + 1] < h_angle; h_i++) {
  }
  for (v_i = 0; v_i + 2 < v_num && ies[ofs + h_num + v_i + 1] < v_angle; v_i++) {
  }
  const float h_frac = ies_inverse_lerp(ies[ofs + h_i], ies[ofs + h_i + 1], h_angle);
  const float v_frac = ies_inverse_lerp(ies[ofs + h_num + v_i], ies[ofs + h_num + v_i + 1], v_angle);
  ofs += h_num + v_num;
  const float a = interpolate_ies_vertical(ies, ofs, v_i, v_num, v_frac, (h_i == 0) ? h_num - 2 : h_i - 1);
  const float b = interpolate_ies_vertical(ies, ofs, v_i, v_num, v_frac, h_i);
  const float c = interpolate_ies_vertical(ies, ofs, v_i, v_num, v_frac, h_i + 1);
  const float d = interpolate_ies_vertical(ies, ofs, v_i, v_num, v_frac, (h_i + 2 == h_num) ? 1 : h_i + 2);
  return fmaxf(ies_cubic_interp(a, b, c, d, h_frac), 0.0f);
}

/* svm_ies.h:97-117 svm_node_ies: NODE_IES (strength, vector, fac), slot, strength */
CY_FN void svm_node_ies(const float *ies, CySvmStack stack, hc_uint4 node, uint *err)
{
  const uint strength_offset = node.y & 0xFF, vector_offset = (node.y >> 8) & 0xFF;
  const uint fac_offset = (node.y >> 16) & 0xFF, slot = node.z;
  cfloat3 vector = svm_load3(stack, vector_offset, err);
  const float strength = (strength_offset == SVM_STACK_INVALID) ? as_float(node.w) :
                                                                  svm_load(stack, strength_offset, err);
  vector = normalize3(vector);
  const float v_angle = safe_acosf(-vector.z);
  const float h_angle = cy_atan2f(vector.x, vector.y) + CY_PI_F;
  const float fac = strength * kernel_ies_interp(ies, (int)slot, h_angle, v_angle);
  if (fac_offset != SVM_STACK_INVALID) {
    svm_store(stack, fac_offset, fac, err);
  }
}

#endif /* CY_SVM_IES_H */
