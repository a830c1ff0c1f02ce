/*
 * cy_attribute.h — geometry attributes on triangles: the attribute map lookup
 * and the barycentric interpolation of per-face / per-vertex / per-corner
 * values, as the SVM's Attribute, Texture Coordinate (UV, Generated) and
 * Vertex Color nodes read them.
 *   find_attribute                         kernel/geom/geom_attribute.h:40-95
 *   triangle_attribute_float/2/3/4         kernel/geom/geom_triangle.h:114-360
 *   primitive_surface_attribute_* (meshes) kernel/geom/geom_primitive.h:57-241
 *   svm_node_attr                          kernel/svm/svm_attribute.h:21-95
 *   svm_node_vertex_color                  kernel/svm/svm_vertex_color.h:19-36
 *   svm_node_normal_map, svm_node_tangent  kernel/svm/svm_tex_coord.h:255-392
 *   ensure_valid_reflection                kernel/kernel_montecarlo.h:196-298
 *   svm_node_object_info                   kernel/svm/svm_geometry.h:104-139
 *   svm_node_particle_info                 kernel/svm/svm_geometry.h:141-202
 *   svm_node_hair_info, curve_thickness,
 *   curve_tangent_normal                   kernel/svm/svm_geometry.h:204-243, geom/geom_curve.h:263-323
 *   curve_attribute_float / float2 / float3 kernel/geom/geom_curve.h:28-200
 *   svm_node_attr_bump_dx / _dy            kernel/svm/svm_attribute.h:92-188
 *   svm_node_vertex_color_bump_dx / _dy    kernel/svm/svm_vertex_color.h:38-90
 *   svm_node_set_bump                      kernel/svm/svm_displace.h:21-84
 * The host packs attributes for triangle meshes without subdivision
 * (`__tri_patch` is all ~0, so attribute_primitive_type is always
 * ATTR_PRIM_GEOMETRY) and float / float2 / float3 attributes of curves (per
 * curve or per key, e.g. the Hair Info node's intercept and random); an RGBA
 * attribute found on a curve raises CY_ERR_FEATURE.  Per-object maps: KernelObject.attribute_map_offset into
 * `__attributes_map`, two rows (geometry, subdivision) per attribute, closed
 * by ATTR_STD_NONE.
 */
#ifndef CY_ATTRIBUTE_H
#define CY_ATTRIBUTE_H

enum {
  NODE_ATTR = 16,
  NODE_VERTEX_COLOR = 17,
  NODE_SET_BUMP = 26,
  NODE_OBJECT_INFO = 48,
  NODE_PARTICLE_INFO = 49,
  NODE_HAIR_INFO = 50,
  NODE_TANGENT = 70,
  NODE_NORMAL_MAP = 71
};
/* AttributeStandard ids read by the kernel itself (kernel_types.h:750-779) */
#define ATTR_STD_VERTEX_NORMAL 1u

/* AttributeElement (kernel_types.h:735-748) and NodeAttributeType (svm_types.h:160-166) */
enum {
  ATTR_ELEMENT_NONE = 0,
  ATTR_ELEMENT_OBJECT = 1,
  ATTR_ELEMENT_MESH = 2,
  ATTR_ELEMENT_FACE = 3,
  ATTR_ELEMENT_VERTEX = 4,
  ATTR_ELEMENT_VERTEX_MOTION = 5,
  ATTR_ELEMENT_CORNER = 6,
  ATTR_ELEMENT_CORNER_BYTE = 7,
  ATTR_ELEMENT_CURVE = 8,
  ATTR_ELEMENT_CURVE_KEY = 9,
  ATTR_ELEMENT_CURVE_KEY_MOTION = 10,
  ATTR_ELEMENT_VOXEL = 11
};
enum { NODE_ATTR_FLOAT = 0, NODE_ATTR_FLOAT2 = 1, NODE_ATTR_FLOAT3 = 2, NODE_ATTR_RGBA = 3 };
#define ATTR_STD_NOT_FOUND (~0)
#define ATTR_PRIM_TYPES 2

typedef struct CyAttr {
  int element;
  int type;
  int offset; /* ATTR_STD_NOT_FOUND when absent */
} CyAttr;

CY_FN CyAttr attribute_not_found()
{
  CyAttr a;
  a.element = ATTR_ELEMENT_NONE;
  a.type = 0;
  a.offset = ATTR_STD_NOT_FOUND;
  return a;
}

/* find_attribute: the object's map row with this id (prim PRIM_NONE: only
 * mesh / object / voxel elements) */
CY_FN CyAttr find_attribute(const CyGlobals *kg, int object, int prim, uint id)
{
  if (object == OBJECT_NONE || kg->__attributes_map == nullptr) {
    return attribute_not_found();
  }
  uint attr_offset = kg->__objects[object].attribute_map_offset; /* + ATTR_PRIM_GEOMETRY */
  hc_uint4 attr_map = kg->__attributes_map[attr_offset];
  while (attr_map.x != id) {
    if (attr_map.x == 0u) { /* ATTR_STD_NONE */
      return attribute_not_found();
    }
    attr_offset += ATTR_PRIM_TYPES;
    attr_map = kg->__attributes_map[attr_offset];
  }
  CyAttr desc;
  desc.element = (int)attr_map.y;
  if (prim == PRIM_NONE && desc.element != ATTR_ELEMENT_MESH && desc.element != ATTR_ELEMENT_VOXEL &&
      desc.element != ATTR_ELEMENT_OBJECT) {
    return attribute_not_found();
  }
  desc.offset = (attr_map.y == ATTR_ELEMENT_NONE) ? (int)ATTR_STD_NOT_FOUND : (int)attr_map.z;
  desc.type = (int)(attr_map.w & 0xffu);
  return desc;
}

/* color_uchar4_to_float4 (util_color.h) */
CY_FN void uchar4_to_float4(uint c, float f[4])
{
  f[0] = (float)(c & 0xffu) * (1.0f / 255.0f);
  f[1] = (float)((c >> 8) & 0xffu) * (1.0f / 255.0f);
  f[2] = (float)((c >> 16) & 0xffu) * (1.0f / 255.0f);
  f[3] = (float)(c >> 24) * (1.0f / 255.0f);
}

/* one value of an n-component attribute array */
CY_FN void attr_fetch(const CyGlobals *kg, int n, bool bytes, int i, float f[4])
{
  if (bytes) {
    uchar4_to_float4(kg->__attributes_uchar4[i], f);
  }
  else if (n == 1) {
    f[0] = kg->__attributes_float[i];
  }
  else if (n == 2) {
    const hc_float2 a = kg->__attributes_float2[i];
    f[0] = a.x;
    f[1] = a.y;
  }
  else {
    const hc_float4 a = kg->__attributes_float3[i];
    f[0] = a.x;
    f[1] = a.y;
    f[2] = a.z;
    f[3] = a.w;
  }
}

/* triangle_attribute_float / float2 / float3 / float4 (n = 1, 2, 3, 4) of
 * the triangle at (u, v): u*f0 + v*f1 + (1-u-v)*f2 per component for
 * per-vertex and per-corner elements, the stored value for per-face and
 * per-object ones, 0 for elements the reference's reader of that width
 * does not handle.  With dd = {du, dv} (one axis of the shading point's
 * differentials) the value plus its derivative, du*f0 + dv*f1 - (du+dv)*f2
 * for interpolated elements and 0 otherwise (the *_BUMP_DX / _DY nodes) */
CY_FN void triangle_attribute(const CyGlobals *kg, const CyAttr &desc, int prim, float u, float v, int n, float out[4],
                              const float *dd = nullptr)
{
  int idx[3] = {0, 0, 0};
  int m = 0;
  bool bytes = false;
  const int e = desc.element;
  if (n == 4) {
    if (e == ATTR_ELEMENT_CORNER_BYTE) {
      const int tri = desc.offset + prim * 3;
      idx[0] = tri;
      idx[1] = tri + 1;
      idx[2] = tri + 2;
      m = 3;
      bytes = true;
    }
    else if (e == ATTR_ELEMENT_VERTEX) {
      const hc_uint4 t = kg->__tri_vindex[prim];
      idx[0] = desc.offset + (int)t.x;
      idx[1] = desc.offset + (int)t.y;
      idx[2] = desc.offset + (int)t.z;
      m = 3;
    }
    else if (e == ATTR_ELEMENT_OBJECT || e == ATTR_ELEMENT_MESH) {
      idx[0] = desc.offset;
      m = 1;
      bytes = true;
    }
  }
  else if (e == ATTR_ELEMENT_FACE) {
    idx[0] = desc.offset + prim;
    m = 1;
  }
  else if (e == ATTR_ELEMENT_VERTEX || e == ATTR_ELEMENT_VERTEX_MOTION) {
    const hc_uint4 t = kg->__tri_vindex[prim];
    idx[0] = desc.offset + (int)t.x;
    idx[1] = desc.offset + (int)t.y;
    idx[2] = desc.offset + (int)t.z;
    m = 3;
  }
  else if (e == ATTR_ELEMENT_CORNER) {
    const int tri = desc.offset + prim * 3;
    idx[0] = tri;
    idx[1] = tri + 1;
    idx[2] = tri + 2;
    m = 3;
  }
  else if (e == ATTR_ELEMENT_OBJECT || e == ATTR_ELEMENT_MESH) {
    idx[0] = desc.offset;
    m = 1;
  }
  float f[3][4] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
  for (int k = 0; k < m; k++) {
    attr_fetch(kg, n, bytes, idx[k], f[k]);
  }
  const float w = 1.0f - u - v;
  for (int c = 0; c < n; c++) {
    out[c] = (m == 3) ? u * f[0][c] + v * f[1][c] + w * f[2][c] : (m == 1) ? f[0][c] : 0.0f;
  }
  if (dd) {
    for (int c = 0; c < n; c++) {
      const float d = (m == 3) ? dd[0] * f[0][c] + dd[1] * f[1][c] - (dd[0] + dd[1]) * f[2][c] : 0.0f;
      out[c] = out[c] + d;
    }
  }
}

/* curve_attribute_float / float2 / float3 (geom_curve.h:28-200) of the curve
 * segment at parameter u: per-key values interpolated (1 - u) * f0 + u * f1
 * between the segment's keys, per-curve and per-object ones as stored, 0
 * otherwise.  du_dx (the bump X form) adds du.dx * (f1 - f0) for per-key
 * values; the Y form's derivative is 0 on curves. */
CY_FN void curve_attribute(const CyGlobals *kg, const CyAttr &desc, int prim, int type, float u, int n, float out[4],
                           const float *du_dx = nullptr)
{
  int idx[2] = {0, 0};
  int m = 0;
  const int e = desc.element;
  if (e == ATTR_ELEMENT_CURVE) {
    idx[0] = desc.offset + prim;
    m = 1;
  }
  else if (e == ATTR_ELEMENT_CURVE_KEY || e == ATTR_ELEMENT_CURVE_KEY_MOTION) {
    const int k0 = as_int(kg->__curves[prim].x) + (int)CY_PRIMITIVE_UNPACK_SEGMENT((uint)type);
    idx[0] = desc.offset + k0;
    idx[1] = desc.offset + k0 + 1;
    m = 2;
  }
  else if (e == ATTR_ELEMENT_OBJECT || e == ATTR_ELEMENT_MESH) {
    idx[0] = desc.offset;
    m = 1;
  }
  float f[2][4] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
  for (int k = 0; k < m; k++) {
    attr_fetch(kg, n, false, idx[k], f[k]);
  }
  for (int c = 0; c < n; c++) {
    out[c] = (m == 2) ? (1.0f - u) * f[0][c] + u * f[1][c] : (m == 1) ? f[0][c] : 0.0f;
    if (du_dx && m == 2) {
      out[c] = out[c] + *du_dx * (f[1][c] - f[0][c]);
    }
  }
}

/* svm_node_attr: the attribute read with the stored type, converted to the
 * node's output type (float: the average of a colour / vector) */
CY_FN void svm_node_attr(const CyGlobals *kg, int object, int prim, int type, float u, float v, CySvmStack stack,
                         hc_uint4 node, uint *err, const float *dd = nullptr, int bump_axis = 0)
{
  const uint out_offset = node.z;
  const int out_type = (int)node.w;
  CyAttr desc;
  if (object != OBJECT_NONE) {
    desc = find_attribute(kg, object, prim, node.y);
    if (desc.offset == (int)ATTR_STD_NOT_FOUND) {
      desc = attribute_not_found();
      desc.offset = 0;
      desc.type = out_type;
    }
  }
  else {
    desc = attribute_not_found();
    desc.offset = 0;
    desc.type = out_type;
  }
  const bool tri = (type & PRIMITIVE_ALL_TRIANGLE) != 0;
  const bool curve = !tri && (type & PRIMITIVE_ALL_CURVE);
  float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const int n = (desc.type == NODE_ATTR_FLOAT) ? 1 : (desc.type == NODE_ATTR_FLOAT2) ? 2 :
                (desc.type == NODE_ATTR_RGBA)  ? 4 :
                                                 3;
  if (curve && n == 4 && desc.element != ATTR_ELEMENT_NONE) {
    cy_set_error(err, CY_ERR_FEATURE, 11); /* RGBA attributes of curves are not packed */
  }
  if (tri) {
    triangle_attribute(kg, desc, prim, u, v, n, f, dd);
  }
  else if (curve && n < 4) {
    curve_attribute(kg, desc, prim, type, u, n, f, (dd && bump_axis == 1) ? &dd[0] : nullptr);
  }
  if (n == 1) {
    if (out_type == NODE_ATTR_FLOAT) {
      svm_store(stack, out_offset, f[0], err);
    }
    else {
      svm_store3(stack, out_offset, mk3(f[0], f[0], f[0]), err);
    }
  }
  else if (n == 2) {
    if (out_type == NODE_ATTR_FLOAT) {
      svm_store(stack, out_offset, f[0], err);
    }
    else {
      svm_store3(stack, out_offset, mk3(f[0], f[1], 0.0f), err);
    }
  }
  else {
    const cfloat3 c = mk3(f[0], f[1], f[2]);
    if (out_type == NODE_ATTR_FLOAT) {
      svm_store(stack, out_offset, average3(c), err);
    }
    else {
      svm_store3(stack, out_offset, c, err);
    }
  }
}

CY_FN void svm_node_vertex_color(const CyGlobals *kg, int object, int prim, int type, float u, float v,
                                 CySvmStack stack, uint layer_id, uint color_offset, uint alpha_offset, uint *err,
                                 const float *dd = nullptr)
{
  const CyAttr desc = find_attribute(kg, object, prim, layer_id);
  if (desc.offset != (int)ATTR_STD_NOT_FOUND) {
    float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (type & PRIMITIVE_ALL_TRIANGLE) {
      triangle_attribute(kg, desc, prim, u, v, 4, f, dd);
    }
    else if (type & PRIMITIVE_ALL_CURVE) {
      cy_set_error(err, CY_ERR_FEATURE, 11);
    }
    svm_store3(stack, color_offset, mk3(f[0], f[1], f[2]), err);
    svm_store(stack, alpha_offset, f[3], err);
  }
  else {
    svm_store3(stack, color_offset, mk3(0.0f, 0.0f, 0.0f), err);
    svm_store(stack, alpha_offset, 0.0f, err);
  }
}

/* the shading point as the geometry-aware nodes read it */
typedef struct CyAttrIn {
  cfloat3 P, N, Ng, I;
  float u, v;
  int object, prim, type, flag, shader;
#if CY_CLOSURE_EXT
  cfloat3 dPdu;
  /* the Bump node's dP.dx / dP.dy; a bump form's du, dv along its axis */
  cfloat3 dPdx, dPdy;
  float bump_du, bump_dv;
  int bump;
#endif
#ifdef CY_DBG_X
  bool dbg = false;
#endif
} CyAttrIn;

/* primitive_surface_attribute_float / float2 / float3 (geom_primitive.h:57-241):
 * triangles interpolate, curves carry no packed attributes (error when one is
 * found), anything else reads 0 */
CY_FN void surface_attribute(const CyGlobals *kg, const CyAttrIn &in, const CyAttr &desc, int n, float f[4],
                             uint *err)
{
  f[0] = f[1] = f[2] = f[3] = 0.0f;
  if (in.type & PRIMITIVE_ALL_TRIANGLE) {
    triangle_attribute(kg, desc, in.prim, in.u, in.v, n, f);
  }
  else if ((in.type & PRIMITIVE_ALL_CURVE) && n < 4) {
    curve_attribute(kg, desc, in.prim, in.type, in.u, n, f);
  }
  else if ((in.type & PRIMITIVE_ALL_CURVE) && desc.element != ATTR_ELEMENT_NONE) {
    cy_set_error(err, CY_ERR_FEATURE, 11);
  }
}

/* kernel_montecarlo.h:196-298: N tilted towards Ng just enough that the
 * reflection of I stays above the surface */
CY_FN cfloat3 ensure_valid_reflection(cfloat3 Ng, cfloat3 I, cfloat3 N)
{
  const cfloat3 R = sub3(mul3f(N, 2.0f * dot3(N, I)), I);
  const float threshold = cmin(0.9f * dot3(Ng, I), 0.01f);
  if (dot3(Ng, R) >= threshold) {
    return N;
  }
  const float NdotNg = dot3(N, Ng);
  const cfloat3 X = normalize3(sub3(N, mul3f(Ng, NdotNg)));
  const float Ix = dot3(I, X), Iz = dot3(I, Ng);
  const float Ix2 = sqr(Ix), Iz2 = sqr(Iz);
  const float a = Ix2 + Iz2;
  const float b = safe_sqrtf(Ix2 * (a - sqr(threshold)));
  const float c = Iz * threshold + a;
  const float fac = 0.5f / a;
  const float N1_z2 = fac * (b + c), N2_z2 = fac * (-b + c);
  bool valid1 = (N1_z2 > 1e-5f) && (N1_z2 <= (1.0f + 1e-5f));
  bool valid2 = (N2_z2 > 1e-5f) && (N2_z2 <= (1.0f + 1e-5f));
  float nx, nz;
  if (valid1 && valid2) {
    const float N1x = safe_sqrtf(1.0f - N1_z2), N1y = safe_sqrtf(N1_z2);
    const float N2x = safe_sqrtf(1.0f - N2_z2), N2y = safe_sqrtf(N2_z2);
    const float R1 = 2.0f * (N1x * Ix + N1y * Iz) * N1y - Iz;
    const float R2 = 2.0f * (N2x * Ix + N2y * Iz) * N2y - Iz;
    valid1 = (R1 >= 1e-5f);
    valid2 = (R2 >= 1e-5f);
    const bool first = (valid1 && valid2) ? (R1 < R2) : (R1 > R2);
    nx = first ? N1x : N2x;
    nz = first ? N1y : N2y;
  }
  else if (valid1 || valid2) {
    const float Nz2 = valid1 ? N1_z2 : N2_z2;
    nx = safe_sqrtf(1.0f - Nz2);
    nz = safe_sqrtf(Nz2);
  }
  else {
    return Ng;
  }
  return add3(mul3f(X, nx), mul3f(Ng, nz));
}

/* object_normal_transform / object_inverse_normal_transform (geom_object.h,
 * __OBJECT_MOTION__ form: the object's static transforms) */
CY_FN cfloat3 attr_object_normal_transform(const CyGlobals *kg, int object, cfloat3 N)
{
  return normalize3(transform_direction_transposed(object_itfm(kg, object), N));
}
CY_FN cfloat3 attr_object_inverse_normal_transform(const CyGlobals *kg, int object, cfloat3 N)
{
  return (object != OBJECT_NONE) ? normalize3(transform_direction_transposed(object_tfm(kg, object), N)) : N;
}

/* svm_tex_coord.h:255-345 */
CY_FN void svm_node_normal_map(const CyGlobals *kg, const CyAttrIn &in, CySvmStack stack, hc_uint4 node, uint *err)
{
  uint color_offset, strength_offset, normal_offset, space;
  svm_unpack4(node.y, &color_offset, &strength_offset, &normal_offset, &space);
  cfloat3 color = svm_load3(stack, color_offset, err);
  color = mul3f(mk3(color.x - 0.5f, color.y - 0.5f, color.z - 0.5f), 2.0f);
  const bool is_backfacing = (in.flag & SD_BACKFACING) != 0;
  cfloat3 N;
  if (space == 0) { /* NODE_NORMAL_MAP_TANGENT */
    if (in.object == OBJECT_NONE) {
      svm_store3(stack, normal_offset, mk3(0.0f, 0.0f, 0.0f), err);
      return;
    }
    const CyAttr attr = find_attribute(kg, in.object, in.prim, node.z);
    const CyAttr attr_sign = find_attribute(kg, in.object, in.prim, node.w);
    const CyAttr attr_normal = find_attribute(kg, in.object, in.prim, ATTR_STD_VERTEX_NORMAL);
    if (attr.offset == (int)ATTR_STD_NOT_FOUND || attr_sign.offset == (int)ATTR_STD_NOT_FOUND ||
        attr_normal.offset == (int)ATTR_STD_NOT_FOUND) {
      svm_store3(stack, normal_offset, mk3(0.0f, 0.0f, 0.0f), err);
      return;
    }
    float f[4];
    surface_attribute(kg, in, attr, 3, f, err);
    const cfloat3 tangent = mk3(f[0], f[1], f[2]);
    surface_attribute(kg, in, attr_sign, 1, f, err);
    const float sign = f[0];
    cfloat3 normal;
    if ((uint)in.shader & SHADER_SMOOTH_NORMAL) {
      surface_attribute(kg, in, attr_normal, 3, f, err);
      normal = mk3(f[0], f[1], f[2]);
    }
    else {
      normal = is_backfacing ? neg3(in.Ng) : in.Ng;
      normal = attr_object_inverse_normal_transform(kg, in.object, normal);
    }
    const cfloat3 B = mul3f(cross3(normal, tangent), sign);
    N = safe_normalize3(add3(add3(mul3f(tangent, color.x), mul3f(B, color.y)), mul3f(normal, color.z)));
    N = attr_object_normal_transform(kg, in.object, N);
  }
  else {
    if (space == 3 || space == 4) { /* BLENDER_OBJECT / BLENDER_WORLD */
      color.y = -color.y;
      color.z = -color.z;
    }
    N = color;
    if (space == 1 || space == 3) { /* OBJECT / BLENDER_OBJECT */
      if (in.object == OBJECT_NONE) {
        cy_set_error(err, CY_ERR_SVM_NODE, 1000 + NODE_NORMAL_MAP); /* no object transform to apply */
      }
      else {
        N = attr_object_normal_transform(kg, in.object, N);
      }
    }
    else {
      N = safe_normalize3(N);
    }
  }
  if (is_backfacing) {
    N = neg3(N);
  }
  float strength = svm_load(stack, strength_offset, err);
  if (strength != 1.0f) {
    strength = cmax(strength, 0.0f);
    N = safe_normalize3(add3(in.N, mul3f(sub3(N, in.N), strength)));
  }
  N = ensure_valid_reflection(in.Ng, in.I, N);
  if (is_zero3(N)) {
    N = in.N;
  }
  svm_store3(stack, normal_offset, N, err);
}

/* svm_tex_coord.h:347-390 */
CY_FN void svm_node_tangent(const CyGlobals *kg, const CyAttrIn &in, CySvmStack stack, hc_uint4 node, uint *err)
{
  uint tangent_offset, direction_type, axis;
  svm_unpack3(node.y, &tangent_offset, &direction_type, &axis);
  cfloat3 tangent;
  cfloat3 attribute_value = mk3(0.0f, 0.0f, 0.0f);
  const CyAttr desc = find_attribute(kg, in.object, in.prim, node.z);
  if (desc.offset != (int)ATTR_STD_NOT_FOUND) {
    float f[4];
    if (desc.type == NODE_ATTR_FLOAT2) {
      surface_attribute(kg, in, desc, 2, f, err);
      attribute_value = mk3(f[0], f[1], 0.0f);
    }
    else {
      surface_attribute(kg, in, desc, 3, f, err);
      attribute_value = mk3(f[0], f[1], f[2]);
    }
  }
  if (direction_type == 1) { /* NODE_TANGENT_UVMAP */
    tangent = (desc.offset == (int)ATTR_STD_NOT_FOUND) ? mk3(0.0f, 0.0f, 0.0f) : attribute_value;
  }
  else { /* radial */
    const cfloat3 generated = (desc.offset == (int)ATTR_STD_NOT_FOUND) ? in.P : attribute_value;
    if (axis == 0) {
      tangent = mk3(0.0f, -(generated.z - 0.5f), (generated.y - 0.5f));
    }
    else if (axis == 1) {
      tangent = mk3(-(generated.z - 0.5f), 0.0f, (generated.x - 0.5f));
    }
    else {
      tangent = mk3(-(generated.y - 0.5f), (generated.x - 0.5f), 0.0f);
    }
  }
  if (in.object == OBJECT_NONE) {
    cy_set_error(err, CY_ERR_SVM_NODE, 1000 + NODE_TANGENT); /* no object transform to apply */
  }
  else {
    tangent = attr_object_normal_transform(kg, in.object, tangent);
  }
  tangent = cross3(in.N, normalize3(cross3(tangent, in.N)));
  svm_store3(stack, tangent_offset, tangent, err);
}

/* svm_geometry.h:104-139 (surfaces: sd->lamp is LAMP_NONE) */
CY_FN void svm_node_object_info(const CyGlobals *kg, const CyAttrIn &in, CySvmStack stack, uint type, uint out_offset,
                                uint *err)
{
  const int object = in.object;
  float data;
  switch (type) {
    case 0: { /* NODE_INFO_OB_LOCATION: object_location (ob_tfm translation) */
      cfloat3 loc = mk3(0.0f, 0.0f, 0.0f);
      if (object != OBJECT_NONE) {
        const struct cy_tfm *t = object_tfm(kg, object);
        loc = mk3(t->x.w, t->y.w, t->z.w);
      }
      svm_store3(stack, out_offset, loc, err);
      return;
    }
    case 1: { /* NODE_INFO_OB_COLOR */
      cfloat3 col = mk3(0.0f, 0.0f, 0.0f);
      if (object != OBJECT_NONE) {
        const hc_KernelObject &ko = kg->__objects[object];
        col = mk3(ko.color[0], ko.color[1], ko.color[2]);
      }
      svm_store3(stack, out_offset, col, err);
      return;
    }
    case 2: /* NODE_INFO_OB_INDEX */
      data = (object != OBJECT_NONE) ? kg->__objects[object].pass_id : 0.0f;
      break;
    case 3: /* NODE_INFO_MAT_INDEX: shader_pass_id */
      data = (float)kg->__shaders[(uint)in.shader & SHADER_MASK].pass_id;
      break;
    case 4: /* NODE_INFO_OB_RANDOM */
      data = (object != OBJECT_NONE) ? kg->__objects[object].random_number : 0.0f;
      break;
    default:
      data = 0.0f;
      break;
  }
  svm_store(stack, out_offset, data, err);
}

/* svm_node_particle_info (svm_geometry.h:141-202): the record of the object's
 * particle (object_particle_id, geom_object.h:267-273; particle 0 for no object) */
CY_FN void svm_node_particle_info(const CyGlobals *kg, const CyAttrIn &in, CySvmStack stack, uint type,
                                  uint out_offset, uint *err)
{
  const int id = (in.object == OBJECT_NONE) ? 0 : kg->__objects[in.object].particle_index;
  const hc_KernelParticle &p = kg->__particles[id];
  switch (type) {
    case 0: /* NODE_INFO_PAR_INDEX: particle_index is a uint */
      svm_store(stack, out_offset, (float)(uint)p.index, err);
      break;
    case 1: /* NODE_INFO_PAR_RANDOM: hash_uint2_to_float(particle_index, 0) */
      svm_store(stack, out_offset, (float)hash_uint2((uint)p.index, 0u) / (float)0xFFFFFFFFu, err);
      break;
    case 2:
      svm_store(stack, out_offset, p.age, err);
      break;
    case 3:
      svm_store(stack, out_offset, p.lifetime, err);
      break;
    case 4:
      svm_store3(stack, out_offset, mk3(p.location.x, p.location.y, p.location.z), err);
      break;
    case 6:
      svm_store(stack, out_offset, p.size, err);
      break;
    case 7:
      svm_store3(stack, out_offset, mk3(p.velocity.x, p.velocity.y, p.velocity.z), err);
      break;
    case 8:
      svm_store3(stack, out_offset, mk3(p.angular_velocity.x, p.angular_velocity.y, p.angular_velocity.z), err);
      break;
  }
}

#if CY_CLOSURE_EXT
/* svm_node_hair_info (svm_geometry.h:204-243): strand flag, curve_thickness
 * (geom_curve.h:263-286: twice the radius interpolated between the segment's
 * keys) and curve_tangent_normal (:307-323); intercept and random are curve
 * attributes (NODE_ATTR) */
CY_FN void svm_node_hair_info(const CyGlobals *kg, const CyAttrIn &in, CySvmStack stack, uint type, uint out_offset,
                              uint *err)
{
  const bool curve = (in.type & PRIMITIVE_ALL_CURVE) != 0;
  switch (type) {
    case 0: /* NODE_INFO_CURVE_IS_STRAND */
      svm_store(stack, out_offset, curve ? 1.0f : 0.0f, err);
      break;
    case 2: { /* NODE_INFO_CURVE_THICKNESS */
      float r = 0.0f;
      if (curve) {
        const int k0 = as_int(kg->__curves[in.prim].x) + (int)CY_PRIMITIVE_UNPACK_SEGMENT((uint)in.type);
        const hc_float4 P0 = kg->__curve_keys[k0], P1 = kg->__curve_keys[k0 + 1];
        r = (P1.w - P0.w) * in.u + P0.w;
      }
      svm_store(stack, out_offset, r * 2.0f, err);
      break;
    }
    case 3: { /* NODE_INFO_CURVE_TANGENT_NORMAL */
      cfloat3 tgN = mk3(0.0f, 0.0f, 0.0f);
      if (curve) {
        const cfloat3 mI = neg3(in.I);
        tgN = neg3(sub3(mI, mul3f(in.dPdu, dot3(in.dPdu, mI) / len_squared3(in.dPdu))));
        tgN = normalize3(tgN);
      }
      svm_store3(stack, out_offset, tgN, err);
      break;
    }
  }
}
#endif

/* svm_geometry.h NODE_GEOM_T: primitive_tangent (geom_primitive.h:292-320),
 * the spherical tangent of the generated coordinates around Z, else (and on
 * curves) the normalised surface derivative dPdu */
CY_FN void svm_node_geometry_tangent(const CyGlobals *kg, const CyAttrIn &in, CySvmStack stack, uint out_offset,
                                     uint *err)
{
  cfloat3 T = mk3(0.0f, 0.0f, 0.0f);
  const CyAttr desc = (in.type & PRIMITIVE_ALL_CURVE) ? attribute_not_found() :
                                                        find_attribute(kg, in.object, in.prim, 7u /* GENERATED */);
  if (desc.offset != (int)ATTR_STD_NOT_FOUND) {
    float f[4];
    surface_attribute(kg, in, desc, 3, f, err);
    cfloat3 data = mk3(-(f[1] - 0.5f), (f[0] - 0.5f), 0.0f);
    data = attr_object_normal_transform(kg, in.object, data);
    T = cross3(in.N, normalize3(cross3(data, in.N)));
  }
  else {
#if CY_CLOSURE_EXT
    T = normalize3(in.dPdu);
#else
    cy_set_error(err, CY_ERR_SVM_NODE, 2000 + 2); /* tangent from surface derivatives (sd->dPdu) */
#endif
  }
  svm_store3(stack, out_offset, T, err);
}

#if CY_CLOSURE_EXT
/* svm_displace.h:21-84 svm_node_set_bump: the normal tilted by the height's
 * differences across the shading point's dP.dx / dP.dy (the graph's
 * SampleX / SampleY copies were evaluated at P + dP.dx / dy) */
CY_FN void svm_node_set_bump(const CyGlobals *kg, const CyAttrIn &in, CySvmStack stack, hc_uint4 node, uint *err)
{
  uint normal_offset, scale_offset, invert, use_object_space;
  svm_unpack4(node.y, &normal_offset, &scale_offset, &invert, &use_object_space);
  cfloat3 normal_in = (normal_offset != SVM_STACK_INVALID) ? svm_load3(stack, normal_offset, err) : in.N;
  cfloat3 dPdx = in.dPdx;
  cfloat3 dPdy = in.dPdy;
  if (use_object_space) {
    normal_in = attr_object_inverse_normal_transform(kg, in.object, normal_in);
    if (in.object != OBJECT_NONE) {
      dPdx = transform_direction(object_itfm(kg, in.object), dPdx);
      dPdy = transform_direction(object_itfm(kg, in.object), dPdy);
    }
  }
  /* surface tangents from the normal */
  const cfloat3 Rx = cross3(dPdy, normal_in);
  const cfloat3 Ry = cross3(normal_in, dPdx);
  uint c_offset, x_offset, y_offset, strength_offset;
  svm_unpack4(node.z, &c_offset, &x_offset, &y_offset, &strength_offset);
  const float h_c = svm_load(stack, c_offset, err);
  const float h_x = svm_load(stack, x_offset, err);
  const float h_y = svm_load(stack, y_offset, err);
  /* surface gradient and determinant */
  const float det = dot3(dPdx, Rx);
  const cfloat3 surfgrad = add3(mul3f(Rx, h_x - h_c), mul3f(Ry, h_y - h_c));
  const float absdet = fabsf(det);
  float strength = svm_load(stack, strength_offset, err);
  float scale = svm_load(stack, scale_offset, err);
  if (invert) {
    scale *= -1.0f;
  }
  strength = cmax(strength, 0.0f);
  cfloat3 normal_out = safe_normalize3(sub3(mul3f(normal_in, absdet), mul3f(surfgrad, scale * signf(det))));
  if (is_zero3(normal_out)) {
    normal_out = normal_in;
  }
  else {
    normal_out = normalize3(add3(mul3f(normal_out, strength), mul3f(normal_in, 1.0f - strength)));
  }
  if (use_object_space) {
    normal_out = attr_object_normal_transform(kg, in.object, normal_out);
  }
  normal_out = ensure_valid_reflection(in.Ng, in.I, normal_out);
  CY_DBG3(&in, "bump h", mk3(h_c, h_x, h_y));
  CY_DBG3(&in, "bump dPdx", dPdx);
  CY_DBG3(&in, "bump dPdy", dPdy);
  CY_DBG3(&in, "bump N in", normal_in);
  CY_DBG3(&in, "bump det str scale", mk3(det, strength, scale));
  CY_DBG3(&in, "bump N out", normal_out);
  svm_store3(stack, node.w, normal_out, err);
}
#endif

#if CY_CLOSURE_EXT
/* svm_bump.h:21-46 svm_node_enter_bump_eval, the part after the saved state:
 * the shading point as if undisplaced -- ATTR_STD_POSITION_UNDISPLACED
 * (primitive_surface_attribute_float3 with its derivatives along the ray
 * differentials, geom_triangle.h:241-298) moved to world space by the object's
 * transform (object_position_transform / object_dir_transform; the CPU
 * kernel's sd->ob_tfm is the object transform for objects without motion).
 * found = 0 when the object has no such attribute (the state stays). */
typedef struct CyBumpEval {
  cfloat3 P, dPdx, dPdy;
  int found;
} CyBumpEval;

CY_NOINLINE CyBumpEval svm_bump_undisplaced(const hc_KernelObject *objects, const hc_uint4 *attributes_map,
                                            const hc_float4 *attributes_float3, const hc_uint4 *tri_vindex,
                                            CyAttrIn in, float du_dx, float du_dy, float dv_dx, float dv_dy)
{
  CyGlobals kgv;
  kgv.__objects = objects;
  kgv.__attributes_map = attributes_map;
  kgv.__attributes_float3 = attributes_float3;
  kgv.__tri_vindex = tri_vindex;
  const CyGlobals *kg = &kgv;
  CyBumpEval r;
  r.found = 0;
  r.P = r.dPdx = r.dPdy = mk3(0.0f, 0.0f, 0.0f);
  const CyAttr desc = (in.object != OBJECT_NONE) ? find_attribute(kg, in.object, in.prim, 10u /* UNDISPLACED */) :
                                                   attribute_not_found();
  if (desc.offset == (int)ATTR_STD_NOT_FOUND) {
    return r;
  }
  r.found = 1;
  if (in.type & PRIMITIVE_ALL_TRIANGLE) {
    const int e = desc.element;
    cfloat3 f[3] = {mk3(0.0f, 0.0f, 0.0f), mk3(0.0f, 0.0f, 0.0f), mk3(0.0f, 0.0f, 0.0f)};
    bool interp = false;
    if (e == ATTR_ELEMENT_VERTEX || e == ATTR_ELEMENT_VERTEX_MOTION) {
      const hc_uint4 t = kg->__tri_vindex[in.prim];
      const int idx[3] = {desc.offset + (int)t.x, desc.offset + (int)t.y, desc.offset + (int)t.z};
      for (int k = 0; k < 3; k++) {
        const hc_float4 a = kg->__attributes_float3[idx[k]];
        f[k] = mk3(a.x, a.y, a.z);
      }
      interp = true;
    }
    else if (e == ATTR_ELEMENT_CORNER) {
      const int tri = desc.offset + in.prim * 3;
      for (int k = 0; k < 3; k++) {
        const hc_float4 a = kg->__attributes_float3[tri + k];
        f[k] = mk3(a.x, a.y, a.z);
      }
      interp = true;
    }
    else if (e == ATTR_ELEMENT_FACE || e == ATTR_ELEMENT_OBJECT || e == ATTR_ELEMENT_MESH) {
      const hc_float4 a = kg->__attributes_float3[desc.offset + (e == ATTR_ELEMENT_FACE ? in.prim : 0)];
      r.P = mk3(a.x, a.y, a.z);
    }
    if (interp) {
      r.dPdx = sub3(add3(mul3f(f[0], du_dx), mul3f(f[1], dv_dx)), mul3f(f[2], du_dx + dv_dx));
      r.dPdy = sub3(add3(mul3f(f[0], du_dy), mul3f(f[1], dv_dy)), mul3f(f[2], du_dy + dv_dy));
      r.P = add3(add3(mul3f(f[0], in.u), mul3f(f[1], in.v)), mul3f(f[2], 1.0f - in.u - in.v));
    }
  }
  /* curves carry no undisplaced positions (Mesh::add_undisplaced only) */
  const struct cy_tfm *tfm = object_tfm(kg, in.object);
  r.P = transform_point(tfm, r.P);
  r.dPdx = transform_direction(tfm, r.dPdx);
  r.dPdy = transform_direction(tfm, r.dPdy);
  return r;
}
#endif

/* NODE_ATTR / NODE_VERTEX_COLOR / NODE_NORMAL_MAP / NODE_TANGENT /
 * NODE_OBJECT_INFO / NODE_SET_BUMP out of line: the arrays they read in a local CyGlobals, so
 * the shading kernels' register allocation does not carry them */
CY_NOINLINE void svm_eval_attribute_node(const hc_KernelObject *objects,
                                         const hc_KernelShader *shaders,
                                         const hc_uint4 *attributes_map,
                                         const float *attributes_float,
                                         const hc_float2 *attributes_float2,
                                         const hc_float4 *attributes_float3,
                                         const uint32_t *attributes_uchar4,
                                         const hc_uint4 *tri_vindex,
                                         const hc_float4 *curves,
                                         const hc_float4 *curve_keys,
                                         const hc_KernelParticle *particles,
                                         CyAttrIn in,
                                         CySvmStack stack,
                                         hc_uint4 node,
                                         uint *err)
{
  CyGlobals kgv;
  kgv.__curves = curves;
  kgv.__curve_keys = curve_keys;
  kgv.__particles = particles;
  kgv.__objects = objects;
  kgv.__shaders = shaders;
  kgv.__attributes_map = attributes_map;
  kgv.__attributes_float = attributes_float;
  kgv.__attributes_float2 = attributes_float2;
  kgv.__attributes_float3 = attributes_float3;
  kgv.__attributes_uchar4 = attributes_uchar4;
  kgv.__tri_vindex = tri_vindex;
  const CyGlobals *kg = &kgv;
#if CY_CLOSURE_EXT
  const float dd[2] = {in.bump_du, in.bump_dv};
  const float *ddp = in.bump ? dd : nullptr;
#else
  const float *ddp = nullptr;
#endif
  switch (node.x) {
    case NODE_ATTR:
#if CY_CLOSURE_EXT
      svm_node_attr(kg, in.object, in.prim, in.type, in.u, in.v, stack, node, err, ddp, in.bump);
#else
      svm_node_attr(kg, in.object, in.prim, in.type, in.u, in.v, stack, node, err, ddp);
#endif
      break;
    case NODE_VERTEX_COLOR:
      svm_node_vertex_color(kg, in.object, in.prim, in.type, in.u, in.v, stack, node.y, node.z, node.w, err, ddp);
      break;
#if CY_CLOSURE_EXT
    case NODE_SET_BUMP:
      svm_node_set_bump(kg, in, stack, node, err);
      break;
#endif
    case NODE_NORMAL_MAP:
      svm_node_normal_map(kg, in, stack, node, err);
      break;
    case NODE_TANGENT:
      svm_node_tangent(kg, in, stack, node, err);
      break;
    case NODE_OBJECT_INFO:
      svm_node_object_info(kg, in, stack, node.y, node.z, err);
      break;
    case NODE_PARTICLE_INFO:
      svm_node_particle_info(kg, in, stack, node.y, node.z, err);
      break;
#if CY_CLOSURE_EXT
    case NODE_HAIR_INFO:
      svm_node_hair_info(kg, in, stack, node.y, node.z, err);
      break;
#endif
    case NODE_GEOMETRY: /* NODE_GEOM_T only */
      svm_node_geometry_tangent(kg, in, stack, node.z, err);
      break;
  }
}

#endif /* CY_ATTRIBUTE_H */
