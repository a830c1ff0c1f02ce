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
 * The host packs attributes only for triangle meshes without subdivision
 * (`__tri_patch` is all ~0, so attribute_primitive_type is always
 * ATTR_PRIM_GEOMETRY); an attribute found on a curve raises
 * CY_ERR_FEATURE.  Per-object maps: KernelObject.attribute_map_offset into
 * `__attributes_map`, two rows (geometry, subdivision) per attribute, closed
 * by ATTR_STD_NONE.
 */
#ifndef CY_ATTRIBUTE_H
#define CY_ATTRIBUTE_H

enum {
  NODE_ATTR = 16,
  NODE_VERTEX_COLOR = 17
};

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
 * does not handle */
CY_FN void triangle_attribute(const CyGlobals *kg, const CyAttr &desc, int prim, float u, float v, int n, float out[4])
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
}

/* svm_node_attr: the attribute read with the stored type, converted to the
 * node's output type (float: the average of a colour / vector) */
CY_FN void svm_node_attr(const CyGlobals *kg, int object, int prim, int type, float u, float v, CySvmStack stack,
                         hc_uint4 node, uint *err)
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
  if (!tri && (type & PRIMITIVE_ALL_CURVE) && desc.element != ATTR_ELEMENT_NONE) {
    cy_set_error(err, CY_ERR_FEATURE, 11); /* curve attributes are not packed */
  }
  float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const int n = (desc.type == NODE_ATTR_FLOAT) ? 1 : (desc.type == NODE_ATTR_FLOAT2) ? 2 :
                (desc.type == NODE_ATTR_RGBA)  ? 4 :
                                                 3;
  if (tri) {
    triangle_attribute(kg, desc, prim, u, v, n, f);
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
                                 CySvmStack stack, uint layer_id, uint color_offset, uint alpha_offset, uint *err)
{
  const CyAttr desc = find_attribute(kg, object, prim, layer_id);
  if (desc.offset != (int)ATTR_STD_NOT_FOUND) {
    float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (type & PRIMITIVE_ALL_TRIANGLE) {
      triangle_attribute(kg, desc, prim, u, v, 4, f);
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

/* NODE_ATTR / NODE_VERTEX_COLOR out of line: the arrays they read in a local
 * CyGlobals, so the shading kernels' register allocation does not carry them */
CY_NOINLINE void svm_eval_attribute_node(const hc_KernelObject *objects,
                                         const hc_uint4 *attributes_map,
                                         const float *attributes_float,
                                         const hc_float2 *attributes_float2,
                                         const hc_float4 *attributes_float3,
                                         const uint32_t *attributes_uchar4,
                                         const hc_uint4 *tri_vindex,
                                         int object,
                                         int prim,
                                         int type,
                                         float u,
                                         float v,
                                         CySvmStack stack,
                                         hc_uint4 node,
                                         uint *err)
{
  CyGlobals kgv;
  kgv.__objects = objects;
  kgv.__attributes_map = attributes_map;
  kgv.__attributes_float = attributes_float;
  kgv.__attributes_float2 = attributes_float2;
  kgv.__attributes_float3 = attributes_float3;
  kgv.__attributes_uchar4 = attributes_uchar4;
  kgv.__tri_vindex = tri_vindex;
  const CyGlobals *kg = &kgv;
  if (node.x == NODE_ATTR) {
    svm_node_attr(kg, object, prim, type, u, v, stack, node, err);
  }
  else {
    svm_node_vertex_color(kg, object, prim, type, u, v, stack, node.y, node.z, node.w, err);
  }
}

#endif /* CY_ATTRIBUTE_H */
