/*
 * cy_svm_extra.h — input / vector / converter nodes of the SVM beyond the
 * texture set (cy_svm_nodes.h), each with the reference's arithmetic:
 *   Camera Data        kernel/svm/svm_camera.h:19-45
 *   Normal             kernel/svm/svm_normal.h:19-45
 *   RGB / Vector Curves kernel/svm/svm_ramp.h:21-109 (extrapolated lookups)
 *   Vector Rotate      kernel/svm/svm_vector_rotate.h:21-79
 *   Vector Transform   kernel/svm/svm_vector_transform.h:21-104
 * (__OBJECT_MOTION__ forms of the object transforms: the object's static
 * tfm / itfm, geom_object.h).
 */
#ifndef CY_SVM_EXTRA_H
#define CY_SVM_EXTRA_H

enum {
  NODE_CAMERA = 54,
  NODE_NORMAL = 65,
  NODE_RGB_CURVES = 68,
  NODE_VECTOR_CURVES = 69,
  NODE_VECTOR_ROTATE = 78,
  NODE_VECTOR_TRANSFORM = 79
};

/* svm_camera.h:19-45 */
CY_FN void svm_node_camera(const CyGlobals *kg, const CySD *sd, CySvmStack stack, uint out_vector, uint out_zdepth,
                           uint out_distance, uint *err)
{
  const struct cy_tfm *tfm = (const struct cy_tfm *)&KD->cam.worldtocamera;
  const cfloat3 vector = transform_point(tfm, sd->P);
  const float zdepth = vector.z;
  const float distance = len3(vector);
  if (out_vector != SVM_STACK_INVALID) {
    svm_store3(stack, out_vector, normalize3(vector), err);
  }
  if (out_zdepth != SVM_STACK_INVALID) {
    svm_store(stack, out_zdepth, zdepth, err);
  }
  if (out_distance != SVM_STACK_INVALID) {
    svm_store(stack, out_distance, distance, err);
  }
}

/* svm_normal.h:19-45: the node's direction (extra node) and its dot product
 * with the normalised input */
CY_FN void svm_node_normal(const CyGlobals *kg, CySvmStack stack, uint in_normal_offset, uint out_normal_offset,
                           uint out_dot_offset, int *offset, uint *err)
{
  const hc_uint4 node1 = kg->__svm_nodes[*offset];
  (*offset)++;
  const cfloat3 normal = svm_load3(stack, in_normal_offset, err);
  const cfloat3 direction = normalize3(mk3(as_float(node1.x), as_float(node1.y), as_float(node1.z)));
  if (out_normal_offset != SVM_STACK_INVALID) {
    svm_store3(stack, out_normal_offset, direction, err);
  }
  if (out_dot_offset != SVM_STACK_INVALID) {
    svm_store(stack, out_dot_offset, dot3(direction, normalize3(normal)), err);
  }
}

/* svm_ramp.h:21-54 rgb_ramp_lookup with extrapolation (curves) */
CY_FN hc_float4 curves_lookup(const CyGlobals *kg, int offset, float f, int table_size)
{
  if (f < 0.0f || f > 1.0f) {
    hc_float4 t0, t1;
    if (f < 0.0f) {
      t0 = svm_node_float4(kg, offset);
      t1 = svm_node_float4(kg, offset + 1);
      f = -f;
    }
    else {
      t0 = svm_node_float4(kg, offset + table_size - 1);
      t1 = svm_node_float4(kg, offset + table_size - 2);
      f = f - 1.0f;
    }
    /* t0 + dy * f * (table_size - 1), dy = t0 - t1 */
    const float n = (float)(table_size - 1);
    return svm_f4(t0.x + (t0.x - t1.x) * f * n, t0.y + (t0.y - t1.y) * f * n, t0.z + (t0.z - t1.z) * f * n,
                  t0.w + (t0.w - t1.w) * f * n);
  }
  return rgb_ramp_lookup(kg, offset, f, true, table_size);
}

/* svm_ramp.h:84-109 svm_node_curves (RGB Curves and Vector Curves) */
CY_FN void svm_node_curves(const CyGlobals *kg, CySvmStack stack, hc_uint4 node, int *offset, uint *err)
{
  uint fac_offset, color_offset, out_offset;
  svm_unpack3(node.y, &fac_offset, &color_offset, &out_offset);
  const int table_size = (int)kg->__svm_nodes[*offset].x;
  (*offset)++;
  const float fac = svm_load(stack, fac_offset, err);
  cfloat3 color = svm_load3(stack, color_offset, err);
  const float min_x = as_float(node.z), max_x = as_float(node.w);
  const float range_x = max_x - min_x;
  /* (color - min_x) / range_x: float3 / float multiplies by the reciprocal */
  const float inv_range = 1.0f / range_x;
  const cfloat3 relpos = mul3f(sub3(color, mk3(min_x, min_x, min_x)), inv_range);
  const float r = curves_lookup(kg, *offset, relpos.x, table_size).x;
  const float g = curves_lookup(kg, *offset, relpos.y, table_size).y;
  const float b = curves_lookup(kg, *offset, relpos.z, table_size).z;
  color = add3(mul3f(color, 1.0f - fac), mul3f(mk3(r, g, b), fac));
  svm_store3(stack, out_offset, color, err);
  *offset += table_size;
}

/* util_transform.h:151-178 euler_to_transform */
CY_FN struct cy_tfm euler_to_tfm(cfloat3 rotation)
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
  return t;
}

/* svm_vector_rotate.h:21-79 */
CY_FN void svm_node_vector_rotate(CySvmStack stack, uint input_stack_offsets, uint axis_stack_offsets,
                                  uint result_stack_offset, uint *err)
{
  uint type, vector_stack_offset, rotation_stack_offset, invert;
  svm_unpack4(input_stack_offsets, &type, &vector_stack_offset, &rotation_stack_offset, &invert);
  uint center_stack_offset, axis_stack_offset, angle_stack_offset;
  svm_unpack3(axis_stack_offsets, &center_stack_offset, &axis_stack_offset, &angle_stack_offset);
  if (result_stack_offset == SVM_STACK_INVALID) {
    return;
  }
  const cfloat3 vector = svm_load3(stack, vector_stack_offset, err);
  const cfloat3 center = svm_load3(stack, center_stack_offset, err);
  cfloat3 result;
  if (type == 4) { /* NODE_VECTOR_ROTATE_TYPE_EULER_XYZ */
    const struct cy_tfm t = euler_to_tfm(svm_load3(stack, rotation_stack_offset, err));
    const cfloat3 v = sub3(vector, center);
    result = add3(invert ? transform_direction_transposed(&t, v) : transform_direction(&t, v), center);
  }
  else {
    cfloat3 axis;
    switch (type) {
      case 1:
        axis = mk3(1.0f, 0.0f, 0.0f);
        break;
      case 2:
        axis = mk3(0.0f, 1.0f, 0.0f);
        break;
      case 3:
        axis = mk3(0.0f, 0.0f, 1.0f);
        break;
      default:
        axis = normalize3(svm_load3(stack, axis_stack_offset, err));
        break;
    }
    float angle = svm_load(stack, angle_stack_offset, err);
    angle = invert ? -angle : angle;
    result = (dot3(axis, axis) != 0.0f) ? add3(rotate_around_axis(sub3(vector, center), axis, angle), center) :
                                          vector;
  }
  svm_store3(stack, result_stack_offset, result, err);
}

/* svm_vector_transform.h:21-104 */
CY_FN void svm_node_vector_transform(const CyGlobals *kg, const CySD *sd, CySvmStack stack, hc_uint4 node, uint *err)
{
  uint itype, ifrom, ito;
  svm_unpack3(node.y, &itype, &ifrom, &ito);
  const uint vector_in = node.z & 0xFF, vector_out = (node.z >> 8) & 0xFF;
  cfloat3 in = svm_load3(stack, vector_in, err);
  const bool is_object = (sd->object != OBJECT_NONE);
  const bool is_direction = (itype == 0 || itype == 2); /* VECTOR, NORMAL */
  const struct cy_tfm *w2c = (const struct cy_tfm *)&KD->cam.worldtocamera;
  const struct cy_tfm *c2w = (const struct cy_tfm *)&KD->cam.cameratoworld;
  if (ifrom == 0) { /* from world */
    if (ito == 2) {
      in = is_direction ? transform_direction(w2c, in) : transform_point(w2c, in);
    }
    else if (ito == 1 && is_object) { /* object_inverse_dir / position_transform */
      const struct cy_tfm *it = object_itfm(kg, sd->object);
      in = is_direction ? transform_direction(it, in) : transform_point(it, in);
    }
  }
  else if (ifrom == 2) { /* from camera */
    if (ito == 0 || ito == 1) {
      in = is_direction ? transform_direction(c2w, in) : transform_point(c2w, in);
    }
    if (ito == 1 && is_object) {
      const struct cy_tfm *it = object_itfm(kg, sd->object);
      in = is_direction ? transform_direction(it, in) : transform_point(it, in);
    }
  }
  else if (ifrom == 1) { /* from object */
    if ((ito == 0 || ito == 2) && is_object) { /* object_dir / position_transform */
      const struct cy_tfm *t = object_tfm(kg, sd->object);
      in = is_direction ? transform_direction(t, in) : transform_point(t, in);
    }
    if (ito == 2) {
      in = is_direction ? transform_direction(w2c, in) : transform_point(w2c, in);
    }
  }
  if (itype == 2) {
    in = normalize3(in);
  }
  if (vector_out != SVM_STACK_INVALID) {
    svm_store3(stack, vector_out, in, err);
  }
}

#endif /* CY_SVM_EXTRA_H */
