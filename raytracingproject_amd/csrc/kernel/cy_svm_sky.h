/*
 * cy_svm_sky.h — the Sky Texture node (kernel/svm/svm_sky.h:21-330) for the HIP
 * device: Preetham and Hosek-Wilkie analytic skies from the host-precomputed
 * model parameters the node carries, and the Nishita sky from its precomputed
 * texture plus the sun disc.  Every libm call is the glibc restatement of
 * cy_math.h; expressions keep the reference's operation order.  Included by
 * cy_path.h after cy_svm_image.h.
 */
#ifndef CY_SVM_SKY_H
#define CY_SVM_SKY_H

enum { NODE_TEX_SKY = 56 };

/* kernel_projection.h:40-46 */
CY_FN void sky_direction_to_spherical(cfloat3 dir, float *theta, float *phi)
{
  *theta = safe_acosf(dir.z);
  *phi = cy_atan2f(dir.x, dir.y);
}

/* kernel_color.h xyz_to_rgb: rows of the scene's XYZ -> RGB matrix (film) */
CY_FN cfloat3 sky_xyz_to_rgb(const CyGlobals *kg, cfloat3 xyz)
{
  return mk3(dot3(mk3(KD->film.xyz_to_r.x, KD->film.xyz_to_r.y, KD->film.xyz_to_r.z), xyz),
             dot3(mk3(KD->film.xyz_to_g.x, KD->film.xyz_to_g.y, KD->film.xyz_to_g.z), xyz),
             dot3(mk3(KD->film.xyz_to_b.x, KD->film.xyz_to_b.y, KD->film.xyz_to_b.z), xyz));
}

/* util_color.h:168-186 */
CY_FN cfloat3 sky_xyY_to_xyz(float x, float y, float Y)
{
  const float X = (y != 0.0f) ? (x / y) * Y : 0.0f;
  const float Z = (y != 0.0f && Y != 0.0f) ? (1.0f - x - y) / y * Y : 0.0f;
  return mk3(X, Y, Z);
}

/* svm_sky.h:21-25 */
CY_FN float sky_angle_between(float thetav, float phiv, float theta, float phi)
{
  const float cospsi = cy_sinf(thetav) * cy_sinf(theta) * cy_cosf(phi - phiv) + cy_cosf(thetav) * cy_cosf(theta);
  return safe_acosf(cospsi);
}

/* svm_sky.h:31-38 (Preetham) */
CY_FN float sky_perez_function(const float *lam, float theta, float gamma)
{
  const float ctheta = cy_cosf(theta);
  const float cgamma = cy_cosf(gamma);
  return (1.0f + lam[0] * cy_expf(lam[1] / ctheta)) *
         (1.0f + lam[2] * cy_expf(lam[3] * gamma) + lam[4] * cgamma * cgamma);
}

/* svm_sky.h:76-91 (Hosek-Wilkie) */
CY_FN float sky_radiance_internal(const float *c, float theta, float gamma)
{
  const float ctheta = cy_cosf(theta);
  const float cgamma = cy_cosf(gamma);
  const float expM = cy_expf(c[4] * gamma);
  const float rayM = cgamma * cgamma;
  const float mieM = (1.0f + rayM) / cy_powf((1.0f + c[8] * c[8] - 2.0f * c[8] * cgamma), 1.5f);
  const float zenith = sqrtf(ctheta);
  return (1.0f + c[0] * cy_expf(c[1] / (ctheta + 0.01f))) *
         (c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith);
}

/* svm_sky.h:40-122: the two analytic models share their parameter block */
CY_FN cfloat3 sky_radiance_analytic(const CyGlobals *kg, cfloat3 dir, int model, const float *p)
{
  const float sunphi = p[0], suntheta = p[1];
  const float *config_x = p + 5, *config_y = p + 14, *config_z = p + 23;
  float theta, phi;
  sky_direction_to_spherical(dir, &theta, &phi);
  const float gamma = sky_angle_between(theta, phi, suntheta, sunphi);
  theta = fminf(theta, CY_PI_2_F - 0.001f);
  if (model == 0) {
    /* radiance_x/y/z hold the zenith Y / x / y (nodes.cpp:645-705) */
    const float x = p[3] * sky_perez_function(config_y, theta, gamma);
    const float y = p[4] * sky_perez_function(config_z, theta, gamma);
    const float Y = p[2] * sky_perez_function(config_x, theta, gamma);
    return sky_xyz_to_rgb(kg, sky_xyY_to_xyz(x, y, Y));
  }
  const float x = sky_radiance_internal(config_x, theta, gamma) * p[2];
  const float y = sky_radiance_internal(config_y, theta, gamma) * p[3];
  const float z = sky_radiance_internal(config_z, theta, gamma) * p[4];
  return mul3f(sky_xyz_to_rgb(kg, mk3(x, y, z)), CY_2PI_F / 683.0f);
}

/* svm_sky.h:125-128 (std::cos / std::sin of a float: glibc cosf / sinf) */
CY_FN cfloat3 sky_geographical_to_direction(float lat, float lon)
{
  return mk3(cy_cosf(lat) * cy_cosf(lon), cy_cosf(lat) * cy_sinf(lon), cy_sinf(lat));
}

/* util_math.h:795-798 */
CY_FN float sky_precise_angle(cfloat3 a, cfloat3 b)
{
  return 2.0f * cy_atan2f(len3(sub3(a, b)), len3(add3(a, b)));
}

CY_FN cfloat3 sky_interp3(cfloat3 a, cfloat3 b, float t)
{
  return add3(a, mul3f(sub3(b, a), t));
}

/* svm_sky.h:130-210 */
CY_FN cfloat3 sky_radiance_nishita(const CyGlobals *kg, const hc_TextureInfo *texture_info, cfloat3 dir,
                                   const float *nishita_data, uint texture_id)
{
  const float sun_elevation = nishita_data[6];
  const float sun_rotation = nishita_data[7];
  const float angular_diameter = nishita_data[8];
  const float sun_intensity = nishita_data[9];
  const bool sun_disc = (angular_diameter >= 0.0f);
  cfloat3 xyz = mk3(0.0f, 0.0f, 0.0f);
  float dtheta, dphi;
  sky_direction_to_spherical(dir, &dtheta, &dphi);
  if (dir.z >= 0.0f) {
    const cfloat3 sun_dir = sky_geographical_to_direction(sun_elevation, sun_rotation + CY_PI_2_F);
    const float sun_dir_angle = sky_precise_angle(dir, sun_dir);
    const float half_angular = angular_diameter / 2.0f;
    const float dir_elevation = CY_PI_2_F - dtheta;
    if (sun_disc && sun_dir_angle < half_angular) {
      const cfloat3 pixel_bottom = mk3(nishita_data[0], nishita_data[1], nishita_data[2]);
      const cfloat3 pixel_top = mk3(nishita_data[3], nishita_data[4], nishita_data[5]);
      if (sun_elevation - half_angular > 0.0f) {
        if (sun_elevation + half_angular > 0.0f) {
          const float y = ((dir_elevation - sun_elevation) / angular_diameter) + 0.5f;
          xyz = mul3f(sky_interp3(pixel_bottom, pixel_top, y), sun_intensity);
        }
      }
      else {
        if (sun_elevation + half_angular > 0.0f) {
          const float y = dir_elevation / (sun_elevation + half_angular);
          xyz = mul3f(sky_interp3(pixel_bottom, pixel_top, y), sun_intensity);
        }
      }
      /* limb darkening, coefficient 0.6 */
      const float limb_darkening = (1.0f - 0.6f * (1.0f - sqrtf(1.0f - sqr(sun_dir_angle / half_angular))));
      xyz = mul3f(xyz, limb_darkening);
    }
    else {
      float x = (dphi + CY_PI_F + sun_rotation) / CY_2PI_F;
      const float y = safe_sqrtf(dir_elevation / CY_PI_2_F);
      if (x > 1.0f) {
        x -= 1.0f;
      }
      const hc_float4 t = kernel_tex_image_interp(texture_info, (int)texture_id, x, y);
      xyz = mk3(t.x, t.y, t.z);
    }
  }
  else {
    if (dir.z < -0.4f) {
      xyz = mk3(0.0f, 0.0f, 0.0f);
    }
    else {
      /* black ground fade */
      float fade = 1.0f + dir.z * 2.5f;
      fade = sqr(fade) * fade;
      float x = (dphi + CY_PI_F + sun_rotation) / CY_2PI_F;
      if (x > 1.0f) {
        x -= 1.0f;
      }
      const hc_float4 t = kernel_tex_image_interp(texture_info, (int)texture_id, x, -0.5f);
      xyz = mul3f(mk3(t.x, t.y, t.z), fade);
    }
  }
  return sky_xyz_to_rgb(kg, xyz);
}

/* svm_sky.h:212-330 svm_node_tex_sky: NODE_TEX_SKY (vector, out, model) and
 * 8 parameter nodes (Preetham / Hosek: sunphi, suntheta, radiance xyz, the
 * three 9-entry configurations) or 3 (Nishita: 10 floats + texture slot). */
CY_FN void svm_node_tex_sky(const CyGlobals *kg, const hc_TextureInfo *texture_info, CySvmStack stack,
                            hc_uint4 node, int *offset, uint *err)
{
  const uint dir_offset = node.y, out_offset = node.z;
  const int sky_model = (int)node.w;
  const cfloat3 dir = svm_load3(stack, dir_offset, err);
  cfloat3 f;
  if (sky_model == 0 || sky_model == 1) {
    float p[32];
    for (int k = 0; k < 8; k++) {
      const hc_uint4 d = kg->__svm_nodes[*offset];
      *offset += 1;
      p[4 * k + 0] = as_float(d.x);
      p[4 * k + 1] = as_float(d.y);
      p[4 * k + 2] = as_float(d.z);
      p[4 * k + 3] = as_float(d.w);
    }
    f = sky_radiance_analytic(kg, dir, sky_model, p);
  }
  else {
    float nishita_data[10];
    const hc_uint4 d0 = kg->__svm_nodes[*offset];
    const hc_uint4 d1 = kg->__svm_nodes[*offset + 1];
    const hc_uint4 d2 = kg->__svm_nodes[*offset + 2];
    *offset += 3;
    nishita_data[0] = as_float(d0.x);
    nishita_data[1] = as_float(d0.y);
    nishita_data[2] = as_float(d0.z);
    nishita_data[3] = as_float(d0.w);
    nishita_data[4] = as_float(d1.x);
    nishita_data[5] = as_float(d1.y);
    nishita_data[6] = as_float(d1.z);
    nishita_data[7] = as_float(d1.w);
    nishita_data[8] = as_float(d2.x);
    nishita_data[9] = as_float(d2.y);
    f = sky_radiance_nishita(kg, texture_info, dir, nishita_data, d2.z);
  }
  svm_store3(stack, out_offset, f, err);
}

#endif /* CY_SVM_SKY_H */
