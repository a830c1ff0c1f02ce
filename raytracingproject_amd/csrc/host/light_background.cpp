/*
 * light_background.cpp — the background importance map's CDFs, the host step
 * of LightManager::device_update_background (render/light.cpp:530-565
 * background_cdf, 676-716 marginal CDF).  The map itself is the world shader
 * evaluated by the device's SHADER task (hipcy_shader_eval,
 * SHADER_EVAL_BACKGROUND at ((x + 0.5) / w, (y + 0.5) / h)); this turns it into
 * the __light_background_conditional_cdf / __light_background_marginal_cdf
 * arrays the kernels sample (kernel_light_background.h:26-131).
 *
 * Each CDF entry is a float pair: .x the function value (luminance * sin
 * theta), .y the running CDF; the entry after the last holds the total in .x
 * and 1 in .y.  float32 arithmetic in the reference's order (no contraction:
 * built with -ffp-contract=off), sinf from the C library as the reference.
 */
#include <math.h>
#include <stdint.h>

extern "C" {

void hcb_background_cdf(const float *pixels, int res_x, int res_y, float *marg_cdf, float *cond_cdf)
{
  const float pi = 3.14159265358979323846f;
  const int cdf_width = res_x + 1;
  /* conditional CDFs (rows, U direction) */
  for (int i = 0; i < res_y; i++) {
    float *row = cond_cdf + 2 * (size_t)i * cdf_width;
    const float sin_theta = sinf(pi * ((float)i + 0.5f) / (float)res_y);
    for (int j = 0; j < res_x; j++) {
      const float *px = pixels + 4 * ((size_t)i * res_x + j);
      const float ave_luminance = (px[0] + px[1] + px[2]) * (1.0f / 3.0f); /* average() */
      row[2 * j] = ave_luminance * sin_theta;
      row[2 * j + 1] = (j == 0) ? 0.0f : row[2 * (j - 1) + 1] + row[2 * (j - 1)] / (float)res_x;
    }
    const float cdf_total = row[2 * (res_x - 1) + 1] + row[2 * (res_x - 1)] / (float)res_x;
    const float cdf_total_inv = 1.0f / cdf_total;
    row[2 * res_x] = cdf_total;
    if (cdf_total > 0.0f) {
      for (int j = 1; j < res_x; j++) {
        row[2 * j + 1] *= cdf_total_inv;
      }
    }
    row[2 * res_x + 1] = 1.0f;
  }
  /* marginal CDF (column, V direction, sum of rows) */
  marg_cdf[0] = cond_cdf[2 * res_x];
  marg_cdf[1] = 0.0f;
  for (int i = 1; i < res_y; i++) {
    marg_cdf[2 * i] = cond_cdf[2 * ((size_t)i * cdf_width + res_x)];
    marg_cdf[2 * i + 1] = marg_cdf[2 * (i - 1) + 1] + marg_cdf[2 * (i - 1)] / (float)res_y;
  }
  const float cdf_total = marg_cdf[2 * (res_y - 1) + 1] + marg_cdf[2 * (res_y - 1)] / (float)res_y;
  marg_cdf[2 * res_y] = cdf_total;
  if (cdf_total > 0.0f) {
    for (int i = 1; i < res_y; i++) {
      marg_cdf[2 * i + 1] /= cdf_total;
    }
  }
  marg_cdf[2 * res_y + 1] = 1.0f;
}

}  // extern "C"
