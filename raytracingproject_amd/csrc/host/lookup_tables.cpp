/*
 * lookup_tables.cpp — host-built lookup tables the kernel reads from
 * __lookup_table (render/tables.cpp LookupTables).
 *
 * cyh_beckmann_table: the Beckmann visible-slope sampling table of
 * render/shader.cpp:52-135 (beckmann_table_rows; Heitz & d'Eon 2014,
 * supplemental 2/2), BECKMANN_TABLE_SIZE^2 floats.  Row i is the inverse CDF
 * of the marginal visible slope distribution P22_wi(x) for cos(theta_i) =
 * i / (SIZE - 1), sampled at SIZE values of U.  Arithmetic as the reference:
 * float expf per P22 term, float per-slope sums, double CDF and inversion.
 * Built with -ffp-contract=off like the reference host.
 */
#include <cmath>
#include <vector>

namespace {

constexpr int kBeckmannTableSize = 256;
constexpr int kDataTmpSize = 512;
constexpr float kSlopeMax = 6.0f; /* range holding 99.99 % of the distribution */

float p22(float slope_x, float slope_y)
{
  return expf(-(slope_x * slope_x + slope_y * slope_y));
}

void beckmann_rows(float *table, int row_from, int row_to)
{
  std::vector<double> slope_x(kDataTmpSize), cdf(kDataTmpSize);
  for (int index_theta = row_from; index_theta < row_to; index_theta++) {
    const float cos_theta = index_theta / (kBeckmannTableSize - 1.0f);
    const float s2 = 1.0f - cos_theta * cos_theta;
    const float sin_theta = sqrtf(s2 > 0.0f ? s2 : 0.0f);
    slope_x[0] = (double)-kSlopeMax;
    cdf[0] = 0;
    for (int ix = 1; ix < kDataTmpSize; ++ix) {
      slope_x[ix] = (double)(-kSlopeMax + 2.0f * kSlopeMax * ix / (kDataTmpSize - 1.0f));
      float dot_product = fmaxf(0.0f, -(float)slope_x[ix] * sin_theta + cos_theta);
      float marginal = 0.0f;
      for (int j = 0; j < 100; ++j) {
        float slope_y = -kSlopeMax + 2.0f * kSlopeMax * j * (1.0f / 99.0f);
        marginal += dot_product * p22((float)slope_x[ix], slope_y);
      }
      cdf[ix] = cdf[ix - 1] + (double)marginal;
    }
    for (int ix = 1; ix < kDataTmpSize; ++ix) {
      cdf[ix] /= cdf[kDataTmpSize - 1];
    }
    int ix = 0;
    for (int index_U = 0; index_U < kBeckmannTableSize; ++index_U) {
      const double U = 0.0000001 + 0.9999998 * index_U / (double)(kBeckmannTableSize - 1);
      while (cdf[ix] <= U) {
        ++ix;
      }
      const double interp = (cdf[ix] - U) / (cdf[ix] - cdf[ix - 1]);
      table[index_U + index_theta * kBeckmannTableSize] =
          (float)(interp * slope_x[ix - 1] + (1.0 - interp) * slope_x[ix]);
    }
  }
}

}  // namespace

extern "C" int cyh_beckmann_table_size()
{
  return kBeckmannTableSize;
}

/* out: kBeckmannTableSize^2 floats */
extern "C" void cyh_beckmann_table(float *out)
{
  beckmann_rows(out, 0, kBeckmannTableSize);
}
