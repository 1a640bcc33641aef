// gauss_host.hpp -- the Gaussian coefficients of SIFT_NCL, host side, no HIP.
//
// One definition shared by the library (the tables every blur kernel uses,
// api.hip / blur.hip) and by gen_sym_coefs.cpp, which prints the same tables
// as compile-time constants for the symmetric octave blur (blur.hip).  The
// library re-checks at context creation that the compiled-in tables equal the
// ones it computes, entry for entry.
#pragma once

#include <math.h>

namespace sift {

constexpr int kLayers = 2;                // nOctaveLayers
constexpr double kSigma = 1.6;            // src/sift.cpp:6
constexpr double kRefPi = 3.14159265359;  // src/sift.cpp:7

// getGaussianKernel(float sigma), src/sift.cpp:95-108: a (2w+1)^2 table,
// w = floor(3 sigma), K[a][b] = (float)(8192 * norm * exp(-(a^2+b^2) / den))
// with norm in double and den = (double)(2 sigma sigma) from a float product.
// Returns the table side 2w+1; writes the table when coeff is non-null.
inline int gaussian_kernel_host(float sigma, float* coeff) {
  const int w = (int)floor(3 * sigma);
  const int size = 2 * w + 1;
  const double norm = 1. / (2 * kRefPi * sigma * sigma);  // double chain
  const double den = (double)(2 * sigma * sigma);          // float chain, then double
  if (coeff)
    for (int a = -w; a <= w; ++a)
      for (int b = -w; b <= w; ++b) {
        double g = norm * exp(-(a * a + b * b) * 1. / den);
        g = g * 8192;
        coeff[(a + w) * size + (b + w)] = (float)g;
      }
  return size;
}

// SIFT_FLAG_FAST's 1-D taps: g(a) = exp(-a^2 / (2 sigma^2)) / sqrt(2 pi sigma^2)
// for a in [-w, w], the square root of getGaussianKernel's normalisation
// (src/sift.cpp:103, same float 2*sigma*sigma chain and PI), so that
// K[a][b] / 8192 = g(a) g(b) up to float rounding.  Returns 2w+1.
inline int fast_taps_host(float sigma, float* g) {
  const int w = (int)floor(3 * sigma);
  const double den = (double)(2 * sigma * sigma);
  const double nrm = 1. / sqrt(2 * kRefPi * sigma * sigma);
  if (g)
    for (int a = -w; a <= w; ++a) g[a + w] = (float)(nrm * exp(-(a * a) * 1. / den));
  return 2 * w + 1;
}

// The five blur sigmas of SIFT_NCL: the base sqrt(1.6^2 + 0.2^2)
// (src/sift.cpp:237) and sig[1..4] (:240-245).
inline void sift_sigmas(float* base, float* sig) {
  *base = (float)sqrt(kSigma * kSigma + 0.2 * 0.2);
  const double k = pow(2.0, 1.0 / kLayers);
  for (int i = 1; i <= 4; ++i) {
    const double tot = pow(k * 1.0, (double)i) * kSigma;
    sig[i - 1] = (float)sqrt(tot * tot - kSigma * kSigma);
  }
}

}  // namespace sift
