// homography.hip -- the reference application's last step,
// host code: findHomography(obj, scene, RANSAC) and perspectiveTransform
// (src/main.cpp:44-62).  A few hundred matches and at most 2000 four-point
// hypotheses: microseconds of CPU work that a GPU launch would only slow
// down, so this stays on the host behind the same C ABI.
//
// Restated from OpenCV 4.x calib3d (not in this image; parity against it is
// unpinned):
//   * RANSACPointSetRegistrator::run with modelPoints 4, threshold 3,
//     confidence 0.995, maxIters 2000, RNG((uint64)-1) (multiply-with-carry,
//     uniform(a, b) = a + next() % (b - a)), getSubset without partial checks
//     (10000 attempts), RANSACUpdateNumIters after every better model;
//   * HomographyEstimatorCallback: checkSubset (haveCollinearPoints on the last
//     point, the 4-triangle orientation test), runKernel (normalised DLT: the
//     eigenvector of the smallest eigenvalue of LtL, here by cyclic Jacobi),
//     computeError (float reprojection error against threshold^2);
//   * then a DLT refit on the inliers and 10 Levenberg-Marquardt iterations on
//     the 8 free entries (a plain LM here, not OpenCV's LMSolver);
//   * perspectiveTransform: w = h20 x + h21 y + h22, (0, 0) when |w| <= FLT_EPSILON.
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "common.hpp"

namespace sift {

namespace {

struct Rng {  // cv::RNG
  uint64_t state;
  unsigned next() {
    state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
    return (unsigned)state;
  }
  int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a)) + a; }
};

struct P2 {
  float x, y;
};

bool collinear_last(const P2* p, int count) {
  const int i = count - 1;
  for (int j = 0; j < i; ++j) {
    const double dx1 = p[j].x - p[i].x, dy1 = p[j].y - p[i].y;
    for (int k = 0; k < j; ++k) {
      const double dx2 = p[k].x - p[i].x, dy2 = p[k].y - p[i].y;
      if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
        return true;
    }
  }
  return false;
}

double det3(double a0, double a1, double b0, double b1, double c0, double c1) {
  // | a0 a1 1 ; b0 b1 1 ; c0 c1 1 |
  return a0 * (b1 - c1) - a1 * (b0 - c0) + (b0 * c1 - b1 * c0);
}

bool check_subset(const P2* s, const P2* d) {
  if (collinear_last(s, 4) || collinear_last(d, 4)) return false;
  static const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
  int negative = 0;
  for (int i = 0; i < 4; ++i) {
    const int* t = tt[i];
    const double A = det3(s[t[0]].x, s[t[0]].y, s[t[1]].x, s[t[1]].y, s[t[2]].x, s[t[2]].y);
    const double B = det3(d[t[0]].x, d[t[0]].y, d[t[1]].x, d[t[1]].y, d[t[2]].x, d[t[2]].y);
    negative += A * B < 0;
  }
  return negative == 0 || negative == 4;
}

// Symmetric 9x9 eigen decomposition (cyclic Jacobi); returns the eigenvector
// of the smallest eigenvalue.
void smallest_eigvec(double A[9][9], double v[9]) {
  double V[9][9];
  for (int i = 0; i < 9; ++i)
    for (int j = 0; j < 9; ++j) V[i][j] = i == j;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int i = 0; i < 9; ++i)
      for (int j = i + 1; j < 9; ++j) off += A[i][j] * A[i][j];
    if (off < 1e-300) break;
    for (int p = 0; p < 9; ++p)
      for (int q = p + 1; q < 9; ++q) {
        if (fabs(A[p][q]) < 1e-300) continue;
        const double th = (A[q][q] - A[p][p]) / (2 * A[p][q]);
        const double t = (th >= 0 ? 1 : -1) / (fabs(th) + sqrt(th * th + 1));
        const double c = 1 / sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < 9; ++k) {
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 9; ++k) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 9; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int m = 0;
  for (int i = 1; i < 9; ++i)
    if (A[i][i] < A[m][m]) m = i;
  for (int i = 0; i < 9; ++i) v[i] = V[i][m];
}

void mat3mul(const double* a, const double* b, double* c) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c[i * 3 + j] = a[i * 3] * b[j] + a[i * 3 + 1] * b[3 + j] + a[i * 3 + 2] * b[6 + j];
}

// HomographyEstimatorCallback::runKernel: H mapping M (src) to m (dst).
bool run_kernel(const P2* M, const P2* m, int count, double* H) {
  double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
  for (int i = 0; i < count; ++i) {
    cmx += m[i].x;
    cmy += m[i].y;
    cMx += M[i].x;
    cMy += M[i].y;
  }
  cmx /= count;
  cmy /= count;
  cMx /= count;
  cMy /= count;
  for (int i = 0; i < count; ++i) {
    smx += fabs(m[i].x - cmx);
    smy += fabs(m[i].y - cmy);
    sMx += fabs(M[i].x - cMx);
    sMy += fabs(M[i].y - cMy);
  }
  if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
    return false;
  smx = count / smx;
  smy = count / smy;
  sMx = count / sMx;
  sMy = count / sMy;
  const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
  const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
  double LtL[9][9];
  memset(LtL, 0, sizeof(LtL));
  for (int i = 0; i < count; ++i) {
    const double x = (m[i].x - cmx) * smx, y = (m[i].y - cmy) * smy;
    const double X = (M[i].x - cMx) * sMx, Y = (M[i].y - cMy) * sMy;
    const double Lx[] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
    const double Ly[] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
    for (int j = 0; j < 9; ++j)
      for (int k = j; k < 9; ++k) LtL[j][k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
  }
  for (int j = 0; j < 9; ++j)
    for (int k = 0; k < j; ++k) LtL[j][k] = LtL[k][j];
  double H0[9], T[9], R[9];
  smallest_eigvec(LtL, H0);
  mat3mul(invHnorm, H0, T);
  mat3mul(T, Hnorm2, R);
  if (fabs(R[8]) < DBL_MIN) return false;
  for (int i = 0; i < 9; ++i) H[i] = R[i] / R[8];
  return true;
}

// computeError + findInliers: float reprojection error <= (float)(thr^2).
int find_inliers(const P2* s, const P2* d, int n, const double* H, double thr, unsigned char* mask) {
  const float t = (float)(thr * thr);
  int count = 0;
  for (int i = 0; i < n; ++i) {
    const float ww = 1.f / (H[6] * s[i].x + H[7] * s[i].y + 1.f);
    const float dx = (H[0] * s[i].x + H[1] * s[i].y + H[2]) * ww - d[i].x;
    const float dy = (H[3] * s[i].x + H[4] * s[i].y + H[5]) * ww - d[i].y;
    const float e = dx * dx + dy * dy;
    mask[i] = e <= t;
    count += mask[i];
  }
  return count;
}

int update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = std::min(std::max(p, 0.), 1.);
  ep = std::min(std::max(ep, 0.), 1.);
  double num = std::max(1. - p, DBL_MIN);
  double denom = 1. - pow(1. - ep, model_points);
  if (denom < DBL_MIN) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)lrint(num / denom);
}

// 10 Levenberg-Marquardt iterations on h[0..7] (h[8] = 1), residuals
// (H s)_xy / (H s)_z - d over the inliers.
void refine_lm(const P2* s, const P2* d, int n, double* H) {
  double lambda = 1e-3;
  auto cost = [&](const double* h) {
    double c = 0;
    for (int i = 0; i < n; ++i) {
      const double w = h[6] * s[i].x + h[7] * s[i].y + 1;
      const double ex = (h[0] * s[i].x + h[1] * s[i].y + h[2]) / w - d[i].x;
      const double ey = (h[3] * s[i].x + h[4] * s[i].y + h[5]) / w - d[i].y;
      c += ex * ex + ey * ey;
    }
    return c;
  };
  double c0 = cost(H);
  for (int it = 0; it < 10; ++it) {
    double JtJ[8][8] = {}, Jtr[8] = {};
    for (int i = 0; i < n; ++i) {
      const double X = s[i].x, Y = s[i].y;
      const double w = H[6] * X + H[7] * Y + 1, iw = 1 / w;
      const double u = (H[0] * X + H[1] * Y + H[2]) * iw, v = (H[3] * X + H[4] * Y + H[5]) * iw;
      const double Jx[8] = {X * iw, Y * iw, iw, 0, 0, 0, -X * u * iw, -Y * u * iw};
      const double Jy[8] = {0, 0, 0, X * iw, Y * iw, iw, -X * v * iw, -Y * v * iw};
      const double rx = u - d[i].x, ry = v - d[i].y;
      for (int a = 0; a < 8; ++a) {
        Jtr[a] += Jx[a] * rx + Jy[a] * ry;
        for (int b = 0; b < 8; ++b) JtJ[a][b] += Jx[a] * Jx[b] + Jy[a] * Jy[b];
      }
    }
    double A[8][9];
    for (int a = 0; a < 8; ++a) {
      for (int b = 0; b < 8; ++b) A[a][b] = JtJ[a][b] + (a == b ? lambda * JtJ[a][a] : 0);
      A[a][8] = -Jtr[a];
    }
    bool ok = true;
    for (int c = 0; c < 8 && ok; ++c) {  // Gaussian elimination, partial pivoting
      int piv = c;
      for (int r = c + 1; r < 8; ++r)
        if (fabs(A[r][c]) > fabs(A[piv][c])) piv = r;
      if (fabs(A[piv][c]) < 1e-300) {
        ok = false;
        break;
      }
      if (piv != c)
        for (int k = 0; k < 9; ++k) std::swap(A[c][k], A[piv][k]);
      for (int r = c + 1; r < 8; ++r) {
        const double f = A[r][c] / A[c][c];
        for (int k = c; k < 9; ++k) A[r][k] -= f * A[c][k];
      }
    }
    if (!ok) break;
    double dx[8];
    for (int c = 7; c >= 0; --c) {
      double v = A[c][8];
      for (int k = c + 1; k < 8; ++k) v -= A[c][k] * dx[k];
      dx[c] = v / A[c][c];
    }
    double Hn[9];
    for (int k = 0; k < 8; ++k) Hn[k] = H[k] + dx[k];
    Hn[8] = 1;
    const double c1 = cost(Hn);
    if (c1 < c0) {
      memcpy(H, Hn, sizeof(Hn));
      c0 = c1;
      lambda = std::max(lambda * 0.1, 1e-12);
    } else {
      lambda *= 10;
    }
  }
}

}  // namespace

int find_homography_ransac(const float* src_xy, const float* dst_xy, int n, double thr, int max_iters,
                           double confidence, double* H, unsigned char* mask_out) {
  if (n < 4 || !(confidence > 0 && confidence < 1) || max_iters < 1) return 0;
  const P2* s = reinterpret_cast<const P2*>(src_xy);
  const P2* d = reinterpret_cast<const P2*>(dst_xy);
  std::vector<unsigned char> best_mask(n, 0), mask(n);
  double best[9] = {0}, model[9];
  bool result = false;
  if (n == 4) {
    if (!run_kernel(s, d, 4, best)) return 0;
    std::fill(best_mask.begin(), best_mask.end(), 1);
    result = true;
  } else {
    Rng rng{~0ull};
    int niters = max_iters, max_good = 0;
    for (int iter = 0; iter < niters; ++iter) {
      // getSubset (no partial checks, 10000 attempts)
      int idx[4];
      P2 ms[4], md[4];
      int i = 0, attempts = 0;
      for (; attempts < 10000; ++attempts) {
        for (i = 0; i < 4;) {
          int idx_i, j;
          for (;;) {
            idx_i = idx[i] = rng.uniform(0, n);
            for (j = 0; j < i; ++j)
              if (idx_i == idx[j]) break;
            if (j == i) break;
          }
          ms[i] = s[idx_i];
          md[i] = d[idx_i];
          ++i;
        }
        if (!check_subset(ms, md)) continue;
        break;
      }
      if (!(i == 4 && attempts < 10000)) {
        if (iter == 0) return 0;
        break;
      }
      if (!run_kernel(ms, md, 4, model)) continue;
      const int good = find_inliers(s, d, n, model, thr, mask.data());
      if (good > std::max(max_good, 3)) {
        best_mask.swap(mask);
        memcpy(best, model, sizeof(best));
        max_good = good;
        niters = update_num_iters(confidence, (double)(n - good) / n, 4, niters);
      }
    }
    result = max_good > 0;
  }
  if (!result) return 0;
  if (n > 4) {  // refit on the inliers, then LM (findHomography, fundam.cpp)
    std::vector<P2> si, di;
    for (int i = 0; i < n; ++i)
      if (best_mask[i]) {
        si.push_back(s[i]);
        di.push_back(d[i]);
      }
    if (!si.empty()) {
      double refit[9];
      if (run_kernel(si.data(), di.data(), (int)si.size(), refit)) memcpy(best, refit, sizeof(best));
      refine_lm(si.data(), di.data(), (int)si.size(), best);
    }
  }
  for (int i = 0; i < 9; ++i) H[i] = best[i] / best[8];
  if (mask_out) memcpy(mask_out, best_mask.data(), n);
  return 1;
}

void perspective_transform(const double* H, const float* xy, int n, float* out) {
  for (int i = 0; i < n; ++i) {
    const double x = xy[2 * i], y = xy[2 * i + 1];
    const double w = H[6] * x + H[7] * y + H[8];
    if (fabs(w) > FLT_EPSILON) {
      const double iw = 1. / w;
      out[2 * i] = (float)((H[0] * x + H[1] * y + H[2]) * iw);
      out[2 * i + 1] = (float)((H[3] * x + H[4] * y + H[5]) * iw);
    } else {
      out[2 * i] = out[2 * i + 1] = 0.f;
    }
  }
}

}  // namespace sift
