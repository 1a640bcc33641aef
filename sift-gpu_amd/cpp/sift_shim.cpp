// sift_shim.cpp -- the reference's C++ API (include/sift.hpp) on top of the
// C ABI (include/sift_hip.h).  Only plain pointers cross into the GPU library;
// this file converts cv::Mat / std::vector<KeyPoint> to packed host buffers.
#include "sift.hpp"

#include <stdlib.h>
#include <string.h>

#include <memory>
#include <stdexcept>
#include <string>

#include "sift_hip.h"

static_assert(sizeof(KeyPoint) == sizeof(sift_keypoint), "cv::KeyPoint layout must match sift_keypoint");

namespace {

struct CtxHolder {
  sift_ctx* ctx = nullptr;
  int rows = 0, cols = 0;
  ~CtxHolder() {
    if (ctx) sift_ctx_destroy(ctx);
  }
};

thread_local CtxHolder g_ctx;

[[noreturn]] void raise(const char* fn, int rc, sift_ctx* c) {
  throw std::runtime_error(std::string(fn) + ": " + (c ? sift_last_error(c) : "") + " (code " +
                           std::to_string(rc) + ")");
}

// One context per thread, grown to the largest image seen.
sift_ctx* ctx_for(int rows, int cols) {
  if (g_ctx.ctx && rows <= g_ctx.rows && cols <= g_ctx.cols) return g_ctx.ctx;
  const int r = std::max(rows, g_ctx.rows), c = std::max(cols, g_ctx.cols);
  if (g_ctx.ctx) sift_ctx_destroy(g_ctx.ctx);
  g_ctx.ctx = nullptr;
  const char* dev = getenv("SIFT_HIP_DEVICE");
  const char* verb = getenv("SIFT_HIP_VERBOSE");
  unsigned flags = (verb && atoi(verb)) ? SIFT_FLAG_VERBOSE : 0u;
  int rc = sift_ctx_create(dev ? atoi(dev) : 0, r, c, 1, flags, &g_ctx.ctx);
  if (rc) raise("sift_ctx_create", rc, nullptr);
  g_ctx.rows = r;
  g_ctx.cols = c;
  return g_ctx.ctx;
}

void require_f32(const Mat& m, const char* fn) {
  if (m.empty()) throw std::runtime_error(std::string(fn) + ": empty image");
  if (m.type() != CV_32FC1) throw std::runtime_error(std::string(fn) + ": expected CV_32FC1 (DATATYPE)");
  if (!m.isContinuous()) throw std::runtime_error(std::string(fn) + ": expected a continuous Mat");
}

std::vector<float> pack(std::vector<Mat>& planes, int rows, int cols, int n_oct, int per,
                        const char* fn) {
  std::vector<float> buf(sift_packed_size(rows, cols, n_oct, per));
  if ((int)planes.size() < n_oct * per) throw std::runtime_error(std::string(fn) + ": too few planes");
  std::vector<int> orows(n_oct), ocols(n_oct);
  sift_octave_shapes(rows, cols, n_oct, orows.data(), ocols.data());
  size_t off = 0;
  for (int o = 0; o < n_oct; ++o)
    for (int s = 0; s < per; ++s) {
      Mat& m = planes[o * per + s];
      require_f32(m, fn);
      if (m.rows != orows[o] || m.cols != ocols[o])
        throw std::runtime_error(std::string(fn) + ": plane size does not match the octave shape");
      memcpy(buf.data() + off, m.ptr<float>(0), sizeof(float) * m.rows * m.cols);
      off += (size_t)m.rows * m.cols;
    }
  return buf;
}

void unpack(const std::vector<float>& buf, std::vector<Mat>& planes, int rows, int cols, int n_oct,
            int per) {
  planes.resize((size_t)n_oct * per);
  std::vector<int> orows(n_oct), ocols(n_oct);
  sift_octave_shapes(rows, cols, n_oct, orows.data(), ocols.data());
  size_t off = 0;
  for (int o = 0; o < n_oct; ++o)
    for (int s = 0; s < per; ++s) {
      Mat m(orows[o], ocols[o], CV_32FC1);
      memcpy(m.ptr<float>(0), buf.data() + off, sizeof(float) * m.rows * m.cols);
      off += (size_t)m.rows * m.cols;
      planes[o * per + s] = m;
    }
}

}  // namespace

// src/sift.cpp:49-57 -- a third-party algorithm (opencv_contrib SIFT).
void SITF_BuildIn_OpenCV(InputArray image, std::vector<KeyPoint>& keypoints, OutputArray descriptors) {
#if defined(SIFT_HIP_HAVE_OPENCV) && defined(CV_VERSION_MAJOR) && (CV_VERSION_MAJOR >= 4) && \
    (CV_VERSION_MINOR >= 4 || CV_VERSION_MAJOR > 4)
  Ptr<SIFT> det = SIFT::create();
  Mat mask;
  det->detectAndCompute(image, mask, keypoints, descriptors, false);
#else
  (void)image;
  (void)keypoints;
  (void)descriptors;
  throw std::runtime_error("SITF_BuildIn_OpenCV: OpenCV's SIFT is not available in this build");
#endif
}

// src/sift.cpp:59-91
void SIFT_NCL(InputArray image, std::vector<KeyPoint>& keypoints, OutputArray descriptors) {
  Mat img = image.getMat();
  require_f32(img, "SIFT_NCL");
  sift_ctx* c = ctx_for(img.rows, img.cols);
  int n = 0;
  int rc = sift_detect_compute(c, img.ptr<float>(0), img.rows, img.cols, sizeof(float) * img.cols,
                               nullptr, nullptr, 0, &n);
  if (rc != SIFT_OK && rc != SIFT_E_CAPACITY) raise("SIFT_NCL", rc, c);
  keypoints.resize(n);
  descriptors.create(n, SIFT_DESC_LEN, CV_32F);
  Mat d = descriptors.getMat();
  if (n > 0) {
    rc = sift_copy_results(c, reinterpret_cast<sift_keypoint*>(keypoints.data()), d.ptr<float>(0), n, &n);
    if (rc) raise("SIFT_NCL", rc, c);
  }
}

// src/sift.cpp:123-153
void Gaussian_Blur(Mat& src, Mat& dst, double sigma) {
  require_f32(src, "Gaussian_Blur");
  Mat out(src.rows, src.cols, CV_32FC1);
  sift_ctx* c = ctx_for(src.rows, src.cols);
  int rc = sift_gaussian_blur(c, src.ptr<float>(0), src.rows, src.cols, sigma, out.ptr<float>(0));
  if (rc) raise("Gaussian_Blur", rc, c);
  dst = out;
}

// src/sift.cpp:170-217
void Gaussian_Blur_1D(Mat& src, Mat& dst, double sigma) {
  require_f32(src, "Gaussian_Blur_1D");
  Mat out(src.rows, src.cols, CV_32FC1);
  sift_ctx* c = ctx_for(src.rows, src.cols);
  int rc = sift_gaussian_blur_1d(c, src.ptr<float>(0), src.rows, src.cols, sigma, out.ptr<float>(0));
  if (rc) raise("Gaussian_Blur_1D", rc, c);
  dst = out;
}

// src/sift.cpp:229-263
void buildGaussianPyramid(Mat& image, std::vector<Mat>& gpyr, int nOctaves) {
  require_f32(image, "buildGaussianPyramid");
  sift_ctx* c = ctx_for(image.rows, image.cols);
  std::vector<float> buf(sift_packed_size(image.rows, image.cols, nOctaves, SIFT_N_SCALES));
  int rc = sift_build_gaussian_pyramid(c, image.ptr<float>(0), image.rows, image.cols, nOctaves,
                                       buf.data());
  if (rc) raise("buildGaussianPyramid", rc, c);
  unpack(buf, gpyr, image.rows, image.cols, nOctaves, SIFT_N_SCALES);
}

// src/sift.cpp:265-283
void buildDoGPyramid(std::vector<Mat>& gpyr, std::vector<Mat>& dogpyr, int nOctaves) {
  if (gpyr.empty()) throw std::runtime_error("buildDoGPyramid: empty pyramid");
  const int rows = gpyr[0].rows, cols = gpyr[0].cols;
  std::vector<float> g = pack(gpyr, rows, cols, nOctaves, SIFT_N_SCALES, "buildDoGPyramid");
  std::vector<float> d(sift_packed_size(rows, cols, nOctaves, SIFT_N_DOG));
  sift_ctx* c = ctx_for(rows, cols);
  int rc = sift_build_dog_pyramid(c, g.data(), rows, cols, nOctaves, d.data());
  if (rc) raise("buildDoGPyramid", rc, c);
  unpack(d, dogpyr, rows, cols, nOctaves, SIFT_N_DOG);
}

// src/sift.cpp:547-577
void findScaleSpaceExtrema(std::vector<Mat>& gpyr, std::vector<Mat>& dogpyr,
                           std::vector<KeyPoint>& keypoints, int nOctaves) {
  if (gpyr.empty()) throw std::runtime_error("findScaleSpaceExtrema: empty pyramid");
  const int rows = gpyr[0].rows, cols = gpyr[0].cols;
  std::vector<float> g = pack(gpyr, rows, cols, nOctaves, SIFT_N_SCALES, "findScaleSpaceExtrema");
  std::vector<float> d = pack(dogpyr, rows, cols, nOctaves, SIFT_N_DOG, "findScaleSpaceExtrema");
  sift_ctx* c = ctx_for(rows, cols);
  int n = 0;
  int rc = sift_find_scale_space_extrema(c, g.data(), d.data(), rows, cols, nOctaves, nullptr, 0, &n);
  if (rc != SIFT_OK && rc != SIFT_E_CAPACITY) raise("findScaleSpaceExtrema", rc, c);
  keypoints.clear();
  keypoints.resize(n);
  if (n > 0) {
    rc = sift_copy_results(c, reinterpret_cast<sift_keypoint*>(keypoints.data()), nullptr, n, &n);
    if (rc) raise("findScaleSpaceExtrema", rc, c);
  }
}

// src/sift.cpp:733-753
void calDescriptor(std::vector<Mat>& gpyr, std::vector<KeyPoint>& keypoints, Mat& descriptors,
                   int firstOctave) {
  if (gpyr.empty()) throw std::runtime_error("calDescriptor: empty pyramid");
  const int rows = gpyr[0].rows, cols = gpyr[0].cols;
  const int n_oct = (int)gpyr.size() / SIFT_N_SCALES;
  std::vector<float> g = pack(gpyr, rows, cols, n_oct, SIFT_N_SCALES, "calDescriptor");
  const int n = (int)keypoints.size();
  if (descriptors.rows != n || descriptors.cols != SIFT_DESC_LEN) descriptors.create(n, SIFT_DESC_LEN, CV_32F);
  if (n == 0) return;
  sift_ctx* c = ctx_for(rows, cols);
  int rc = sift_calc_descriptors(c, g.data(), rows, cols, n_oct,
                                 reinterpret_cast<const sift_keypoint*>(keypoints.data()), n,
                                 descriptors.ptr<float>(0), firstOctave);
  if (rc) raise("calDescriptor", rc, c);
}
