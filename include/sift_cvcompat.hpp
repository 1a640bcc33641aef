/*
 * sift_cvcompat.hpp -- the minimal slice of OpenCV types that the reference
 * API (canhld94/SIFT-GPU include/sift.hpp) exposes: cv::Mat (CV_32FC1 and
 * CV_8UC1, refcounted, continuous), cv::KeyPoint, cv::Point2f, and the
 * InputArray / OutputArray parameter adapters.  Used only when the real
 * OpenCV headers are not available; with OpenCV installed, include/sift.hpp
 * uses the real types and this header is never included.
 */
#ifndef SIFT_CVCOMPAT_HPP_
#define SIFT_CVCOMPAT_HPP_

#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <vector>

namespace cv {

typedef unsigned char uchar;

enum { CV_8U = 0, CV_32F = 5 };
#define CV_8UC1 0
#define CV_32FC1 5

struct Point2f {
  float x, y;
  Point2f() : x(0), y(0) {}
  Point2f(float x_, float y_) : x(x_), y(y_) {}
};

/* cv::KeyPoint: {Point2f pt; float size, angle, response; int octave, class_id;} */
class KeyPoint {
 public:
  KeyPoint() : pt(0, 0), size(0), angle(-1), response(0), octave(0), class_id(-1) {}
  KeyPoint(Point2f p, float sz, float ang = -1, float resp = 0, int oct = 0, int cls = -1)
      : pt(p), size(sz), angle(ang), response(resp), octave(oct), class_id(cls) {}
  Point2f pt;
  float size;
  float angle;
  float response;
  int octave;
  int class_id;
};

struct MatSize {
  int r, c;
  bool operator==(const MatSize& o) const { return r == o.r && c == o.c; }
  bool operator!=(const MatSize& o) const { return !(*this == o); }
};

class Mat {
 public:
  int rows = 0, cols = 0;
  uchar* data = nullptr;
  MatSize size{0, 0};

  Mat() {}
  Mat(int r, int c, int type) { create(r, c, type); }
  Mat(int r, int c, int type, void* ext) : rows(r), cols(c), size{r, c}, type_(type) {
    data = static_cast<uchar*>(ext);
  }

  void create(int r, int c, int type) {
    if (r == rows && c == cols && type == type_ && data) return;
    if (type != CV_32F && type != CV_8U) throw std::runtime_error("cvcompat: unsupported Mat type");
    const size_t n = (size_t)r * c * elem(type);
    buf_ = std::shared_ptr<uchar>(new uchar[n ? n : 1], std::default_delete<uchar[]>());
    data = buf_.get();
    rows = r;
    cols = c;
    size = MatSize{r, c};
    type_ = type;
  }
  void release() {
    buf_.reset();
    data = nullptr;
    rows = cols = 0;
    size = MatSize{0, 0};
  }
  int type() const { return type_; }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  bool isContinuous() const { return true; }
  size_t elemSize() const { return elem(type_); }
  size_t step1() const { return (size_t)cols; }
  size_t total() const { return (size_t)rows * cols; }
  template <typename T>
  T* ptr(int i = 0) {
    return reinterpret_cast<T*>(data + (size_t)i * cols * elem(type_));
  }
  template <typename T>
  const T* ptr(int i = 0) const {
    return reinterpret_cast<const T*>(data + (size_t)i * cols * elem(type_));
  }
  template <typename T>
  T& at(int i, int j) {
    return ptr<T>(i)[j];
  }
  template <typename T>
  const T& at(int i, int j) const {
    return ptr<T>(i)[j];
  }
  Mat clone() const {
    Mat m(rows, cols, type_);
    std::copy(data, data + total() * elem(type_), m.data);
    return m;
  }
  /* dst = a - b for CV_32FC1 (used by the DoG, src/sift.cpp:280). */
  friend Mat operator-(const Mat& a, const Mat& b) {
    if (a.size != b.size || a.type_ != CV_32F || b.type_ != CV_32F)
      throw std::runtime_error("cvcompat: operator- needs equal-size CV_32FC1 Mats");
    Mat d(a.rows, a.cols, CV_32F);
    const float *pa = a.ptr<float>(), *pb = b.ptr<float>();
    float* pd = d.ptr<float>();
    for (size_t i = 0; i < a.total(); ++i) pd[i] = pa[i] - pb[i];
    return d;
  }

 private:
  static size_t elem(int t) { return t == CV_32F ? 4 : 1; }
  std::shared_ptr<uchar> buf_;
  int type_ = CV_32F;
};

class _InputArray {
 public:
  _InputArray(const Mat& m) : m_(&m) {}
  Mat getMat() const { return *m_; }

 private:
  const Mat* m_;
};

class _OutputArray {
 public:
  _OutputArray(Mat& m) : m_(&m) {}
  void create(int r, int c, int type) const { m_->create(r, c, type); }
  Mat& getMatRef() const { return *m_; }
  Mat getMat() const { return *m_; }

 private:
  Mat* m_;
};

typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;

namespace xfeatures2d {}  // keeps `using namespace cv::xfeatures2d;` valid

}  // namespace cv

#endif /* SIFT_CVCOMPAT_HPP_ */
