// main_shape.cpp -- a caller shaped like the reference application
// (src/main.cpp): it includes ONLY "sift.hpp" and relies on what that header
// brings in transitively -- std::cout / std::endl (<iostream>), gettimeofday
// (<sys/time.h>), exit (<stdlib.h>), printf (<stdio.h>), omp_get_max_threads
// (<omp.h>, when the compiler has it) and the cv:: types -- exactly as
// src/main.cpp does.  Built in compat mode (no OpenCV in this image), where
// imread / imshow / BFMatcher / findHomography do not exist; with OpenCV
// installed src/main.cpp itself compiles against this header.
#include "sift.hpp"

static double now_ms() {
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return tv.tv_sec * 1e3 + tv.tv_usec * 1e-3;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::cout << "Usage: ./sift <rows> [cols] " << std::endl;
    exit(0);
  }
  const int rows = atoi(argv[1]), cols = argc > 2 ? atoi(argv[2]) : rows;
  Mat gray(rows, cols, DATATYPE);
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) gray.at<data_t>(i, j) = (data_t)((i * 7 + j * 13) % 251);
#ifdef _OPENMP
  printf("omp threads %d\n", omp_get_max_threads());
#endif
  std::vector<KeyPoint> kp;
  Mat desc;
  const double t0 = now_ms();
  SIFT_NCL(gray, kp, desc);
  std::cout << kp.size() << " keypoints, " << desc.rows << " x " << desc.cols << " descriptors in "
            << now_ms() - t0 << " ms" << std::endl;
  return 0;
}
