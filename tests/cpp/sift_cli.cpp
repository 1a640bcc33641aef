// sift_cli.cpp -- a caller written against the reference API (include/sift.hpp),
// the way canhld94/SIFT-GPU src/main.cpp uses it, minus the GUI/matching.
//   sift_cli <in.pgm> <out.bin> [modules]
// Runs SIFT_NCL (or, with "modules", the sub-module chain buildGaussianPyramid
// -> buildDoGPyramid -> findScaleSpaceExtrema -> calDescriptor) and writes
// int32 n, n x 28-byte KeyPoints, n x 128 float descriptors.
#include <stdio.h>
#include <string.h>

#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "sift.hpp"

static bool read_pgm(const char* path, Mat& gray) {
  std::ifstream f(path, std::ios::binary);
  std::string magic;
  int w = 0, h = 0, mx = 0;
  f >> magic >> w >> h >> mx;
  f.get();
  if (magic != "P5" || mx != 255 || w <= 0 || h <= 0) return false;
  std::vector<unsigned char> px((size_t)w * h);
  f.read(reinterpret_cast<char*>(px.data()), px.size());
  if (!f) return false;
  gray = Mat(h, w, DATATYPE);  // CV_32FC1, as readImage's convertTo (src/main.cpp:85)
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) gray.at<data_t>(i, j) = (data_t)px[(size_t)i * w + j];
  return true;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cout << "Usage: ./sift_cli <in.pgm> <out.bin> [modules]" << std::endl;
    return -1;
  }
  Mat gray;
  if (!read_pgm(argv[1], gray)) {
    std::cout << " --(!) Error reading images " << std::endl;
    return 1;
  }
  std::vector<KeyPoint> keypoints;
  Mat descriptors;
  try {
    if (argc > 3 && std::string(argv[3]) == "modules") {
      std::vector<Mat> gpyr, dogpyr;
      buildGaussianPyramid(gray, gpyr, 5);
      buildDoGPyramid(gpyr, dogpyr, 5);
      findScaleSpaceExtrema(gpyr, dogpyr, keypoints, 5);
      descriptors = Mat((int)keypoints.size(), 128, CV_32F);
      calDescriptor(gpyr, keypoints, descriptors, 0);
    } else {
      SIFT_NCL(gray, keypoints, descriptors);
    }
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << std::endl;
    return 2;
  }
  FILE* out = fopen(argv[2], "wb");
  if (!out) return 3;
  int n = (int)keypoints.size();
  fwrite(&n, sizeof(int), 1, out);
  if (n) {
    fwrite(keypoints.data(), sizeof(KeyPoint), n, out);
    fwrite(descriptors.ptr<float>(0), sizeof(float) * 128, n, out);
  }
  fclose(out);
  printf("%d keypoints\n", n);
  return 0;
}
