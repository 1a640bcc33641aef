/*
 * sift.hpp -- drop-in replacement for canhld94/SIFT-GPU include/sift.hpp.
 *
 * Same eight functions, same argument meaning (include/sift.hpp:36-67 of the
 * reference), implemented on the MI355X C ABI (include/sift_hip.h).  The
 * reference's vestigial `#include <cuda.h>` (:13) is dropped.  With OpenCV
 * available the real cv:: types are used; otherwise a minimal compatible
 * subset (sift_cvcompat.hpp).
 *
 * Behavioural differences, all deliberate:
 *  - errors throw std::runtime_error instead of exit(0) (src/sift.cpp:278);
 *  - the pyramid uses the correct o*5+s plane index for any nOctaves (the
 *    reference's gpyr[o*nOctaves+i], src/sift.cpp:248, is only valid at 5);
 *  - no per-call timing printfs unless SIFT_HIP_VERBOSE=1 is set.
 * The device used is $SIFT_HIP_DEVICE (default 0); one context per thread.
 */
#ifndef SIFT_HPP_
#define SIFT_HPP_

#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>  // the reference header's own includes (include/sift.hpp:11-26)

#include <iostream>
#include <vector>

#if defined(__has_include)
#if __has_include(<opencv2/core.hpp>) && !defined(SIFT_HIP_NO_OPENCV)
#define SIFT_HIP_HAVE_OPENCV 1
#endif
#if __has_include(<omp.h>)
#include <omp.h>
#endif
#endif

#ifdef SIFT_HIP_HAVE_OPENCV
// The reference's OpenCV include set (include/sift.hpp:14-23) minus cuda.h, so
// a caller like src/main.cpp (imread, imshow, findHomography, cvPoint, ...)
// compiles against this header unchanged.
#include <opencv2/core.hpp>
#include <opencv2/core/hal/hal.hpp>
#include <opencv2/core/types_c.h>
#include <opencv2/core/utility.hpp>
#include <opencv2/features2d.hpp>
#include <opencv2/imgproc.hpp>
#if __has_include(<opencv2/imgcodecs.hpp>)
#include <opencv2/imgcodecs.hpp>
#endif
#if __has_include(<opencv2/highgui.hpp>)
#include <opencv2/highgui.hpp>
#endif
#if __has_include(<opencv2/calib3d/calib3d.hpp>)
#include <opencv2/calib3d/calib3d.hpp>
#endif
#if __has_include(<opencv2/xfeatures2d.hpp>)
#include <opencv2/xfeatures2d.hpp>
#else
namespace cv { namespace xfeatures2d {} }
#endif
#else
#include "sift_cvcompat.hpp"
#endif

using namespace cv;
using namespace cv::xfeatures2d;

typedef float data_t;  // data type used in the filters

#define DATATYPE CV_32FC1

/* SIFT built-in OpenCV function (needs opencv_contrib; throws otherwise). */
void SITF_BuildIn_OpenCV(InputArray image, std::vector<KeyPoint>& keypoints,
                         OutputArray descriptors);

/* NCL SIFT: the hot path, on the GPU. */
void SIFT_NCL(InputArray image, std::vector<KeyPoint>& keypoints, OutputArray descriptors);

/* Sub modules */
void Gaussian_Blur(Mat& src, Mat& dst, double sigma);

void Gaussian_Blur_1D(Mat& src, Mat& dst, double sigma);

void buildGaussianPyramid(Mat& image, std::vector<Mat>& gpyr, int nOctaves);

void buildDoGPyramid(std::vector<Mat>& gpyr, std::vector<Mat>& dogpyr, int nOctaves);

void findScaleSpaceExtrema(std::vector<Mat>& gpyr, std::vector<Mat>& dogpyr,
                           std::vector<KeyPoint>& keypoints, int nOctaves);

void calDescriptor(std::vector<Mat>& gpyr, std::vector<KeyPoint>& keypoints, Mat& descriptors,
                   int firstOctave);

#endif /* SIFT_HPP_ */
