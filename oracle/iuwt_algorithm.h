// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// CPU restatement of IuwtDeconvolutionAlgorithm
// (cpp/algorithms/iuwt_deconvolution_algorithm.{h,cc}), its IuwtMask
// (cpp/algorithms/iuwt/iuwt_mask.h) and image_analysis flood fills
// (cpp/algorithms/iuwt/image_analysis.cc), on top of the IUWT restatement in
// iuwt.cc and the double-precision circular convolution in fft.cc.
//
// Parity notes (parity unpinned: the reference's own tests mark this
// algorithm as failing, cpp/test/test_radler.cc:101, and no fixture pins it):
//  - float sums (DotProduct, Snr) run sequentially with the FMA contraction
//    of the reference's -O3 -march=native build, as written;
//  - aocommon Image::RMS is not in /root/reference: sqrt(sum(v^2)/n) with a
//    double sum is used (an assumption, stated here and in DESIGN.md);
//  - MeasureRMSPerScale's Gaussian fits and flood fills only feed fields
//    the algorithm never reads (b_major/b_minor/b_pa, convolved_area) and
//    are left out;
//  - schaapcommon::math::Convolve is the double-precision circular
//    convolution of fft.cc (FFTW float in the reference).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "oracle.h"

namespace oracle {

struct IuwtAlgoSettings {
  float minor_loop_gain = 0.1f;
  float major_loop_gain = 1.0f;
  float clean_border = 0.0f;
  bool allow_negative = true;
  const bool* mask = nullptr;
  float absolute_threshold = 0.0f;
  float threshold_sigma_level = 4.0f;
  float tolerance = 0.75f;
};

// One step of the outer loop, for trace comparisons.
struct IuwtStep {
  int32_t succeeded;      // FindAndDeconvolveStructure result
  int32_t scale;          // most significant scale (-1: none)
  uint32_t x, y;          // its position (full-image coordinates)
  int32_t end_scale;      // curEndScale of the step
  int32_t min_scale;      // curMinScale of the step
  uint64_t area;          // SelectStructures area size (0 if not reached)
  float max_value;        // maxValue after the step (0 if not updated)
  uint32_t trimmed_width; // width of the trimmed box (0: not trimmed)
};

// IuwtDeconvolution::ExecuteMajorIteration (cpp/algorithms/iuwt_deconvolution.h:22-39)
// with PerformMajorIteration (iuwt_deconvolution_algorithm.cc:800-918).
// Returns maxValue; iteration_number is advanced like the reference's.
float IuwtExecute(const IuwtAlgoSettings& s, size_t& iteration_number,
                  size_t max_iterations, ImageSet& dirty, ImageSet& model,
                  const std::vector<const float*>& psfs,
                  bool& another_iteration_required, std::vector<IuwtStep>* steps);

// IuwtDecomposition::EndScale (iuwt_decomposition.h:306-308)
int IuwtEndScale(size_t max_image_dimension);

}  // namespace oracle
