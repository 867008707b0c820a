// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
// ParallelDeconvolution tiling restatement (see tiling.cc).
#pragma once

#include <limits>
#include <memory>
#include <vector>

#include "oracle.h"

namespace oracle {

// cpp/algorithms/parallel_deconvolution.h (SubImage)
struct SubImage {
  size_t index = 0, x = 0, y = 0, width = 0, height = 0;
  std::vector<unsigned char> mask, boundary_mask;  // bool per pixel
  double peak = 0.0;
  bool reached_major_threshold = false;
  // test harness: decision margin after the last component of the clean pass
  float end_margin = std::numeric_limits<float>::infinity();
};

// One subimage's algorithm (the reference clones the first algorithm per
// subimage, parallel_deconvolution.cc:227-242): persistent settings,
// iteration count and multiscale state.
struct TiledAlgorithm {
  int kind = 0;  // 0 GenericClean, 1 MultiScale, 2 IUWT
  AlgoSettings settings;
  size_t iteration_number = 0;
  std::unique_ptr<MultiScale> ms;
  Result Execute(ImageSet& data, ImageSet& model,
                 const std::vector<const float*>& psfs,
                 std::vector<Component>* trace);
};

// ParallelDeconvolution's auto-mask state (parallel_deconvolution.cc:
// 260-268, 359-390, 425-462): full-image masks per scale, 0/1 bytes.
// Per-run state ParallelDeconvolution keeps across subimages: the per-scale
// auto-masks (parallel_deconvolution.cc:359-462) and the full-image RMS
// factor trimmed to each subimage (:244-250, 332-337, 421-423).
struct ParallelMasks {
  bool track = false, use = false;
  std::vector<std::vector<unsigned char>> scale_masks;
  std::vector<float> rms_factor;  // width x height, empty = none
};

struct ParallelResult {
  bool another_iteration_required = false;
  double start_peak = 0.0, end_peak = 0.0;
};

std::vector<SubImage> MakeSubImages(const float* image, size_t width,
                                    size_t height, const bool* user_mask,
                                    size_t grid_w, size_t grid_h);

ParallelResult ParallelRun(std::vector<TiledAlgorithm>& algorithms,
                           size_t grid_w, size_t grid_h, const SetDesc& desc,
                           ImageSet& data, ImageSet& model,
                           const std::vector<const float*>& psfs,
                           double major_loop_gain, double divergence_limit,
                           const bool* user_mask, std::vector<SubImage>* out_subs,
                           std::vector<std::vector<Component>>* traces,
                           bool snapshot = false, ParallelMasks* masks = nullptr);

}  // namespace oracle
