// radler::algorithms::IuwtDeconvolution (reference:
// cpp/algorithms/iuwt_deconvolution.h, iuwt_deconvolution_algorithm.{h,cc},
// iuwt/iuwt_mask.h, iuwt/image_analysis.cc) on the device: the wavelet
// transforms, masks, convolutions, conjugate-gradient updates and reductions
// run as HIP kernels on device-resident planes; the host keeps the scalar
// control flow (scale choice, thresholds, bounding boxes) and the
// connected-component walk of the joined-channel refit.
#pragma once

#include <memory>

#include "deconvolution_algorithm.h"

namespace radler::algorithms {

class IuwtDeconvolution final : public DeconvolutionAlgorithm {
 public:
  IuwtDeconvolution() = default;
  IuwtDeconvolution(const IuwtDeconvolution& o) : DeconvolutionAlgorithm(o) {}

  /// iuwt_deconvolution.h:22-39: a fresh IuwtDeconvolutionAlgorithm per
  /// major iteration (PSF responses re-measured, scales restart at 2).
  DeconvolutionResult ExecuteMajorIteration(ImageSet& data_image, ImageSet& model_image,
                                            const gpu::Planes& psf_images) final;
  std::unique_ptr<DeconvolutionAlgorithm> Clone() const final {
    return std::make_unique<IuwtDeconvolution>(*this);
  }

  /// One step of the outer loop of the last ExecuteMajorIteration (the
  /// oracle's IuwtStep), for parity tests.
  struct Step {
    int32_t succeeded, scale;
    uint32_t x, y;
    int32_t end_scale, min_scale;
    uint64_t area;
    float max_value;
    uint32_t trimmed_width;  // width of the trimmed box (0: not trimmed)
  };
  const std::vector<Step>& Steps() const { return steps_; }

 private:
  std::vector<Step> steps_;
};

}  // namespace radler::algorithms
