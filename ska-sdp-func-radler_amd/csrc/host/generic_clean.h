// radler::algorithms::GenericClean on the device (reference:
// cpp/algorithms/generic_clean.{h,cc}): Högbom CLEAN, or Clark-like with the
// sub-minor loop and an FFT residual correction.
#pragma once

#include <memory>

#include "deconvolution_algorithm.h"

namespace radler::algorithms {

class GenericClean final : public DeconvolutionAlgorithm {
 public:
  explicit GenericClean(bool use_sub_minor_optimization);
  GenericClean(const GenericClean&) = default;

  DeconvolutionResult ExecuteMajorIteration(ImageSet& dirty_set,
                                            ImageSet& model_set,
                                            const gpu::Planes& psfs) final;
  std::unique_ptr<DeconvolutionAlgorithm> Clone() const final {
    return std::make_unique<GenericClean>(*this);
  }

  /// x, y, scale(=0) of every component of the last ExecuteMajorIteration.
  const std::vector<uint32_t>& LastTrace() const { return trace_; }

 private:
  rdl_peak FindPeak(gpu::Session& s, const float* d_image, size_t width,
                    size_t height, const uint8_t* d_mask);
  void RunComponentOptimization(ImageSet& residual_set, ImageSet& model_set,
                                const gpu::Planes& psfs);
  void FitSpectra(ImageSet& model_set);

  const float convolution_padding_;
  bool use_sub_minor_optimization_;
  std::vector<uint32_t> trace_;
  std::shared_ptr<gpu::Buffer> rms_scratch_;  // image x RMS factor
};

}  // namespace radler::algorithms
