// radler::algorithms::MultiScaleAlgorithm on the device (reference:
// cpp/algorithms/multiscale_algorithm.{h,cc}; Offringa & Smirnov 2017).
// All images, convolved PSFs and kernel spectra stay in HBM for the whole
// major iteration; the host only sees per-scale peaks and loop scalars.
// Device-side caching the reference does not do (results are the same
// convolutions): the forward FFT of the integrated image is shared by all
// active scales, twice-convolved PSFs and padded PSF spectra are computed once
// per scale per major iteration.
#pragma once

#include <map>
#include <memory>
#include <optional>
#include <vector>

#include "deconvolution_algorithm.h"
#include "multiscale_transforms.h"

namespace radler::algorithms {

class MultiScaleAlgorithm final : public DeconvolutionAlgorithm {
 public:
  MultiScaleAlgorithm(const Settings::Multiscale& settings, double beam_size,
                      double pixel_scale_x, double pixel_scale_y,
                      bool track_components);
  MultiScaleAlgorithm(const MultiScaleAlgorithm& other);

  std::unique_ptr<DeconvolutionAlgorithm> Clone() const final {
    return std::make_unique<MultiScaleAlgorithm>(*this);
  }

  DeconvolutionResult ExecuteMajorIteration(ImageSet& data_image,
                                            ImageSet& model_image,
                                            const gpu::Planes& psf_images) final;

  struct ScaleInfo {
    float scale = 0.0;
    float psf_peak = 0.0;
    float kernel_peak = 0.0;
    float bias_factor = 0.0;
    float gain = 0.0;
    float max_normalized_image_value = 0.0;
    float max_unnormalized_image_value = 0.0;
    float rms = 0.0;
    size_t max_image_value_x = 0;
    size_t max_image_value_y = 0;
    bool is_active = false;
    size_t n_components_cleaned = 0;
    float total_flux_cleaned = 0.0;
  };

  size_t ScaleCount() const { return scale_infos_.size(); }
  float ScaleSize(size_t i) const { return scale_infos_[i].scale; }
  const std::vector<ScaleInfo>& ScaleInfos() const { return scale_infos_; }
  /// x, y, scale index of every component of the last major iteration.
  const std::vector<uint32_t>& LastTrace() const { return trace_; }

 private:
  void FindActiveScaleConvolvedMaxima(const ImageSet& image_set,
                                      float* d_integrated, bool report_rms);
  void FindPeakDirect(const float* d_image, size_t scale_index);
  void ActivateScales(size_t scale_with_last_peak);

  const Settings::Multiscale& settings_;
  double beam_size_in_pixels_;
  bool track_components_;
  std::vector<ScaleInfo> scale_infos_;
  std::vector<uint32_t> trace_;

  // per-major-iteration device state
  gpu::Session* session_ = nullptr;
  std::unique_ptr<multiscale::MultiScaleTransforms> transforms_;
  const uint8_t* d_mask_ = nullptr;
  std::shared_ptr<gpu::Buffer> scratch_;  // W x H
  std::shared_ptr<gpu::Buffer> spectrum_, spectrum_work_;
  // One image with the identity integration (ImageSet copy fast path): the
  // integrated image IS the residual, so the scale-convolved images that
  // FindActiveScaleConvolvedMaxima computes are the next outer iteration's
  // individually convolved image for that scale (same input, same FFT plan,
  // same kernel spectrum: bit-identical to a fresh Transform). They are kept
  // per scale and swapped in instead of convolving again.
  std::vector<gpu::Planes> scale_images_;
  std::vector<bool> scale_image_valid_;
};

// multiscale_algorithm.cc:90-151 (free functions in the reference)
void InitializeScales(std::vector<MultiScaleAlgorithm::ScaleInfo>& scales,
                      double beam_size_in_pixels, size_t min_width_height,
                      MultiscaleShape shape, size_t max_scales,
                      const std::vector<double>& scale_list);
std::optional<size_t> SelectMaximumScale(
    const std::vector<MultiScaleAlgorithm::ScaleInfo>& scales);

}  // namespace radler::algorithms
