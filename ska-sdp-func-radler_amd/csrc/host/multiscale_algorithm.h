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

#include "component_list.h"
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
  /// Joined channels over the ranks of `comm` (one process per GPU): every
  /// rank runs the integrated-image work (integration, the scales' peak
  /// searches, the selection and the sub-minor loop: identical inputs give
  /// identical results) and the per-image residual correction and model
  /// update of the images it owns (image i: rank i % size); the corrected
  /// residual planes are then broadcast from their owners, the model planes
  /// at the end of the major iteration. Same operations on the same data as
  /// one process: bit-identical residuals, models and traces.
  void SetChannelShard(Communicator* comm) final { shard_ = comm; }

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
  /// multiscale_algorithm.h:72-79: the components of the major iterations
  /// so far (save_source_list), per scale with one value per image.
  const ComponentList& GetComponentList() const { return *component_list_; }
  bool HasComponentList() const { return component_list_ != nullptr; }
  void ClearComponentList() { component_list_.reset(); }
  float ScaleSize(size_t i) const { return scale_infos_[i].scale; }
  const std::vector<ScaleInfo>& ScaleInfos() const { return scale_infos_; }
  /// x, y, scale index of every component of the last major iteration.
  const std::vector<uint32_t>& LastTrace() const { return trace_; }

  /// Auto-masking (multiscale_algorithm.h:41-55): track = grow one mask per
  /// scale from the components; use = clean each scale inside its mask only
  /// (the clean mask is then ignored). Masks persist across major
  /// iterations: canonical host copies (0/1 bytes, width x height), device
  /// working copies uploaded when changed.
  void SetAutoMaskMode(bool track_per_scale_masks, bool use_per_scale_masks) {
    track_masks_ = track_per_scale_masks;
    use_masks_ = use_per_scale_masks;
  }
  size_t GetScaleMaskCount() const { return host_masks_.size(); }
  void SetScaleMaskCount(size_t n) {
    host_masks_.resize(n);
    masks_dirty_ = true;
  }
  /// Mutable access (ParallelDeconvolution fills subimage boxes).
  std::vector<uint8_t>& GetScaleMask(size_t index) {
    masks_dirty_ = true;
    return host_masks_[index];
  }

 private:
  void FindActiveScaleConvolvedMaxima(const ImageSet& image_set,
                                      float* d_integrated, bool report_rms);
  void FindPeakDirect(const float* d_image, size_t scale_index);
  void RunFullComponentFitter(ImageSet& residual_set, ImageSet& model_set,
                              const gpu::Planes& psfs);
  void ActivateScales(size_t scale_with_last_peak);
  void UploadScaleMasks(gpu::Session& s, size_t n_pixels);
  void DownloadScaleMasks();
  /// the mask the peak searches and the sub-minor loop of `scale` use
  const uint8_t* MaskFor(size_t scale) const {
    if (use_masks_ && scale < dev_masks_.size())
      return static_cast<const uint8_t*>(dev_masks_[scale].Ptr());
    return d_mask_;
  }

  const Settings::Multiscale& settings_;
  double beam_size_in_pixels_;
  bool track_components_;
  std::unique_ptr<ComponentList> component_list_;
  std::vector<ScaleInfo> scale_infos_;
  std::vector<uint32_t> trace_;

  // per-major-iteration device state
  gpu::Session* session_ = nullptr;
  Communicator* shard_ = nullptr;  // SetChannelShard (not copied by Clone)
  std::unique_ptr<multiscale::MultiScaleTransforms> transforms_;
  const uint8_t* d_mask_ = nullptr;
  std::shared_ptr<gpu::Buffer> scratch_;  // W x H
  std::shared_ptr<gpu::Buffer> rms_scratch_;  // W x H: image x RMS factor
  /// d_image, or d_image x the RMS factor (multiscale_algorithm.cc:707-713)
  /// FindActiveScaleConvolvedMaxima through the fused multi-scale launch
  void FindMaximaFused(const float* d_source, bool identity, std::vector<size_t> pending);
  const float* PeakSearchInput(const float* d_image, size_t w, size_t h);
  /// unnormalized / factor at the peak (:736-743), the value itself without
  float Normalized(float value, size_t x, size_t y, size_t w) const;
  std::shared_ptr<gpu::Buffer> spectrum_, spectrum_work_;
  // the second session lane's work spectrum (FindActiveScaleConvolvedMaxima
  // alternates the scales' fused inverse transforms over two lanes)
  std::shared_ptr<gpu::Buffer> spectrum_work2_;
  // the fused multi-scale path (MultiScaleTransforms::Fused): one inner
  // inverse spectrum per active scale, made by one launch
  std::vector<std::shared_ptr<gpu::Buffer>> scale_u_;
  // One image with the identity integration (ImageSet copy fast path): the
  // integrated image IS the residual, so the scale-convolved images that
  // FindActiveScaleConvolvedMaxima computes are the next outer iteration's
  // individually convolved image for that scale (same input, same FFT plan,
  // same kernel spectrum: bit-identical to a fresh Transform). They are kept
  // per scale and swapped in instead of convolving again.
  std::vector<gpu::Planes> scale_images_;
  std::vector<bool> scale_image_valid_;

  bool track_masks_ = false, use_masks_ = false;
  std::vector<std::vector<uint8_t>> host_masks_;
  std::vector<gpu::Buffer> dev_masks_;
  gpu::Session* masks_session_ = nullptr;
  bool masks_dirty_ = true;
};

// multiscale_algorithm.cc:90-151 (free functions in the reference)
void InitializeScales(std::vector<MultiScaleAlgorithm::ScaleInfo>& scales,
                      double beam_size_in_pixels, size_t min_width_height,
                      MultiscaleShape shape, size_t max_scales,
                      const std::vector<double>& scale_list);
std::optional<size_t> SelectMaximumScale(
    const std::vector<MultiScaleAlgorithm::ScaleInfo>& scales);

}  // namespace radler::algorithms
