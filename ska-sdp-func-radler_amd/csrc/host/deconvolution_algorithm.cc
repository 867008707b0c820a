#include "deconvolution_algorithm.h"

#include <stdexcept>

namespace radler::algorithms {

const uint8_t* DeconvolutionAlgorithm::DeviceCleanMask(gpu::Session& s,
                                                       size_t width,
                                                       size_t height) {
  if (!settings_.clean_mask) return nullptr;
  const size_t n = width * height;
  if (!mask_buffer_ || mask_buffer_->Bytes() < n || mask_session_ != &s) {
    mask_buffer_ = std::make_shared<gpu::Buffer>(s, n);
    mask_session_ = &s;
  }
  // bool is one byte holding 0/1: upload as uint8
  s.H2D(mask_buffer_->Ptr(), settings_.clean_mask, n);
  return static_cast<const uint8_t*>(mask_buffer_->Ptr());
}

void DeconvolutionAlgorithm::PerformSpectralFit(float* values, size_t x,
                                                size_t y) const {
  if (!spectral_fitter_) return;
  const size_t n = spectral_fitter_->Frequencies().size();
  std::vector<float> channel(n), scratch;
  for (size_t p = 0; p != n_polarizations_; ++p) {
    for (size_t ch = 0; ch != n; ++ch) channel[ch] = values[ch * n_polarizations_ + p];
    spectral_fitter_->FitAndEvaluate(channel.data(), x, y, scratch);
    for (size_t ch = 0; ch != n; ++ch) values[ch * n_polarizations_ + p] = channel[ch];
  }
}

const float* DeconvolutionAlgorithm::DeviceSpectralMap(gpu::Session& s,
                                                       size_t n_images) {
  if (!spectral_fitter_) return nullptr;
  if (spectral_map_images_ != n_images || spectral_map_session_ != &s) {
    spectral_map_images_ = n_images;
    spectral_map_session_ = &s;
    spectral_map_.reset();
    const std::vector<float> g = ComponentFitMatrix(*spectral_fitter_, n_polarizations_);
    spectral_map_identity_ = g.empty();
    if (!g.empty()) {
      if (g.size() != n_images * n_images)
        throw std::runtime_error(
            "Spectral fitting: the image set does not match the fitter's "
            "channels");
      spectral_map_ = std::make_shared<gpu::Buffer>(s, g.size() * sizeof(float));
      s.H2D(spectral_map_->Ptr(), g.data(), g.size() * sizeof(float));
    }
  }
  return spectral_map_identity_ ? nullptr : spectral_map_->F();
}

const float* DeconvolutionAlgorithm::DeviceRmsFactor(gpu::Session& s, size_t width,
                                                     size_t height) {
  if (!rms_factor_) return nullptr;
  const size_t n = width * height;
  if (rms_factor_->size() != n)
    throw std::runtime_error("RMS factor image does not match the image size");
  if (!rms_device_ || rms_device_session_ != &s) {
    rms_device_ = std::make_shared<gpu::Buffer>(s, n * sizeof(float));
    s.H2D(rms_device_->Ptr(), rms_factor_->data(), n * sizeof(float));
    rms_device_session_ = &s;
  }
  return rms_device_->F();
}

const float* DeconvolutionAlgorithm::RmsWeighted(gpu::Session& s, const float* d_image,
                                                 float* d_scratch, size_t width,
                                                 size_t height) {
  const float* rms = DeviceRmsFactor(s, width, height);
  if (!rms) return d_image;
  gpu::Check(rdl_multiply(s.Handle(), d_scratch, d_image, rms, width * height),
             "rdl_multiply");
  return d_scratch;
}

}  // namespace radler::algorithms
