#include "deconvolution_algorithm.h"

namespace radler::algorithms {

const uint8_t* DeconvolutionAlgorithm::DeviceCleanMask(gpu::Session& s,
                                                       size_t width,
                                                       size_t height) {
  if (!settings_.clean_mask) return nullptr;
  const size_t n = width * height;
  if (!mask_buffer_ || mask_buffer_->Bytes() < n)
    mask_buffer_ = std::make_shared<gpu::Buffer>(s, n);
  // bool is one byte holding 0/1: upload as uint8
  s.H2D(mask_buffer_->Ptr(), settings_.clean_mask, n);
  return static_cast<const uint8_t*>(mask_buffer_->Ptr());
}

}  // namespace radler::algorithms
