// Multiscale scale kernels and their circular convolution on the device
// (reference: cpp/algorithms/multiscale/multiscale_transforms.{h,cc}).
// Kernels are generated on the host with the reference's float/double mix;
// their W x H spectra are cached per scale, so Transform() costs one forward
// FFT, one spectrum product and one inverse FFT per image.
#pragma once

#include <map>
#include <memory>
#include <vector>

#include "device.h"
#include "settings.h"

namespace radler::algorithms::multiscale {

class MultiScaleTransforms {
 public:
  using Shape = radler::MultiscaleShape;
  MultiScaleTransforms(gpu::Session& s, size_t width, size_t height,
                       Shape shape);

  size_t Width() const { return width_; }
  size_t Height() const { return height_; }
  gpu::Fft& Fft() { return fft_; }

  /// Spectrum of the scale kernel placed at the origin (cached).
  const void* KernelSpectrum(float scale);
  /// The scale's n x n shape kernel on the device (cached), for direct
  /// stamping of sparse models.
  const float* ShapeKernel(float scale, size_t& n);
  /// In-place convolution of one W x H plane with the scale kernel
  /// (multiscale_transforms.cc:9-21).
  void Transform(float* d_image, float scale);

  // multiscale_transforms.h:41-195
  static std::vector<float> MakeShapeFunction(float scale, size_t& n,
                                              size_t max_n, Shape shape);
  static float KernelPeakValue(double scale, size_t max_n, Shape shape);
  static float GaussianSigma(float scale) { return scale * (3.0 / 16.0); }

 private:
  gpu::Session& s_;
  size_t width_, height_;
  Shape shape_;
  gpu::Fft& fft_;
  std::map<float, std::shared_ptr<gpu::Buffer>> spectra_;
  std::map<float, std::pair<std::shared_ptr<gpu::Buffer>, size_t>> shapes_;
};

}  // namespace radler::algorithms::multiscale
