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
  /// Whether this object's kernels, plans and work planes live on `s` (an
  /// algorithm that a different worker session runs next must rebuild them:
  /// work queued on two streams would race).
  bool BoundTo(const gpu::Session& s) const { return &s_ == &s; }

  /// The largest scale the next transforms use. Images whose sides are not
  /// FFT-friendly (even and 7-smooth, utils::CalculateGoodFFTSize) are then
  /// convolved in a periodically extended plane of a friendly size that
  /// holds the largest kernel's radius on every side; the cropped result is
  /// the same circular W x H convolution (rounding aside). Bluestein
  /// transforms of arbitrary subimage sizes cost 3-4x more.
  void SetMaxScale(float scale);
  /// FFT plane size (W x H, or the extended plane).
  size_t PlaneWidth() const { return pw_; }
  size_t PlaneHeight() const { return ph_; }
  size_t SpectrumBytes() { return TheFft().SpectrumBytes(); }

  /// Spectrum of the scale kernel placed at the origin of the plane (cached).
  const void* KernelSpectrum(float scale);
  /// The scale's n x n shape kernel on the device (cached), for direct
  /// stamping of sparse models.
  const float* ShapeKernel(float scale, size_t& n);
  /// In-place convolution of one W x H plane with the scale kernel
  /// (multiscale_transforms.cc:9-21).
  void Transform(float* d_image, float scale);
  /// Forward spectrum of a W x H image (shared by several ConvolveSpectrum).
  void Forward(const float* d_image, void* d_spectrum);
  /// d_out (W x H) = image of d_spectrum convolved with the scale kernel;
  /// d_spectrum is preserved, d_work is spectrum-sized scratch.
  void ConvolveSpectrum(const void* d_spectrum, float scale, void* d_work, float* d_out);
  /// ConvolveSpectrum with the peak search fused (Fft::ConvolveSpectrumPeak);
  /// false (nothing done) for the periodically extended planes and plans
  /// without the fused form.
  bool ConvolveSpectrumPeak(const void* d_spectrum, float scale, void* d_work, float* d_out,
                            uint32_t h_border, uint32_t v_border, bool allow_negative,
                            const uint8_t* d_mask, uint32_t slot);

  /// The fused multi-scale path (Fft::FusedScales) for this plane: the
  /// forward half of an image (periodically extended where the plane is),
  /// the scales' real kernel spectra (cached), every listed scale's inner
  /// inverse into d_outs (spectrum-sized each), and per scale the outer
  /// inverse + inverse rows with the fused peak search into the W x H d_out.
  bool Fused();
  const void* RealKernelSpectrum(float scale);
  void ForwardHalf(const float* d_image, void* d_half);
  void Scales(const void* d_half, const std::vector<float>& scales,
              const std::vector<void*>& d_outs);
  void FinishPeak(const void* d_u, float scale, void* d_work, float* d_out, uint32_t h_border,
                  uint32_t v_border, bool allow_negative, const uint8_t* d_mask, uint32_t slot);

  // multiscale_transforms.h:41-195
  static std::vector<float> MakeShapeFunction(float scale, size_t& n,
                                              size_t max_n, Shape shape);
  static float KernelPeakValue(double scale, size_t max_n, Shape shape);
  static float GaussianSigma(float scale) { return scale * (3.0 / 16.0); }

 private:
  bool Extended() const { return pw_ != width_ || ph_ != height_; }
  /// The plane's FFT, planned on first use (an unfriendly W x H is never
  /// planned itself: its transforms run in the extended plane).
  gpu::Fft& TheFft();
  size_t KernelRadius(float scale) const;
  void Plan(size_t radius);
  float* Plane();
  void Crop(float* d_out);

  gpu::Session& s_;
  size_t width_, height_;
  Shape shape_;
  size_t pw_, ph_, radius_ = 0;  // FFT plane and the margin it holds
  gpu::Fft* fft_;
  std::shared_ptr<gpu::Buffer> plane_;
  std::map<float, std::shared_ptr<gpu::Buffer>> spectra_;
  std::map<float, std::shared_ptr<gpu::Buffer>> real_spectra_;  // RealKernelSpectrum
  std::map<float, std::pair<std::shared_ptr<gpu::Buffer>, size_t>> shapes_;
};

}  // namespace radler::algorithms::multiscale
