#include "multiscale_transforms.h"

#include <cmath>
#include <stdexcept>

#include "fft_sizes.h"

namespace radler::algorithms::multiscale {

namespace {
// multiscale_transforms.h:186-194
float HannWindow(float x, size_t n) {
  return (x * 2 <= float(n + 1))
             ? float(0.5 * (1.0 + std::cos(2.0 * M_PI * x / double(n + 1))))
             : 0.0f;
}
float ShapeFunction(float x) {
  if (x < 1.0f) {
    const float xx = x * x;
    return float(1.0 - double(xx));
  }
  return 0.0f;
}
// multiscale_transforms.h:118-185. The reference's GCC build contracts
// dx*dx + dydy into an FMA (exact here: dx is a half-integer).
std::vector<float> TaperedQuadratic(double scale, size_t& n) {
  n = size_t(std::ceil(scale * 0.5) * 2.0) + 1;
  std::vector<float> out(n * n, 0.0f);
  if (scale == 0.0) {
    out[0] = 1.0f;
    return out;
  }
  float sum = 0.0f;
  for (int y = 0; y != int(n); ++y) {
    const float dy = float(y - 0.5 * double(n - 1));
    const float dydy = dy * dy;
    for (int x = 0; x != int(n); ++x) {
      const float dx = float(x - 0.5 * double(n - 1));
      const float r = std::sqrt(std::fma(dx, dx, dydy));
      const float v = HannWindow(r, n) * ShapeFunction(float(double(r) / scale));
      out[x + y * n] = v;
      sum += v;
    }
  }
  const float norm = float(1.0 / double(sum));
  for (float& v : out) v *= norm;
  return out;
}
// multiscale_transforms.h:127-161
std::vector<float> Gaussian(double scale, size_t& n, size_t max_n) {
  float sigma = MultiScaleTransforms::GaussianSigma(float(scale));
  n = int(std::ceil(sigma * 12.0 / 2.0)) * 2 + 1;
  if (n > max_n) {
    n = max_n;
    if ((n % 2) == 0 && n > 0) --n;
  }
  if (n < 1) n = 1;
  if (sigma == 0.0f) {
    sigma = 1.0f;
    n = 1;
  }
  std::vector<float> out(n * n);
  const float mu = float(int(n / 2));
  const float two_sigma_sq = float(2.0 * sigma * sigma);
  std::vector<float> g(n);
  for (int i = 0; i != int(n); ++i) {
    const float v = float(i) - mu;
    g[i] = std::exp(-v * v / two_sigma_sq);
  }
  float sum = 0.0f;
  for (size_t y = 0; y != n; ++y)
    for (size_t x = 0; x != n; ++x) {
      const float v = g[x] * g[y];
      out[x + y * n] = v;
      sum += v;
    }
  const float norm = float(1.0 / double(sum));
  for (float& v : out) v *= norm;
  return out;
}
}  // namespace

std::vector<float> MultiScaleTransforms::MakeShapeFunction(float scale,
                                                           size_t& n,
                                                           size_t max_n,
                                                           Shape shape) {
  if (shape == Shape::kGaussianShape) return Gaussian(scale, n, max_n);
  return TaperedQuadratic(scale, n);
}

float MultiScaleTransforms::KernelPeakValue(double scale, size_t max_n,
                                            Shape shape) {
  size_t n;
  const std::vector<float> k = MakeShapeFunction(float(scale), n, max_n, shape);
  return k[n / 2 + (n / 2) * n];
}

MultiScaleTransforms::MultiScaleTransforms(gpu::Session& s, size_t width,
                                           size_t height, Shape shape)
    : s_(s),
      width_(width),
      height_(height),
      shape_(shape),
      pw_(width),
      ph_(height),
      fft_(nullptr) {}

namespace {
// A coarse ladder of FFT-friendly plane sides for the periodically extended
// transforms: subimages of slightly different sizes (Dijkstra boundaries)
// then share a few FFT plans instead of planning one per subimage.
size_t CanonicalFftSize(size_t n) {
  const size_t step = n > 2048 ? 512 : n > 1024 ? 256 : n > 256 ? 64 : 2;
  size_t m = (n + step - 1) / step * step;
  while (utils::CalculateGoodFFTSize(m) != m) m += step;
  return m;
}
}  // namespace

gpu::Fft& MultiScaleTransforms::TheFft() {
  if (!fft_) Plan(radius_);
  return *fft_;
}

size_t MultiScaleTransforms::KernelRadius(float scale) const {
  size_t n;
  MakeShapeFunction(scale, n, std::min(width_, height_), shape_);
  return n / 2;
}

void MultiScaleTransforms::Plan(size_t radius) {
  const bool friendly = utils::CalculateGoodFFTSize(width_) == width_ &&
                        utils::CalculateGoodFFTSize(height_) == height_;
  size_t pw = width_, ph = height_;
  if (!friendly && radius < width_ && radius < height_) {
    pw = std::max(width_, CanonicalFftSize(width_ + 2 * radius));
    ph = std::max(height_, CanonicalFftSize(height_ + 2 * radius));
  }
  radius_ = radius;
  if (fft_ && pw == pw_ && ph == ph_) return;
  pw_ = pw;
  ph_ = ph;
  fft_ = &s_.GetFft(pw_, ph_);
  spectra_.clear();
  real_spectra_.clear();
  plane_.reset();
}

void MultiScaleTransforms::SetMaxScale(float scale) {
  const size_t r = KernelRadius(scale);
  if (!fft_ || r > radius_ || pw_ == width_) Plan(r);
}

float* MultiScaleTransforms::Plane() {
  if (!plane_) plane_ = std::make_shared<gpu::Buffer>(s_, pw_ * ph_ * sizeof(float));
  return plane_->F();
}

void MultiScaleTransforms::Crop(float* d_out) {
  gpu::Check(rdl_box(s_.Handle(), d_out, uint32_t(width_), 0, 0, Plane(), uint32_t(pw_),
                     uint32_t(radius_), uint32_t(radius_), uint32_t(width_),
                     uint32_t(height_), nullptr, RDL_BOX_COPY),
             "rdl_box");
}

const void* MultiScaleTransforms::KernelSpectrum(float scale) {
  TheFft();
  if (Extended() && KernelRadius(scale) > radius_) Plan(KernelRadius(scale));
  auto it = spectra_.find(scale);
  if (it != spectra_.end()) return it->second->Ptr();
  size_t n;
  const std::vector<float> k =
      MakeShapeFunction(scale, n, std::min(width_, height_), shape_);
  gpu::Buffer placed(s_, pw_ * ph_ * sizeof(float));
  // schaapcommon::math::PrepareSmallConvolutionKernel
  gpu::Check(rdl_prepare_small_kernel(s_.Handle(), placed.F(), uint32_t(pw_),
                                      uint32_t(ph_), k.data(), uint32_t(n)),
             "rdl_prepare_small_kernel");
  auto spectrum = std::make_shared<gpu::Buffer>(s_, fft_->SpectrumBytes());
  fft_->Forward(placed.F(), spectrum->Ptr());
  s_.Sync();
  spectra_[scale] = spectrum;
  return spectrum->Ptr();
}

const float* MultiScaleTransforms::ShapeKernel(float scale, size_t& n) {
  auto it = shapes_.find(scale);
  if (it == shapes_.end()) {
    size_t kn;
    const std::vector<float> k =
        MakeShapeFunction(scale, kn, std::min(width_, height_), shape_);
    auto buf = std::make_shared<gpu::Buffer>(s_, k.size() * sizeof(float));
    s_.H2D(buf->Ptr(), k.data(), k.size() * sizeof(float));
    it = shapes_.emplace(scale, std::make_pair(buf, kn)).first;
  }
  n = it->second.second;
  return it->second.first->F();
}

void MultiScaleTransforms::Transform(float* d_image, float scale) {
  const void* spectrum = KernelSpectrum(scale);
  if (!Extended()) {
    fft_->Convolve(d_image, spectrum);
    return;
  }
  float* plane = Plane();
  gpu::Check(rdl_periodic_extend(s_.Handle(), plane, uint32_t(pw_), uint32_t(ph_),
                                 d_image, uint32_t(width_), uint32_t(height_),
                                 uint32_t(radius_), uint32_t(radius_)),
             "rdl_periodic_extend");
  // the window of the convolved plane straight into the image (no Crop pass)
  if (fft_->ConvolveWindow(plane, spectrum, d_image, width_, height_, radius_, radius_)) return;
  fft_->Convolve(plane, spectrum);
  Crop(d_image);
}

void MultiScaleTransforms::Forward(const float* d_image, void* d_spectrum) {
  TheFft();
  if (!Extended()) {
    fft_->Forward(d_image, d_spectrum);
    return;
  }
  float* plane = Plane();
  gpu::Check(rdl_periodic_extend(s_.Handle(), plane, uint32_t(pw_), uint32_t(ph_),
                                 d_image, uint32_t(width_), uint32_t(height_),
                                 uint32_t(radius_), uint32_t(radius_)),
             "rdl_periodic_extend");
  fft_->Forward(plane, d_spectrum);
}

void MultiScaleTransforms::ConvolveSpectrum(const void* d_spectrum, float scale,
                                            void* d_work, float* d_out) {
  if (Extended() && KernelRadius(scale) > radius_)
    throw std::logic_error("ConvolveSpectrum: scale larger than the planned margin");
  const void* kernel = KernelSpectrum(scale);
  if (!Extended()) {
    fft_->ConvolveSpectrum(d_spectrum, kernel, d_work, d_out);
    return;
  }
  if (fft_->ConvolveSpectrumWindow(d_spectrum, kernel, d_work, d_out, width_, height_,
                                   radius_, radius_))
    return;
  fft_->ConvolveSpectrum(d_spectrum, kernel, d_work, Plane());
  Crop(d_out);
}

bool MultiScaleTransforms::ConvolveSpectrumPeak(const void* d_spectrum, float scale,
                                                void* d_work, float* d_out,
                                                uint32_t h_border, uint32_t v_border,
                                                bool allow_negative, const uint8_t* d_mask,
                                                uint32_t slot) {
  if (Extended() && KernelRadius(scale) > radius_)
    throw std::logic_error("ConvolveSpectrumPeak: scale larger than the planned margin");
  const void* kernel = KernelSpectrum(scale);
  if (!Extended())
    return fft_->ConvolveSpectrumPeak(d_spectrum, kernel, d_work, d_out, h_border, v_border,
                                      allow_negative, d_mask, slot);
  return fft_->ConvolveSpectrumWindowPeak(d_spectrum, kernel, d_work, d_out, width_, height_,
                                          radius_, radius_, h_border, v_border,
                                          allow_negative, d_mask, slot);
}

bool MultiScaleTransforms::Fused() { return TheFft().FusedScales(); }

const void* MultiScaleTransforms::RealKernelSpectrum(float scale) {
  TheFft();
  if (Extended() && KernelRadius(scale) > radius_) Plan(KernelRadius(scale));
  auto it = real_spectra_.find(scale);
  if (it != real_spectra_.end()) return it->second->Ptr();
  size_t n;
  const std::vector<float> k =
      MakeShapeFunction(scale, n, std::min(width_, height_), shape_);
  auto spectrum = std::make_shared<gpu::Buffer>(s_, fft_->RealKernelBytes());
  fft_->RealKernel(k.data(), n, spectrum->Ptr());
  real_spectra_[scale] = spectrum;
  return spectrum->Ptr();
}

void MultiScaleTransforms::ForwardHalf(const float* d_image, void* d_half) {
  TheFft();
  if (!Extended()) {
    fft_->ForwardHalf(d_image, d_half);
    return;
  }
  float* plane = Plane();
  gpu::Check(rdl_periodic_extend(s_.Handle(), plane, uint32_t(pw_), uint32_t(ph_),
                                 d_image, uint32_t(width_), uint32_t(height_),
                                 uint32_t(radius_), uint32_t(radius_)),
             "rdl_periodic_extend");
  fft_->ForwardHalf(plane, d_half);
}

void MultiScaleTransforms::Scales(const void* d_half, const std::vector<float>& scales,
                                  const std::vector<void*>& d_outs) {
  std::vector<const void*> kernels;
  for (float sc : scales) {
    if (Extended() && KernelRadius(sc) > radius_)
      throw std::logic_error("Scales: scale larger than the planned margin");
    kernels.push_back(RealKernelSpectrum(sc));
  }
  fft_->Scales(d_half, kernels, d_outs);
}

void MultiScaleTransforms::FinishPeak(const void* d_u, float scale, void* d_work, float* d_out,
                                      uint32_t h_border, uint32_t v_border,
                                      bool allow_negative, const uint8_t* d_mask,
                                      uint32_t slot) {
  (void)scale;
  const size_t ox = Extended() ? radius_ : 0, oy = Extended() ? radius_ : 0;
  fft_->ScaleFinishWindowPeak(d_u, d_work, d_out, width_, height_, ox, oy, h_border, v_border,
                              allow_negative, d_mask, slot);
}

}  // namespace radler::algorithms::multiscale
