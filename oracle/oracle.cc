// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
// CPU restatement of Radler's CLEAN hot path; see oracle.h.
#include <chrono>
#include "oracle.h"

#include "component_optimization.h"

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "fft.h"

namespace oracle {

// ---------------------------------------------------------------------------
// Peak finding — cpp/math/peak_finder.cc
// ---------------------------------------------------------------------------
namespace {
void Box(size_t width, size_t height, size_t start_y, size_t end_y,
         size_t hb, size_t vb, size_t& xs, size_t& xe, size_t& ys,
         size_t& ye) {
  // peak_finder.cc:27-32 (unsigned arithmetic as in the reference)
  xs = hb;
  xe = width - hb;
  ys = std::max(start_y, vb);
  ye = std::min(end_y, height - vb);
  if (xe < xs) xe = xs;
  if (ye < ys) ye = ys;
}
}  // namespace

Peak FindPeakAvx(const float* image, size_t width, size_t height,
                 bool allow_negative, size_t start_y, size_t end_y, size_t hb,
                 size_t vb) {
  // peak_finder.cc:199-253: sequential strict '>' scan from FLT_MIN, first
  // index wins, peakIndex starts at 0 so "no peak" returns image[0].
  float peak_max = std::numeric_limits<float>::min();
  size_t peak_index = 0;
  size_t xs, xe, ys, ye;
  Box(width, height, start_y, end_y, hb, vb, xs, xe, ys, ye);
  for (size_t yi = ys; yi != ye; ++yi) {
    size_t index = yi * width + xs;
    for (size_t xi = xs; xi != xe; ++xi) {
      float value = image[index];
      if (allow_negative) value = std::fabs(value);
      if (value > peak_max) {
        peak_index = index;
        peak_max = std::fabs(image[index]);
      }
      ++index;
    }
  }
  Peak p;
  p.has = true;
  p.x = peak_index % width;
  p.y = peak_index / width;
  p.value = image[p.x + p.y * width];
  return p;
}

Peak FindPeakSimple(const float* image, size_t width, size_t height,
                    bool allow_negative, size_t start_y, size_t end_y,
                    size_t hb, size_t vb) {
  float peak_max = std::numeric_limits<float>::min();
  size_t peak_index = width * height;
  size_t xs, xe, ys, ye;
  Box(width, height, start_y, end_y, hb, vb, xs, xe, ys, ye);
  for (size_t yi = ys; yi != ye; ++yi) {
    size_t index = yi * width + xs;
    for (size_t xi = xs; xi != xe; ++xi) {
      float value = image[index];
      if (allow_negative) value = std::fabs(value);
      if (value > peak_max) {
        peak_index = index;
        peak_max = std::fabs(value);
      }
      ++index;
    }
  }
  Peak p;
  if (peak_index == width * height) {
    p.has = false;
    p.x = width;
    p.y = height;
    return p;
  }
  p.has = true;
  p.x = peak_index % width;
  p.y = peak_index / width;
  p.value = image[p.x + p.y * width];
  return p;
}

Peak FindPeakWithMask(const float* image, size_t width, size_t height,
                      bool allow_negative, size_t start_y, size_t end_y,
                      const bool* mask, size_t hb, size_t vb) {
  float peak_max = std::numeric_limits<float>::min();
  Peak p;
  p.x = width;
  p.y = height;
  size_t xs, xe, ys, ye;
  Box(width, height, start_y, end_y, hb, vb, xs, xe, ys, ye);
  for (size_t yi = ys; yi != ye; ++yi) {
    for (size_t xi = xs; xi != xe; ++xi) {
      float value = image[yi * width + xi];
      if (allow_negative) value = std::fabs(value);
      if (value > peak_max && mask[yi * width + xi]) {
        p.x = xi;
        p.y = yi;
        peak_max = std::fabs(value);
      }
    }
  }
  if (p.y == height) {
    p.has = false;
    return p;
  }
  p.has = true;
  p.value = image[p.x + p.y * width];
  return p;
}

// ---------------------------------------------------------------------------
// PSF subtraction — cpp/algorithms/simple_clean.cc:96-131
// ---------------------------------------------------------------------------
void PartialSubtractImage(float* image, const float* psf, size_t width,
                          size_t height, size_t x, size_t y, float factor,
                          size_t start_y, size_t end_y) {
  size_t start_x, end_x;
  const int offset_x = static_cast<int>(x) - static_cast<int>(width / 2);
  const int offset_y = static_cast<int>(y) - static_cast<int>(height / 2);
  start_x = offset_x > 0 ? size_t(offset_x) : 0;
  if (offset_y > static_cast<int>(start_y)) start_y = offset_y;
  end_x = x + width / 2;
  if (end_x > width) end_x = width;
  end_y = std::min(y + height / 2, end_y);
  // The pairwise-unrolled body plus scalar tail of the reference together
  // cover [start_x, end_x) once; GCC contracts each update into an FMA.
  for (size_t ypos = start_y; ypos < end_y; ++ypos) {
    float* img = image + ypos * width;
    const float* p = psf + (ypos - offset_y) * width - offset_x;
    for (size_t xpos = start_x; xpos < end_x; ++xpos)
      img[xpos] = std::fmaf(-p[xpos], factor, img[xpos]);
  }
}

void SubtractImage(float* image, const float* psf, size_t width, size_t height,
                   size_t x, size_t y, float factor) {
  ParallelFor(0, height, [&](size_t a, size_t b) {
    PartialSubtractImage(image, psf, width, height, x, y, factor, a, b);
  });
}

// ---------------------------------------------------------------------------
// FFT sizes — cpp/utils/fft_size_calculations.h:15-50
// ---------------------------------------------------------------------------
size_t CalculateGoodFFTSize(size_t minimum_size) {
  size_t best = 2 * minimum_size;
  for (size_t f2 = 2; f2 < best; f2 *= 2)
    for (size_t f23 = f2; f23 < best; f23 *= 3)
      for (size_t f235 = f23; f235 < best; f235 *= 5)
        for (size_t f2357 = f235; f2357 < best; f2357 *= 7)
          if (f2357 >= minimum_size) best = f2357;
  return best;
}

size_t GetConvolutionSize(double scale, size_t original_size, double padding) {
  return CalculateGoodFFTSize(
      std::ceil(padding * (scale * 1.5 + original_size)));
}

// ---------------------------------------------------------------------------
// Convolution helpers (schaapcommon / aocommon contracts)
// ---------------------------------------------------------------------------
void PrepareSmallConvolutionKernel(float* dest, size_t width, size_t height,
                                   const float* kernel, size_t n) {
  if (n > width || n > height)
    throw std::runtime_error("Kernel size is larger than the image size");
  for (size_t y = 0; y != n; ++y) {
    long dy = long(y) - long(n / 2);
    if (dy < 0) dy += height;
    for (size_t x = 0; x != n; ++x) {
      long dx = long(x) - long(n / 2);
      if (dx < 0) dx += width;
      dest[dx + dy * width] = kernel[x + y * n];
    }
  }
}

void PrepareConvolutionKernel(float* dest, const float* source, size_t width,
                              size_t height) {
  for (size_t y = 0; y != height; ++y) {
    const size_t sy = (y + height / 2) % height;
    for (size_t x = 0; x != width; ++x) {
      const size_t sx = (x + width / 2) % width;
      dest[x + y * width] = source[sx + sy * width];
    }
  }
}

void Untrim(float* dest, size_t out_w, size_t out_h, const float* src,
            size_t in_w, size_t in_h) {
  std::fill_n(dest, out_w * out_h, 0.0f);
  const size_t sx = (out_w - in_w) / 2, sy = (out_h - in_h) / 2;
  for (size_t y = 0; y != in_h; ++y)
    std::copy_n(src + y * in_w, in_w, dest + (y + sy) * out_w + sx);
}

void Trim(float* dest, size_t out_w, size_t out_h, const float* src,
          size_t in_w, size_t in_h) {
  const size_t sx = (in_w - out_w) / 2, sy = (in_h - out_h) / 2;
  for (size_t y = 0; y != out_h; ++y)
    std::copy_n(src + (y + sy) * in_w + sx, out_w, dest + y * out_w);
}

// ---------------------------------------------------------------------------
// Scale kernels — cpp/algorithms/multiscale/multiscale_transforms.h
// ---------------------------------------------------------------------------
namespace {
float HannWindow(float x, size_t n) {  // .h:186-190
  return (x * 2 <= float(n + 1))
             ? float(0.5 * (1.0 + std::cos(2.0 * M_PI * x / double(n + 1))))
             : 0.0f;
}
float ShapeFn(float x) {  // .h:192-194
  if (x < 1.0f) {
    const float xx = x * x;
    return float(1.0 - double(xx));
  }
  return 0.0f;
}

std::vector<float> TaperedQuadratic(double scale, size_t& n) {  // .h:122-185
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
      const float r = std::sqrt(std::fmaf(dx, dx, dydy));
      const float v = HannWindow(r, n) * ShapeFn(float(double(r) / scale));
      out[x + y * n] = v;
      sum += v;
    }
  }
  const float norm = float(1.0 / double(sum));
  for (float& v : out) v *= norm;
  return out;
}

std::vector<float> Gaussian(double scale, size_t& n, size_t max_n) {
  float sigma = float(float(scale) * (3.0 / 16.0));  // .h:114-116
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
  float sum = 0.0f;
  std::vector<float> g(n);
  for (int i = 0; i != int(n); ++i) {
    const float v = float(i) - mu;
    g[i] = std::exp(-v * v / two_sigma_sq);
  }
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

std::vector<float> MakeShapeFunction(float scale, size_t& n, size_t max_n,
                                     Shape shape) {
  if (shape == Shape::kGaussian) return Gaussian(scale, n, max_n);
  return TaperedQuadratic(scale, n);
}

float KernelPeakValue(double scale, size_t max_n, Shape shape) {
  size_t n;
  std::vector<float> k = MakeShapeFunction(float(scale), n, max_n, shape);
  return k[n / 2 + (n / 2) * n];
}

void AddShapeComponent(float* image, size_t width, size_t height, float scale,
                       size_t x, size_t y, float gain, Shape shape) {
  size_t n;  // multiscale_transforms.h:62-89
  std::vector<float> kernel =
      MakeShapeFunction(scale, n, std::min(width, height), shape);
  const int left = x > n / 2 ? int(x - n / 2) : 0;
  const int top = y > n / 2 ? int(y - n / 2) : 0;
  const size_t right = std::min(x + (n + 1) / 2, width);
  const size_t bottom = std::min(y + (n + 1) / 2, height);
  for (size_t yi = top; yi != bottom; ++yi) {
    float* img = &image[yi * width];
    const float* k = &kernel[(yi + n / 2 - y) * n + left + n / 2 - x];
    for (size_t xi = left; xi != right; ++xi) {
      img[xi] = std::fmaf(*k, gain, img[xi]);
      ++k;
    }
  }
}

void MsTransform(std::vector<float*>& images, size_t width, size_t height,
                 float scale, Shape shape) {
  size_t n;
  std::vector<float> k =
      MakeShapeFunction(scale, n, std::min(width, height), shape);
  std::vector<float> kernel(width * height, 0.0f);
  PrepareSmallConvolutionKernel(kernel.data(), width, height, k.data(), n);
  for (float* img : images) ConvolveCircular(img, kernel.data(), width, height);
}

// ---------------------------------------------------------------------------
// ImageSet integration — cpp/image_set.cc
// ---------------------------------------------------------------------------
void GetLinearIntegrated(const ImageSet& set, float* dest) {
  const SetDesc& d = *set.desc;
  const size_t n = set.width * set.height;
  if (d.squared_joins) {
    GetSquareIntegrated(set, dest);
    return;
  }
  if (d.n_channels == 1 && d.n_pol == 1) {  // image_set.cc:425-430
    std::copy_n(set.images[0], n, dest);
    return;
  }
  bool is_first = true;
  double weight_sum = 0.0;
  for (size_t ch = 0; ch != d.n_channels; ++ch) {
    const float w = d.weights[ch];
    if (w != 0.0f) {
      weight_sum += w;
      for (size_t p = 0; p != d.n_pol; ++p) {
        const float* img = set.images[ch * d.n_pol + p];
        if (is_first) {  // AssignMultiply, image_set.cc:16-24
          for (size_t i = 0; i != n; ++i) dest[i] = img[i] * w;
          is_first = false;
        } else {  // aocommon AddWithFactor (contracted)
          for (size_t i = 0; i != n; ++i) dest[i] = std::fmaf(img[i], w, dest[i]);
        }
      }
    }
  }
  if (weight_sum > 0.0) {
    const float f = float(double(d.pol_factor) / weight_sum);
    for (size_t i = 0; i != n; ++i) dest[i] *= f;
  } else {
    std::fill_n(dest, n, 0.0f);
  }
}

void GetSquareIntegrated(const ImageSet& set, float* dest) {
  const SetDesc& d = *set.desc;
  const size_t n = set.width * set.height;
  if (d.squared_joins) {
    // image_set.cc:363-390 (aocommon SquareWithFactor / AddSquared orders
    // are not in /root/reference: parity unpinned for this branch)
    bool is_first = true;
    double weight_sum = 0.0;
    for (size_t ch = 0; ch != d.n_channels; ++ch) {
      const float w = d.weights[ch];
      if (w != 0.0f) {
        weight_sum += w;
        for (size_t p = 0; p != d.n_pol; ++p) {
          const float* img = set.images[ch * d.n_pol + p];
          if (is_first) {
            for (size_t i = 0; i != n; ++i) dest[i] = img[i] * img[i] * w;
            is_first = false;
          } else {
            for (size_t i = 0; i != n; ++i)
              dest[i] = std::fmaf(img[i] * img[i], w, dest[i]);
          }
        }
      }
    }
    if (weight_sum > 0.0) {
      const float f = float(std::sqrt(double(d.pol_factor) / weight_sum));
      for (size_t i = 0; i != n; ++i) dest[i] = std::sqrt(dest[i]) * f;
    } else {
      std::fill_n(dest, n, 0.0f);
    }
    return;
  }
  if (d.n_channels == 1) {  // image_set.cc:289-311
    if (d.n_pol == 1) {
      std::copy_n(set.images[0], n, dest);
    } else {
      for (size_t i = 0; i != n; ++i) dest[i] = set.images[0][i] * set.images[0][i];
      for (size_t p = 1; p != d.n_pol; ++p)
        for (size_t i = 0; i != n; ++i)
          dest[i] = std::fmaf(set.images[p][i], set.images[p][i], dest[i]);
      const float f = std::sqrt(d.pol_factor);
      for (size_t i = 0; i != n; ++i) dest[i] = std::sqrt(dest[i]) * f;
    }
    return;
  }
  std::vector<float> scratch(n);
  double weight_sum = 0.0;
  for (size_t ch = 0; ch != d.n_channels; ++ch) {
    const float w = d.weights[ch];
    if (w != 0.0f) {
      weight_sum += w;
      if (d.n_pol == 1) {
        std::copy_n(set.images[ch], n, scratch.data());
      } else {
        const float* first = set.images[ch * d.n_pol];
        for (size_t i = 0; i != n; ++i) scratch[i] = first[i] * first[i];
        for (size_t p = 1; p != d.n_pol; ++p) {
          const float* img = set.images[ch * d.n_pol + p];
          for (size_t i = 0; i != n; ++i)
            scratch[i] = std::fmaf(img[i], img[i], scratch[i]);
        }
        for (size_t i = 0; i != n; ++i) scratch[i] = std::sqrt(scratch[i]);
      }
    } else {
      std::fill(scratch.begin(), scratch.end(), 0.0f);
    }
    if (ch == 0) {
      for (size_t i = 0; i != n; ++i) dest[i] = scratch[i] * w;
    } else {
      for (size_t i = 0; i != n; ++i) dest[i] = std::fmaf(scratch[i], w, dest[i]);
    }
  }
  const float f = float(double(std::sqrt(d.pol_factor)) / weight_sum);
  for (size_t i = 0; i != n; ++i) dest[i] *= f;
}

void GetIntegratedPsf(const SetDesc& d, const std::vector<const float*>& psfs,
                      size_t n, float* dest) {
  if (d.n_channels == 1) {  // image_set.cc:504-505
    std::copy_n(psfs[0], n, dest);
    return;
  }
  bool is_first = true;
  double weight_sum = 0.0;
  for (size_t ch = 0; ch != d.n_channels; ++ch) {
    const float w = d.weights[ch];
    if (w != 0.0f) {
      weight_sum += w;
      if (is_first) {
        for (size_t i = 0; i != n; ++i) dest[i] = psfs[ch][i] * w;
        is_first = false;
      } else {
        for (size_t i = 0; i != n; ++i) dest[i] = std::fmaf(psfs[ch][i], w, dest[i]);
      }
    }
  }
  const float f = float(weight_sum == 0.0 ? 0.0 : 1.0 / weight_sum);
  for (size_t i = 0; i != n; ++i) dest[i] *= f;
}

// ---------------------------------------------------------------------------
// SubMinorLoop — cpp/algorithms/subminor_loop.cc
// ---------------------------------------------------------------------------
size_t SubMinorLoop::GetMaxComponent(std::vector<float>& scratch,
                                     float& max_value) const {
  // subminor_loop.cc:13-36
  ImageSet set;
  set.desc = desc_;
  set.width = positions_.size();
  set.height = 1;
  for (const auto& r : residual_) set.images.push_back(const_cast<float*>(r.data()));
  GetLinearIntegrated(set, scratch.data());
  if (!rms_selected_.empty())
    for (size_t i = 0; i != positions_.size(); ++i) scratch[i] *= rms_selected_[i];
  size_t max_component = 0;
  max_value = scratch[0];
  for (size_t i = 0; i != positions_.size(); ++i) {
    const float value = allow_negative ? std::fabs(scratch[i]) : scratch[i];
    if (value > max_value) {
      max_component = i;
      max_value = value;
    }
  }
  max_value = scratch[max_component];
  return max_component;
}

void SubMinorLoop::NoteArgmaxMargin(const std::vector<float>& scratch,
                                    size_t chosen) const {
  const auto value = [&](size_t i) {
    return allow_negative ? std::fabs(scratch[i]) : scratch[i];
  };
  bool any = false;
  float second = 0.0f;
  for (size_t i = 0; i != positions_.size(); ++i)
    if (i != chosen && (!any || value(i) > second)) {
      second = value(i);
      any = true;
    }
  if (any) margins->Note(value(chosen), second);
}

SubMinorLoop::RunResult SubMinorLoop::Run(
    ImageSet& convolved_residual,
    const std::vector<const float*>& twice_convolved_psfs) {
  desc_ = convolved_residual.desc;
  positions_.clear();
  // findPeakPositions, subminor_loop.cc:143-184
  {
    std::vector<float> integrated(width_ * height_);
    GetLinearIntegrated(convolved_residual, integrated.data());
    if (rms_factor)  // subminor_loop.cc:147-149
      for (size_t i = 0; i != width_ * height_; ++i) integrated[i] *= rms_factor[i];
    const size_t xs = horizontal_border;
    const size_t xe = std::max<long>(xs, long(width_) - long(horizontal_border));
    const size_t ys = vertical_border;
    const size_t ye = std::max<long>(ys, long(height_) - long(vertical_border));
    for (size_t y = ys; y != ye; ++y) {
      for (size_t x = xs; x != xe; ++x) {
        const float v = integrated[y * width_ + x];
        const float value = allow_negative ? std::fabs(v) : v;
        if (value >= threshold && (!mask || mask[y * width_ + x]))
          positions_.emplace_back(x, y);
      }
    }
  }
  // MakeSets, subminor_loop.cc:119-132
  const size_t n_img = convolved_residual.Size();
  residual_.assign(n_img, std::vector<float>(positions_.size()));
  model_.assign(n_img, std::vector<float>(positions_.size(), 0.0f));
  for (size_t i = 0; i != n_img; ++i)
    for (size_t p = 0; p != positions_.size(); ++p)
      residual_[i][p] =
          convolved_residual.images[i][positions_[p].second * width_ +
                                       positions_[p].first];
  rms_selected_.clear();
  if (rms_factor)  // SubMinorModel::MakeRmsFactorImage (subminor_loop.cc:134-141)
    for (const auto& p : positions_)
      rms_selected_.push_back(rms_factor[p.second * width_ + p.first]);
  if (positions_.empty()) return {false, false, 0.0f};

  std::vector<float> scratch(positions_.size());
  float max_value;
  size_t max_component = GetMaxComponent(scratch, max_value);
  const float max_value_at_start = std::fabs(max_value);
  bool diverging = false;
  std::vector<float> component_values(n_img);
  for (;;) {
    if (margins) margins->Note(std::fabs(max_value), threshold);
    if (!(std::fabs(max_value) > threshold &&
          current_iteration < max_iterations &&
          (!stop_on_negative || max_value >= 0.0f) && !diverging))
      break;
    if (margins) NoteArgmaxMargin(scratch, max_component);
    for (size_t i = 0; i != n_img; ++i)
      component_values[i] = residual_[i][max_component] * gain;
    flux_cleaned += max_value * gain;
    const size_t x = positions_[max_component].first;
    const size_t y = positions_[max_component].second;
    if (trace)
      trace->push_back({uint32_t(x), uint32_t(y), trace_scale,
                        margins ? margins->Take()
                                : std::numeric_limits<float>::infinity(),
                        std::fabs(max_value)});
    PerformSpectralFit(convolved_residual.desc->fitter.get(),
                       convolved_residual.desc->n_pol, component_values.data());
    for (size_t i = 0; i != n_img; ++i)
      model_[i][max_component] += component_values[i];
    for (size_t i = 0; i != n_img; ++i) {
      float* image = residual_[i].data();
      const float* psf = twice_convolved_psfs[convolved_residual.PsfIndex(i)];
      const float f = component_values[i];
      for (size_t px = 0; px != positions_.size(); ++px) {
        const int psf_x = int(positions_[px].first) - int(x) + int(width_ / 2);
        const int psf_y = int(positions_[px].second) - int(y) + int(height_ / 2);
        if (psf_x >= 0 && psf_x < int(width_) && psf_y >= 0 &&
            psf_y < int(height_))
          image[px] = std::fmaf(-psf[psf_x + psf_y * width_], f, image[px]);
      }
    }
    max_component = GetMaxComponent(scratch, max_value);
    if (divergence_limit != 0.0f)
      diverging = std::fabs(max_value) > max_value_at_start * divergence_limit;
    ++current_iteration;
  }
  return {diverging, true, max_value};
}

void SubMinorLoop::GetFullIndividualModel(size_t image_index,
                                          float* dest) const {
  std::fill_n(dest, width_ * height_, 0.0f);  // subminor_loop.cc:186-193
  for (size_t p = 0; p != positions_.size(); ++p)
    dest[positions_[p].first + positions_[p].second * width_] =
        model_[image_index][p];
}

void SubMinorLoop::UpdateAutoMask(bool* mask) const {
  for (size_t i = 0; i != model_.size(); ++i)
    for (size_t p = 0; p != positions_.size(); ++p)
      if (model_[i][p] != 0.0f)
        mask[positions_[p].first + positions_[p].second * width_] = true;
}

void SubMinorLoop::CorrectResidualDirty(size_t image_index, float* residual,
                                        const float* psf) const {
  // subminor_loop.cc:195-218
  const size_t pn = padded_width_ * padded_height_;
  std::vector<float> a(pn), b(pn), c(width_ * height_);
  Untrim(a.data(), padded_width_, padded_height_, psf, width_, height_);
  PrepareConvolutionKernel(b.data(), a.data(), padded_width_, padded_height_);
  GetFullIndividualModel(image_index, c.data());
  Untrim(a.data(), padded_width_, padded_height_, c.data(), width_, height_);
  ConvolveCircular(a.data(), b.data(), padded_width_, padded_height_);
  Trim(c.data(), width_, height_, a.data(), padded_width_, padded_height_);
  for (size_t i = 0; i != width_ * height_; ++i) residual[i] -= c[i];
}

// ---------------------------------------------------------------------------
// GenericClean — cpp/algorithms/generic_clean.cc:56-277
// ---------------------------------------------------------------------------
namespace {
Peak GenericFindPeak(const AlgoSettings& s, const float* image, size_t w,
                     size_t h) {
  // generic_clean.cc:255-277 via peak_finder.h:99-107 (border by round())
  const size_t hb = std::round(w * s.clean_border_ratio);
  const size_t vb = std::round(h * s.clean_border_ratio);
  std::vector<float> scratch;
  if (s.rms_factor) {  // generic_clean.cc:258-264
    scratch.assign(image, image + w * h);
    for (size_t i = 0; i != w * h; ++i) scratch[i] *= s.rms_factor[i];
    image = scratch.data();
  }
  if (!s.clean_mask)
    return FindPeakAvx(image, w, h, s.allow_negative, 0, h, hb, vb);
  return FindPeakWithMask(image, w, h, s.allow_negative, 0, h, s.clean_mask,
                          hb, vb);
}
}  // namespace

Result GenericCleanExecute(const AlgoSettings& s_in, size_t& iteration_number,
                           ImageSet& dirty, ImageSet& model,
                           const std::vector<const float*>& psfs,
                           std::vector<Component>* trace) {
  AlgoSettings s = s_in;
  const size_t width = dirty.width, height = dirty.height;
  const size_t start_iter = iteration_number;
  if (s.stop_on_negative) s.allow_negative = true;
  size_t conv_w = std::ceil(1.1f * width);
  size_t conv_h = std::ceil(1.1f * height);
  if (conv_w % 2 != 0) ++conv_w;
  if (conv_h % 2 != 0) ++conv_h;

  std::vector<float> integrated(width * height);
  GetLinearIntegrated(dirty, integrated.data());
  Peak max_value = GenericFindPeak(s, integrated.data(), width, height);
  Result result;
  result.has_starting_peak = max_value.has;
  result.starting_peak = max_value.value;
  result.final_peak = max_value.has ? max_value.value : 0.0f;
  if (!max_value.has) return result;
  if (iteration_number >= s.max_iterations) return result;
  if (s.component_optimization != 0) {  // generic_clean.cc:89-95
    for (size_t i = 0; i != dirty.Size(); ++i)  // RunComponentOptimization (:26-48)
      GradientDescent(model.images[i], dirty.images[i], psfs[dirty.PsfIndex(i)], width,
                      height, 2 * width, 2 * height);
    if (dirty.desc->fitter) {  // FitSpectra (:278-297)
      std::vector<float> values(model.Size());
      for (size_t p = 0; p != width * height; ++p) {
        for (size_t i = 0; i != model.Size(); ++i) values[i] = model.images[i][p];
        PerformSpectralFit(dirty.desc->fitter.get(), dirty.desc->n_pol, values.data());
        for (size_t i = 0; i != model.Size(); ++i) model.images[i][p] = values[i];
      }
    }
    return result;
  }

  const float initial_max_value = std::fabs(max_value.value);
  float first_threshold = s.threshold;
  const float major_iter_threshold = std::max(
      s.major_iteration_threshold, initial_max_value * (1.0f - s.major_loop_gain));
  if (major_iter_threshold > first_threshold) first_threshold = major_iter_threshold;

  bool diverging = false;
  if (s.use_sub_minor_optimization) {
    SubMinorLoop sub(width, height, conv_w, conv_h);
    sub.current_iteration = iteration_number;
    sub.max_iterations = s.max_iterations;
    sub.threshold = first_threshold;
    sub.gain = s.minor_loop_gain;
    sub.allow_negative = s.allow_negative;
    sub.stop_on_negative = s.stop_on_negative;
    sub.divergence_limit = s.divergence_limit;
    sub.mask = s.clean_mask;
    sub.rms_factor = s.rms_factor;  // generic_clean.cc:126-128
    sub.horizontal_border = std::round(width * s.clean_border_ratio);
    sub.vertical_border = std::round(height * s.clean_border_ratio);
    sub.trace = trace;
    SubMinorLoop::RunResult r = sub.Run(dirty, psfs);
    diverging = r.diverging;
    max_value.has = r.has_peak;
    max_value.value = r.peak;
    iteration_number = sub.current_iteration;
    std::vector<float> scratch(width * height);
    for (size_t i = 0; i != dirty.Size(); ++i) {
      // CorrectResidualDirty leaves the trimmed convolved model of the last
      // image in `integrated` (generic_clean.cc:141-143: scratch_c=integrated)
      sub.CorrectResidualDirty(i, dirty.images[i], psfs[dirty.PsfIndex(i)]);
      sub.GetFullIndividualModel(i, scratch.data());
      float* m = model.images[i];
      for (size_t p = 0; p != width * height; ++p) m[p] += scratch[p];
    }
    if (!max_value.has) {
      // generic_clean.cc:150-157. CorrectResidualDirty used `integrated` as
      // its scratch_c (generic_clean.cc:141-143), so it now holds the trimmed
      // convolution of the last image's sub-minor model. Run() returns no
      // peak only when no pixel was selected, so that model is all zeros.
      std::fill(integrated.begin(), integrated.end(), 0.0f);
      max_value = GenericFindPeak(s, integrated.data(), width, height);
    }
  } else {
    size_t peak_index = max_value.x + max_value.y * width;
    std::vector<float> peak_values(dirty.Size());
    while (max_value.has && std::fabs(max_value.value) > first_threshold &&
           iteration_number < s.max_iterations &&
           !(max_value.value < 0.0f && s.stop_on_negative) && !diverging) {
      if (trace)
        trace->push_back({uint32_t(peak_index % width),
                          uint32_t(peak_index / width), 0});
      for (size_t i = 0; i != dirty.Size(); ++i)
        peak_values[i] = dirty.images[i][peak_index];
      PerformSpectralFit(dirty.desc->fitter.get(), dirty.desc->n_pol,
                         peak_values.data());  // generic_clean.cc:186
      const size_t cx = peak_index % width, cy = peak_index / width;
      for (size_t i = 0; i != dirty.Size(); ++i) {
        peak_values[i] *= s.minor_loop_gain;
        model.images[i][peak_index] += peak_values[i];
        SubtractImage(dirty.images[i], psfs[dirty.PsfIndex(i)], width, height,
                      cx, cy, peak_values[i]);
      }
      GetSquareIntegrated(dirty, integrated.data());
      max_value = GenericFindPeak(s, integrated.data(), width, height);
      peak_index = max_value.x + max_value.y * width;
      if (max_value.has && s.divergence_limit != 0.0f)
        diverging =
            std::fabs(max_value.value) > initial_max_value * s.divergence_limit;
      ++iteration_number;
    }
  }
  if (diverging) {
    if (max_value.has) result.final_peak = max_value.value;
    result.another_iteration_required = false;
    result.is_diverging = true;
  } else if (max_value.has) {
    const bool final_threshold_reached =
        std::fabs(max_value.value) <= s.threshold || max_value.value == 0.0f;
    const bool negative_reached = max_value.value < 0.0f && s.stop_on_negative;
    const bool mgain_reached = std::fabs(max_value.value) <= major_iter_threshold;
    const bool did_work = (iteration_number - start_iter) != 0;
    result.another_iteration_required =
        mgain_reached && did_work && !negative_reached && !final_threshold_reached;
    result.final_peak = max_value.value;
  } else {
    result.another_iteration_required = false;
  }
  return result;
}

// ---------------------------------------------------------------------------
// MultiScaleAlgorithm — cpp/algorithms/multiscale_algorithm.cc
// ---------------------------------------------------------------------------
void InitializeScales(std::vector<ScaleInfo>& scales, double beam_px,
                      size_t min_wh, Shape shape, size_t max_scales,
                      const std::vector<double>& scale_list) {
  if (scale_list.empty()) {  // multiscale_algorithm.cc:90-131
    if (scales.empty()) {
      size_t scale_index = 0;
      double scale = beam_px * 2.0;
      do {
        ScaleInfo& e = scales.emplace_back();
        e.scale = scale_index == 0 ? 0.0f : float(scale);
        e.kernel_peak = KernelPeakValue(scale, min_wh, shape);
        scale *= 2.0;
        ++scale_index;
      } while (scale < min_wh * 0.5 &&
               (max_scales == 0 || scale_index < max_scales));
    } else {
      while (!scales.empty() && scales.back().scale >= min_wh * 0.5)
        scales.pop_back();
    }
  } else if (scales.empty()) {
    std::vector<double> sorted = scale_list;
    std::sort(sorted.begin(), sorted.end());
    for (double sc : sorted) {
      ScaleInfo& e = scales.emplace_back();
      e.scale = float(sc);
      e.kernel_peak = KernelPeakValue(e.scale, min_wh, shape);
    }
  }
}

bool SelectMaximumScale(const std::vector<ScaleInfo>& scales, size_t& index) {
  std::map<float, size_t> peak_to_scale;  // multiscale_algorithm.cc:133-151
  for (size_t i = 0; i != scales.size(); ++i) {
    if (scales[i].is_active) {
      const float v = std::fabs(scales[i].max_unnormalized_image_value *
                                scales[i].bias_factor);
      peak_to_scale.insert(std::make_pair(v, i));
    }
  }
  if (peak_to_scale.empty()) return false;
  index = peak_to_scale.rbegin()->second;
  return true;
}

namespace {
// ConvolvePsfs, multiscale_algorithm.cc:29-88
void ConvolvePsfs(std::vector<std::vector<float>>& out, const float* psf,
                  size_t w, size_t h, bool is_integrated,
                  std::vector<ScaleInfo>& scales, double beam_px,
                  double scale_bias, double minor_loop_gain, Shape shape) {
  out.assign(scales.size(), std::vector<float>());
  const double first_auto_scale_size = beam_px * 2.0;
  for (size_t si = 0; si != scales.size(); ++si) {
    ScaleInfo& e = scales[si];
    out[si].assign(psf, psf + w * h);
    if (e.scale != 0.0f) {
      std::vector<float*> l{out[si].data()};
      MsTransform(l, w, h, e.scale, shape);
    }
    if (is_integrated) {
      e.psf_peak = out[si][w / 2 + (h / 2) * w];
      double exp_term;
      if (e.scale == 0.0f || scales.size() < 2)
        exp_term = 0.0;
      else
        exp_term = std::log2(e.scale / first_auto_scale_size);
      e.bias_factor = float(std::pow(scale_bias, -exp_term));
      e.gain = float(minor_loop_gain / e.psf_peak);
      e.is_active = true;
    }
  }
}

float Rms(const float* image, size_t n) {  // threaded_deconvolution_tools.h:40
  float result = 0.0f;
  for (size_t i = 0; i != n; ++i) result = std::fmaf(image[i], image[i], result);
  return std::sqrt(result / float(n));
}
}  // namespace

void MultiScale::FindPeakDirect(const float* image, size_t w, size_t h,
                                size_t scale_index) {
  ScaleInfo& info = scales_[scale_index];  // multiscale_algorithm.cc:700-748
  const size_t hb = std::round(w * s_.clean_border_ratio);
  const size_t vb = std::round(h * s_.clean_border_ratio);
  std::vector<float> scratch;
  if (s_.rms_factor) {  // :707-713
    scratch.assign(image, image + w * h);
    for (size_t i = 0; i != w * h; ++i) scratch[i] *= s_.rms_factor[i];
    image = scratch.data();
  }
  Peak p;
  if (use_scale_masks)
    p = FindPeakWithMask(image, w, h, s_.allow_negative, 0, h,
                         ScaleMask(scale_index), hb, vb);
  else if (!s_.clean_mask)
    p = FindPeakAvx(image, w, h, s_.allow_negative, 0, h, hb, vb);
  else
    p = FindPeakWithMask(image, w, h, s_.allow_negative, 0, h, s_.clean_mask,
                         hb, vb);
  info.max_image_value_x = p.x;
  info.max_image_value_y = p.y;
  if (p.has) {
    info.max_unnormalized_image_value = p.value;
    info.max_normalized_image_value =
        s_.rms_factor ? p.value / s_.rms_factor[p.x + p.y * w] : p.value;
  } else {
    info.max_unnormalized_image_value = 0.0f;
    info.max_normalized_image_value = 0.0f;
  }
}

void MultiScale::FindActiveScaleConvolvedMaxima(const ImageSet& set,
                                                float* integrated,
                                                bool report_rms) {
  // multiscale_algorithm.cc:578-634 + threaded_deconvolution_tools.cc:30-107
  const size_t w = set.width, h = set.height;
  GetLinearIntegrated(set, integrated);
  for (size_t si = 0; si != scales_.size(); ++si) {
    ScaleInfo& e = scales_[si];
    if (!e.is_active) continue;
    if (e.scale == 0.0f) {
      FindPeakDirect(integrated, w, h, si);
      if (report_rms) e.rms = Rms(integrated, w * h);
    } else {
      std::vector<float> copy(integrated, integrated + w * h);
      std::vector<float*> l{copy.data()};
      MsTransform(l, w, h, e.scale, s_.shape);
      const size_t border_scale = std::ceil(e.scale * 0.5);
      const size_t xb = std::max<size_t>(std::round(w * s_.clean_border_ratio),
                                         border_scale);
      const size_t yb = std::max<size_t>(std::round(h * s_.clean_border_ratio),
                                         border_scale);
      if (report_rms) e.rms = Rms(copy.data(), w * h);
      if (s_.rms_factor)  // threaded_deconvolution_tools.cc:84-87
        for (size_t i = 0; i != w * h; ++i) copy[i] *= s_.rms_factor[i];
      Peak p;
      // threaded_deconvolution_tools.cc:43-44: the scale's mask replaces the
      // clean mask when scale masks are in use
      const bool* mask = use_scale_masks ? ScaleMask(si) : s_.clean_mask;
      if (!mask)
        p = FindPeakAvx(copy.data(), w, h, s_.allow_negative, 0, h, xb, yb);
      else
        p = FindPeakWithMask(copy.data(), w, h, s_.allow_negative, 0, h, mask,
                             xb, yb);
      e.max_normalized_image_value =
          p.has ? (s_.rms_factor ? p.value / s_.rms_factor[p.x + p.y * w] : p.value)
                : 0.0f;
      e.max_unnormalized_image_value = p.has ? p.value : 0.0f;
      e.max_image_value_x = p.x;
      e.max_image_value_y = p.y;
    }
  }
}

void MultiScale::NoteScaleSelection() {
  // SelectMaximumScale's std::map<float, size_t> keys (test margins)
  float first = -1.0f, second = -1.0f;
  for (const ScaleInfo& e : scales_) {
    if (!e.is_active) continue;
    const float key = std::fabs(e.max_unnormalized_image_value * e.bias_factor);
    if (key > first) {
      second = first;
      first = key;
    } else if (key > second) {
      second = key;
    }
  }
  if (second >= 0.0f) margins.Note(first, second);
}

void MultiScale::ActivateScales(size_t last) {  // .cc:636-656
  for (size_t i = 0; i != scales_.size(); ++i) {
    if (i != last)
      margins.Note(std::fabs(scales_[i].max_unnormalized_image_value) *
                       scales_[i].bias_factor,
                   std::fabs(scales_[last].max_unnormalized_image_value) *
                       (1.0 - s_.minor_loop_gain) * scales_[last].bias_factor);
    const bool activate =
        i == last ||
        std::fabs(scales_[i].max_unnormalized_image_value) *
                scales_[i].bias_factor >
            std::fabs(scales_[last].max_unnormalized_image_value) *
                (1.0 - s_.minor_loop_gain) * scales_[last].bias_factor;
    scales_[i].is_active = activate;
  }
}

Result MultiScale::Execute(ImageSet& data, ImageSet& model,
                           const std::vector<const float*>& psfs,
                           std::vector<Component>* trace) {
  // multiscale_algorithm.cc:183-576
  const auto setup_start = std::chrono::steady_clock::now();
  const size_t width = data.width, height = data.height;
  const size_t npx = width * height;
  if (s_.stop_on_negative) s_.allow_negative = true;
  InitializeScales(scales_, s_.beam_size_in_pixels, std::min(width, height),
                   s_.shape, s_.max_scales, s_.scale_list);
  if (track_scale_masks) {  // :214-226
    for (const auto& m : scale_masks)
      if (m.size() != npx)
        throw std::runtime_error("Invalid automask size in multiscale algorithm");
    while (scale_masks.size() < scales_.size()) scale_masks.emplace_back(npx, 0);
  }
  bool has_hit_threshold_in_sub_loop = false;
  size_t threshold_countdown = std::max(size_t{8}, scales_.size() * 3 / 2);

  std::vector<float> integrated(npx);
  const size_t n_psf = data.desc->n_channels;
  std::vector<std::vector<std::vector<float>>> convolved_psfs(n_psf);
  GetIntegratedPsf(*data.desc, psfs, npx, integrated.data());
  ConvolvePsfs(convolved_psfs[0], integrated.data(), width, height, true,
               scales_, s_.beam_size_in_pixels, s_.scale_bias,
               s_.minor_loop_gain, s_.shape);
  if (n_psf > 1) {
    for (size_t i = 0; i != n_psf; ++i)
      ConvolvePsfs(convolved_psfs[i], psfs[i], width, height, false, scales_,
                   s_.beam_size_in_pixels, s_.scale_bias, s_.minor_loop_gain,
                   s_.shape);
  }

  FindActiveScaleConvolvedMaxima(data, integrated.data(), true);
  setup_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                setup_start).count();
  const size_t setup_iteration = iteration_number;
  const auto clean_start = std::chrono::steady_clock::now();
  switch_seconds = 0.0;
  switch_components = 0;
  bool switched = clean_threads == 0;
  Result result;
  size_t scale_with_peak;
  margins = MarginTracker();
  end_margin = std::numeric_limits<float>::infinity();
  NoteScaleSelection();
  if (!SelectMaximumScale(scales_, scale_with_peak)) {
    result.another_iteration_required = false;
    return result;
  }
  bool is_final_threshold = false;
  const float initial_peak_value =
      std::fabs(scales_[scale_with_peak].max_unnormalized_image_value *
                scales_[scale_with_peak].bias_factor);
  float m_gain_threshold = initial_peak_value * (1.0 - s_.major_loop_gain);
  m_gain_threshold = std::max(m_gain_threshold, s_.major_iteration_threshold);
  float first_threshold = m_gain_threshold;
  if (s_.threshold > first_threshold) {
    first_threshold = s_.threshold;
    is_final_threshold = true;
  }

  std::vector<std::vector<float>> individual(data.Size(),
                                             std::vector<float>(npx));
  ImageSet individual_set;
  individual_set.desc = data.desc;
  individual_set.width = width;
  individual_set.height = height;
  for (auto& v : individual) individual_set.images.push_back(v.data());
  bool diverging = false;

  size_t outer_iteration = 0;
  for (;;) {
    if (stop_after_outer && outer_iteration == stop_after_outer) break;
    ++outer_iteration;
    if (!switched && outer_iteration > switch_after) {
      // bench.py's cpu_baseline: the rest of the run on clean_threads
      switch_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                     clean_start).count();
      switch_components = iteration_number - setup_iteration;
      SetNThreads(clean_threads);
      switched = true;
    }
    margins.Note(std::fabs(scales_[scale_with_peak].max_unnormalized_image_value *
                           scales_[scale_with_peak].bias_factor),
                 first_threshold);
    if (!(iteration_number < s_.max_iterations &&
          std::fabs(scales_[scale_with_peak].max_unnormalized_image_value *
                    scales_[scale_with_peak].bias_factor) > first_threshold &&
          (!s_.stop_on_negative ||
           scales_[scale_with_peak].max_unnormalized_image_value >= 0.0f) &&
          threshold_countdown > 0 && !diverging))
      break;
    const ScaleInfo& sinfo = scales_[scale_with_peak];
    std::vector<std::vector<float>> twice(n_psf);
    std::vector<float*> transform_list;
    for (size_t i = 0; i != n_psf; ++i) {
      twice[i] = convolved_psfs[i][scale_with_peak];
      transform_list.push_back(twice[i].data());
    }
    for (size_t i = 0; i != data.Size(); ++i) {
      std::copy_n(data.images[i], npx, individual[i].data());
      transform_list.push_back(individual[i].data());
    }
    if (sinfo.scale != 0.0f)
      MsTransform(transform_list, width, height, sinfo.scale, s_.shape);

    const float sub_iteration_gain_threshold =
        std::fabs(sinfo.max_unnormalized_image_value * sinfo.bias_factor) *
        (1.0 - s_.sub_minor_loop_gain);
    float first_sub_iteration_threshold = sub_iteration_gain_threshold;
    margins.Note(first_threshold, first_sub_iteration_threshold);
    if (first_threshold > first_sub_iteration_threshold) {
      first_sub_iteration_threshold = first_threshold;
      if (!has_hit_threshold_in_sub_loop) has_hit_threshold_in_sub_loop = true;
      threshold_countdown--;
    }
    if (s_.fast_sub_minor_loop) {
      const size_t sub_start = iteration_number;
      const size_t conv_w =
          GetConvolutionSize(sinfo.scale, width, s_.convolution_padding);
      const size_t conv_h =
          GetConvolutionSize(sinfo.scale, height, s_.convolution_padding);
      SubMinorLoop sub(width, height, conv_w, conv_h);
      sub.current_iteration = iteration_number;
      sub.max_iterations = s_.max_iterations;
      sub.threshold = first_sub_iteration_threshold / sinfo.bias_factor;
      sub.gain = sinfo.gain;
      sub.divergence_limit = s_.divergence_limit;
      sub.allow_negative = s_.allow_negative;
      sub.stop_on_negative = s_.stop_on_negative;
      const size_t scale_border = std::ceil(sinfo.scale * 0.5);
      sub.horizontal_border =
          std::max<size_t>(std::round(width * s_.clean_border_ratio), scale_border);
      sub.vertical_border =
          std::max<size_t>(std::round(height * s_.clean_border_ratio), scale_border);
      sub.mask = use_scale_masks ? ScaleMask(scale_with_peak) : s_.clean_mask;
      sub.rms_factor = s_.rms_factor;  // multiscale_algorithm.cc:401-402
      sub.trace = trace;
      sub.trace_scale = uint32_t(scale_with_peak);
      sub.margins = &margins;
      std::vector<const float*> twice_ptrs;
      for (auto& t : twice) twice_ptrs.push_back(t.data());
      SubMinorLoop::RunResult r = sub.Run(individual_set, twice_ptrs);
      diverging = r.diverging;
      if (s_.divergence_limit != 0.0f && r.has_peak)
        diverging = diverging ||
                    std::fabs(r.peak) > initial_peak_value * s_.divergence_limit;
      if (!r.has_peak) break;
      iteration_number = sub.current_iteration;
      scales_[scale_with_peak].n_components_cleaned += iteration_number - sub_start;
      scales_[scale_with_peak].total_flux_cleaned += sub.flux_cleaned;
      std::vector<float> scratch(npx);
      for (size_t i = 0; i != data.Size(); ++i) {
        const float* psf = convolved_psfs[data.PsfIndex(i)][scale_with_peak].data();
        sub.CorrectResidualDirty(i, data.images[i], psf);
        sub.GetFullIndividualModel(i, scratch.data());
        if (i == 0 && track_scale_masks)  // :444-445
          sub.UpdateAutoMask(
              reinterpret_cast<bool*>(scale_masks[scale_with_peak].data()));
        if (scales_[scale_with_peak].scale != 0.0f) {
          std::vector<float*> l{scratch.data()};
          MsTransform(l, width, height, scales_[scale_with_peak].scale, s_.shape);
        }
        float* m = model.images[i];
        for (size_t p = 0; p != npx; ++p) m[p] += scratch[p];
      }
    } else {
      // multiscale_algorithm.cc:463-519
      ScaleInfo& mi = scales_[scale_with_peak];
      while (iteration_number < s_.max_iterations &&
             std::fabs(mi.max_unnormalized_image_value * mi.bias_factor) >
                 first_sub_iteration_threshold &&
             (!s_.stop_on_negative || mi.max_unnormalized_image_value >= 0.0f) &&
             !diverging) {
        std::vector<float> cv(data.Size());
        for (size_t i = 0; i != data.Size(); ++i)
          cv[i] = individual[i][mi.max_image_value_x + mi.max_image_value_y * width];
        const size_t x = mi.max_image_value_x, y = mi.max_image_value_y;
        if (trace)
          trace->push_back(
              {uint32_t(x), uint32_t(y), uint32_t(scale_with_peak), margins.Take(),
               std::fabs(mi.max_unnormalized_image_value * mi.bias_factor)});
        PerformSpectralFit(data.desc->fitter.get(), data.desc->n_pol,
                           cv.data());  // multiscale_algorithm.cc:477
        for (size_t i = 0; i != data.Size(); ++i) {
          cv[i] = cv[i] * mi.gain;
          const float* psf = convolved_psfs[data.PsfIndex(i)][scale_with_peak].data();
          SubtractImage(data.images[i], psf, width, height, x, y, cv[i]);
          SubtractImage(individual[i].data(), twice[data.PsfIndex(i)].data(),
                        width, height, x, y, cv[i]);
          if (mi.scale == 0.0f)
            model.images[i][x + width * y] += cv[i];
          else
            AddShapeComponent(model.images[i], width, height, mi.scale, x, y,
                              cv[i], s_.shape);
          mi.n_components_cleaned++;
          mi.total_flux_cleaned += cv[i];
          if (track_scale_masks)  // :695-696
            scale_masks[scale_with_peak][x + width * y] = 1;
        }
        GetLinearIntegrated(individual_set, integrated.data());
        FindPeakDirect(integrated.data(), width, height, scale_with_peak);
        const float abs_peak =
            std::fabs(mi.max_unnormalized_image_value * mi.bias_factor);
        if (s_.divergence_limit != 0.0f)
          diverging = abs_peak > initial_peak_value * s_.divergence_limit;
        ++iteration_number;
      }
    }
    ActivateScales(scale_with_peak);
    FindActiveScaleConvolvedMaxima(data, integrated.data(), false);
    if (std::getenv("ORACLE_DEBUG")) {
      std::fprintf(stderr, "[ms] it=%zu", iteration_number);
      for (const ScaleInfo& e : scales_)
        std::fprintf(stderr, " | s=%g a=%d v=%.9g x=%zu y=%zu", e.scale,
                     int(e.is_active), e.max_unnormalized_image_value * e.bias_factor,
                     e.max_image_value_x, e.max_image_value_y);
      std::fprintf(stderr, "\n");
    }
    NoteScaleSelection();
    if (!SelectMaximumScale(scales_, scale_with_peak)) {
      result.another_iteration_required = false;
      end_margin = margins.Take();
      return result;
    }
  }
  end_margin = margins.Take();
  const bool max_iter_reached = iteration_number >= s_.max_iterations;
  const bool negative_reached =
      s_.stop_on_negative &&
      scales_[scale_with_peak].max_unnormalized_image_value < 0.0f;
  result.is_diverging = diverging;
  result.another_iteration_required =
      !max_iter_reached && !is_final_threshold && !negative_reached && !diverging;
  result.final_peak = scales_[scale_with_peak].max_unnormalized_image_value *
                      scales_[scale_with_peak].bias_factor;
  return result;
}

}  // namespace oracle
