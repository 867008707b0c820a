// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
// Line references: cpp/algorithms/iuwt_deconvolution_algorithm.cc unless
// stated otherwise. See iuwt_algorithm.h for the parity notes.
#include "iuwt_algorithm.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <memory>
#include <stack>

#include "fft.h"
#include "iuwt.h"

namespace oracle {

namespace {

using Plane = std::vector<float>;

// IuwtMask (cpp/algorithms/iuwt/iuwt_mask.h:17-90)
struct Mask {
  Mask(size_t n, size_t w, size_t h) : m(n, std::vector<char>(w * h, 0)), w(w), h(h) {}
  std::vector<std::vector<char>> m;
  size_t w, h;
  Mask Trimmed(size_t x1, size_t y1, size_t x2, size_t y2) const {
    Mask out(m.size(), x2 - x1, y2 - y1);
    for (size_t s = 0; s != m.size(); ++s)
      for (size_t y = y1; y != y2; ++y)
        for (size_t x = x1; x != x2; ++x)
          out.m[s][(y - y1) * (x2 - x1) + (x - x1)] = m[s][y * w + x];
    return out;
  }
};

// IuwtDecomposition (cpp/algorithms/iuwt/iuwt_decomposition.h:37-351)
struct Iuwt {
  Iuwt(int n, size_t w, size_t h) : scales(n + 1), n(n), w(w), h(h) {}
  std::vector<Plane> scales;
  int n;
  size_t w, h;
  // DecomposeMt (iuwt_decomposition.cc:9-54); input may alias scratch, and
  // may point into one of this decomposition's own scales (it is copied first)
  void Decompose(const float* input, float* scratch, bool include_largest) {
    if (input != scratch) {
      const Plane in(input, input + w * h);
      IuwtDecompose(in.data(), scratch, w, h, size_t(n), scales, include_largest);
    } else {
      IuwtDecompose(scratch, scratch, w, h, size_t(n), scales, include_largest);
    }
  }
  // Recompose (iuwt_decomposition.h:121-146)
  void Recompose(Plane& out, bool include_largest) const {
    out.assign(w * h, 0.0f);
    IuwtRecompose(scales, w, h, size_t(n), include_largest, out.data());
  }
  // ApplyMask (:284-291)
  void ApplyMask(const Mask& mask) {
    for (int s = 0; s != n; ++s)
      for (size_t i = 0; i != w * h; ++i)
        if (!mask.m[s][i]) scales[s][i] = 0.0f;
    scales[n].assign(w * h, 0.0f);
  }
  // CreateTrimmed (:58-68): the largest scale becomes a zero image of the
  // untrimmed size
  Iuwt Trimmed(int new_n, size_t x1, size_t y1, size_t x2, size_t y2) const {
    Iuwt out(new_n, x2 - x1, y2 - y1);
    for (int s = 0; s != new_n; ++s) {
      out.scales[s].assign((x2 - x1) * (y2 - y1), 0.0f);
      for (size_t y = y1; y != y2; ++y)
        for (size_t x = x1; x != x2; ++x)
          out.scales[s][(y - y1) * (x2 - x1) + (x - x1)] = scales[s][y * w + x];
    }
    out.scales.back().assign(w * h, 0.0f);
    return out;
  }
  float& At(int s, size_t i) { return scales[s][i]; }
  float At(int s, size_t i) const { return scales[s][i]; }
};

struct C3 {
  size_t x, y;
  int scale;
};
struct C2 {
  size_t x, y;
};

// image_analysis.cc:9-19
bool ExceedsThreshold(float val, float threshold) {
  if (threshold >= 0.0) return val > threshold;
  return val < threshold || val > -threshold;
}
bool ExceedsThresholdAbs(float val, float threshold) {
  return std::fabs(val) > threshold;
}

// Floodfill / MaskedFloodfill (image_analysis.cc:81-225)
void Floodfill(const Iuwt& iuwt, Mask& mask, const std::vector<float>& thr,
               size_t min_scale, size_t end_scale, C3 comp, float clean_border,
               const bool* prior, size_t& area) {
  const size_t width = iuwt.w, height = iuwt.h;
  const size_t xb = size_t(clean_border * width), yb = size_t(clean_border * height);
  const size_t min_x = xb, max_x = width - xb, min_y = yb, max_y = height - yb;
  area = 0;
  end_scale = std::min<size_t>(end_scale, size_t(iuwt.n));
  std::stack<C3> todo;
  todo.push(comp);
  mask.m[comp.scale][comp.x + comp.y * width] = 1;
  auto ok = [&](int s, size_t idx) {
    return ExceedsThreshold(iuwt.At(s, idx), thr[s]) && !mask.m[s][idx] &&
           (prior == nullptr || prior[idx]);
  };
  while (!todo.empty()) {
    const C3 c = todo.top();
    ++area;
    todo.pop();
    const size_t idx = c.x + c.y * width;
    if (c.x > min_x && ok(c.scale, idx - 1)) {
      mask.m[c.scale][idx - 1] = 1;
      todo.push({c.x - 1, c.y, c.scale});
    }
    if (c.x < max_x - 1 && ok(c.scale, idx + 1)) {
      mask.m[c.scale][idx + 1] = 1;
      todo.push({c.x + 1, c.y, c.scale});
    }
    if (c.y > min_y && ok(c.scale, idx - width)) {
      mask.m[c.scale][idx - width] = 1;
      todo.push({c.x, c.y - 1, c.scale});
    }
    if (c.y < max_y - 1 && ok(c.scale, idx + width)) {
      mask.m[c.scale][idx + width] = 1;
      todo.push({c.x, c.y + 1, c.scale});
    }
    if (c.scale > int(min_scale) && ok(c.scale - 1, idx)) {
      mask.m[c.scale - 1][idx] = 1;
      todo.push({c.x, c.y, c.scale - 1});
    }
    if (c.scale < int(end_scale) - 1 && ok(c.scale + 1, idx)) {
      mask.m[c.scale + 1][idx] = 1;
      todo.push({c.x, c.y, c.scale + 1});
    }
  }
}

// SelectStructures (image_analysis.cc:227-259)
void SelectStructures(const Iuwt& iuwt, Mask& mask, const std::vector<float>& thr,
                      size_t min_scale, size_t end_scale, float clean_border,
                      const bool* prior, size_t& area) {
  const size_t width = iuwt.w, height = iuwt.h;
  const size_t xb = size_t(clean_border * width), yb = size_t(clean_border * height);
  area = 0;
  for (size_t s = min_scale; s != end_scale; ++s)
    for (size_t y = yb; y != height - yb; ++y)
      for (size_t x = xb; x != width - xb; ++x) {
        const size_t idx = x + y * width;
        const bool in_prior = prior == nullptr || prior[idx];
        if (ExceedsThreshold(iuwt.At(int(s), idx), thr[s]) && !mask.m[s][idx] &&
            in_prior) {
          size_t sub = 0;
          Floodfill(iuwt, mask, thr, min_scale, end_scale, {x, y, int(s)},
                    clean_border, prior, sub);
          area += sub;
        }
      }
}

// FloodFill2D, area-collecting form (image_analysis.cc:292-333)
void FloodFill2D(const float* image, std::vector<char>& mask, float threshold,
                 C2 comp, size_t width, size_t height, std::vector<C2>& area) {
  area.clear();
  std::stack<C2> todo;
  todo.push(comp);
  mask[comp.x + comp.y * width] = 1;
  while (!todo.empty()) {
    const C2 c = todo.top();
    area.push_back(c);
    todo.pop();
    const size_t idx = c.x + c.y * width;
    if (c.x > 0 && ExceedsThresholdAbs(image[idx - 1], threshold) && !mask[idx - 1]) {
      mask[idx - 1] = 1;
      todo.push({c.x - 1, c.y});
    }
    if (c.x < width - 1 && ExceedsThresholdAbs(image[idx + 1], threshold) &&
        !mask[idx + 1]) {
      mask[idx + 1] = 1;
      todo.push({c.x + 1, c.y});
    }
    if (c.y > 0 && ExceedsThresholdAbs(image[idx - width], threshold) &&
        !mask[idx - width]) {
      mask[idx - width] = 1;
      todo.push({c.x, c.y - 1});
    }
    if (c.y < height - 1 && ExceedsThresholdAbs(image[idx + width], threshold) &&
        !mask[idx + width]) {
      mask[idx + width] = 1;
      todo.push({c.x, c.y + 1});
    }
  }
}

// aocommon::Image::RMS (not in /root/reference; double sum assumed)
float Rms(const Plane& p) {
  double sum = 0.0;
  for (float v : p) sum += double(v) * double(v);
  return float(std::sqrt(sum / double(p.size())));
}

// schaapcommon::math::PrepareConvolutionKernel + Convolve at the image size
Plane PsfKernel(const float* psf, size_t w, size_t h) {
  Plane k(w * h);
  PrepareConvolutionKernel(k.data(), psf, w, h);
  return k;
}
void Convolve(Plane& image, const Plane& kernel, size_t w, size_t h) {
  ConvolveCircular(image.data(), kernel.data(), w, h);
}

// aocommon Image::AddWithFactor (contracted: fma(other, factor, this))
void AddWithFactor(Plane& dst, const Plane& src, float factor) {
  for (size_t i = 0; i != dst.size(); ++i) dst[i] = std::fma(src[i], factor, dst[i]);
}

class Algorithm {
 public:
  Algorithm(size_t w, size_t h, const IuwtAlgoSettings& s)
      : width_(w), height_(h), s_(s) {}

  float PerformMajorIteration(size_t& iter_counter, size_t n_iter, ImageSet& model_set,
                              ImageSet& dirty_set, const std::vector<const float*>& psfs,
                              bool& reached, std::vector<IuwtStep>* steps);

 private:
  struct ScaleResponse {
    float rms = 0.0f, peak_response = 0.0f, peak_response_to_next_scale = 0.0f;
  };
  struct Val {
    size_t x = 0, y = 0;
    int scale = 0;
    float val = 0.0f;
  };

  float CentralPeak(const Plane& d) const { return d[width_ / 2 + (height_ / 2) * width_]; }

  // :42-102 (the fields the algorithm reads)
  void MeasureRmsPerScale(const Plane& psf, size_t end_scale) {
    Iuwt iuwt(int(end_scale), width_, height_);
    Plane scratch(width_ * height_);
    iuwt.Decompose(psf.data(), scratch.data(), false);
    psf_response_.assign(end_scale, ScaleResponse());
    for (size_t s = 0; s != end_scale; ++s) {
      psf_response_[s].rms = Rms(iuwt.scales[s]);
      psf_response_[s].peak_response = CentralPeak(iuwt.scales[s]);
    }
    iuwt.Decompose(iuwt.scales[1].data(), scratch.data(), false);
    for (size_t s = 0; s != end_scale; ++s)
      psf_response_[s].peak_response_to_next_scale = CentralPeak(iuwt.scales[s]);
  }

  // :104-110
  float Mad(const Plane& d) const {
    Plane v(d.size());
    for (size_t i = 0; i != d.size(); ++i) v[i] = std::fabs(d[i]);
    const size_t mid = d.size() / 2;
    std::nth_element(v.begin(), v.begin() + mid, v.end());
    return float(v[mid] / 0.674559);
  }

  // :112-167 (full-image width; the data may be a trimmed plane only when
  // width_ matches it, as in the reference's calls)
  float GetMaxAbs(const Plane& data, size_t& x, size_t& y, size_t width) const {
    const size_t height = data.size() / width;
    const size_t xb = size_t(s_.clean_border * width), yb = size_t(s_.clean_border * height);
    x = width;
    y = height;
    float max_val = std::numeric_limits<float>::lowest();
    for (size_t yi = yb; yi != height - yb; ++yi)
      for (size_t xi = xb; xi != width - xb; ++xi) {
        if (s_.mask && !s_.mask[yi * width + xi]) continue;
        const float v = s_.allow_negative ? std::fabs(data[yi * width + xi])
                                          : data[yi * width + xi];
        if (v > max_val) {
          max_val = v;
          x = xi;
          y = yi;
        }
      }
    return max_val;
  }

  // :169-174 (contracted float sum)
  static float Dot(const Plane& a, const Plane& b) {
    float sum = 0.0f;
    for (size_t i = 0; i != a.size(); ++i) sum = std::fma(a[i], b[i], sum);
    return sum;
  }

  // :180-214
  static void BoundingBox(size_t& x1, size_t& y1, size_t& x2, size_t& y2,
                          const Plane& image, size_t width, size_t height) {
    const float mp = *std::max_element(image.begin(), image.end());
    const float mn = *std::min_element(image.begin(), image.end());
    const float m = std::max(mp, -mn);
    x1 = width;
    x2 = 0;
    y1 = height;
    y2 = 0;
    for (size_t y = 0; y != height; ++y) {
      const float* p = image.data() + y * width;
      for (size_t x = 0; x != x1; ++x)
        if (std::fabs(p[x]) > m * 0.01) {
          x1 = x;
          break;
        }
      for (size_t x = width - 1; x != x2; --x)
        if (std::fabs(p[x]) > m * 0.01) {
          x2 = x;
          break;
        }
    }
    x2++;
    for (size_t y = 0; y != height; ++y) {
      const float* p = image.data() + y * width;
      for (size_t x = 0; x != width; ++x)
        if (std::fabs(p[x]) > m * 0.01) {
          if (y1 > y) y1 = y;
          if (y2 < y) y2 = y + 1;
        }
    }
  }

  // :216-260
  static void AdjustBox(size_t& x1, size_t& y1, size_t& x2, size_t& y2, size_t width,
                        size_t height, int end_scale) {
    const int min_box = std::max<int>(128, int((size_t(1) << (end_scale + 3)) * 3 / 2));
    const int bw = int(x2 - x1), bh = int(y2 - y1);
    int nx1 = int(x1 - 0.5 * bw), nx2 = int(x2 + 0.5 * bw);
    int ny1 = int(y1 - 0.5 * bh), ny2 = int(y2 + 0.5 * bh);
    if (nx2 - nx1 < min_box) {
      const int mid = int(0.5 * (int(x1) + int(x2)));
      nx1 = mid - min_box / 2;
      nx2 = mid + min_box / 2;
    }
    if (ny2 - ny1 < min_box) {
      const int mid = int(0.5 * (int(y1) + int(y2)));
      ny1 = mid - min_box / 2;
      ny2 = mid + min_box / 2;
    }
    x1 = nx1 >= 0 ? size_t(nx1) : 0;
    x2 = nx2 < int(width) ? size_t(nx2) : width;
    y1 = ny1 >= 0 ? size_t(ny1) : 0;
    y2 = ny2 < int(height) ? size_t(ny2) : height;
    while ((x2 - x1) % 8 != 0) x2--;
    while ((y2 - y1) % 8 != 0) y2--;
  }

  // :262-274
  static Plane Trim(const float* src, size_t old_w, size_t x1, size_t y1, size_t x2,
                    size_t y2) {
    Plane out((x2 - x1) * (y2 - y1));
    for (size_t y = y1; y != y2; ++y)
      for (size_t x = x1; x != x2; ++x) out[(y - y1) * (x2 - x1) + (x - x1)] = src[y * old_w + x];
    return out;
  }
  // TrimPsf (.h:109-115)
  static Plane TrimPsf(const Plane& psf, size_t old_w, size_t old_h, size_t nw, size_t nh) {
    return Trim(psf.data(), old_w, (old_w - nw) / 2, (old_h - nh) / 2, (old_w + nw) / 2,
                (old_h + nh) / 2);
  }
  // :276-306
  static Plane Untrim(const Plane& small, size_t width, size_t height, size_t x1,
                      size_t y1, size_t x2, size_t y2) {
    Plane out(width * height, 0.0f);
    for (size_t y = y1; y != y2; ++y)
      for (size_t x = x1; x != x2; ++x)
        out[y * width + x] = small[(y - y1) * (x2 - x1) + (x - x1)];
    return out;
  }

  // :308-321 (contracted float sums)
  static float Snr(const Iuwt& noisy, const Iuwt& model) {
    float m_sum = 0.0f, n_sum = 0.0f;
    for (int s = 0; s != noisy.n; ++s) {
      const Plane& n = noisy.scales[s];
      const Plane& m = model.scales[s];
      for (size_t i = 0; i != n.size(); ++i) {
        m_sum = std::fma(m[i], m[i], m_sum);
        const float d = m[i] - n[i];
        n_sum = std::fma(d, d, n_sum);
      }
    }
    return m_sum / n_sum;
  }

  // :323-412
  bool RunConjugateGradient(Iuwt& iuwt, const Mask& mask, Plane& masked_dirty,
                            Plane& structure_model, Plane& scratch, const Plane& psf_kernel,
                            size_t width, size_t height) {
    Plane gradient = masked_dirty;
    float model_snr = 0.0f;
    const Iuwt initial(iuwt);
    for (size_t it = 0; it != 20; ++it) {
      scratch = gradient;
      Convolve(scratch, psf_kernel, width, height);
      iuwt.Decompose(scratch.data(), scratch.data(), false);
      iuwt.ApplyMask(mask);
      iuwt.Recompose(scratch, false);
      const float g_dot_s = Dot(gradient, scratch);
      if (g_dot_s == 0.0f) return false;
      const float step = Dot(masked_dirty, masked_dirty) / g_dot_s;
      AddWithFactor(structure_model, gradient, step);
      const float den = Dot(masked_dirty, masked_dirty);
      if (den == 0.0f) return false;
      AddWithFactor(masked_dirty, scratch, -step);
      const float grad_step = Dot(masked_dirty, masked_dirty) / den;
      scratch = gradient;
      gradient = masked_dirty;
      AddWithFactor(gradient, scratch, grad_step);
      scratch = structure_model;
      Convolve(scratch, psf_kernel, width, height);
      iuwt.Decompose(scratch.data(), scratch.data(), false);
      iuwt.ApplyMask(mask);
      const float previous = model_snr;
      model_snr = Snr(iuwt, initial);
      if (model_snr > 100 && it > 2) return true;
      if (model_snr < previous && it > 5 && model_snr > 3) return true;
    }
    if (model_snr <= 3.0f) {
      structure_model.assign(width * height, 0.0f);
      return false;
    }
    return true;
  }

  bool FindAndDeconvolveStructure(Iuwt& iuwt, Plane& dirty, const Plane& psf,
                                  const Plane& psf_kernel,
                                  const std::vector<const float*>& psfs, Plane& scratch,
                                  std::vector<Plane>& structure_model, size_t end_scale,
                                  size_t min_scale, std::vector<Val>& max_components,
                                  IuwtStep& step);
  bool FillAndDeconvolveStructure(Iuwt& iuwt, Plane& dirty,
                                  std::vector<Plane>& structure_model_full,
                                  Plane& scratch, const Plane& psf, const Plane& psf_kernel,
                                  const std::vector<const float*>& psfs, size_t end_scale,
                                  size_t min_scale, size_t width, size_t height,
                                  const std::vector<float>& thresholds, const C3& max_comp,
                                  bool allow_trimming, const bool* prior_mask,
                                  IuwtStep& step);
  void PerformSubImageFitAll(Iuwt& iuwt, const Mask& mask, const Plane& structure_model,
                             Plane& scratch_a, Plane& scratch_b, const C3& max_comp,
                             std::vector<Plane>& fitted_model, const Plane& psf,
                             const std::vector<const float*>& psfs, const Plane& dirty);
  void PerformSubImageFitSingle(Iuwt& iuwt, const Mask& mask, const Plane& structure_model,
                                Plane& scratch_b, const C3& max_comp, const Plane& psf,
                                Plane& sub_dirty, float* fitted_sub_model,
                                std::vector<float>& correction_factor);
  float ComponentFitBoxed(Iuwt& iuwt, const Mask& mask, const std::vector<C2>& area,
                          Plane& model, Plane& masked_dirty, const Plane& psf,
                          const Plane& psf_kernel, size_t x1, size_t y1, size_t x2,
                          size_t y2);
  float ComponentFit(Iuwt& iuwt, const Mask& mask, const std::vector<C2>& area,
                     Plane& model, Plane& masked_dirty, const Plane& psf_kernel,
                     size_t x_offset, size_t y_offset);

  size_t width_, height_;
  size_t box_x1_ = 0, box_x2_ = 0, box_y1_ = 0, box_y2_ = 0;
  IuwtAlgoSettings s_;
  std::vector<float> rmses_;
  std::vector<ScaleResponse> psf_response_;
  ImageSet* dirty_set_ = nullptr;
};

// :414-497
bool Algorithm::FindAndDeconvolveStructure(Iuwt& iuwt, Plane& dirty, const Plane& psf,
                                           const Plane& psf_kernel,
                                           const std::vector<const float*>& psfs,
                                           Plane& scratch,
                                           std::vector<Plane>& structure_model,
                                           size_t end_scale, size_t min_scale,
                                           std::vector<Val>& max_components,
                                           IuwtStep& step) {
  iuwt.Decompose(dirty.data(), scratch.data(), false);
  std::vector<float> thresholds(end_scale);
  rmses_.resize(end_scale);
  for (size_t s = 0; s != end_scale; ++s) {
    const float r = Mad(iuwt.scales[s]);
    rmses_[s] = r;
    // threshold_sigma_level_ * 4.0 / 5.0 is a double expression
    thresholds[s] = float(double(r) * (double(s_.threshold_sigma_level) * 4.0 / 5.0));
  }
  scratch = dirty;
  max_components.assign(end_scale, Val());
  for (size_t s = 0; s != end_scale; ++s) {
    size_t x, y;
    const float v = GetMaxAbs(iuwt.scales[s], x, y, width_);
    max_components[s] = {x, y, int(s), v};
  }
  float max_val = -1.0f;
  size_t max_x = 0, max_y = 0;
  int max_scale = -1;
  for (size_t s = 0; s != end_scale; ++s) {
    const Val& v = max_components[s];
    const float abs_coef = v.val / psf_response_[s].rms;
    if (s >= min_scale && abs_coef > max_val && v.val > rmses_[s] * s_.threshold_sigma_level &&
        v.val > rmses_[s] / rmses_[0] * s_.absolute_threshold) {
      max_x = v.x;
      max_y = v.y;
      max_scale = int(s);
      if (s == 0) {
        const float lowest = std::min(psf_response_[0].rms, psf_response_[1].rms);
        max_val = v.val / lowest * psf_response_[1].peak_response /
                  psf_response_[0].peak_response_to_next_scale;
      } else {
        max_val = abs_coef;
      }
    }
  }
  step.scale = max_scale;
  if (max_scale == -1) return false;
  step.x = uint32_t(max_x);
  step.y = uint32_t(max_y);
  max_val = iuwt.At(max_scale, max_x + max_y * width_);
  if (std::fabs(max_val) < thresholds[max_scale]) return false;
  const float scale_max_abs = std::fabs(max_val);
  for (size_t s = 0; s != end_scale; ++s) {
    if (thresholds[s] < s_.tolerance * scale_max_abs) thresholds[s] = s_.tolerance * scale_max_abs;
    if (max_val < 0.0f) thresholds[s] = -thresholds[s];
  }
  return FillAndDeconvolveStructure(iuwt, dirty, structure_model, scratch, psf, psf_kernel,
                                    psfs, end_scale, min_scale, width_, height_, thresholds,
                                    {max_x, max_y, max_scale}, true, s_.mask, step);
}

// :499-606
bool Algorithm::FillAndDeconvolveStructure(
    Iuwt& iuwt, Plane& dirty, std::vector<Plane>& structure_model_full, Plane& scratch,
    const Plane& psf, const Plane& psf_kernel, const std::vector<const float*>& psfs,
    size_t end_scale, size_t min_scale, size_t width, size_t height,
    const std::vector<float>& thresholds, const C3& max_comp, bool allow_trimming,
    const bool* prior_mask, IuwtStep& step) {
  Mask mask(end_scale, width, height);
  size_t area = 0;
  SelectStructures(iuwt, mask, thresholds, min_scale, end_scale, s_.clean_border,
                   prior_mask, area);
  if (allow_trimming) step.area = area;
  iuwt.ApplyMask(mask);
  iuwt.Recompose(scratch, false);
  size_t x1, y1, x2, y2;
  BoundingBox(x1, y1, x2, y2, scratch, width, height);
  AdjustBox(x1, y1, x2, y2, width, height, max_comp.scale + 1);
  if (allow_trimming && ((x2 - x1) < width || (y2 - y1) < height)) {
    box_x1_ = x1;
    box_x2_ = x2;
    box_y1_ = y1;
    box_y2_ = y2;
    const size_t nw = x2 - x1, nh = y2 - y1;
    step.trimmed_width = uint32_t(nw);
    dirty = Trim(dirty.data(), width, x1, y1, x2, y2);
    const Plane small_psf = TrimPsf(psf, width, height, nw, nh);
    const Plane small_kernel = PsfKernel(small_psf.data(), nw, nh);
    scratch.assign(nw * nh, 0.0f);
    const int fit_end = std::max(IuwtEndScale(std::min(nw, nh)), max_comp.scale + 1);
    if (fit_end < int(end_scale)) end_scale = size_t(fit_end);
    Iuwt trimmed = iuwt.Trimmed(int(end_scale), x1, y1, x2, y2);
    std::vector<Plane> trimmed_model;
    for (const Plane& p : structure_model_full)
      trimmed_model.push_back(Trim(p.data(), width, x1, y1, x2, y2));
    std::vector<char> trimmed_prior;
    const bool* trimmed_prior_ptr = nullptr;
    if (prior_mask) {
      trimmed_prior.resize(nw * nh);
      for (size_t y = 0; y != nh; ++y)
        for (size_t x = 0; x != nw; ++x)
          trimmed_prior[y * nw + x] = prior_mask[(y + y1) * width + x + x1];
      trimmed_prior_ptr = reinterpret_cast<const bool*>(trimmed_prior.data());
    }
    const bool result = FillAndDeconvolveStructure(
        trimmed, dirty, trimmed_model, scratch, small_psf, small_kernel, psfs, end_scale,
        min_scale, nw, nh, thresholds, {max_comp.x - x1, max_comp.y - y1, max_comp.scale},
        false, trimmed_prior_ptr, step);
    for (size_t i = 0; i != structure_model_full.size(); ++i)
      structure_model_full[i] = Untrim(trimmed_model[i], width, height, x1, y1, x2, y2);
    dirty.assign(width * height, 0.0f);
    scratch.assign(width * height, 0.0f);
    box_x1_ = 0;
    box_x2_ = width;
    box_y1_ = 0;
    box_y2_ = height;
    return result;
  }
  iuwt.Decompose(dirty.data(), scratch.data(), false);
  iuwt.ApplyMask(mask);
  iuwt.Recompose(scratch, false);
  Plane masked_dirty = scratch;
  Plane structure_model(width * height, 0.0f);
  if (!RunConjugateGradient(iuwt, mask, masked_dirty, structure_model, scratch, psf_kernel,
                            width, height))
    return false;
  const float rms_before = Rms(dirty);
  scratch = structure_model;
  Convolve(scratch, psf_kernel, width, height);
  masked_dirty = dirty;
  AddWithFactor(masked_dirty, scratch, -s_.minor_loop_gain);
  const float rms_after = Rms(masked_dirty);
  if (rms_after > rms_before) return false;
  PerformSubImageFitAll(iuwt, mask, structure_model, scratch, masked_dirty, max_comp,
                        structure_model_full, psf, psfs, dirty);
  return true;
}

// :608-656
void Algorithm::PerformSubImageFitAll(Iuwt& iuwt, const Mask& mask,
                                      const Plane& structure_model, Plane& scratch_a,
                                      Plane& scratch_b, const C3& max_comp,
                                      std::vector<Plane>& fitted_model, const Plane& psf,
                                      const std::vector<const float*>& psfs,
                                      const Plane& dirty) {
  const size_t width = iuwt.w, height = iuwt.h;
  if (dirty_set_->Size() == 1) {
    fitted_model[0] = structure_model;
    return;
  }
  std::vector<float> factors;
  scratch_a = dirty;
  PerformSubImageFitSingle(iuwt, mask, structure_model, scratch_b, max_comp, psf, scratch_a,
                           nullptr, factors);
  for (Plane& p : fitted_model) p.assign(width * height, 0.0f);
  for (size_t i = 0; i != dirty_set_->Size(); ++i) {
    const float* sub_psf = psfs[dirty_set_->PsfIndex(i)];
    scratch_a = Trim(dirty_set_->images[i], width_, box_x1_, box_y1_, box_x2_, box_y2_);
    Plane small_sub_psf;
    if (width_ != width || height_ != height)
      small_sub_psf = TrimPsf(Plane(sub_psf, sub_psf + width_ * height_), width_, height_,
                              width, height);
    else
      small_sub_psf.assign(sub_psf, sub_psf + width_ * height_);
    PerformSubImageFitSingle(iuwt, mask, structure_model, scratch_b, max_comp, small_sub_psf,
                             scratch_a, fitted_model[i].data(), factors);
  }
}

// :658-741
void Algorithm::PerformSubImageFitSingle(Iuwt& iuwt, const Mask& mask,
                                         const Plane& structure_model, Plane& scratch_b,
                                         const C3& max_comp, const Plane& psf,
                                         Plane& sub_dirty, float* fitted_sub_model,
                                         std::vector<float>& correction_factor) {
  const size_t width = iuwt.w, height = iuwt.h;
  const Plane psf_kernel = PsfKernel(psf.data(), width, height);
  Plane& masked_dirty = scratch_b;
  iuwt.Decompose(sub_dirty.data(), sub_dirty.data(), false);
  iuwt.ApplyMask(mask);
  iuwt.Recompose(masked_dirty, false);
  std::vector<char> mask2d(structure_model.size(), 0);
  const float peak = std::fabs(structure_model[max_comp.y * width + max_comp.x]);
  size_t comp_index = 0;
  for (size_t y = 0; y != height; ++y)
    for (size_t x = 0; x != width; ++x) {
      if (mask2d[y * width + x] || !(std::fabs(structure_model[y * width + x]) > peak * 1e-4))
        continue;
      std::vector<C2> area;
      FloodFill2D(structure_model.data(), mask2d, float(peak * 1e-4), {x, y}, width, height,
                  area);
      sub_dirty.assign(width * height, 0.0f);
      size_t bx1 = width, bx2 = 0, by1 = height, by2 = 0;
      for (const C2& a : area) {
        const size_t idx = a.x + a.y * width;
        bx1 = std::min(a.x, bx1);
        bx2 = std::max(a.x, bx2);
        by1 = std::min(a.y, by1);
        by2 = std::max(a.y, by2);
        sub_dirty[idx] = structure_model[idx];
      }
      AdjustBox(bx1, by1, bx2, by2, width, height, iuwt.n);
      const float factor = ComponentFitBoxed(iuwt, mask, area, sub_dirty, masked_dirty, psf,
                                             psf_kernel, bx1, by1, bx2, by2);
      if (fitted_sub_model) {
        const float integrated = correction_factor[comp_index];
        if (std::isfinite(factor) && std::isfinite(integrated) && integrated != 0.0f)
          for (const C2& a : area) {
            const size_t idx = a.x + a.y * width;
            fitted_sub_model[idx] += structure_model[idx] * factor / integrated;
          }
        ++comp_index;
      } else {
        correction_factor.push_back(factor);
      }
    }
}

// :743-771
float Algorithm::ComponentFitBoxed(Iuwt& iuwt, const Mask& mask, const std::vector<C2>& area,
                                   Plane& model, Plane& masked_dirty, const Plane& psf,
                                   const Plane& psf_kernel, size_t x1, size_t y1, size_t x2,
                                   size_t y2) {
  const size_t width = iuwt.w, height = iuwt.h;
  if (x1 > 0 || y1 > 0 || x2 < width || y2 < height) {
    const size_t nw = x2 - x1, nh = y2 - y1;
    Iuwt small(iuwt.n, nw, nh);
    const Mask small_mask = mask.Trimmed(x1, y1, x2, y2);
    Plane small_model = Trim(model.data(), width, x1, y1, x2, y2);
    const Plane small_psf = TrimPsf(psf, width, height, nw, nh);
    const Plane small_kernel = PsfKernel(small_psf.data(), nw, nh);
    Plane small_dirty = Trim(masked_dirty.data(), width, x1, y1, x2, y2);
    return ComponentFit(small, small_mask, area, small_model, small_dirty, small_kernel, x1, y1);
  }
  return ComponentFit(iuwt, mask, area, model, masked_dirty, psf_kernel, 0, 0);
}

// :773-798
float Algorithm::ComponentFit(Iuwt& iuwt, const Mask& mask, const std::vector<C2>& area,
                              Plane& model, Plane& masked_dirty, const Plane& psf_kernel,
                              size_t x_offset, size_t y_offset) {
  const size_t width = iuwt.w, height = iuwt.h;
  Convolve(model, psf_kernel, width, height);
  iuwt.Decompose(model.data(), model.data(), false);
  iuwt.ApplyMask(mask);
  iuwt.Recompose(model, false);
  float model_sum = 0.0f, dirty_sum = 0.0f;
  for (const C2& a : area) {
    const size_t idx = (a.x - x_offset) + (a.y - y_offset) * width;
    model_sum += model[idx];
    dirty_sum += masked_dirty[idx];
  }
  if (model_sum == 0.0f || !std::isfinite(dirty_sum) || !std::isfinite(model_sum)) return 0.0f;
  return dirty_sum / model_sum;
}

// :800-918
float Algorithm::PerformMajorIteration(size_t& iter_counter, size_t n_iter,
                                       ImageSet& model_set, ImageSet& dirty_set,
                                       const std::vector<const float*>& psfs, bool& reached,
                                       std::vector<IuwtStep>* steps) {
  reached = false;
  if (iter_counter == n_iter) return 0.0f;
  dirty_set_ = &dirty_set;
  box_x1_ = 0;
  box_x2_ = width_;
  box_y1_ = 0;
  box_y2_ = height_;
  const size_t n = width_ * height_;
  Plane dirty(n), psf(n);
  GetLinearIntegrated(dirty_set, dirty.data());
  GetIntegratedPsf(*dirty_set.desc, psfs, n, psf.data());
  const int max_scale = IuwtEndScale(std::min(width_, height_));
  int end_scale = 2;
  Plane psf_kernel = PsfKernel(psf.data(), width_, height_);
  MeasureRmsPerScale(psf, size_t(max_scale));
  std::vector<Plane> structure_model(model_set.Size(), Plane(n, 0.0f));
  auto iuwt = std::make_unique<Iuwt>(end_scale, width_, height_);
  float max_value = 0.0f;
  size_t min_scale = 0;
  bool do_continue = true;
  std::vector<Val> initial;
  do {
    const Plane dirty_before = dirty;
    psf_kernel = PsfKernel(psf.data(), width_, height_);
    std::vector<Val> max_components;
    Plane scratch(n);
    IuwtStep step{};
    step.scale = -1;
    step.end_scale = end_scale;
    step.min_scale = int(min_scale);
    const bool ok = FindAndDeconvolveStructure(*iuwt, dirty, psf, psf_kernel, psfs, scratch,
                                               structure_model, size_t(end_scale), min_scale,
                                               max_components, step);
    step.succeeded = ok ? 1 : 0;
    if (ok) {
      for (Plane& p : structure_model)
        for (float& v : p) v *= s_.minor_loop_gain;
      for (size_t i = 0; i != model_set.Size(); ++i)
        for (size_t k = 0; k != n; ++k) model_set.images[i][k] += structure_model[i][k];
      for (size_t i = 0; i != dirty_set.Size(); ++i) {
        scratch = structure_model[i];
        const Plane kernel = PsfKernel(psfs[dirty_set.PsfIndex(i)], width_, height_);
        Convolve(scratch, kernel, width_, height_);
        for (size_t k = 0; k != n; ++k) dirty_set.images[i][k] -= scratch[k];
      }
      GetLinearIntegrated(dirty_set, dirty.data());
      while (max_components.size() > initial.size())
        initial.push_back(max_components[initial.size()]);
      max_value = 0.0f;
      for (size_t c = 0; c != initial.size(); ++c) {
        max_value = std::max(max_value, max_components[c].val);
        if (std::fabs(max_components[c].val) <
            std::fabs(initial[c].val) * (1.0 - s_.major_loop_gain))
          reached = true;
      }
      step.max_value = max_value;
      if (steps) steps->push_back(step);
      if (reached) break;  // before ++iter_counter, as the reference
    } else {
      if (int(min_scale) + 1 < end_scale) {
        ++min_scale;
      } else {
        min_scale = 0;
        if (end_scale != max_scale) {
          ++end_scale;
          iuwt = std::make_unique<Iuwt>(end_scale, width_, height_);
        } else {
          do_continue = false;
        }
      }
      dirty = dirty_before;
      if (steps) steps->push_back(step);
    }
    ++iter_counter;
  } while (iter_counter != n_iter && do_continue);
  return max_value;
}

}  // namespace

int IuwtEndScale(size_t max_image_dimension) {
  return std::max(int(std::log2(double(max_image_dimension))) - 3, 2);
}

float IuwtExecute(const IuwtAlgoSettings& s, size_t& iteration_number,
                  size_t max_iterations, ImageSet& dirty, ImageSet& model,
                  const std::vector<const float*>& psfs,
                  bool& another_iteration_required, std::vector<IuwtStep>* steps) {
  Algorithm alg(dirty.width, dirty.height, s);
  const float v = alg.PerformMajorIteration(iteration_number, max_iterations, model, dirty,
                                            psfs, another_iteration_required, steps);
  if (iteration_number >= max_iterations) another_iteration_required = false;
  return v;
}

}  // namespace oracle
