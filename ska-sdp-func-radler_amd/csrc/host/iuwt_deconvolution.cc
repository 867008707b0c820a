// Line references are to the reference's
// cpp/algorithms/iuwt_deconvolution_algorithm.cc unless stated otherwise.
//
// Precision: the convolutions run in double (schaapcommon's FFTW float in the
// reference), dot products and SNR sums accumulate in double (a sequential
// float sum there), Image::RMS is sqrt(sum v^2 / n) with a double sum.
// Selection, masks, IUWT planes, maxima and medians are bit-exact given the
// same inputs.
#include "iuwt_deconvolution.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <stack>
#include <stdexcept>

#include "logger.h"

namespace radler::algorithms {

namespace {

using gpu::Buffer;
using gpu::Check;
using gpu::Session;

// A device float plane.
struct Plane {
  Plane() = default;
  Plane(Session& s, size_t w_, size_t h_) : w(w_), h(h_) {
    buf = std::make_shared<Buffer>(s, std::max<size_t>(1, w * h) * sizeof(float));
  }
  std::shared_ptr<Buffer> buf;
  size_t w = 0, h = 0;
  float* F() const { return buf->F(); }
  size_t N() const { return w * h; }
};

Plane Copy(Session& s, const Plane& p) {
  Plane out(s, p.w, p.h);
  s.D2D(out.F(), p.F(), p.N() * sizeof(float));
  return out;
}
void Assign(Session& s, Plane& dst, const Plane& src) {
  if (!dst.buf || dst.w != src.w || dst.h != src.h) dst = Plane(s, src.w, src.h);
  s.D2D(dst.F(), src.F(), src.N() * sizeof(float));
}
Plane Zeros(Session& s, size_t w, size_t h) {
  Plane p(s, w, h);
  s.Zero(p.F(), p.N() * sizeof(float));
  return p;
}

// :262-274 (Trim) / TrimPsf (.h:109-115) / :276-306 (Untrim)
Plane Trim(Session& s, const float* src, size_t old_w, size_t x1, size_t y1, size_t x2,
           size_t y2) {
  Plane out(s, x2 - x1, y2 - y1);
  Check(rdl_box(s.Handle(), out.F(), uint32_t(out.w), 0, 0, src, uint32_t(old_w),
                uint32_t(x1), uint32_t(y1), uint32_t(out.w), uint32_t(out.h), nullptr,
                RDL_BOX_COPY),
        "rdl_box");
  return out;
}
Plane TrimPsf(Session& s, const Plane& psf, size_t nw, size_t nh) {
  return Trim(s, psf.F(), psf.w, (psf.w - nw) / 2, (psf.h - nh) / 2, (psf.w + nw) / 2,
              (psf.h + nh) / 2);
}
Plane Untrim(Session& s, const Plane& small, size_t width, size_t height, size_t x1,
             size_t y1) {
  Plane out = Zeros(s, width, height);
  Check(rdl_box(s.Handle(), out.F(), uint32_t(width), uint32_t(x1), uint32_t(y1), small.F(),
                uint32_t(small.w), 0, 0, uint32_t(small.w), uint32_t(small.h), nullptr,
                RDL_BOX_COPY),
        "rdl_box");
  return out;
}

// schaapcommon::math::PrepareConvolutionKernel + Convolve at the image size,
// in double: the LDS engine (rows/columns kernels with float in/out) where
// the size allows, rocFFT double otherwise.
class Convolver {
 public:
  Convolver(Session& s, size_t w, size_t h) : s_(s), w_(w), h_(h), fft_(s.GetFft(w, h, true)) {}
  std::shared_ptr<Buffer> Kernel(const float* d_psf) {
    auto spec = std::make_shared<Buffer>(s_, fft_.SpectrumBytes());
    Plane k(s_, w_, h_);
    Check(rdl_prepare_psf_kernel(s_.Handle(), k.F(), uint32_t(w_), uint32_t(h_), d_psf,
                                 uint32_t(w_), uint32_t(h_)),
          "rdl_prepare_psf_kernel");
    if (fft_.UsesLds()) {
      fft_.Forward(k.F(), spec->Ptr());
    } else {
      EnsureDouble();
      Check(rdl_convert(s_.Handle(), k.F(), dbl_.Ptr(), w_ * h_, 1), "rdl_convert");
      fft_.Forward64(dbl_.D(), spec->Ptr());
    }
    return spec;
  }
  void Convolve(float* d_image, const Buffer& spectrum) {
    if (fft_.UsesLds()) {
      fft_.Convolve(d_image, spectrum.Ptr());
      return;
    }
    EnsureDouble();
    Check(rdl_convert(s_.Handle(), d_image, dbl_.Ptr(), w_ * h_, 1), "rdl_convert");
    fft_.Convolve64(dbl_.D(), spectrum.Ptr());
    Check(rdl_convert(s_.Handle(), dbl_.Ptr(), d_image, w_ * h_, 0), "rdl_convert");
  }

 private:
  void EnsureDouble() {
    if (dbl_.Bytes() < w_ * h_ * sizeof(double)) dbl_.Resize(s_, w_ * h_ * sizeof(double));
  }
  Session& s_;
  size_t w_, h_;
  gpu::Fft& fft_;
  Buffer dbl_;
};

// IuwtDecomposition (iuwt/iuwt_decomposition.h:37-351): n detail planes and
// the approximation plane (used as the transform's i1 buffer).
struct Iuwt {
  Iuwt(Session& s, int n_, size_t w_, size_t h_) : n(n_), w(w_), h(h_) {
    coeffs = std::make_shared<Buffer>(s, size_t(n + 1) * w * h * sizeof(float));
  }
  int n;
  size_t w, h;
  std::shared_ptr<Buffer> coeffs;
  float* Scale(int s) const { return coeffs->F() + size_t(s) * w * h; }
  // DecomposeMt (iuwt_decomposition.cc:9-54), include_largest = false
  void Decompose(Session& s, float* input, float* scratch) {
    Check(rdl_iuwt_decompose(s.Handle(), input, scratch, uint32_t(w), uint32_t(h),
                             uint32_t(n), coeffs->F(), 0),
          "rdl_iuwt_decompose");
  }
  // Recompose (iuwt_decomposition.h:121-146), include_largest = false
  void Recompose(Session& s, Plane& out) const {
    if (!out.buf || out.w != w || out.h != h) out = Plane(s, w, h);
    Check(rdl_iuwt_recompose(s.Handle(), coeffs->F(), uint32_t(w), uint32_t(h), uint32_t(n),
                             0, out.F()),
          "rdl_iuwt_recompose");
  }
  // ApplyMask (iuwt_decomposition.h:284-291): the approximation plane is
  // zeroed there too; nothing reads it with include_largest = false
  void ApplyMask(Session& s, const Buffer& mask) {
    Check(rdl_iuwt_apply_mask(s.Handle(), coeffs->F(), static_cast<const uint8_t*>(mask.Ptr()),
                              uint32_t(w), uint32_t(h), uint32_t(n)),
          "rdl_iuwt_apply_mask");
  }
  // CreateTrimmed (iuwt_decomposition.h:58-68)
  Iuwt Trimmed(Session& s, int new_n, size_t x1, size_t y1, size_t x2, size_t y2) const {
    Iuwt out(s, new_n, x2 - x1, y2 - y1);
    for (int k = 0; k != new_n; ++k)
      Check(rdl_box(s.Handle(), out.Scale(k), uint32_t(out.w), 0, 0, Scale(k), uint32_t(w),
                    uint32_t(x1), uint32_t(y1), uint32_t(out.w), uint32_t(out.h), nullptr,
                    RDL_BOX_COPY),
            "rdl_box");
    return out;
  }
  Iuwt Clone(Session& s) const {
    Iuwt out(s, n, w, h);
    s.D2D(out.Coeffs(), coeffs->F(), size_t(n) * w * h * sizeof(float));
    return out;
  }
  float* Coeffs() const { return coeffs->F(); }
};

// IuwtMask (iuwt/iuwt_mask.h): n planes of bytes.
struct Mask {
  Mask(Session& s, int n_, size_t w_, size_t h_) : n(n_), w(w_), h(h_) {
    bytes = std::make_shared<Buffer>(s, std::max<size_t>(1, size_t(n) * w * h));
  }
  int n;
  size_t w, h;
  std::shared_ptr<Buffer> bytes;
  uint8_t* B() const { return static_cast<uint8_t*>(bytes->Ptr()); }
};

struct C3 {
  size_t x, y;
  int scale;
};
struct C2 {
  size_t x, y;
};

class Algorithm {
 public:
  Algorithm(Session& s, size_t w, size_t h, const IuwtDeconvolution& a,
            const uint8_t* d_clean_mask)
      : s_(s),
        width_(w),
        height_(h),
        minor_loop_gain_(a.MinorLoopGain()),
        major_loop_gain_(a.MajorLoopGain()),
        clean_border_(a.CleanBorderRatio()),
        allow_negative_(a.AllowNegativeComponents()),
        mask_(a.CleanMask()),
        d_mask_(d_clean_mask),
        absolute_threshold_(a.Threshold()) {}

  float PerformMajorIteration(size_t& iter_counter, size_t n_iter, ImageSet& model_set,
                              ImageSet& dirty_set, const gpu::Planes& psfs, bool& reached,
                              std::vector<IuwtDeconvolution::Step>& steps);

 private:
  struct ScaleResponse {
    float rms = 0.0f, peak_response = 0.0f, peak_response_to_next_scale = 0.0f;
  };
  struct Val {
    size_t x = 0, y = 0;
    int scale = 0;
    float val = 0.0f;
  };
  using Step = IuwtDeconvolution::Step;

  Convolver& Conv(size_t w, size_t h) {
    auto key = std::make_pair(w, h);
    auto it = convolvers_.find(key);
    if (it == convolvers_.end())
      it = convolvers_.emplace(key, std::make_unique<Convolver>(s_, w, h)).first;
    return *it->second;
  }
  std::shared_ptr<Buffer> KernelOf(const Plane& psf) { return Conv(psf.w, psf.h).Kernel(psf.F()); }
  void Convolve(Plane& p, const Buffer& spec) { Conv(p.w, p.h).Convolve(p.F(), spec); }

  float CentralPeak(const float* d, size_t w, size_t h) {
    return s_.ReadFloat(d + w / 2 + (h / 2) * w);
  }
  float Rms(const Plane& p) {
    float v = 0.0f;
    Check(rdl_rms(s_.Handle(), p.F(), p.N(), &v), "rdl_rms");
    return v;
  }
  float Dot(const Plane& a, const Plane& b) {
    double d = 0.0;
    Check(rdl_dot(s_.Handle(), a.F(), b.F(), a.N(), &d), "rdl_dot");
    return float(d);
  }
  void AddWithFactor(Plane& dst, const Plane& src, float factor) {
    Check(rdl_axpy(s_.Handle(), dst.F(), src.F(), dst.N(), factor, 0), "rdl_axpy");
  }
  // :104-110
  float Mad(const float* d, size_t n) {
    float v = 0.0f;
    Check(rdl_select_kth(s_.Handle(), d, n, 1, 0.0f, n / 2, &v), "rdl_select_kth");
    return float(v / 0.674559);
  }
  // :112-167
  float GetMaxAbs(const float* data, size_t& x, size_t& y) {
    const size_t xb = size_t(clean_border_ * width_), yb = size_t(clean_border_ * height_);
    rdl_peak p{};
    Check(rdl_max_abs(s_.Handle(), data, uint32_t(width_), uint32_t(height_), uint32_t(xb),
                      uint32_t(yb), allow_negative_ ? 1 : 0, d_mask_, &p),
          "rdl_max_abs");
    x = p.x;
    y = p.y;
    return p.value;
  }
  // :180-214 (the per-row scans on the device, the reference's loop logic here)
  void BoundingBox(size_t& x1, size_t& y1, size_t& x2, size_t& y2, const Plane& img) {
    std::vector<int32_t> first(img.h), last(img.h);
    Check(rdl_bbox_rows(s_.Handle(), img.F(), uint32_t(img.w), uint32_t(img.h), first.data(),
                        last.data()),
          "rdl_bbox_rows");
    x1 = img.w;
    x2 = 0;
    y1 = img.h;
    y2 = 0;
    for (size_t y = 0; y != img.h; ++y) {
      if (first[y] >= 0 && size_t(first[y]) < x1) x1 = size_t(first[y]);
      if (last[y] >= 0 && size_t(last[y]) > x2) x2 = size_t(last[y]);
    }
    x2++;
    for (size_t y = 0; y != img.h; ++y)
      if (first[y] >= 0) {
        if (y1 > y) y1 = y;
        if (y2 < y) y2 = y + 1;
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

  // :42-102: the fields the algorithm reads (rms, peak responses)
  void MeasureRmsPerScale(const Plane& psf, int end_scale) {
    Iuwt iuwt(s_, end_scale, width_, height_);
    Plane scratch(s_, width_, height_);
    iuwt.Decompose(s_, psf.F(), scratch.F());
    psf_response_.assign(size_t(end_scale), ScaleResponse());
    Plane plane(s_, width_, height_);
    for (int k = 0; k != end_scale; ++k) {
      s_.D2D(plane.F(), iuwt.Scale(k), plane.N() * sizeof(float));
      psf_response_[k].rms = Rms(plane);
      psf_response_[k].peak_response = CentralPeak(iuwt.Scale(k), width_, height_);
    }
    // decompose the scale-1 coefficients (a copy: the reference reads the old
    // plane before the decomposition replaces it)
    s_.D2D(plane.F(), iuwt.Scale(1), plane.N() * sizeof(float));
    iuwt.Decompose(s_, plane.F(), scratch.F());
    for (int k = 0; k != end_scale; ++k)
      psf_response_[k].peak_response_to_next_scale = CentralPeak(iuwt.Scale(k), width_, height_);
  }

  // :323-412
  bool RunConjugateGradient(Iuwt& iuwt, const Mask& mask, Plane& masked_dirty,
                            Plane& structure_model, Plane& scratch, const Buffer& psf_kernel) {
    Plane gradient = Copy(s_, masked_dirty);
    float model_snr = 0.0f;
    const Iuwt initial = iuwt.Clone(s_);
    const size_t coeff_n = size_t(iuwt.n) * iuwt.w * iuwt.h;
    for (size_t it = 0; it != 20; ++it) {
      Assign(s_, scratch, gradient);
      Convolve(scratch, psf_kernel);
      iuwt.Decompose(s_, scratch.F(), scratch.F());
      iuwt.ApplyMask(s_, *mask.bytes);
      iuwt.Recompose(s_, scratch);
      const float g_dot_s = Dot(gradient, scratch);
      if (g_dot_s == 0.0f) return false;
      const float md_md = Dot(masked_dirty, masked_dirty);
      const float step = md_md / g_dot_s;
      AddWithFactor(structure_model, gradient, step);
      const float den = md_md;  // <masked_dirty, masked_dirty> again (:366)
      if (den == 0.0f) return false;
      AddWithFactor(masked_dirty, scratch, -step);
      const float grad_step = Dot(masked_dirty, masked_dirty) / den;
      std::swap(scratch, gradient);  // scratch = old gradient
      Assign(s_, gradient, masked_dirty);
      AddWithFactor(gradient, scratch, grad_step);
      Assign(s_, scratch, structure_model);
      Convolve(scratch, psf_kernel);
      iuwt.Decompose(s_, scratch.F(), scratch.F());
      iuwt.ApplyMask(s_, *mask.bytes);
      const float previous = model_snr;
      double m_sum = 0.0, n_sum = 0.0;
      Check(rdl_iuwt_snr_sums(s_.Handle(), iuwt.Coeffs(), initial.Coeffs(), coeff_n, &m_sum,
                              &n_sum),
            "rdl_iuwt_snr_sums");
      model_snr = float(m_sum) / float(n_sum);
      if (model_snr > 100 && it > 2) return true;
      if (model_snr < previous && it > 5 && model_snr > 3) return true;
    }
    if (model_snr <= 3.0f) {
      s_.Zero(structure_model.F(), structure_model.N() * sizeof(float));
      return false;
    }
    return true;
  }

  bool FindAndDeconvolveStructure(Iuwt& iuwt, Plane& dirty, const Plane& psf,
                                  const Buffer& psf_kernel, const gpu::Planes& psfs,
                                  Plane& scratch, std::vector<Plane>& structure_model,
                                  int end_scale, size_t min_scale,
                                  std::vector<Val>& max_components, Step& step);
  bool FillAndDeconvolveStructure(Iuwt& iuwt, Plane& dirty, std::vector<Plane>& model_full,
                                  Plane& scratch, const Plane& psf, const Buffer& psf_kernel,
                                  const gpu::Planes& psfs, int end_scale, size_t min_scale,
                                  size_t width, size_t height,
                                  const std::vector<float>& thresholds, const C3& max_comp,
                                  bool allow_trimming, const bool* prior_host,
                                  const uint8_t* prior_dev, Step& step);
  void PerformSubImageFitAll(Iuwt& iuwt, const Mask& mask, const Plane& structure_model,
                             Plane& scratch_a, Plane& scratch_b, const C3& max_comp,
                             std::vector<Plane>& fitted_model, const Plane& psf,
                             const gpu::Planes& psfs, const Plane& dirty);
  void PerformSubImageFitSingle(Iuwt& iuwt, const Mask& mask, const Plane& structure_model,
                                Plane& scratch_b, const C3& max_comp, const Plane& psf,
                                Plane& sub_dirty, std::vector<float>* fitted_sub_model,
                                std::vector<float>& correction_factor);

  Session& s_;
  size_t width_, height_;
  size_t box_x1_ = 0, box_x2_ = 0, box_y1_ = 0, box_y2_ = 0;
  float minor_loop_gain_, major_loop_gain_, clean_border_;
  bool allow_negative_;
  const bool* mask_;
  const uint8_t* d_mask_;
  float absolute_threshold_;
  const float threshold_sigma_level_ = 4.0f;
  const float tolerance_ = 0.75f;
  std::vector<float> rmses_;
  std::vector<ScaleResponse> psf_response_;
  ImageSet* dirty_set_ = nullptr;
  std::map<std::pair<size_t, size_t>, std::unique_ptr<Convolver>> convolvers_;
};

// :414-497
bool Algorithm::FindAndDeconvolveStructure(Iuwt& iuwt, Plane& dirty, const Plane& psf,
                                           const Buffer& psf_kernel, const gpu::Planes& psfs,
                                           Plane& scratch, std::vector<Plane>& structure_model,
                                           int end_scale, size_t min_scale,
                                           std::vector<Val>& max_components, Step& step) {
  iuwt.Decompose(s_, dirty.F(), scratch.F());
  std::vector<float> thresholds(static_cast<size_t>(end_scale));
  rmses_.resize(size_t(end_scale));
  for (int k = 0; k != end_scale; ++k) {
    const float r = Mad(iuwt.Scale(k), width_ * height_);
    rmses_[k] = r;
    // threshold_sigma_level_ * 4.0 / 5.0 is a double expression
    thresholds[k] = float(double(r) * (double(threshold_sigma_level_) * 4.0 / 5.0));
  }
  Assign(s_, scratch, dirty);
  max_components.assign(size_t(end_scale), Val());
  for (int k = 0; k != end_scale; ++k) {
    size_t x, y;
    const float v = GetMaxAbs(iuwt.Scale(k), x, y);
    max_components[k] = {x, y, k, v};
  }
  float max_val = -1.0f;
  size_t max_x = 0, max_y = 0;
  int max_scale = -1;
  for (int k = 0; k != end_scale; ++k) {
    const Val& v = max_components[k];
    const float abs_coef = v.val / psf_response_[k].rms;
    if (size_t(k) >= min_scale && abs_coef > max_val &&
        v.val > rmses_[k] * threshold_sigma_level_ &&
        v.val > rmses_[k] / rmses_[0] * absolute_threshold_) {
      max_x = v.x;
      max_y = v.y;
      max_scale = k;
      if (k == 0) {
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
  max_val = s_.ReadFloat(iuwt.Scale(max_scale) + max_x + max_y * width_);
  log::Debug() << "IUWT: most significant pixel " << max_x << ',' << max_y << '=' << max_val
               << " on scale " << max_scale << '\n';
  if (std::fabs(max_val) < thresholds[max_scale]) return false;
  const float scale_max_abs = std::fabs(max_val);
  for (int k = 0; k != end_scale; ++k) {
    if (thresholds[k] < tolerance_ * scale_max_abs) thresholds[k] = tolerance_ * scale_max_abs;
    if (max_val < 0.0f) thresholds[k] = -thresholds[k];
  }
  return FillAndDeconvolveStructure(iuwt, dirty, structure_model, scratch, psf, psf_kernel,
                                    psfs, end_scale, min_scale, width_, height_, thresholds,
                                    {max_x, max_y, max_scale}, true, mask_, d_mask_, step);
}

// :499-606
bool Algorithm::FillAndDeconvolveStructure(
    Iuwt& iuwt, Plane& dirty, std::vector<Plane>& model_full, Plane& scratch, const Plane& psf,
    const Buffer& psf_kernel, const gpu::Planes& psfs, int end_scale, size_t min_scale,
    size_t width, size_t height, const std::vector<float>& thresholds, const C3& max_comp,
    bool allow_trimming, const bool* prior_host, const uint8_t* prior_dev, Step& step) {
  Mask mask(s_, end_scale, width, height);
  uint64_t area = 0;
  // image_analysis::SelectStructures (iuwt/image_analysis.cc:227-259)
  const size_t xb = size_t(clean_border_ * width), yb = size_t(clean_border_ * height);
  Check(rdl_iuwt_select(s_.Handle(), iuwt.Coeffs(), uint32_t(width), uint32_t(height),
                        uint32_t(min_scale), uint32_t(end_scale), thresholds.data(),
                        uint32_t(xb), uint32_t(yb), prior_dev, mask.B(), &area),
        "rdl_iuwt_select");
  if (allow_trimming) step.area = area;
  iuwt.ApplyMask(s_, *mask.bytes);
  iuwt.Recompose(s_, scratch);
  size_t x1, y1, x2, y2;
  BoundingBox(x1, y1, x2, y2, scratch);
  AdjustBox(x1, y1, x2, y2, width, height, max_comp.scale + 1);
  if (allow_trimming && ((x2 - x1) < width || (y2 - y1) < height)) {
    box_x1_ = x1;
    box_x2_ = x2;
    box_y1_ = y1;
    box_y2_ = y2;
    const size_t nw = x2 - x1, nh = y2 - y1;
    step.trimmed_width = uint32_t(nw);
    dirty = Trim(s_, dirty.F(), width, x1, y1, x2, y2);
    const Plane small_psf = TrimPsf(s_, psf, nw, nh);
    const std::shared_ptr<Buffer> small_kernel = KernelOf(small_psf);
    scratch = Plane(s_, nw, nh);
    // IuwtDecomposition::EndScale (iuwt_decomposition.h:306-308)
    const int fit_end = std::max(std::max(int(std::log2(double(std::min(nw, nh)))) - 3, 2),
                                 max_comp.scale + 1);
    if (fit_end < end_scale) end_scale = fit_end;
    Iuwt trimmed = iuwt.Trimmed(s_, end_scale, x1, y1, x2, y2);
    std::vector<Plane> trimmed_model;
    for (const Plane& p : model_full) trimmed_model.push_back(Trim(s_, p.F(), width, x1, y1, x2, y2));
    std::vector<char> trimmed_prior;
    const bool* trimmed_prior_host = nullptr;
    std::unique_ptr<Buffer> trimmed_prior_dev;
    if (prior_host) {
      trimmed_prior.resize(nw * nh);
      for (size_t y = 0; y != nh; ++y)
        for (size_t x = 0; x != nw; ++x)
          trimmed_prior[y * nw + x] = prior_host[(y + y1) * width + x + x1] ? 1 : 0;
      trimmed_prior_host = reinterpret_cast<const bool*>(trimmed_prior.data());
      trimmed_prior_dev = std::make_unique<Buffer>(s_, nw * nh);
      s_.H2D(trimmed_prior_dev->Ptr(), trimmed_prior.data(), nw * nh);
    }
    const bool result = FillAndDeconvolveStructure(
        trimmed, dirty, trimmed_model, scratch, small_psf, *small_kernel, psfs, end_scale,
        min_scale, nw, nh, thresholds, {max_comp.x - x1, max_comp.y - y1, max_comp.scale}, false,
        trimmed_prior_host,
        trimmed_prior_dev ? static_cast<const uint8_t*>(trimmed_prior_dev->Ptr()) : nullptr,
        step);
    for (size_t i = 0; i != model_full.size(); ++i)
      model_full[i] = Untrim(s_, trimmed_model[i], width, height, x1, y1);
    dirty = Zeros(s_, width, height);
    scratch = Zeros(s_, width, height);
    box_x1_ = 0;
    box_x2_ = width;
    box_y1_ = 0;
    box_y2_ = height;
    return result;
  }
  iuwt.Decompose(s_, dirty.F(), scratch.F());
  iuwt.ApplyMask(s_, *mask.bytes);
  iuwt.Recompose(s_, scratch);
  Plane masked_dirty = Copy(s_, scratch);
  Plane structure_model = Zeros(s_, width, height);
  if (!RunConjugateGradient(iuwt, mask, masked_dirty, structure_model, scratch, psf_kernel))
    return false;
  const float rms_before = Rms(dirty);
  Assign(s_, scratch, structure_model);
  Convolve(scratch, psf_kernel);
  Assign(s_, masked_dirty, dirty);
  AddWithFactor(masked_dirty, scratch, -minor_loop_gain_);
  const float rms_after = Rms(masked_dirty);
  if (rms_after > rms_before) {
    log::Debug() << "IUWT: RMS got worse: " << rms_before << " -> " << rms_after << '\n';
    return false;
  }
  PerformSubImageFitAll(iuwt, mask, structure_model, scratch, masked_dirty, max_comp,
                        model_full, psf, psfs, dirty);
  return true;
}

// :608-656
void Algorithm::PerformSubImageFitAll(Iuwt& iuwt, const Mask& mask,
                                      const Plane& structure_model, Plane& scratch_a,
                                      Plane& scratch_b, const C3& max_comp,
                                      std::vector<Plane>& fitted_model, const Plane& psf,
                                      const gpu::Planes& psfs, const Plane& dirty) {
  const size_t width = iuwt.w, height = iuwt.h;
  if (dirty_set_->Size() == 1) {
    fitted_model[0] = Copy(s_, structure_model);
    return;
  }
  std::vector<float> factors;
  Assign(s_, scratch_a, dirty);
  PerformSubImageFitSingle(iuwt, mask, structure_model, scratch_b, max_comp, psf, scratch_a,
                           nullptr, factors);
  for (size_t i = 0; i != dirty_set_->Size(); ++i) {
    const float* sub_psf = psfs.Plane(dirty_set_->PsfIndex(i));
    scratch_a = Trim(s_, dirty_set_->Data(i), width_, box_x1_, box_y1_, box_x2_, box_y2_);
    Plane full_psf(s_, width_, height_);
    s_.D2D(full_psf.F(), sub_psf, full_psf.N() * sizeof(float));
    const Plane small_sub_psf =
        (width_ != width || height_ != height) ? TrimPsf(s_, full_psf, width, height) : full_psf;
    std::vector<float> fitted(width * height, 0.0f);
    PerformSubImageFitSingle(iuwt, mask, structure_model, scratch_b, max_comp, small_sub_psf,
                             scratch_a, &fitted, factors);
    fitted_model[i] = Plane(s_, width, height);
    s_.H2D(fitted_model[i].F(), fitted.data(), fitted.size() * sizeof(float));
  }
}

// :658-798 (connected components walked on the host, in the reference's
// FloodFill2D order; per component the boxed fit runs on the device)
void Algorithm::PerformSubImageFitSingle(Iuwt& iuwt, const Mask& mask,
                                         const Plane& structure_model, Plane& scratch_b,
                                         const C3& max_comp, const Plane& psf,
                                         Plane& sub_dirty, std::vector<float>* fitted_sub_model,
                                         std::vector<float>& correction_factor) {
  const size_t width = iuwt.w, height = iuwt.h, n = width * height;
  const std::shared_ptr<Buffer> psf_kernel = KernelOf(psf);
  Plane& masked_dirty = scratch_b;
  iuwt.Decompose(s_, sub_dirty.F(), sub_dirty.F());
  iuwt.ApplyMask(s_, *mask.bytes);
  iuwt.Recompose(s_, masked_dirty);
  std::vector<float> model(n), mdirty(n);
  s_.D2H(model.data(), structure_model.F(), n * sizeof(float));
  s_.D2H(mdirty.data(), masked_dirty.F(), n * sizeof(float));
  std::vector<uint8_t> mask_host(size_t(mask.n) * n);
  s_.D2H(mask_host.data(), mask.B(), mask_host.size());
  std::vector<char> mask2d(n, 0);
  const float peak = std::fabs(model[max_comp.y * width + max_comp.x]);
  const float fill_threshold = float(peak * 1e-4);
  size_t comp_index = 0;
  for (size_t y = 0; y != height; ++y)
    for (size_t x = 0; x != width; ++x) {
      if (mask2d[y * width + x] || !(std::fabs(model[y * width + x]) > peak * 1e-4)) continue;
      // image_analysis::FloodFill2D, area-collecting form (image_analysis.cc:292-333)
      std::vector<C2> area;
      std::stack<C2> todo;
      todo.push({x, y});
      mask2d[x + y * width] = 1;
      while (!todo.empty()) {
        const C2 c = todo.top();
        area.push_back(c);
        todo.pop();
        const size_t idx = c.x + c.y * width;
        auto visit = [&](size_t j, C2 next) {
          if (std::fabs(model[j]) > fill_threshold && !mask2d[j]) {
            mask2d[j] = 1;
            todo.push(next);
          }
        };
        if (c.x > 0) visit(idx - 1, {c.x - 1, c.y});
        if (c.x < width - 1) visit(idx + 1, {c.x + 1, c.y});
        if (c.y > 0) visit(idx - width, {c.x, c.y - 1});
        if (c.y < height - 1) visit(idx + width, {c.x, c.y + 1});
      }
      std::vector<float> sub(n, 0.0f);
      size_t bx1 = width, bx2 = 0, by1 = height, by2 = 0;
      for (const C2& a : area) {
        const size_t idx = a.x + a.y * width;
        bx1 = std::min(a.x, bx1);
        bx2 = std::max(a.x, bx2);
        by1 = std::min(a.y, by1);
        by2 = std::max(a.y, by2);
        sub[idx] = model[idx];
      }
      AdjustBox(bx1, by1, bx2, by2, width, height, iuwt.n);
      // PerformSubImageComponentFitBoxed / PerformSubImageComponentFit (:743-798)
      const bool boxed = bx1 > 0 || by1 > 0 || bx2 < width || by2 < height;
      const size_t nw = boxed ? bx2 - bx1 : width, nh = boxed ? by2 - by1 : height;
      const size_t ox = boxed ? bx1 : 0, oy = boxed ? by1 : 0;
      Plane comp_model(s_, nw, nh);
      std::vector<float> small(nw * nh);
      for (size_t yy = 0; yy != nh; ++yy)
        std::copy_n(sub.data() + (yy + oy) * width + ox, nw, small.data() + yy * nw);
      s_.H2D(comp_model.F(), small.data(), small.size() * sizeof(float));
      Iuwt fit_iuwt(s_, iuwt.n, nw, nh);
      Mask fit_mask(s_, mask.n, nw, nh);
      {
        std::vector<uint8_t> m(size_t(mask.n) * nw * nh);
        for (int k = 0; k != mask.n; ++k)
          for (size_t yy = 0; yy != nh; ++yy)
            std::copy_n(mask_host.data() + size_t(k) * n + (yy + oy) * width + ox, nw,
                        m.data() + size_t(k) * nw * nh + yy * nw);
        s_.H2D(fit_mask.B(), m.data(), m.size());
      }
      std::shared_ptr<Buffer> kernel = psf_kernel;
      if (boxed) kernel = KernelOf(TrimPsf(s_, psf, nw, nh));
      Convolve(comp_model, *kernel);
      fit_iuwt.Decompose(s_, comp_model.F(), comp_model.F());
      fit_iuwt.ApplyMask(s_, *fit_mask.bytes);
      fit_iuwt.Recompose(s_, comp_model);
      std::vector<float> fitted(nw * nh);
      s_.D2H(fitted.data(), comp_model.F(), fitted.size() * sizeof(float));
      float model_sum = 0.0f, dirty_sum = 0.0f;
      for (const C2& a : area) {
        model_sum += fitted[(a.x - ox) + (a.y - oy) * nw];
        dirty_sum += mdirty[a.x + a.y * width];
      }
      const float factor =
          (model_sum == 0.0f || !std::isfinite(dirty_sum) || !std::isfinite(model_sum))
              ? 0.0f
              : dirty_sum / model_sum;
      if (fitted_sub_model) {
        const float integrated = correction_factor[comp_index];
        if (std::isfinite(factor) && std::isfinite(integrated) && integrated != 0.0f)
          for (const C2& a : area) {
            const size_t idx = a.x + a.y * width;
            (*fitted_sub_model)[idx] += model[idx] * factor / integrated;
          }
        ++comp_index;
      } else {
        correction_factor.push_back(factor);
      }
    }
}

// :800-918
float Algorithm::PerformMajorIteration(size_t& iter_counter, size_t n_iter, ImageSet& model_set,
                                       ImageSet& dirty_set, const gpu::Planes& psfs,
                                       bool& reached, std::vector<Step>& steps) {
  reached = false;
  if (iter_counter == n_iter) return 0.0f;
  dirty_set_ = &dirty_set;
  box_x1_ = 0;
  box_x2_ = width_;
  box_y1_ = 0;
  box_y2_ = height_;
  const size_t n = width_ * height_;
  Plane dirty(s_, width_, height_), psf(s_, width_, height_);
  dirty_set.GetLinearIntegrated(dirty.F());
  dirty_set.GetIntegratedPsf(psf.F(), psfs);
  const int max_scale = std::max(int(std::log2(double(std::min(width_, height_)))) - 3, 2);
  int end_scale = 2;
  const std::shared_ptr<Buffer> psf_kernel = KernelOf(psf);
  MeasureRmsPerScale(psf, max_scale);
  std::vector<Plane> structure_model;
  for (size_t i = 0; i != model_set.Size(); ++i) structure_model.push_back(Zeros(s_, width_, height_));
  auto iuwt = std::make_unique<Iuwt>(s_, end_scale, width_, height_);
  std::map<size_t, std::shared_ptr<Buffer>> image_kernels;
  float max_value = 0.0f;
  size_t min_scale = 0;
  bool do_continue = true;
  std::vector<Val> initial;
  do {
    const Plane dirty_before = Copy(s_, dirty);
    std::vector<Val> max_components;
    Plane scratch(s_, width_, height_);
    Step step{};
    step.scale = -1;
    step.end_scale = end_scale;
    step.min_scale = int(min_scale);
    const bool ok = FindAndDeconvolveStructure(*iuwt, dirty, psf, *psf_kernel, psfs, scratch,
                                               structure_model, end_scale, min_scale,
                                               max_components, step);
    step.succeeded = ok ? 1 : 0;
    if (ok) {
      for (size_t i = 0; i != model_set.Size(); ++i) {
        Plane& p = structure_model[i];
        Check(rdl_scale(s_.Handle(), p.F(), n, minor_loop_gain_), "rdl_scale");
        Check(rdl_add(s_.Handle(), model_set.Data(i), p.F(), n), "rdl_add");
      }
      // dirty = dirty - structureModel (x) psf, per image (:868-877)
      for (size_t i = 0; i != dirty_set.Size(); ++i) {
        const size_t pi = dirty_set.PsfIndex(i);
        auto it = image_kernels.find(pi);
        if (it == image_kernels.end()) {
          Plane p(s_, width_, height_);
          s_.D2D(p.F(), psfs.Plane(pi), n * sizeof(float));
          it = image_kernels.emplace(pi, KernelOf(p)).first;
        }
        Assign(s_, scratch, structure_model[i]);
        Convolve(scratch, *it->second);
        Check(rdl_axpy(s_.Handle(), dirty_set.Data(i), scratch.F(), n, -1.0f, 0), "rdl_axpy");
      }
      dirty_set.GetLinearIntegrated(dirty.F());
      while (max_components.size() > initial.size()) initial.push_back(max_components[initial.size()]);
      max_value = 0.0f;
      for (size_t c = 0; c != initial.size(); ++c) {
        max_value = std::max(max_value, max_components[c].val);
        if (std::fabs(max_components[c].val) < std::fabs(initial[c].val) * (1.0 - major_loop_gain_))
          reached = true;
      }
      step.max_value = max_value;
      steps.push_back(step);
      if (reached) break;  // before ++iter_counter, as the reference
    } else {
      if (int(min_scale) + 1 < end_scale) {
        ++min_scale;
      } else {
        min_scale = 0;
        if (end_scale != max_scale) {
          ++end_scale;
          iuwt = std::make_unique<Iuwt>(s_, end_scale, width_, height_);
        } else {
          do_continue = false;
        }
      }
      dirty = dirty_before;
      steps.push_back(step);
    }
    ++iter_counter;
  } while (iter_counter != n_iter && do_continue);
  return max_value;
}

}  // namespace

DeconvolutionResult IuwtDeconvolution::ExecuteMajorIteration(ImageSet& data_image,
                                                             ImageSet& model_image,
                                                             const gpu::Planes& psf_images) {
  Session& s = data_image.Session();
  const size_t width = data_image.Width(), height = data_image.Height();
  if (psf_images.width != width || psf_images.height != height)
    throw std::runtime_error("IUWT: PSFs must have the image size");
  const uint8_t* d_mask = DeviceCleanMask(s, width, height);
  Algorithm algorithm(s, width, height, *this, d_mask);
  size_t iteration_number = IterationNumber();
  DeconvolutionResult result;
  steps_.clear();
  result.final_peak_value = algorithm.PerformMajorIteration(
      iteration_number, MaxIterations(), model_image, data_image, psf_images,
      result.another_iteration_required, steps_);
  SetIterationNumber(iteration_number);
  if (IterationNumber() >= MaxIterations()) result.another_iteration_required = false;
  s.Sync();
  return result;
}

}  // namespace radler::algorithms
