// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// CPU restatement of Radler's CLEAN hot path (ska-sdp-func-radler snapshot
// 2025-04-10 at /root/reference). Each function cites the reference lines it
// restates. Compiled with -ffp-contract=off; every site where the reference's
// GCC -O3 -march=native build contracts `a - b*c` / `a + b*c` into an FMA is
// written as an explicit std::fmaf here.
//
// Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline.
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <limits>
#include <map>
#include <memory>
#include <vector>

#include "spectral.h"

namespace oracle {

struct Peak {
  bool has = false;
  float value = 0.0f;
  size_t x = 0, y = 0;
};

// cpp/math/peak_finder.cc:199-253 (Avx<bool>, the x86 default of Find()).
Peak FindPeakAvx(const float* image, size_t width, size_t height,
                 bool allow_negative, size_t start_y, size_t end_y,
                 size_t horizontal_border, size_t vertical_border);
// cpp/math/peak_finder.cc:19-56
Peak FindPeakSimple(const float* image, size_t width, size_t height,
                    bool allow_negative, size_t start_y, size_t end_y,
                    size_t horizontal_border, size_t vertical_border);
// cpp/math/peak_finder.cc:97-131
Peak FindPeakWithMask(const float* image, size_t width, size_t height,
                      bool allow_negative, size_t start_y, size_t end_y,
                      const bool* mask, size_t horizontal_border,
                      size_t vertical_border);

// cpp/algorithms/simple_clean.cc:96-131
void PartialSubtractImage(float* image, const float* psf, size_t width,
                          size_t height, size_t x, size_t y, float factor,
                          size_t start_y, size_t end_y);
// cpp/algorithms/threaded_deconvolution_tools.cc:18-28
void SubtractImage(float* image, const float* psf, size_t width, size_t height,
                   size_t x, size_t y, float factor);

// cpp/utils/fft_size_calculations.h:15-50
size_t CalculateGoodFFTSize(size_t minimum_size);
size_t GetConvolutionSize(double scale, size_t original_size, double padding);

// schaapcommon contracts restated from their call sites (see fft.h).
void PrepareSmallConvolutionKernel(float* dest, size_t width, size_t height,
                                   const float* kernel, size_t n);
void PrepareConvolutionKernel(float* dest, const float* source, size_t width,
                              size_t height);
// aocommon::Image::Untrim / Trim (centred embedding / crop).
void Untrim(float* dest, size_t out_w, size_t out_h, const float* src,
            size_t in_w, size_t in_h);
void Trim(float* dest, size_t out_w, size_t out_h, const float* src,
          size_t in_w, size_t in_h);

// cpp/algorithms/multiscale/multiscale_transforms.h:91-195
enum class Shape { kTaperedQuadratic = 0, kGaussian = 1 };
std::vector<float> MakeShapeFunction(float scale, size_t& n, size_t max_n,
                                     Shape shape);
float KernelPeakValue(double scale, size_t max_n, Shape shape);
void AddShapeComponent(float* image, size_t width, size_t height, float scale,
                       size_t x, size_t y, float gain, Shape shape);
// cpp/algorithms/multiscale/multiscale_transforms.cc:9-21
void MsTransform(std::vector<float*>& images, size_t width, size_t height,
                 float scale, Shape shape);

// cpp/image_set.{h,cc}: the [channel][pol] image stack restricted to the
// layout Radler builds for its configs (image index = channel*n_pol + pol,
// PSF index = channel, all polarizations linked).
struct SetDesc {
  size_t n_channels = 1;  // deconvolution channels
  size_t n_pol = 1;
  std::vector<float> weights;  // per deconvolution channel
  float pol_factor = 1.0f;
  bool squared_joins = false;
  // the algorithms' SpectralFitter (deconvolution_algorithm.h:148-161);
  // nullptr = kNoFitting
  std::shared_ptr<const SpectralFit> fitter;
};

struct ImageSet {
  const SetDesc* desc = nullptr;
  size_t width = 0, height = 0;
  std::vector<float*> images;  // n_channels * n_pol views
  size_t Size() const { return images.size(); }
  size_t PsfIndex(size_t i) const { return i / desc->n_pol; }
};

// cpp/image_set.cc:423-462 (GetLinearIntegratedWithNormalChannels)
void GetLinearIntegrated(const ImageSet& set, float* dest);
// cpp/image_set.cc:309-421 (GetSquareIntegrated*)
void GetSquareIntegrated(const ImageSet& set, float* dest);
// cpp/image_set.cc:499-530
void GetIntegratedPsf(const SetDesc& desc, const std::vector<const float*>& psfs,
                      size_t n, float* dest);

struct AlgoSettings {
  float threshold = 0.0f;
  float major_iteration_threshold = 0.0f;
  float minor_loop_gain = 0.1f;
  float major_loop_gain = 1.0f;
  float clean_border_ratio = 0.05f;
  size_t max_iterations = 500;
  float divergence_limit = 4.0f;
  bool allow_negative = true;
  bool stop_on_negative = false;
  const bool* clean_mask = nullptr;
  // DeconvolutionAlgorithm::RmsFactorImage (deconvolution_algorithm.h:163-166):
  // width x height factors multiplied into every peak search; nullptr = none
  const float* rms_factor = nullptr;
  // OptimizationAlgorithm (settings.h): 0 kClean, 2 kGradientDescent
  int component_optimization = 0;
  // generic clean
  bool use_sub_minor_optimization = true;
  // multiscale (cpp/settings.h:465-524)
  bool fast_sub_minor_loop = true;
  double sub_minor_loop_gain = 0.2;
  double scale_bias = 0.6;
  size_t max_scales = 0;
  double convolution_padding = 1.1;
  Shape shape = Shape::kTaperedQuadratic;
  std::vector<double> scale_list;
  double beam_size_in_pixels = 1.0;
};

// cpp/algorithms/deconvolution_algorithm.h:31-58
struct Result {
  bool has_starting_peak = false;
  float starting_peak = 0.0f;
  float final_peak = 0.0f;
  bool another_iteration_required = false;
  bool is_diverging = false;
};

// One CLEAN component: Högbom/Clark record pixel components (scale 0).
// `margin` (test harness, not part of the reference): the smallest gap, in
// the compared quantity's units, between a comparison's two sides over
// every decision taken since the previous component up to and including the
// choice of this one (argmax runner-up, loop-continue thresholds, scale
// selection and activation). A float engine that differs from this one by
// less than that gap makes the same decisions (tests/trace_compare.py).
struct Component {
  uint32_t x, y, scale;
  float margin = std::numeric_limits<float>::infinity();
  float value = 0.0f;  // |integrated peak| that chose it (margin scale)
};

// Decision-margin bookkeeping for the traces above.
struct MarginTracker {
  float pending = std::numeric_limits<float>::infinity();
  // a comparison a > b (or a >= b) was evaluated: record |a - b|
  void Note(double a, double b) {
    const float m = float(std::fabs(a - b));
    if (m < pending) pending = m;
  }
  float Take() {
    const float m = pending;
    pending = std::numeric_limits<float>::infinity();
    return m;
  }
};

// cpp/algorithms/subminor_loop.{h,cc}
class SubMinorLoop {
 public:
  SubMinorLoop(size_t width, size_t height, size_t padded_width,
               size_t padded_height)
      : width_(width),
        height_(height),
        padded_width_(padded_width),
        padded_height_(padded_height) {}
  float threshold = 0.0f, gain = 0.0f, divergence_limit = 0.0f;
  size_t horizontal_border = 0, vertical_border = 0;
  size_t current_iteration = 0, max_iterations = 0;
  bool allow_negative = true, stop_on_negative = false;
  const bool* mask = nullptr;
  const float* rms_factor = nullptr;  // SetRmsFactorImage (full image)
  float flux_cleaned = 0.0f;
  std::vector<Component>* trace = nullptr;
  uint32_t trace_scale = 0;
  MarginTracker* margins = nullptr;  // decision margins (tests only)

  // returns {diverging, has_peak, peak}
  struct RunResult {
    bool diverging;
    bool has_peak;
    float peak;
  };
  RunResult Run(ImageSet& convolved_residual,
                const std::vector<const float*>& twice_convolved_psfs);
  void CorrectResidualDirty(size_t image_index, float* residual,
                            const float* single_convolved_psf) const;
  void GetFullIndividualModel(size_t image_index, float* dest) const;
  // subminor_loop.cc:220-228: every selected pixel with a non-zero model
  // value in any image joins the mask
  void UpdateAutoMask(bool* mask) const;
  size_t NSelected() const { return positions_.size(); }

 private:
  size_t width_, height_, padded_width_, padded_height_;
  std::vector<std::pair<size_t, size_t>> positions_;
  std::vector<std::vector<float>> residual_, model_;
  std::vector<float> rms_selected_;  // SubMinorModel::MakeRmsFactorImage
  const SetDesc* desc_ = nullptr;
  size_t GetMaxComponent(std::vector<float>& scratch, float& max_value) const;
  // gap between the chosen |value| and the runner-up in scratch
  void NoteArgmaxMargin(const std::vector<float>& scratch, size_t chosen) const;
};

// cpp/algorithms/generic_clean.cc:56-253
Result GenericCleanExecute(const AlgoSettings& s, size_t& iteration_number,
                           ImageSet& dirty, ImageSet& model,
                           const std::vector<const float*>& psfs,
                           std::vector<Component>* trace);

// cpp/algorithms/multiscale_algorithm.cc
struct ScaleInfo {
  float scale = 0.0f, psf_peak = 0.0f, kernel_peak = 0.0f, bias_factor = 0.0f,
        gain = 0.0f;
  float max_normalized_image_value = 0.0f, max_unnormalized_image_value = 0.0f,
        rms = 0.0f;
  size_t max_image_value_x = 0, max_image_value_y = 0;
  bool is_active = false;
  size_t n_components_cleaned = 0;
  float total_flux_cleaned = 0.0f;
};

class MultiScale {
 public:
  explicit MultiScale(const AlgoSettings& s) : s_(s) {
    if (s_.beam_size_in_pixels <= 0.0) s_.beam_size_in_pixels = 1.0;
  }
  AlgoSettings& Settings() { return s_; }
  size_t iteration_number = 0;
  // Auto-masking (multiscale_algorithm.h:41-55, .cc:214-226, 403-404,
  // 444-445, 586-610, 695-696, 716-720): track = grow one mask per scale
  // from the components; use = clean each scale inside its mask only (the
  // scale-independent clean mask is then ignored). Masks: one byte (0/1)
  // per pixel, kept across major iterations.
  bool track_scale_masks = false, use_scale_masks = false;
  std::vector<std::vector<uint8_t>> scale_masks;
  Result Execute(ImageSet& data, ImageSet& model,
                 const std::vector<const float*>& psfs,
                 std::vector<Component>* trace);
  const std::vector<ScaleInfo>& Scales() const { return scales_; }
  // decision margins (tests): pending margins after the last component end
  // up in end_margin (the decisions that stopped the run)
  MarginTracker margins;
  float end_margin = std::numeric_limits<float>::infinity();
  // wall seconds of the last Execute's setup (scale PSFs + first peak
  // search), before the outer loop: bench.py's cpu_baseline reports the
  // cleaning rate after setup and the setup separately
  double setup_seconds = 0.0;
  // bench.py's cpu_baseline: when clean_threads is non-zero, the pool
  // switches to clean_threads after switch_after outer iterations;
  // switch_seconds / switch_components record when (seconds since the setup
  // ended) and after how many components. stop_after_outer (non-zero) ends
  // the run after that many outer iterations.
  size_t clean_threads = 0, switch_after = 0, stop_after_outer = 0;
  double switch_seconds = 0.0;
  size_t switch_components = 0;

 private:
  AlgoSettings s_;
  void NoteScaleSelection();
  std::vector<ScaleInfo> scales_;
  void FindActiveScaleConvolvedMaxima(const ImageSet& set, float* integrated,
                                      bool report_rms);
  void FindPeakDirect(const float* image, size_t w, size_t h,
                      size_t scale_index);
  const bool* ScaleMask(size_t i) const {
    return reinterpret_cast<const bool*>(scale_masks[i].data());
  }
  void ActivateScales(size_t scale_with_last_peak);
};

// Single-scale helper used by tests: SelectMaximumScale
// cpp/algorithms/multiscale_algorithm.cc:133-151
bool SelectMaximumScale(const std::vector<ScaleInfo>& scales, size_t& index);
void InitializeScales(std::vector<ScaleInfo>& scales, double beam_px,
                      size_t min_wh, Shape shape, size_t max_scales,
                      const std::vector<double>& scale_list);

}  // namespace oracle
