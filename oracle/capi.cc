// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
// extern "C" surface of the CPU restatement, loaded by tests/ and bench.py
// (cpu_baseline) through ctypes.
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "fft.h"
#include "oracle.h"
#include "tiling.h"
#include "rms_image.h"
#include "component_optimization.h"
#include "iuwt.h"
#include "iuwt_algorithm.h"

using namespace oracle;

extern "C" {

struct orc_set_desc {
  uint64_t width, height, n_channels, n_pol;
  const float* weights;
  float pol_factor;
  int32_t squared_joins;
  // spectral fitting (fit_mode 0 = none, 1 = polynomial over n_channels)
  int32_t fit_mode;
  uint32_t fit_terms;
  const double* fit_frequencies;
  const float* fit_weights;
};

struct orc_algo_settings {
  double threshold, major_iteration_threshold, minor_loop_gain,
      major_loop_gain, border_ratio, divergence_limit;
  uint64_t max_iterations;
  int32_t allow_negative, stop_on_negative, use_sub_minor, fast_sub_minor_loop;
  double sub_minor_loop_gain, scale_bias;
  uint64_t max_scales;
  double convolution_padding;
  int32_t shape, pad0;
  double beam_size_in_pixels;
  const double* scale_list;
  uint64_t n_scale_list;
  const uint8_t* clean_mask;
};

struct orc_result {
  int32_t has_starting_peak;
  float starting_peak;
  float final_peak;
  int32_t another_iteration_required;
  int32_t is_diverging;
  int32_t pad0;
  uint64_t iteration_number;
  uint64_t n_trace;
};

static thread_local std::string g_error;
const char* orc_last_error() { return g_error.c_str(); }

void orc_set_threads(uint64_t n) { SetNThreads(n); }

int orc_find_peak(const float* img, uint64_t w, uint64_t h, int allow_neg,
                  uint64_t start_y, uint64_t end_y, uint64_t hb, uint64_t vb,
                  const uint8_t* mask, int simple, uint64_t* x, uint64_t* y,
                  float* value) {
  Peak p;
  if (mask)
    p = FindPeakWithMask(img, w, h, allow_neg, start_y, end_y,
                         reinterpret_cast<const bool*>(mask), hb, vb);
  else if (simple)
    p = FindPeakSimple(img, w, h, allow_neg, start_y, end_y, hb, vb);
  else
    p = FindPeakAvx(img, w, h, allow_neg, start_y, end_y, hb, vb);
  *x = p.x;
  *y = p.y;
  *value = p.value;
  return p.has ? 1 : 0;
}

void orc_partial_subtract(float* img, const float* psf, uint64_t w, uint64_t h,
                          uint64_t x, uint64_t y, float factor,
                          uint64_t start_y, uint64_t end_y) {
  PartialSubtractImage(img, psf, w, h, x, y, factor, start_y, end_y);
}

void orc_subtract(float* img, const float* psf, uint64_t w, uint64_t h,
                  uint64_t x, uint64_t y, float factor) {
  SubtractImage(img, psf, w, h, x, y, factor);
}

uint64_t orc_good_fft_size(uint64_t n) { return CalculateGoodFFTSize(n); }
uint64_t orc_convolution_size(double scale, uint64_t n, double padding) {
  return GetConvolutionSize(scale, n, padding);
}

void orc_convolve(float* image, const float* kernel, uint64_t w, uint64_t h) {
  ConvolveCircular(image, kernel, w, h);
}

uint64_t orc_shape_function(float scale, uint64_t max_n, int shape,
                            float* out) {
  size_t n;
  std::vector<float> k = MakeShapeFunction(scale, n, max_n, Shape(shape));
  if (out) std::memcpy(out, k.data(), k.size() * sizeof(float));
  return n;
}

float orc_kernel_peak(double scale, uint64_t max_n, int shape) {
  return KernelPeakValue(scale, max_n, Shape(shape));
}

void orc_ms_transform(float* images, uint64_t n_images, uint64_t w, uint64_t h,
                      float scale, int shape) {
  std::vector<float*> l;
  for (uint64_t i = 0; i != n_images; ++i) l.push_back(images + i * w * h);
  MsTransform(l, w, h, scale, Shape(shape));
}

void orc_add_shape_component(float* image, uint64_t w, uint64_t h, float scale,
                             uint64_t x, uint64_t y, float gain, int shape) {
  AddShapeComponent(image, w, h, scale, x, y, gain, Shape(shape));
}

static SetDesc MakeDesc(const orc_set_desc* d) {
  SetDesc desc;
  desc.n_channels = d->n_channels;
  desc.n_pol = d->n_pol;
  desc.weights.assign(d->weights, d->weights + d->n_channels);
  desc.pol_factor = d->pol_factor;
  desc.squared_joins = d->squared_joins != 0;
  if (d->fit_mode != 0)
    desc.fitter = std::make_shared<SpectralFit>(
        d->fit_mode, d->fit_terms,
        std::vector<double>(d->fit_frequencies, d->fit_frequencies + d->n_channels),
        std::vector<float>(d->fit_weights, d->fit_weights + d->n_channels));
  return desc;
}

static ImageSet MakeSet(const SetDesc& desc, const orc_set_desc* d,
                        float* data) {
  ImageSet s;
  s.desc = &desc;
  s.width = d->width;
  s.height = d->height;
  for (uint64_t i = 0; i != d->n_channels * d->n_pol; ++i)
    s.images.push_back(data + i * d->width * d->height);
  return s;
}

void orc_integrate(const orc_set_desc* d, float* images, float* dest,
                   int square) {
  SetDesc desc = MakeDesc(d);
  ImageSet s = MakeSet(desc, d, images);
  if (square)
    GetSquareIntegrated(s, dest);
  else
    GetLinearIntegrated(s, dest);
}

struct OrcAlgo {
  int type;
  AlgoSettings settings;
  std::vector<double> scale_list;
  size_t iteration_number = 0;
  std::unique_ptr<MultiScale> ms;
  std::vector<IuwtStep> iuwt_steps;  // type 2: steps of the last execute
  std::vector<float> rms_factor;     // SetRmsFactorImage (empty = none)
  int component_optimization = 0;    // SetComponentOptimizationAlgorithm
  std::vector<float> margins;        // decision margins of the last trace (+ end)
  std::vector<float> values;         // the components' |peak| (+ the last one)
};

static AlgoSettings MakeSettings(const orc_algo_settings* a) {
  AlgoSettings s;
  s.threshold = a->threshold;
  s.major_iteration_threshold = a->major_iteration_threshold;
  s.minor_loop_gain = a->minor_loop_gain;
  s.major_loop_gain = a->major_loop_gain;
  s.clean_border_ratio = a->border_ratio;
  s.divergence_limit = a->divergence_limit;
  s.max_iterations = a->max_iterations;
  s.allow_negative = a->allow_negative;
  s.stop_on_negative = a->stop_on_negative;
  s.clean_mask = reinterpret_cast<const bool*>(a->clean_mask);
  s.use_sub_minor_optimization = a->use_sub_minor;
  s.fast_sub_minor_loop = a->fast_sub_minor_loop;
  s.sub_minor_loop_gain = a->sub_minor_loop_gain;
  s.scale_bias = a->scale_bias;
  s.max_scales = a->max_scales;
  s.convolution_padding = a->convolution_padding;
  s.shape = Shape(a->shape);
  s.beam_size_in_pixels = a->beam_size_in_pixels;
  if (a->scale_list)
    s.scale_list.assign(a->scale_list, a->scale_list + a->n_scale_list);
  return s;
}

void* orc_algo_create(int type, const orc_algo_settings* a) {
  auto* algo = new OrcAlgo();
  algo->type = type;
  algo->settings = MakeSettings(a);
  if (type == 1) algo->ms = std::make_unique<MultiScale>(algo->settings);
  return algo;
}

void orc_algo_destroy(void* h) { delete static_cast<OrcAlgo*>(h); }

// Steps of the last IUWT (type 2) execute: fills up to cap records, returns
// the count (IuwtStep layout: i32 succeeded, i32 scale, u32 x, u32 y,
// i32 end_scale, i32 min_scale, u64 area, f32 max_value, pad to 40 bytes).
uint64_t orc_iuwt_steps(void* h, IuwtStep* out, uint64_t cap) {
  auto* algo = static_cast<OrcAlgo*>(h);
  const size_t n = std::min<size_t>(cap, algo->iuwt_steps.size());
  for (size_t i = 0; i != n; ++i) out[i] = algo->iuwt_steps[i];
  return algo->iuwt_steps.size();
}

// Update the mutable per-call settings (threshold, max iterations, gains).
void orc_algo_update(void* h, const orc_algo_settings* a) {
  auto* algo = static_cast<OrcAlgo*>(h);
  algo->settings = MakeSettings(a);
  if (algo->ms) {
    algo->ms->Settings() = algo->settings;
    if (algo->ms->Settings().beam_size_in_pixels <= 0.0)
      algo->ms->Settings().beam_size_in_pixels = 1.0;
  }
}

// MultiScaleAlgorithm::SetAutoMaskMode (multiscale_algorithm.h:41-44)
void orc_algo_set_automask(void* h, int track, int use) {
  auto* algo = static_cast<OrcAlgo*>(h);
  if (!algo->ms) return;
  algo->ms->track_scale_masks = track != 0;
  algo->ms->use_scale_masks = use != 0;
}

// copy of scale mask `index` (0/1 bytes, up to n); returns the mask count
uint64_t orc_algo_scale_mask(void* h, uint64_t index, uint8_t* out, uint64_t n) {
  auto* algo = static_cast<OrcAlgo*>(h);
  if (!algo->ms) return 0;
  const auto& masks = algo->ms->scale_masks;
  if (out && index < masks.size())
    std::copy_n(masks[index].data(), std::min<size_t>(n, masks[index].size()), out);
  return masks.size();
}

int orc_algo_execute(void* h, const orc_set_desc* d, float* residual,
                     float* model, const float* psfs, orc_result* out,
                     uint32_t* trace, uint64_t trace_cap) {
  try {
    auto* algo = static_cast<OrcAlgo*>(h);
    SetDesc desc = MakeDesc(d);
    ImageSet res = MakeSet(desc, d, residual);
    ImageSet mod = MakeSet(desc, d, model);
    std::vector<const float*> psf_ptrs;
    for (uint64_t c = 0; c != d->n_channels; ++c)
      psf_ptrs.push_back(psfs + c * d->width * d->height);
    std::vector<Component> tr;
    Result r;
    algo->settings.rms_factor = algo->rms_factor.empty() ? nullptr : algo->rms_factor.data();
    algo->settings.component_optimization = algo->component_optimization;
    if (algo->ms) algo->ms->Settings().rms_factor = algo->settings.rms_factor;
    if (algo->type == 0) {
      r = GenericCleanExecute(algo->settings, algo->iteration_number, res, mod,
                              psf_ptrs, &tr);
    } else if (algo->type == 2) {
      // IuwtDeconvolution::ExecuteMajorIteration (iuwt_deconvolution.h:22-39)
      IuwtAlgoSettings is;
      is.minor_loop_gain = algo->settings.minor_loop_gain;
      is.major_loop_gain = algo->settings.major_loop_gain;
      is.clean_border = algo->settings.clean_border_ratio;
      is.allow_negative = algo->settings.allow_negative;
      is.mask = algo->settings.clean_mask;
      is.absolute_threshold = algo->settings.threshold;
      algo->iuwt_steps.clear();
      bool another = false;
      r.final_peak = IuwtExecute(is, algo->iteration_number, algo->settings.max_iterations,
                                 res, mod, psf_ptrs, another, &algo->iuwt_steps);
      r.another_iteration_required = another;
    } else {
      algo->ms->iteration_number = algo->iteration_number;
      r = algo->ms->Execute(res, mod, psf_ptrs, &tr);
      algo->iteration_number = algo->ms->iteration_number;
    }
    out->has_starting_peak = r.has_starting_peak;
    out->starting_peak = r.starting_peak;
    out->final_peak = r.final_peak;
    out->another_iteration_required = r.another_iteration_required;
    out->is_diverging = r.is_diverging;
    out->iteration_number = algo->iteration_number;
    out->n_trace = tr.size();
    algo->margins.clear();
    algo->values.clear();
    for (const Component& c : tr) {
      algo->margins.push_back(c.margin);
      algo->values.push_back(c.value);
    }
    algo->margins.push_back(algo->ms ? algo->ms->end_margin
                                     : std::numeric_limits<float>::infinity());
    algo->values.push_back(tr.empty() ? 1.0f : tr.back().value);
    if (trace) {
      const size_t n = std::min<size_t>(tr.size(), trace_cap);
      for (size_t i = 0; i != n; ++i) {
        trace[3 * i] = tr[i].x;
        trace[3 * i + 1] = tr[i].y;
        trace[3 * i + 2] = tr[i].scale;
      }
    }
    return 0;
  } catch (std::exception& e) {
    g_error = e.what();
    return 1;
  }
}

// After `after` multiscale outer iterations switch the pool to `n` threads
// (0 = never), and stop after `stop` outer iterations (0 = never);
// orc_algo_switch_info reports when the switch happened.
void orc_algo_set_clean_threads(void* h, uint64_t n, uint64_t after, uint64_t stop) {
  auto* algo = static_cast<OrcAlgo*>(h);
  if (!algo->ms) return;
  algo->ms->clean_threads = n;
  algo->ms->switch_after = after;
  algo->ms->stop_after_outer = stop;
}

void orc_algo_switch_info(void* h, double* seconds, uint64_t* components) {
  auto* algo = static_cast<OrcAlgo*>(h);
  *seconds = algo->ms ? algo->ms->switch_seconds : 0.0;
  *components = algo->ms ? algo->ms->switch_components : 0;
}

// Setup seconds of the last multiscale execute (MultiScale::setup_seconds)
double orc_algo_setup_seconds(void* h) {
  auto* algo = static_cast<OrcAlgo*>(h);
  return algo->ms ? algo->ms->setup_seconds : 0.0;
}

struct orc_parallel_result {
  int32_t another_iteration_required;
  int32_t n_subimages;
  double start_peak, end_peak;
  uint64_t first_iteration_number, total_iterations;
  uint64_t n_trace;
};

// Decision margins of the last execute's trace (oracle.h Component::margin),
// one per component and then the end-of-run margin; returns the count.
// `values` (may be NULL) gets each component's |peak| (the margin's scale).
uint64_t orc_algo_margins(void* h, float* out, float* values, uint64_t cap) {
  auto* algo = static_cast<OrcAlgo*>(h);
  const size_t n = std::min<size_t>(cap, algo->margins.size());
  std::copy_n(algo->margins.data(), n, out);
  if (values) std::copy_n(algo->values.data(), n, values);
  return algo->margins.size();
}

struct OrcParallel {
  std::vector<float> margins;      // per trace entry, in trace order
  std::vector<float> values;       // the components' |peak|
  std::vector<float> end_margins;  // per subimage
  size_t grid_w, grid_h;
  double major_loop_gain_unused = 0.0;
  bool snapshot = false;
  std::vector<TiledAlgorithm> algorithms;
  ParallelMasks masks;
};

// IUWT: coeffs (n_scales + 1) planes; aliased != 0 runs Decompose(x, x, ..)
// with input as the scratch (input is overwritten, like the reference).
int orc_iuwt_decompose(float* input, uint64_t w, uint64_t h, uint64_t n_scales,
                       int aliased, int include_largest, float* coeffs) {
  try {
    std::vector<float> scratch(aliased ? 0 : w * h);
    std::vector<std::vector<float>> c;
    IuwtDecompose(input, aliased ? input : scratch.data(), w, h, n_scales, c,
                  include_largest != 0);
    for (size_t s = 0; s != c.size(); ++s)
      if (!c[s].empty()) std::copy(c[s].begin(), c[s].end(), coeffs + s * w * h);
    return 0;
  } catch (std::exception& e) {
    g_error = e.what();
    return 1;
  }
}

void orc_iuwt_recompose(const float* coeffs, uint64_t w, uint64_t h,
                        uint64_t n_scales, int include_largest, float* out) {
  std::vector<std::vector<float>> c(n_scales + 1);
  for (size_t s = 0; s <= n_scales; ++s)
    if (s < n_scales || include_largest) c[s].assign(coeffs + s * w * h, coeffs + (s + 1) * w * h);
  IuwtRecompose(c, w, h, n_scales, include_largest != 0, out);
}

// MakeSubImages alone (no user mask): boxes 4 x u32 per subimage, labels
// W*H u16 (subimage index + 1 in its boundary mask).
int orc_make_subimages(const float* image, uint64_t w, uint64_t h, uint64_t grid_w,
                       uint64_t grid_h, uint32_t* boxes, uint16_t* labels) {
  try {
    std::vector<SubImage> subs = MakeSubImages(image, w, h, nullptr, grid_w, grid_h);
    std::fill(labels, labels + w * h, uint16_t(0));
    for (const SubImage& s : subs) {
      boxes[4 * s.index] = uint32_t(s.x);
      boxes[4 * s.index + 1] = uint32_t(s.y);
      boxes[4 * s.index + 2] = uint32_t(s.width);
      boxes[4 * s.index + 3] = uint32_t(s.height);
      for (size_t y = 0; y != s.height; ++y)
        for (size_t x = 0; x != s.width; ++x)
          if (s.boundary_mask[y * s.width + x])
            labels[(y + s.y) * w + x + s.x] = uint16_t(s.index + 1);
    }
    return 0;
  } catch (std::exception& e) {
    g_error = e.what();
    return 1;
  }
}

void* orc_parallel_create(int kind, const orc_algo_settings* a, uint64_t grid_w,
                          uint64_t grid_h) {
  auto* p = new OrcParallel();
  p->grid_w = grid_w;
  p->grid_h = grid_h;
  p->algorithms.resize(grid_w * grid_h);
  for (TiledAlgorithm& t : p->algorithms) {
    t.kind = kind;
    t.settings = MakeSettings(a);
    t.settings.clean_mask = nullptr;
  }
  return p;
}

void orc_parallel_destroy(void* h) { delete static_cast<OrcParallel*>(h); }

// DeconvolutionAlgorithm::SetRmsFactorImage (deconvolution_algorithm.h:163-166);
// factor == nullptr clears it
void orc_algo_set_rms(void* h, const float* factor, uint64_t n) {
  auto* algo = static_cast<OrcAlgo*>(h);
  if (factor)
    algo->rms_factor.assign(factor, factor + n);
  else
    algo->rms_factor.clear();
}

// DeconvolutionAlgorithm::SetComponentOptimizationAlgorithm (0 clean, 2 gradient
// descent; generic clean only)
void orc_algo_set_component_optimization(void* h, int algorithm) {
  static_cast<OrcAlgo*>(h)->component_optimization = algorithm;
}

// ParallelDeconvolution::SetRmsFactorImage (parallel_deconvolution.cc:244-250)
void orc_parallel_set_rms(void* h, const float* factor, uint64_t n) {
  auto* p = static_cast<OrcParallel*>(h);
  if (factor)
    p->masks.rms_factor.assign(factor, factor + n);
  else
    p->masks.rms_factor.clear();
}

// Radler::Perform's local-RMS step (cpp/radler.cc:196-216): method 1 =
// kRmsWindow, 2 = kRmsAndMinimumWindow; factor receives the RMS factor image
// and *lowest_rms the value MakeRmsFactorImage returns. rms (may be NULL)
// receives the RMS image before the factor conversion.
int orc_local_rms(const float* integrated, uint64_t width, uint64_t height, int method,
                  double window, double beam, double pixel_scale_x, double pixel_scale_y,
                  double strength, float* rms, float* factor, double* lowest_rms) {
  try {
    std::vector<float> img(width * height);
    if (method == 1)
      RmsImageMake(img.data(), integrated, width, height, window, beam, beam, 0.0L,
                   pixel_scale_x, pixel_scale_y);
    else
      RmsImageMakeWithNegativityLimit(img.data(), integrated, width, height, window,
                                      beam, beam, 0.0L, pixel_scale_x, pixel_scale_y);
    if (rms) std::copy(img.begin(), img.end(), rms);
    *lowest_rms = MakeRmsFactorImage(img.data(), img.size(), strength);
    std::copy(img.begin(), img.end(), factor);
    return 0;
  } catch (const std::exception& e) {
    g_error = e.what();
    return 1;
  }
}

// GenericClean's RunComponentOptimization with kGradientDescent for one
// image (generic_clean.cc:26-48): model += GradientDescent(model, residual,
// psf, 2W x 2H, FFT).
void orc_gradient_descent(float* model, const float* residual, const float* psf,
                          uint64_t width, uint64_t height) {
  GradientDescent(model, residual, psf, width, height, 2 * width, 2 * height);
}

void orc_linear_component_solve(float* model, const float* image, const float* psf,
                                uint64_t width, uint64_t height) {
  LinearComponentSolve(model, image, psf, width, height);
}

// GradientDescentWithVariablePsf: n_psfs lists (counts[p] positions each, x,y
// pairs concatenated), psfs [n_psfs][h][w]; deltas [n_psfs][h][w]
void orc_gradient_descent_variable_psf(const uint32_t* positions, const uint64_t* counts,
                                       uint64_t n_psfs, const float* image,
                                       const float* psfs, uint64_t width, uint64_t height,
                                       uint64_t padded_width, uint64_t padded_height,
                                       float* deltas) {
  std::vector<std::vector<std::pair<size_t, size_t>>> lists(n_psfs);
  std::vector<std::vector<float>> psf_images;
  const size_t n = width * height;
  for (uint64_t p = 0; p != n_psfs; ++p) {
    for (uint64_t i = 0; i != counts[p]; ++i, positions += 2)
      lists[p].emplace_back(positions[0], positions[1]);
    psf_images.emplace_back(psfs + p * n, psfs + (p + 1) * n);
  }
  const std::vector<std::vector<float>> d = GradientDescentWithVariablePsf(
      lists, image, psf_images, width, height, padded_width, padded_height);
  for (uint64_t p = 0; p != n_psfs; ++p) std::copy(d[p].begin(), d[p].end(), deltas + p * n);
}

double orc_make_rms_factor_image(float* rms, uint64_t n, double strength) {
  return MakeRmsFactorImage(rms, n, strength);
}

void orc_padded_convolution(float* image, const float* psf, uint64_t width,
                            uint64_t height, uint64_t padded_width, uint64_t padded_height) {
  PaddedConvolution(image, psf, width, height, padded_width, padded_height);
}

void orc_sliding_minimum(const float* input, uint64_t width, uint64_t height,
                         uint64_t window, float* output) {
  SlidingMinimum(output, input, width, height, window);
}

// ParallelDeconvolution::SetAutoMaskMode (parallel_deconvolution.cc:260-268)
void orc_parallel_set_automask(void* h, int track, int use) {
  auto* p = static_cast<OrcParallel*>(h);
  p->masks.track = track != 0;
  p->masks.use = use != 0;
}

// SetThreshold / SetMinorLoopGain / ... on every subimage algorithm (their
// iteration counts and multiscale state are kept)
void orc_parallel_update(void* h, const orc_algo_settings* a) {
  auto* p = static_cast<OrcParallel*>(h);
  for (TiledAlgorithm& t : p->algorithms) t.settings = MakeSettings(a);
}

// 1: subimages of a pass all trim the residual as it was at the start of the
// pass (the product's concurrent subimage pool, max_threads > 1)
void orc_parallel_set_snapshot(void* h, int snapshot) {
  static_cast<OrcParallel*>(h)->snapshot = snapshot != 0;
}

// sub_boxes: 4 x u32 (x, y, w, h) per subimage; labels (may be NULL): W*H
// u16, subimage index + 1 where the pixel is in that subimage's boundary
// mask; trace: 4 x u32 (subimage, x, y, scale) per component of the run pass.
int orc_parallel_execute(void* h, const orc_set_desc* d, float* residual,
                         float* model, const float* psfs, double major_loop_gain,
                         const uint8_t* user_mask, orc_parallel_result* out,
                         uint32_t* sub_boxes, uint16_t* labels, uint32_t* trace,
                         uint64_t trace_cap) {
  try {
    auto* p = static_cast<OrcParallel*>(h);
    SetDesc desc = MakeDesc(d);
    ImageSet res = MakeSet(desc, d, residual);
    ImageSet mod = MakeSet(desc, d, model);
    std::vector<const float*> psf_ptrs;
    for (uint64_t c = 0; c != d->n_channels; ++c)
      psf_ptrs.push_back(psfs + c * d->width * d->height);
    std::vector<SubImage> subs;
    std::vector<std::vector<Component>> traces;
    const double limit = p->algorithms.front().settings.divergence_limit;
    ParallelResult r = ParallelRun(p->algorithms, p->grid_w, p->grid_h, desc, res,
                                   mod, psf_ptrs, major_loop_gain, limit,
                                   reinterpret_cast<const bool*>(user_mask), &subs,
                                   &traces, p->snapshot, &p->masks);
    out->another_iteration_required = r.another_iteration_required;
    out->n_subimages = int32_t(subs.size());
    out->start_peak = r.start_peak;
    out->end_peak = r.end_peak;
    out->first_iteration_number = p->algorithms.front().iteration_number;
    out->total_iterations = 0;
    for (const TiledAlgorithm& t : p->algorithms)
      out->total_iterations += t.iteration_number;
    if (labels) std::fill(labels, labels + d->width * d->height, uint16_t(0));
    uint64_t n_trace = 0;
    p->margins.clear();
    p->values.clear();
    p->end_margins.assign(subs.size(), std::numeric_limits<float>::infinity());
    for (const SubImage& s : subs) {
      p->end_margins[s.index] = s.end_margin;
      for (const Component& c : traces[s.index]) {
        p->margins.push_back(c.margin);
        p->values.push_back(c.value);
      }
    }
    for (const SubImage& s : subs) {
      if (sub_boxes) {
        sub_boxes[4 * s.index] = uint32_t(s.x);
        sub_boxes[4 * s.index + 1] = uint32_t(s.y);
        sub_boxes[4 * s.index + 2] = uint32_t(s.width);
        sub_boxes[4 * s.index + 3] = uint32_t(s.height);
      }
      if (labels)
        for (size_t y = 0; y != s.height; ++y)
          for (size_t x = 0; x != s.width; ++x)
            if (s.boundary_mask[y * s.width + x])
              labels[(y + s.y) * d->width + x + s.x] = uint16_t(s.index + 1);
      for (const Component& c : traces[s.index]) {
        if (trace && n_trace < trace_cap) {
          trace[4 * n_trace] = uint32_t(s.index);
          trace[4 * n_trace + 1] = c.x;
          trace[4 * n_trace + 2] = c.y;
          trace[4 * n_trace + 3] = c.scale;
        }
        ++n_trace;
      }
    }
    out->n_trace = n_trace;
    return 0;
  } catch (std::exception& e) {
    g_error = e.what();
    return 1;
  }
}

}  // extern "C"

extern "C" {

// SpectralFitter::FitAndEvaluate on one spectrum (n channels), and the fit's
// terms (n_terms floats) when terms != nullptr.
void orc_spectral_fit(int mode, uint32_t n_terms, const double* frequencies,
                      const float* weights, uint64_t n, float* values, float* terms) {
  const SpectralFit fit(mode, n_terms, std::vector<double>(frequencies, frequencies + n),
                        std::vector<float>(weights, weights + n));
  if (terms) {
    std::vector<float> t;
    fit.Fit(t, values);
    std::copy(t.begin(), t.end(), terms);
  }
  fit.FitAndEvaluate(values);
}

// ImageSet::InterpolateAndStoreModel (cpp/image_set.cc:209-288) for one
// polarization: in = n_channels deconvolution planes, out = n_out planes at
// out_frequencies. Zero pixels are not fitted (their terms are zero).
void orc_spectral_interpolate(int mode, uint32_t n_terms, const double* frequencies,
                              const float* weights, uint64_t n_channels,
                              const float* in, uint64_t n_pixels,
                              const double* out_frequencies, uint64_t n_out,
                              float* out) {
  const SpectralFit fit(mode, n_terms,
                        std::vector<double>(frequencies, frequencies + n_channels),
                        std::vector<float>(weights, weights + n_channels));
  std::vector<float> pixel(n_channels), terms;
  std::vector<float> terms_image(n_pixels * n_terms);
  for (uint64_t px = 0; px != n_pixels; ++px) {
    bool is_zero = true;
    for (uint64_t c = 0; c != n_channels; ++c) {
      pixel[c] = in[c * n_pixels + px];
      is_zero = is_zero && pixel[c] == 0.0f;
    }
    float* t = &terms_image[px * n_terms];
    if (is_zero) {
      std::fill_n(t, n_terms, 0.0f);
    } else {
      fit.Fit(terms, pixel.data());
      std::copy_n(terms.begin(), n_terms, t);
    }
  }
  for (uint64_t g = 0; g != n_out; ++g)
    for (uint64_t px = 0; px != n_pixels; ++px) {
      const std::vector<float> t(&terms_image[px * n_terms],
                                 &terms_image[px * n_terms] + n_terms);
      out[g * n_pixels + px] = fit.Evaluate(t, out_frequencies[g]);
    }
}

}  // extern "C"

extern "C" {
// MultiScaleAlgorithm::RunFullComponentFitter for one image: positions are
// (x, y) pairs, counts[s] of them for scale s, in scale order.
void orc_ms_full_component_fitter(float* residual, float* model, const float* psf,
                                  uint64_t width, uint64_t height, const float* scales,
                                  uint64_t n_scales, const uint32_t* positions,
                                  const uint64_t* counts, double padding, int shape) {
  std::vector<std::vector<std::pair<size_t, size_t>>> lists(n_scales);
  size_t k = 0;
  for (uint64_t s = 0; s != n_scales; ++s)
    for (uint64_t i = 0; i != counts[s]; ++i, ++k)
      lists[s].emplace_back(positions[2 * k], positions[2 * k + 1]);
  RunFullComponentFitter(residual, model, psf, width, height,
                         std::vector<float>(scales, scales + n_scales), lists, padding, shape);
}
}  // extern "C"

// Margins of the last orc_parallel_execute: n_trace entries in trace order,
// then one end margin per subimage; returns the total count.
// `values` (may be NULL): the components' |peak| (end entries: 0).
extern "C" uint64_t orc_parallel_margins(void* h, float* out, float* values,
                                         uint64_t cap) {
  auto* p = static_cast<OrcParallel*>(h);
  std::vector<float> all = p->margins;
  all.insert(all.end(), p->end_margins.begin(), p->end_margins.end());
  std::vector<float> vals = p->values;
  vals.resize(all.size(), 0.0f);
  const size_t n = std::min<size_t>(cap, all.size());
  std::copy_n(all.data(), n, out);
  if (values) std::copy_n(vals.data(), n, values);
  return all.size();
}
