// MultiScaleAlgorithm on the device. Line references are to the reference's
// cpp/algorithms/multiscale_algorithm.cc unless stated.
#include "multiscale_algorithm.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <optional>
#include <set>
#include <stdexcept>

#include "communicator.h"
#include "component_optimization.h"
#include "fft_sizes.h"
#include "host_profile.h"
#include "logger.h"
#include "subminor.h"

namespace radler::algorithms {

using multiscale::MultiScaleTransforms;

namespace {
// RDL_SCALE_LANES=1: the scales' inverse transforms on one stream (default 2;
// read per major iteration, so a test can compare both in one process)
int ScaleLanes() {
  const char* e = std::getenv("RDL_SCALE_LANES");
  return e && e[0] == '1' ? 1 : 2;
}

// RDL_FUSED_SCALES=0: the scales' convolutions through the forward spectrum
// and one two-pass column inverse each instead of the fused multi-scale
// launch (read per call, for comparisons)
// RDL_SUBMINOR_DEFER=0: read each sub-minor loop's result before queuing the
// correction (comparison)
bool DeferLoopResult() {
  static const bool on = [] {
    const char* e = std::getenv("RDL_SUBMINOR_DEFER");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool FusedScalesOn() {
  const char* e = std::getenv("RDL_FUSED_SCALES");
  return !(e && e[0] == '0');
}

// joins the session's second lane if a scope exits while it is selected
struct LaneJoin {
  rdl_session* s;
  bool& forked;
  ~LaneJoin() {
    if (forked) (void)rdl_session_join(s);
  }
};
}  // namespace

void InitializeScales(std::vector<MultiScaleAlgorithm::ScaleInfo>& scales,
                      double beam_size_in_pixels, size_t min_width_height,
                      MultiscaleShape shape, size_t max_scales,
                      const std::vector<double>& scale_list) {  // :90-131
  if (scale_list.empty()) {
    if (scales.empty()) {
      size_t scale_index = 0;
      double scale = beam_size_in_pixels * 2.0;
      do {
        MultiScaleAlgorithm::ScaleInfo& e = scales.emplace_back();
        e.scale = scale_index == 0 ? 0.0f : float(scale);
        e.kernel_peak =
            MultiScaleTransforms::KernelPeakValue(scale, min_width_height, shape);
        scale *= 2.0;
        ++scale_index;
      } while (scale < min_width_height * 0.5 &&
               (max_scales == 0 || scale_index < max_scales));
    } else {
      while (!scales.empty() && scales.back().scale >= min_width_height * 0.5) {
        log::Info() << "Scale size " << scales.back().scale
                    << " does not fit in cleaning region: removing scale.\n";
        scales.pop_back();
      }
    }
  } else if (scales.empty()) {
    std::multiset<double> sorted(scale_list.begin(), scale_list.end());
    for (double s : sorted) {
      MultiScaleAlgorithm::ScaleInfo& e = scales.emplace_back();
      e.scale = float(s);
      e.kernel_peak =
          MultiScaleTransforms::KernelPeakValue(e.scale, min_width_height, shape);
    }
  }
}

std::optional<size_t> SelectMaximumScale(
    const std::vector<MultiScaleAlgorithm::ScaleInfo>& scales) {  // :133-151
  std::map<float, size_t> peak_to_scale;
  for (size_t i = 0; i != scales.size(); ++i)
    if (scales[i].is_active)
      peak_to_scale.insert(std::make_pair(
          std::fabs(scales[i].max_unnormalized_image_value *
                    scales[i].bias_factor),
          i));
  if (peak_to_scale.empty()) return std::nullopt;
  return peak_to_scale.rbegin()->second;
}

MultiScaleAlgorithm::MultiScaleAlgorithm(const Settings::Multiscale& settings,
                                         double beam_size, double pixel_scale_x,
                                         double pixel_scale_y,
                                         bool track_components)
    : settings_(settings),
      beam_size_in_pixels_(beam_size / std::max(pixel_scale_x, pixel_scale_y)),
      track_components_(track_components) {
  if (!(beam_size_in_pixels_ > 0.0)) beam_size_in_pixels_ = 1;  // :162
}

MultiScaleAlgorithm::MultiScaleAlgorithm(const MultiScaleAlgorithm& o)
    : DeconvolutionAlgorithm(o),
      settings_(o.settings_),
      beam_size_in_pixels_(o.beam_size_in_pixels_),
      track_components_(o.track_components_),
      component_list_(o.component_list_ ? std::make_unique<ComponentList>(*o.component_list_)
                                        : nullptr),
      scale_infos_(o.scale_infos_),
      track_masks_(o.track_masks_),
      use_masks_(o.use_masks_),
      host_masks_(o.host_masks_) {}

void MultiScaleAlgorithm::UploadScaleMasks(gpu::Session& s, size_t n_pixels) {
  if (!masks_dirty_ && masks_session_ == &s && dev_masks_.size() == host_masks_.size())
    return;
  dev_masks_.clear();
  for (const std::vector<uint8_t>& m : host_masks_) {
    gpu::Buffer& b = dev_masks_.emplace_back(s, n_pixels);
    if (m.size() == n_pixels)
      s.H2D(b.Ptr(), m.data(), n_pixels);
    else
      b.Zero();
  }
  masks_session_ = &s;
  masks_dirty_ = false;
}

void MultiScaleAlgorithm::DownloadScaleMasks() {
  if (!masks_session_) return;
  for (size_t i = 0; i != host_masks_.size() && i != dev_masks_.size(); ++i)
    masks_session_->D2H(host_masks_[i].data(), dev_masks_[i].Ptr(), host_masks_[i].size());
}

void MultiScaleAlgorithm::RunFullComponentFitter(ImageSet& residual_set,
                                                 ImageSet& model_set,
                                                 const gpu::Planes& psfs) {
  // :916-929 over the images, :837-914 per image
  if (ComponentOptimizationAlgorithm() != OptimizationAlgorithm::kGradientDescent)
    throw std::runtime_error(
        "Unsupported optimization algorithm for multiscale clean algorithm");
  if (!component_list_)
    throw std::runtime_error(
        "Multiscale component optimisation fits the component list: it needs "
        "save_source_list");
  gpu::Session& s = residual_set.Session();
  const size_t width = residual_set.Width(), height = residual_set.Height();
  if (!transforms_ || !transforms_->BoundTo(s) || transforms_->Width() != width ||
      transforms_->Height() != height)
    transforms_ = std::make_unique<MultiScaleTransforms>(s, width, height, settings_.shape);
  std::vector<float> scales;
  std::vector<std::vector<std::pair<size_t, size_t>>> lists(scale_infos_.size());
  for (size_t sc = 0; sc != scale_infos_.size(); ++sc) {
    scales.push_back(scale_infos_[sc].scale);
    if (sc < component_list_->NScales())
      for (size_t i = 0; i != component_list_->ComponentCount(sc); ++i)
        lists[sc].push_back(component_list_->GetComponentPosition(sc, i));
  }
  const size_t pw = utils::GetConvolutionSize(scales.back(), width,
                                              settings_.convolution_padding);
  const size_t ph = utils::GetConvolutionSize(scales.back(), height,
                                              settings_.convolution_padding);
  std::vector<float> model(width * height);
  for (size_t i = 0; i != residual_set.Size(); ++i) {
    // :885-897 ("Updating component list") runs before :898-905 ("Updating
    // model"): the list values take the model image's values from before
    // this fit's deltas are added
    s.D2H(model.data(), model_set.Data(i), model.size() * sizeof(float));
    for (size_t sc = 0; sc != lists.size(); ++sc)
      for (size_t c = 0; c != lists[sc].size(); ++c)
        component_list_->Value(sc, c, i) +=
            model[lists[sc][c].second * width + lists[sc][c].first];
    math::RunFullComponentFitter(s, residual_set.Data(i), model_set.Data(i),
                                 psfs.Plane(residual_set.PsfIndex(i)), width, height, scales,
                                 lists, *transforms_, pw, ph);
  }
  // ApplySpectralConstraintsToComponents (deconvolution_algorithm.cc:48-64)
  std::vector<float> values(component_list_->NFrequencies());
  for (size_t sc = 0; sc != component_list_->NScales(); ++sc)
    for (size_t c = 0; c != component_list_->ComponentCount(sc); ++c) {
      size_t x, y;
      component_list_->GetComponent(sc, c, x, y, values.data());
      PerformSpectralFit(values.data(), x, y);
      for (size_t f = 0; f != values.size(); ++f) component_list_->Value(sc, c, f) = values[f];
    }
}

const float* MultiScaleAlgorithm::PeakSearchInput(const float* d_image, size_t w,
                                                 size_t h) {
  if (!RmsFactorImage()) return d_image;
  if (!rms_scratch_ || rms_scratch_->Bytes() < w * h * sizeof(float))
    rms_scratch_ = std::make_shared<gpu::Buffer>(*session_, w * h * sizeof(float));
  return RmsWeighted(*session_, d_image, rms_scratch_->F(), w, h);
}

float MultiScaleAlgorithm::Normalized(float value, size_t x, size_t y, size_t w) const {
  if (!RmsFactorImage()) return value;
  return value / (*RmsFactorImage())[x + y * w];
}

void MultiScaleAlgorithm::FindPeakDirect(const float* d_image,
                                         size_t scale_index) {  // :700-748
  prof::Section prof_section("ms.find_peak_direct");
  ScaleInfo& info = scale_infos_[scale_index];
  const size_t w = transforms_->Width(), h = transforms_->Height();
  d_image = PeakSearchInput(d_image, w, h);
  const uint32_t hb = uint32_t(std::round(w * CleanBorderRatio()));
  const uint32_t vb = uint32_t(std::round(h * CleanBorderRatio()));
  rdl_peak p;
  gpu::Check(rdl_find_peak(session_->Handle(), d_image, uint32_t(w), uint32_t(h),
                           0, uint32_t(h), hb, vb, AllowNegativeComponents(),
                           MaskFor(scale_index), 1, &p),
             "rdl_find_peak");
  info.max_image_value_x = p.x;
  info.max_image_value_y = p.y;
  info.max_unnormalized_image_value = p.found ? p.value : 0.0f;
  info.max_normalized_image_value = p.found ? Normalized(p.value, p.x, p.y, w) : 0.0f;
}

void MultiScaleAlgorithm::FindActiveScaleConvolvedMaxima(
    const ImageSet& image_set, float* d_integrated, bool report_rms) {
  prof::Section prof_section("ms.find_maxima");
  // :578-634 with ThreadedDeconvolutionTools::FindMultiScalePeak /
  // FindSingleScalePeak (threaded_deconvolution_tools.cc:30-107): one forward
  // FFT of the integrated image feeds every active scale.
  rdl_session* s = session_->Handle();
  const size_t w = image_set.Width(), h = image_set.Height();
  const bool identity = image_set.Size() == 1 && image_set.Integration(false).copy_fast_path;
  scale_image_valid_.assign(scale_infos_.size(), false);
  if (identity && scale_images_.size() != scale_infos_.size())
    scale_images_.assign(scale_infos_.size(), gpu::Planes());
  // one image whose integration is the identity: the searches and the
  // forward transform read the residual itself (no integrated copy)
  const float* d_source = d_integrated;
  if (identity)
    d_source = image_set.Data(0);
  else
    image_set.GetLinearIntegrated(d_integrated);
  bool need_fft = false;
  const bool fused_search = !report_rms && !RmsFactorImage();
  // the scale-0 search: queued with the other scales' (one read-back for
  // all) when the convolved scales' searches are queued too
  int direct = -1;
  for (size_t si = 0; si != scale_infos_.size(); ++si) {
    ScaleInfo& e = scale_infos_[si];
    if (!e.is_active) continue;
    if (e.scale == 0.0f) {
      if (fused_search) {
        direct = int(si);
        continue;
      }
      FindPeakDirect(d_source, si);
      if (report_rms)
        gpu::Check(rdl_rms(s, d_source, w * h, &e.rms), "rdl_rms");
    } else {
      need_fft = true;
    }
  }
  if (!need_fft) {
    if (direct >= 0) FindPeakDirect(d_source, size_t(direct));
    return;
  }
  if (scale_infos_.size() + 1 > RDL_PEAK_SLOTS)
    throw std::runtime_error("MultiScaleAlgorithm: too many scales");
  std::vector<size_t> pending;  // scale of each queued peak search (slot = index)
  if (direct >= 0) {  // FindPeakDirect's search (:700-748), collected below
    const uint32_t hb = uint32_t(std::round(w * CleanBorderRatio()));
    const uint32_t vb = uint32_t(std::round(h * CleanBorderRatio()));
    gpu::Check(rdl_find_peak_enqueue(s, d_source, uint32_t(w), uint32_t(h), 0, uint32_t(h), hb,
                                     vb, AllowNegativeComponents(), MaskFor(size_t(direct)), 1,
                                     0),
               "rdl_find_peak_enqueue");
    pending.push_back(size_t(direct));
  }
  if (fused_search && FusedScalesOn() && transforms_->Fused()) {
    FindMaximaFused(d_source, identity, pending);
    return;
  }
  transforms_->Forward(d_source, spectrum_->Ptr());
  // The scales' inverse transforms + fused peak searches are independent
  // (the reference runs them on threads, threaded_deconvolution_tools.cc):
  // with a kept image per scale they alternate over two session lanes, so
  // one scale's latency-bound row pass overlaps the next one's column
  // passes. Every buffer a lane writes is its own (work spectrum, four-step
  // scratch, peak partials slot, scale image); the kernel spectra and the
  // scale images are made before the fork (no allocation on lane 1).
  bool forked = false;
  if (identity && fused_search && spectrum_work2_) {
    size_t n_fft = 0;
    for (size_t si = 0; si != scale_infos_.size(); ++si) {
      const ScaleInfo& e = scale_infos_[si];
      if (!e.is_active || e.scale == 0.0f) continue;
      transforms_->KernelSpectrum(e.scale);
      ++n_fft;
    }
    if (n_fft > 1) {
      for (size_t si = 0; si != scale_infos_.size(); ++si) {
        const ScaleInfo& e = scale_infos_[si];
        if (!e.is_active || e.scale == 0.0f) continue;
        gpu::Planes& kept = scale_images_[si];
        if (!kept.buffer || kept.width != w || kept.height != h)
          kept = gpu::Planes::Make(*session_, w, h, 1);
      }
      gpu::Check(rdl_session_fork(s), "rdl_session_fork");
      forked = true;
    }
  }
  LaneJoin lane_join{s, forked};
  int lane = 0;
  for (size_t si = 0; si != scale_infos_.size(); ++si) {
    ScaleInfo& e = scale_infos_[si];
    if (!e.is_active || e.scale == 0.0f) continue;
    float* d_conv = scratch_->F();
    if (identity) {
      gpu::Planes& kept = scale_images_[si];
      if (!kept.buffer || kept.width != w || kept.height != h)
        kept = gpu::Planes::Make(*session_, w, h, 1);
      d_conv = kept.Base();
      scale_image_valid_[si] = true;
    }
    const size_t border_scale = size_t(std::ceil(e.scale * 0.5));
    const uint32_t xb = uint32_t(
        std::max<size_t>(size_t(std::round(w * CleanBorderRatio())), border_scale));
    const uint32_t yb = uint32_t(
        std::max<size_t>(size_t(std::round(h * CleanBorderRatio())), border_scale));
    if (forked) {
      gpu::Check(rdl_session_lane(s, lane), "rdl_session_lane");
      void* work = lane ? spectrum_work2_->Ptr() : spectrum_work_->Ptr();
      if (transforms_->ConvolveSpectrumPeak(spectrum_->Ptr(), e.scale, work, d_conv, xb, yb,
                                            AllowNegativeComponents(), MaskFor(si),
                                            uint32_t(pending.size()))) {
        pending.push_back(si);
        lane ^= 1;
        continue;
      }
      // no fused kernels for this size (nothing was issued): lane 0 from here
      forked = false;
      gpu::Check(rdl_session_join(s), "rdl_session_join");
    }
    // the peak search fused into the inverse row pass where it can be (the
    // RMS-weighted search reads a weighted copy, so it stays separate)
    if (fused_search &&
        transforms_->ConvolveSpectrumPeak(spectrum_->Ptr(), e.scale, spectrum_work_->Ptr(),
                                          d_conv, xb, yb, AllowNegativeComponents(),
                                          MaskFor(si), uint32_t(pending.size()))) {
      pending.push_back(si);
      continue;
    }
    transforms_->ConvolveSpectrum(spectrum_->Ptr(), e.scale, spectrum_work_->Ptr(),
                                  d_conv);
    if (report_rms)
      gpu::Check(rdl_rms(s, d_conv, w * h, &e.rms), "rdl_rms");
    // the scales' searches queue back to back; one read collects them
    gpu::Check(rdl_find_peak_enqueue(s, PeakSearchInput(d_conv, w, h), uint32_t(w),
                                     uint32_t(h), 0, uint32_t(h), xb, yb,
                                     AllowNegativeComponents(), MaskFor(si), 1,
                                     uint32_t(pending.size())),
               "rdl_find_peak_enqueue");
    pending.push_back(si);
  }
  if (forked) {
    forked = false;
    gpu::Check(rdl_session_join(s), "rdl_session_join");
  }
  std::vector<rdl_peak> peaks(pending.size());
  gpu::Check(rdl_find_peak_collect(s, uint32_t(pending.size()), peaks.data()),
             "rdl_find_peak_collect");
  for (size_t k = 0; k != pending.size(); ++k) {
    ScaleInfo& e = scale_infos_[pending[k]];
    const rdl_peak& p = peaks[k];
    e.max_normalized_image_value = p.found ? Normalized(p.value, p.x, p.y, w) : 0.0f;
    e.max_unnormalized_image_value = p.found ? p.value : 0.0f;
    e.max_image_value_x = p.x;
    e.max_image_value_y = p.y;
  }
}

void MultiScaleAlgorithm::FindMaximaFused(const float* d_source, bool identity,
                                          std::vector<size_t> pending) {
  // The same searches as below, with the scales' convolutions made from ONE
  // forward half by one launch (rdl_conv_scales: the forward spectrum never
  // reaches HBM, the scale kernels are real), then per scale the outer
  // inverse step and the inverse rows with the fused peak search,
  // alternating over two lanes as below.
  rdl_session* s = session_->Handle();
  const size_t w = transforms_->Width(), h = transforms_->Height();
  std::vector<size_t> idx;
  std::vector<float> scales;
  for (size_t si = 0; si != scale_infos_.size(); ++si) {
    const ScaleInfo& e = scale_infos_[si];
    if (!e.is_active || e.scale == 0.0f) continue;
    idx.push_back(si);
    scales.push_back(e.scale);
  }
  // every buffer and kernel spectrum before any fork (no allocation on lane 1)
  const size_t sb = transforms_->SpectrumBytes();
  while (scale_u_.size() < idx.size())
    scale_u_.push_back(std::make_shared<gpu::Buffer>(*session_, sb));
  std::vector<void*> outs;
  for (size_t k = 0; k != idx.size(); ++k) outs.push_back(scale_u_[k]->Ptr());
  for (float sc : scales) transforms_->RealKernelSpectrum(sc);
  std::vector<float*> conv(idx.size(), scratch_->F());
  if (identity)
    for (size_t k = 0; k != idx.size(); ++k) {
      gpu::Planes& kept = scale_images_[idx[k]];
      if (!kept.buffer || kept.width != w || kept.height != h)
        kept = gpu::Planes::Make(*session_, w, h, 1);
      conv[k] = kept.Base();
      scale_image_valid_[idx[k]] = true;
    }
  transforms_->ForwardHalf(d_source, spectrum_->Ptr());
  transforms_->Scales(spectrum_->Ptr(), scales, outs);
  // two lanes only with one image per scale (identity: kept images)
  bool forked = false;
  if (identity && idx.size() > 1 && spectrum_work2_) {
    gpu::Check(rdl_session_fork(s), "rdl_session_fork");
    forked = true;
  }
  LaneJoin lane_join{s, forked};
  int lane = 0;
  for (size_t k = 0; k != idx.size(); ++k) {
    const ScaleInfo& e = scale_infos_[idx[k]];
    const size_t border_scale = size_t(std::ceil(e.scale * 0.5));
    const uint32_t xb = uint32_t(
        std::max<size_t>(size_t(std::round(w * CleanBorderRatio())), border_scale));
    const uint32_t yb = uint32_t(
        std::max<size_t>(size_t(std::round(h * CleanBorderRatio())), border_scale));
    if (forked) gpu::Check(rdl_session_lane(s, lane), "rdl_session_lane");
    void* work = lane ? spectrum_work2_->Ptr() : spectrum_work_->Ptr();
    transforms_->FinishPeak(outs[k], e.scale, work, conv[k], xb, yb, AllowNegativeComponents(),
                            MaskFor(idx[k]), uint32_t(pending.size()));
    pending.push_back(idx[k]);
    if (forked) lane ^= 1;
  }
  if (forked) {
    forked = false;
    gpu::Check(rdl_session_join(s), "rdl_session_join");
  }
  std::vector<rdl_peak> peaks(pending.size());
  gpu::Check(rdl_find_peak_collect(s, uint32_t(pending.size()), peaks.data()),
             "rdl_find_peak_collect");
  for (size_t k = 0; k != pending.size(); ++k) {
    ScaleInfo& e = scale_infos_[pending[k]];
    const rdl_peak& p = peaks[k];
    e.max_normalized_image_value = p.found ? Normalized(p.value, p.x, p.y, w) : 0.0f;
    e.max_unnormalized_image_value = p.found ? p.value : 0.0f;
    e.max_image_value_x = p.x;
    e.max_image_value_y = p.y;
  }
}

void MultiScaleAlgorithm::ActivateScales(size_t last) {  // :636-656
  for (size_t i = 0; i != scale_infos_.size(); ++i) {
    const bool activate =
        i == last ||
        std::fabs(scale_infos_[i].max_unnormalized_image_value) *
                scale_infos_[i].bias_factor >
            std::fabs(scale_infos_[last].max_unnormalized_image_value) *
                (1.0 - MinorLoopGain()) * scale_infos_[last].bias_factor;
    scale_infos_[i].is_active = activate;
  }
}

DeconvolutionResult MultiScaleAlgorithm::ExecuteMajorIteration(
    ImageSet& data_image, ImageSet& model_image, const gpu::Planes& psfs) {
  prof::Section prof_section("ms.execute");
  gpu::Session& session = data_image.Session();
  session_ = &session;
  rdl_session* s = session.Handle();
  const size_t width = data_image.Width();
  const size_t height = data_image.Height();
  const size_t npx = width * height;
  trace_.clear();
  if (StopOnNegativeComponents()) SetAllowNegativeComponents(true);
  InitializeScales(scale_infos_, beam_size_in_pixels_, std::min(width, height),
                   settings_.shape, settings_.max_scales, settings_.scale_list);
  if (track_components_) {  // :228-236
    if (!component_list_)
      component_list_ = std::make_unique<ComponentList>(width, height, scale_infos_.size(),
                                                        data_image.Size());
    else if (component_list_->Width() != width || component_list_->Height() != height)
      throw std::runtime_error("Error in component list dimensions!");
  }
  if (track_masks_) {  // :214-226
    for (const std::vector<uint8_t>& m : host_masks_)
      if (m.size() != npx)
        throw std::runtime_error("Invalid automask size in multiscale algorithm");
    while (host_masks_.size() < scale_infos_.size()) {
      host_masks_.emplace_back(npx, 0);
      masks_dirty_ = true;
    }
  }
  if (track_masks_ || use_masks_) UploadScaleMasks(session, npx);
  // the tracked masks go back to the host copies on every return
  struct MaskSync {
    MultiScaleAlgorithm* a;
    ~MaskSync() {
      if (a->track_masks_) a->DownloadScaleMasks();
    }
  } mask_sync{this};
  if (ComponentOptimizationAlgorithm() != OptimizationAlgorithm::kClean) {  // :242-246
    RunFullComponentFitter(data_image, model_image, psfs);
    return DeconvolutionResult{};
  }

  bool has_hit_threshold_in_sub_loop = false;
  size_t threshold_countdown = std::max(size_t{8}, scale_infos_.size() * 3 / 2);
  // joined channels over the ranks of shard_ (SetChannelShard): image i's
  // residual correction and model update run on rank i % size only
  const int n_ranks = shard_ ? shard_->Size() : 1;
  const int my_rank = shard_ ? shard_->Rank() : 0;
  const bool sharded = n_ranks > 1 && data_image.Size() > 1;
  auto owner = [&](size_t i) { return sharded ? int(i % size_t(n_ranks)) : my_rank; };
  // the owners' planes to every rank (stream-ordered on the session; the
  // ranks issue the same broadcasts in the same order)
  auto share_planes = [&](ImageSet& set) {
    if (!sharded) return;
    prof::Section prof_share("ms.shard_broadcast");
    for (size_t i = 0; i != set.Size(); ++i)
      shard_->Broadcast(session, set.Data(i), npx * sizeof(float), owner(i));
  };

  // rebuilt when another worker session runs this subimage (the ranks'
  // ownership, parallel_deconvolution.cc, changes between major iterations)
  if (!transforms_ || !transforms_->BoundTo(session) || transforms_->Width() != width ||
      transforms_->Height() != height)
    transforms_ = std::make_unique<MultiScaleTransforms>(session, width, height,
                                                         settings_.shape);
  {
    float max_scale = 0.0f;
    for (const ScaleInfo& e : scale_infos_) max_scale = std::max(max_scale, e.scale);
    transforms_->SetMaxScale(max_scale);
  }
  d_mask_ = DeviceCleanMask(session, width, height);
  scratch_ = std::make_shared<gpu::Buffer>(session, npx * sizeof(float));
  gpu::Buffer integrated(session, npx * sizeof(float));
  const size_t spectrum_bytes = transforms_->SpectrumBytes();
  spectrum_ = std::make_shared<gpu::Buffer>(session, spectrum_bytes);
  spectrum_work_ = std::make_shared<gpu::Buffer>(session, spectrum_bytes);
  spectrum_work2_.reset();
  scale_u_.clear();
  // the second lane only on a main session: a subimage pool's workers
  // already keep up to 16 streams busy, and a lane pair per worker adds
  // a spectrum buffer and fork/join events to every small subimage
  if (ScaleLanes() > 1 && !session.IsWorker() && data_image.Size() == 1 &&
      data_image.Integration(false).copy_fast_path)
    spectrum_work2_ = std::make_shared<gpu::Buffer>(session, spectrum_bytes);

  // ConvolvePsfs (:29-88): convolved[psf][scale]
  const size_t n_psf = data_image.PsfCount();
  const size_t n_scales = scale_infos_.size();
  std::vector<gpu::Planes> convolved(n_psf);
  auto convolve_psfs = [&](gpu::Planes& out, const float* d_psf,
                           bool is_integrated) {
    out = gpu::Planes::Make(session, width, height, n_scales);
    const double first_auto_scale_size = beam_size_in_pixels_ * 2.0;
    for (size_t si = 0; si != n_scales; ++si) {
      ScaleInfo& e = scale_infos_[si];
      session.D2D(out.Plane(si), d_psf, npx * sizeof(float));
      if (e.scale != 0.0f) transforms_->Transform(out.Plane(si), e.scale);
      if (is_integrated) {
        e.psf_peak = session.ReadFloat(out.Plane(si) + width / 2 +
                                       (height / 2) * width);
        double exp_term;
        if (e.scale == 0.0f || n_scales < 2)
          exp_term = 0.0;
        else
          exp_term = std::log2(e.scale / first_auto_scale_size);
        e.bias_factor = float(std::pow(settings_.scale_bias, -exp_term));
        e.gain = float(double(MinorLoopGain()) / e.psf_peak);
        e.is_active = true;
        log::Info() << "- Scale " << std::round(e.scale)
                    << ", bias factor=" << std::round(e.bias_factor * 10.0) / 10.0
                    << ", psfpeak=" << e.psf_peak << ", gain=" << e.gain
                    << ", kernel peak=" << e.kernel_peak << '\n';
      }
    }
  };
  {
    prof::Section prof_psfs("ms.convolve_psfs");
    data_image.GetIntegratedPsf(integrated.F(), psfs);
    convolve_psfs(convolved[0], integrated.F(), true);
    if (n_psf > 1)
      for (size_t i = 0; i != n_psf; ++i)
        convolve_psfs(convolved[i], psfs.Plane(i), false);
  }

  FindActiveScaleConvolvedMaxima(data_image, integrated.F(), true);
  DeconvolutionResult result;
  std::optional<size_t> optional_scale = SelectMaximumScale(scale_infos_);
  if (!optional_scale) {
    log::Warn() << "No peak found during multi-scale cleaning! Aborting "
                   "deconvolution.\n";
    result.another_iteration_required = false;
    return result;
  }
  size_t scale_with_peak = *optional_scale;

  bool is_final_threshold = false;
  const float initial_peak_value =
      std::fabs(scale_infos_[scale_with_peak].max_unnormalized_image_value *
                scale_infos_[scale_with_peak].bias_factor);
  float m_gain_threshold = initial_peak_value * (1.0 - MajorLoopGain());
  m_gain_threshold = std::max(m_gain_threshold, MajorIterationThreshold());
  float first_threshold = m_gain_threshold;
  if (Threshold() > first_threshold) {
    first_threshold = Threshold();
    is_final_threshold = true;
  }
  log::Info() << "Starting multi-scale cleaning. Start peak=" << initial_peak_value
              << ", major iteration threshold=" << first_threshold
              << (is_final_threshold ? " (final)\n" : "\n");

  ImageSet individual(data_image, width, height);
  std::map<size_t, gpu::Planes> twice_cache;
  std::map<std::pair<size_t, size_t>, std::shared_ptr<gpu::Buffer>> padded_cache;
  bool diverging = false;

  while (IterationNumber() < MaxIterations() &&
         std::fabs(scale_infos_[scale_with_peak].max_unnormalized_image_value *
                   scale_infos_[scale_with_peak].bias_factor) > first_threshold &&
         (!StopOnNegativeComponents() ||
          scale_infos_[scale_with_peak].max_unnormalized_image_value >= 0.0) &&
         threshold_countdown > 0 && !diverging) {  // :323-543
    ScaleInfo& info = scale_infos_[scale_with_peak];
    bool searched = false;  // the next peak searches already ran (deferred result)
    // twice-convolved PSFs for this scale (:331-350), cached per major iteration
    auto tw = twice_cache.find(scale_with_peak);
    if (tw == twice_cache.end()) {
      prof::Section prof_twice("ms.twice_convolved");
      gpu::Planes t = gpu::Planes::Make(session, width, height, n_psf);
      for (size_t i = 0; i != n_psf; ++i) {
        session.D2D(t.Plane(i), convolved[i].Plane(scale_with_peak),
                    npx * sizeof(float));
        if (info.scale != 0.0f) transforms_->Transform(t.Plane(i), info.scale);
      }
      tw = twice_cache.emplace(scale_with_peak, std::move(t)).first;
    }
    const gpu::Planes& twice = tw->second;
    // individually convolved images (:336-354); at scale 0 the fast sub-minor
    // loop only reads them, so it reads the residual itself
    const bool alias_residual = settings_.fast_sub_minor_loop && info.scale == 0.0f;
    if (info.scale != 0.0f && scale_with_peak < scale_image_valid_.size() &&
        scale_image_valid_[scale_with_peak]) {
      // the residual has not changed since FindActiveScaleConvolvedMaxima
      // convolved it with this scale: take that image
      gpu::Planes previous = individual.Planes();
      individual.SetPlanes(scale_images_[scale_with_peak]);
      scale_images_[scale_with_peak] = previous;
      scale_image_valid_[scale_with_peak] = false;
    } else if (!alias_residual) {
      individual.CopyFrom(data_image);
      if (info.scale != 0.0f)
        for (size_t i = 0; i != data_image.Size(); ++i)
          transforms_->Transform(individual.Data(i), info.scale);
    }

    const float sub_iteration_gain_threshold =
        std::fabs(info.max_unnormalized_image_value * info.bias_factor) *
        (1.0 - settings_.sub_minor_loop_gain);
    float first_sub_iteration_threshold = sub_iteration_gain_threshold;
    if (first_threshold > first_sub_iteration_threshold) {
      first_sub_iteration_threshold = first_threshold;
      if (!has_hit_threshold_in_sub_loop) {
        log::Info() << "Subminor loop is near minor loop threshold. "
                       "Initiating countdown.\n";
        has_hit_threshold_in_sub_loop = true;
      }
      threshold_countdown--;
    }

    if (settings_.fast_sub_minor_loop) {  // :377-462
      const size_t sub_start = IterationNumber();
      const size_t conv_w = utils::GetConvolutionSize(
          info.scale, width, settings_.convolution_padding);
      const size_t conv_h = utils::GetConvolutionSize(
          info.scale, height, settings_.convolution_padding);
      SubMinorLoop sub(session, width, height, conv_w, conv_h);
      sub.SetIterationInfo(IterationNumber(), MaxIterations());
      sub.SetThreshold(first_sub_iteration_threshold / info.bias_factor);
      sub.SetGain(info.gain);
      sub.SetDivergenceLimit(DivergenceLimit());
      sub.SetAllowNegativeComponents(AllowNegativeComponents());
      sub.SetStopOnNegativeComponent(StopOnNegativeComponents());
      const size_t scale_border = size_t(std::ceil(info.scale * 0.5));
      sub.SetCleanBorders(
          std::max<size_t>(size_t(std::round(width * CleanBorderRatio())),
                           scale_border),
          std::max<size_t>(size_t(std::round(height * CleanBorderRatio())),
                           scale_border));
      sub.SetMask(MaskFor(scale_with_peak));
      sub.SetSpectralMap(DeviceSpectralMap(session, data_image.Size()));
      sub.SetLogPolyFit(LogPolyFit());
      sub.SetRmsFactor(DeviceRmsFactor(session, width, height));  // :401-402
      std::vector<uint32_t> xy;
      if (RecordTrace()) sub.SetTrace(&xy);
      // Without a trace or a component list, the loop's result (its
      // component count, last peak, divergence) is read only after the work
      // that does not depend on it is queued: the correction, the model
      // update and the next peak searches (:436-462, :521-524) run behind the
      // loop on the stream instead of after a host round trip.
      const bool defer = !RecordTrace() && !track_components_ && DeferLoopResult();
      SubMinorLoop::RunResult r;
      {
        prof::Section prof_run("ms.subminor_run");
        if (defer)
          r = {false, sub.Launch(alias_residual ? data_image : individual, twice), 0.0f};
        else
          r = sub.Run(alias_residual ? data_image : individual, twice);
      }
      for (size_t c = 0; c + 1 < xy.size(); c += 2) {
        trace_.push_back(xy[c]);
        trace_.push_back(xy[c + 1]);
        trace_.push_back(uint32_t(scale_with_peak));
      }
      if (!r.has_peak) {
        log::Warn() << "Could not continue multi-scale clean, because the "
                       "sub-minor loop failed to find components.\n";
        break;
      }
      auto account = [&](const SubMinorLoop::RunResult& rr) {
        diverging = rr.diverging;
        if (DivergenceLimit() != 0.0f)
          diverging = diverging ||
                      std::fabs(rr.peak) > initial_peak_value * DivergenceLimit();
        SetIterationNumber(sub.CurrentIteration());
        info.n_components_cleaned += IterationNumber() - sub_start;
        info.total_flux_cleaned += sub.FluxCleaned();
      };
      if (!defer) account(r);
      std::optional<prof::Section> prof_correct(std::in_place, "ms.correct_and_model");
      if (track_masks_ && scale_with_peak < dev_masks_.size())  // :444-445
        sub.UpdateAutoMask(static_cast<uint8_t*>(dev_masks_[scale_with_peak].Ptr()));
      for (size_t i = 0; i != data_image.Size(); ++i) {
        if (owner(i) != my_rank) continue;  // another rank's image
        const size_t psf_index = data_image.PsfIndex(i);
        auto key = std::make_pair(psf_index, scale_with_peak);
        auto pc = padded_cache.find(key);
        if (pc == padded_cache.end())
          pc = padded_cache
                   .emplace(key, SubMinorLoop::MakeCorrectionPsfSpectrum(
                                     session, convolved[psf_index].Plane(scale_with_peak),
                                     width, height, conv_w, conv_h))
                   .first;
        sub.CorrectResidualDirtyWithSpectrum(i, data_image.Data(i),
                                             pc->second->Ptr());
        if (info.scale != 0.0f) {
          // the sub-minor model is a few hundred components: stamping the
          // shape kernel costs n_sel * n^2 multiply-adds against two
          // full-image FFTs (:451-460 convolves with the same kernel)
          size_t n_kernel = 0;
          const float* d_kernel = transforms_->ShapeKernel(info.scale, n_kernel);
          if (double(sub.NSelected()) * double(n_kernel) * double(n_kernel) <= 1e9) {
            sub.AddShapeModel(i, d_kernel, n_kernel, model_image.Data(i));
          } else {
            sub.GetFullIndividualModel(i, scratch_->F());
            transforms_->Transform(scratch_->F(), info.scale);
            gpu::Check(rdl_add(s, model_image.Data(i), scratch_->F(), npx),
                       "rdl_add");
          }
        } else {
          sub.AddIndividualModel(i, model_image.Data(i));
        }
      }
      if (track_components_)  // :447-448
        sub.UpdateComponentList(*component_list_, scale_with_peak);
      prof_correct.reset();
      share_planes(data_image);  // the corrected residuals, from their owners
      if (defer) {
        ActivateScales(scale_with_peak);
        FindActiveScaleConvolvedMaxima(data_image, integrated.F(), false);
        searched = true;
        account(sub.Collect());
      }
    } else {  // :463-519
      size_t n_kernel = 0;
      std::vector<float> shape_kernel;
      if (info.scale != 0.0f)
        shape_kernel = MultiScaleTransforms::MakeShapeFunction(
            info.scale, n_kernel, std::min(width, height), settings_.shape);
      else
        shape_kernel = {1.0f}, n_kernel = 1;
      std::vector<float> cv(data_image.Size());
      while (IterationNumber() < MaxIterations() &&
             std::fabs(info.max_unnormalized_image_value * info.bias_factor) >
                 first_sub_iteration_threshold &&
             (!StopOnNegativeComponents() ||
              info.max_unnormalized_image_value >= 0.0) &&
             !diverging) {
        const size_t x = info.max_image_value_x, y = info.max_image_value_y;
        for (size_t i = 0; i != data_image.Size(); ++i)
          cv[i] = session.ReadFloat(individual.Data(i) + x + y * width);
        PerformSpectralFit(cv.data(), x, y);  // :477
        trace_.push_back(uint32_t(x));
        trace_.push_back(uint32_t(y));
        trace_.push_back(uint32_t(scale_with_peak));
        for (size_t i = 0; i != data_image.Size(); ++i) {
          cv[i] = cv[i] * info.gain;
          const size_t pi = data_image.PsfIndex(i);
          gpu::Check(rdl_subtract_psf(s, data_image.Data(i),
                                      convolved[pi].Plane(scale_with_peak),
                                      uint32_t(width), uint32_t(height),
                                      uint32_t(x), uint32_t(y), cv[i]),
                     "rdl_subtract_psf");
          gpu::Check(rdl_subtract_psf(s, individual.Data(i), twice.Plane(pi),
                                      uint32_t(width), uint32_t(height),
                                      uint32_t(x), uint32_t(y), cv[i]),
                     "rdl_subtract_psf");
          // AddComponentToModel (:676-698): scale 0 adds the value itself
          // (fma(1, v, m) == m + v), larger scales stamp the shape kernel.
          gpu::Check(rdl_add_shape_component(
                         s, model_image.Data(i), uint32_t(width),
                         uint32_t(height), shape_kernel.data(),
                         uint32_t(n_kernel), uint32_t(x), uint32_t(y), cv[i]),
                     "rdl_add_shape_component");
          info.n_components_cleaned++;
          info.total_flux_cleaned += cv[i];
          if (track_masks_ && scale_with_peak < dev_masks_.size()) {  // :695-696
            const uint8_t one = 1;
            session.H2D(static_cast<uint8_t*>(dev_masks_[scale_with_peak].Ptr()) + x +
                            width * y,
                        &one, 1);
          }
        }
        if (track_components_)  // :502-504
          component_list_->Add(x, y, scale_with_peak, cv.data());
        individual.GetLinearIntegrated(integrated.F());
        FindPeakDirect(integrated.F(), scale_with_peak);
        const float abs_peak =
            std::fabs(info.max_unnormalized_image_value * info.bias_factor);
        if (DivergenceLimit() != 0.0f)
          diverging = abs_peak > initial_peak_value * DivergenceLimit();
        SetIterationNumber(IterationNumber() + 1);
      }
    }

    if (!searched) {
      ActivateScales(scale_with_peak);
      FindActiveScaleConvolvedMaxima(data_image, integrated.F(), false);
    }
    if (log::Verbosity() >= 3) {
      char buf[256];
      std::string line = "[ms] it=" + std::to_string(IterationNumber());
      for (const ScaleInfo& e : scale_infos_) {
        std::snprintf(buf, sizeof(buf), " | s=%g a=%d v=%.9g x=%zu y=%zu", e.scale,
                      int(e.is_active), e.max_unnormalized_image_value * e.bias_factor,
                      e.max_image_value_x, e.max_image_value_y);
        line += buf;
      }
      std::fprintf(stderr, "%s\n", line.c_str());
    }
    optional_scale = SelectMaximumScale(scale_infos_);
    if (!optional_scale) {
      log::Warn() << "No peak found in main loop of multi-scale cleaning! "
                     "Aborting deconvolution.\n";
      result.another_iteration_required = false;
      share_planes(model_image);
      return result;
    }
    scale_with_peak = *optional_scale;
    log::Info() << "Iteration " << IterationNumber() << ", scale "
                << std::round(scale_infos_[scale_with_peak].scale) << " px : "
                << scale_infos_[scale_with_peak].max_unnormalized_image_value *
                       scale_infos_[scale_with_peak].bias_factor
                << " at " << scale_infos_[scale_with_peak].max_image_value_x
                << ',' << scale_infos_[scale_with_peak].max_image_value_y << '\n';
  }

  const bool max_iter_reached = IterationNumber() >= MaxIterations();
  const bool negative_reached =
      StopOnNegativeComponents() &&
      scale_infos_[scale_with_peak].max_unnormalized_image_value < 0.0;
  if (diverging)
    log::Warn() << "WARNING: Multiscale clean diverged.\n";
  result.is_diverging = diverging;
  result.another_iteration_required =
      !max_iter_reached && !is_final_threshold && !negative_reached && !diverging;
  result.final_peak_value =
      scale_infos_[scale_with_peak].max_unnormalized_image_value *
      scale_infos_[scale_with_peak].bias_factor;
  share_planes(model_image);  // the owners' model updates
  session.Sync();
  return result;
}

}  // namespace radler::algorithms
