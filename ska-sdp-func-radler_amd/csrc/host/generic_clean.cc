// GenericClean::ExecuteMajorIteration on the device. Line references are to
// the reference's cpp/algorithms/generic_clean.cc.
#include "generic_clean.h"

#include <cmath>
#include <stdexcept>

#include "component_optimization.h"
#include "logger.h"
#include "subminor.h"

namespace radler::algorithms {

GenericClean::GenericClean(bool use_sub_minor_optimization)
    : convolution_padding_(1.1f),
      use_sub_minor_optimization_(use_sub_minor_optimization) {}

rdl_peak GenericClean::FindPeak(gpu::Session& s, const float* d_image,
                                size_t width, size_t height,
                                const uint8_t* d_mask) {
  // :255-277 -> peak_finder::Find(border ratio) / FindWithMask, on the image
  // times the RMS factor when there is one
  if (RmsFactorImage()) {
    if (!rms_scratch_ || rms_scratch_->Bytes() < width * height * sizeof(float))
      rms_scratch_ = std::make_shared<gpu::Buffer>(s, width * height * sizeof(float));
    d_image = RmsWeighted(s, d_image, rms_scratch_->F(), width, height);
  }
  const uint32_t hb = uint32_t(std::round(width * CleanBorderRatio()));
  const uint32_t vb = uint32_t(std::round(height * CleanBorderRatio()));
  rdl_peak p;
  gpu::Check(rdl_find_peak(s.Handle(), d_image, uint32_t(width),
                           uint32_t(height), 0, uint32_t(height), hb, vb,
                           AllowNegativeComponents(), d_mask, 1, &p),
             "rdl_find_peak");
  return p;
}

void GenericClean::RunComponentOptimization(ImageSet& residual_set, ImageSet& model_set,
                                            const gpu::Planes& psfs) {
  // :26-48, per image
  gpu::Session& s = residual_set.Session();
  const size_t w = residual_set.Width(), h = residual_set.Height();
  for (size_t i = 0; i != residual_set.Size(); ++i) {
    switch (ComponentOptimizationAlgorithm()) {
      case OptimizationAlgorithm::kGradientDescent:
        math::GradientDescent(s, model_set.Data(i), residual_set.Data(i),
                              psfs.Plane(residual_set.PsfIndex(i)), w, h, 2 * w, 2 * h);
        break;
      case OptimizationAlgorithm::kLinearEquationSolver:
        math::LinearComponentSolve(s, model_set.Data(i), residual_set.Data(i),
                                   psfs.Plane(residual_set.PsfIndex(i)), w, h);
        break;
      case OptimizationAlgorithm::kRegularizedGradientDescent:
        throw std::runtime_error(
            "Regularized gradient descent has not yet been implemented");
      default:
        throw std::runtime_error(
            "Unsupported optimization algorithm for generic clean algorithm");
    }
  }
}

void GenericClean::FitSpectra(ImageSet& model_set) {
  // :278-297: every pixel's spectrum through PerformSpectralFit, which for
  // the polynomial fitter is one linear map (rdl_spectral_interpolate with
  // the per-component matrix)
  gpu::Session& s = model_set.Session();
  const size_t n_img = model_set.Size(), n = model_set.Width() * model_set.Height();
  if (const rdl_logpoly* lp = LogPolyFit()) {
    // the non-linear fit per pixel and polarization, evaluated at the
    // deconvolution channels themselves
    const size_t n_pol = model_set.NPolarizations();
    const std::vector<double> lg(lp->lg, lp->lg + lp->n_channels);
    gpu::Buffer out(s, lp->n_channels * n * sizeof(float));
    for (size_t p = 0; p != n_pol; ++p) {
      gpu::Check(rdl_logpoly_interpolate(s.Handle(), model_set.Data(p), n_pol * n, n, lp,
                                         lg.data(), lp->n_channels, out.F(), n),
                 "rdl_logpoly_interpolate");
      for (size_t c = 0; c != lp->n_channels; ++c)
        s.D2D(model_set.Data(c * n_pol + p), out.F() + c * n, n * sizeof(float));
    }
    return;
  }
  const float* d_map = DeviceSpectralMap(s, n_img);
  if (!d_map) return;
  std::vector<float> map(n_img * n_img);
  s.D2H(map.data(), d_map, map.size() * sizeof(float));
  gpu::Buffer out(s, n_img * n * sizeof(float));
  gpu::Check(rdl_spectral_interpolate(s.Handle(), model_set.Data(0), n, uint32_t(n_img),
                                      map.data(), uint32_t(n_img), out.F(), n),
             "rdl_spectral_interpolate");
  for (size_t i = 0; i != n_img; ++i)
    s.D2D(model_set.Data(i), out.F() + i * n, n * sizeof(float));
}

DeconvolutionResult GenericClean::ExecuteMajorIteration(
    ImageSet& dirty_set, ImageSet& model_set, const gpu::Planes& psfs) {
  gpu::Session& s = dirty_set.Session();
  const size_t width = dirty_set.Width();
  const size_t height = dirty_set.Height();
  const size_t iteration_at_start = IterationNumber();
  trace_.clear();
  if (StopOnNegativeComponents()) SetAllowNegativeComponents(true);
  // :63-66
  size_t conv_w = size_t(std::ceil(convolution_padding_ * width));
  size_t conv_h = size_t(std::ceil(convolution_padding_ * height));
  if (conv_w % 2 != 0) ++conv_w;
  if (conv_h % 2 != 0) ++conv_h;

  const uint8_t* d_mask = DeviceCleanMask(s, width, height);
  gpu::Buffer integrated(s, width * height * sizeof(float));
  dirty_set.GetLinearIntegrated(integrated.F());
  rdl_peak max_value = FindPeak(s, integrated.F(), width, height, d_mask);
  DeconvolutionResult result;
  if (max_value.found) result.starting_peak_value = max_value.value;
  result.final_peak_value = max_value.found ? max_value.value : 0.0f;
  if (!max_value.found) {
    log::Info() << "No peak found.\n";
    return result;
  }
  if (IterationNumber() >= MaxIterations()) return result;
  if (ComponentOptimizationAlgorithm() != OptimizationAlgorithm::kClean) {  // :89-95
    log::Info() << "Running optimization algorithm...\n";
    RunComponentOptimization(dirty_set, model_set, psfs);
    FitSpectra(model_set);
    return result;
  }

  const float initial_max_value = std::fabs(max_value.value);
  float first_threshold = Threshold();
  const float major_iter_threshold = std::max(
      MajorIterationThreshold(), initial_max_value * (1.0f - MajorLoopGain()));
  if (major_iter_threshold > first_threshold) first_threshold = major_iter_threshold;

  bool diverging = false;
  if (use_sub_minor_optimization_) {  // :115-162
    SubMinorLoop sub(s, width, height, conv_w, conv_h);
    sub.SetIterationInfo(IterationNumber(), MaxIterations());
    sub.SetThreshold(first_threshold);
    sub.SetGain(MinorLoopGain());
    sub.SetAllowNegativeComponents(AllowNegativeComponents());
    sub.SetStopOnNegativeComponent(StopOnNegativeComponents());
    sub.SetDivergenceLimit(DivergenceLimit());
    sub.SetMask(d_mask);
    sub.SetSpectralMap(DeviceSpectralMap(s, dirty_set.Size()));
    sub.SetLogPolyFit(LogPolyFit());
    sub.SetRmsFactor(DeviceRmsFactor(s, width, height));  // :126-128
    sub.SetCleanBorders(size_t(std::round(width * CleanBorderRatio())),
                        size_t(std::round(height * CleanBorderRatio())));
    sub.SetTrace(&trace_);  // (kept for GenericClean: not on the headline path)
    const SubMinorLoop::RunResult r = sub.Run(dirty_set, psfs);
    diverging = r.diverging;
    max_value.found = r.has_peak;
    max_value.value = r.peak;
    SetIterationNumber(sub.CurrentIteration());
    for (size_t i = 0; i != dirty_set.Size(); ++i) {
      sub.CorrectResidualDirty(i, dirty_set.Data(i),
                               psfs.Plane(dirty_set.PsfIndex(i)),
                               size_t(dirty_set.PsfIndex(i)));
      sub.AddIndividualModel(i, model_set.Data(i));
    }
    if (!max_value.found) {
      // :150-157 — FindPeak on `integrated`, which CorrectResidualDirty used
      // as scratch: it holds the trimmed convolution of an all-zero model.
      integrated.Zero();
      max_value = FindPeak(s, integrated.F(), width, height, d_mask);
    }
  } else {  // :163-207
    if (dirty_set.Size() > RDL_MAX_IMAGES)
      throw std::runtime_error("GenericClean: too many images");
    rdl_hogbom_params p{};
    p.width = uint32_t(width);
    p.height = uint32_t(height);
    p.n_images = uint32_t(dirty_set.Size());
    p.n_pol = uint32_t(dirty_set.NPolarizations());
    p.integ = dirty_set.Integration(true);
    p.gain = MinorLoopGain();
    p.threshold = first_threshold;
    p.initial_max = initial_max_value;
    p.divergence_limit = DivergenceLimit();
    p.iteration_start = IterationNumber();
    p.max_iterations = MaxIterations();
    p.allow_negative = AllowNegativeComponents();
    p.stop_on_negative = StopOnNegativeComponents();
    p.h_border = uint32_t(std::round(width * CleanBorderRatio()));
    p.v_border = uint32_t(std::round(height * CleanBorderRatio()));
    p.d_mask = d_mask;
    p.d_spectral = DeviceSpectralMap(s, dirty_set.Size());
    p.logpoly = LogPolyFit();
    p.d_rms = DeviceRmsFactor(s, width, height);
    p.start_x = max_value.x;
    p.start_y = max_value.y;
    p.start_value = max_value.value;
    p.start_found = max_value.found;
    const uint64_t cap = MaxIterations() > IterationNumber()
                             ? MaxIterations() - IterationNumber()
                             : 0;
    const uint64_t trace_cap = std::min<uint64_t>(cap, uint64_t(1) << 24);
    trace_.assign(2 * trace_cap, 0);
    rdl_hogbom_result r;
    gpu::Check(rdl_hogbom_run(s.Handle(), dirty_set.Base(), model_set.Base(),
                              psfs.Base(), &p, &r, trace_.data(), trace_cap),
               "rdl_hogbom_run");
    trace_.resize(2 * std::min<uint64_t>(r.iteration - p.iteration_start, trace_cap));
    SetIterationNumber(r.iteration);
    diverging = r.diverging;
    max_value.found = r.found;
    max_value.value = r.peak;
  }
  // trace as (x, y, scale=0) triples, like MultiScaleAlgorithm's
  {
    std::vector<uint32_t> triples;
    triples.reserve(trace_.size() / 2 * 3);
    for (size_t c = 0; c + 1 < trace_.size(); c += 2) {
      triples.push_back(trace_[c]);
      triples.push_back(trace_[c + 1]);
      triples.push_back(0);
    }
    trace_ = std::move(triples);
  }
  // :208-247
  if (diverging) {
    log::Warn() << "WARNING: Stopping clean because of divergence!\n";
    if (max_value.found) result.final_peak_value = max_value.value;
    result.another_iteration_required = false;
    result.is_diverging = true;
  } else if (max_value.found) {
    const bool final_threshold_reached =
        std::fabs(max_value.value) <= Threshold() || max_value.value == 0.0f;
    const bool negative_reached =
        max_value.value < 0.0f && StopOnNegativeComponents();
    const bool mgain_reached = std::fabs(max_value.value) <= major_iter_threshold;
    const bool did_work = (IterationNumber() - iteration_at_start) != 0;
    result.another_iteration_required =
        mgain_reached && did_work && !negative_reached && !final_threshold_reached;
    result.final_peak_value = max_value.value;
  } else {
    result.another_iteration_required = false;
  }
  return result;
}

}  // namespace radler::algorithms
