// radler::algorithms::DeconvolutionAlgorithm — the plugin interface of the
// reference (cpp/algorithms/deconvolution_algorithm.h:31-210), with the same
// settings, setters and result struct. The GPU build passes device-resident
// image sets and PSF planes instead of host aocommon::Images; everything
// else (defaults, Clone(), iteration bookkeeping) is unchanged.
#pragma once

#include <memory>
#include <optional>
#include <vector>

#include "device.h"
#include "image_set.h"
#include "settings.h"
#include "spectral_fitter.h"

namespace radler {
class Communicator;
}

namespace radler::algorithms {

struct DeconvolutionResult {
  std::optional<float> starting_peak_value;
  float final_peak_value = 0.0;
  bool another_iteration_required = false;
  bool is_diverging = false;
};

class DeconvolutionAlgorithm {
 public:
  virtual ~DeconvolutionAlgorithm() = default;
  DeconvolutionAlgorithm& operator=(const DeconvolutionAlgorithm&) = delete;

  virtual DeconvolutionResult ExecuteMajorIteration(
      ImageSet& data_image, ImageSet& model_image,
      const gpu::Planes& psf_images) = 0;
  virtual std::unique_ptr<DeconvolutionAlgorithm> Clone() const = 0;
  /// Process-per-GPU joined channels: the ranks of
  /// `comm` share the per-channel work of ONE image set (MultiScale only;
  /// the others ignore it). nullptr: everything on this rank.
  virtual void SetChannelShard(Communicator* comm) { (void)comm; }

  void SetMaxIterations(size_t v) { settings_.max_iterations = v; }
  void SetThreshold(float v) { settings_.threshold = v; }
  void SetMajorIterationThreshold(float v) {
    settings_.major_iteration_threshold = v;
  }
  void SetMinorLoopGain(float v) { settings_.minor_loop_gain = v; }
  void SetMajorLoopGain(float v) { settings_.major_loop_gain = v; }
  void SetAllowNegativeComponents(bool v) {
    settings_.allow_negative_components = v;
  }
  void SetStopOnNegativeComponents(bool v) {
    settings_.stop_on_negative_component = v;
  }
  void SetCleanBorderRatio(float v) { settings_.clean_border_ratio = v; }
  void SetCleanMask(const bool* mask) { settings_.clean_mask = mask; }
  void SetDivergenceLimit(float v) { settings_.divergence_limit = v; }
  void SetComponentOptimizationAlgorithm(OptimizationAlgorithm a) {
    settings_.component_optimization_algorithm = a;
  }

  size_t MaxIterations() const { return settings_.max_iterations; }
  float Threshold() const { return settings_.threshold; }
  float MajorIterationThreshold() const {
    return settings_.major_iteration_threshold;
  }
  float MinorLoopGain() const { return settings_.minor_loop_gain; }
  float MajorLoopGain() const { return settings_.major_loop_gain; }
  float CleanBorderRatio() const { return settings_.clean_border_ratio; }
  bool AllowNegativeComponents() const {
    return settings_.allow_negative_components;
  }
  bool StopOnNegativeComponents() const {
    return settings_.stop_on_negative_component;
  }
  OptimizationAlgorithm ComponentOptimizationAlgorithm() const {
    return settings_.component_optimization_algorithm;
  }
  const bool* CleanMask() const { return settings_.clean_mask; }
  float DivergenceLimit() const { return settings_.divergence_limit; }
  size_t IterationNumber() const { return iteration_number_; }
  void SetIterationNumber(size_t n) { iteration_number_ = n; }

  // deconvolution_algorithm.h:148-161
  void SetSpectralFitter(
      std::unique_ptr<schaapcommon::fitters::SpectralFitter> fitter,
      size_t n_polarizations) {
    spectral_fitter_ = std::move(fitter);
    n_polarizations_ = n_polarizations;
    spectral_map_.reset();
    has_logpoly_ = spectral_fitter_ && MakeLogPoly(*spectral_fitter_, &logpoly_);
  }
  const schaapcommon::fitters::SpectralFitter& Fitter() const {
    return *spectral_fitter_;
  }
  bool HasSpectralFitter() const { return spectral_fitter_ != nullptr; }

  // deconvolution_algorithm.h:163-166: width x height factors every peak
  // search multiplies in (local-RMS thresholding); nullptr clears it
  void SetRmsFactorImage(std::shared_ptr<const std::vector<float>> image) {
    rms_factor_ = std::move(image);
    rms_device_.reset();
  }
  const std::shared_ptr<const std::vector<float>>& RmsFactorImage() const {
    return rms_factor_;
  }
  /// Keep the component trace of each call (LastTrace(): the parity tests
  /// and DeviceRun); off in Radler::Perform, where nothing reads it and its
  /// per-sub-minor-loop read-back would cost a device round trip.
  void SetRecordTrace(bool on) { record_trace_ = on; }
  bool RecordTrace() const { return record_trace_; }

 protected:
  DeconvolutionAlgorithm() = default;
  // Clones share settings, fitter and iteration count, not device scratch.
  DeconvolutionAlgorithm(const DeconvolutionAlgorithm& o)
      : settings_(o.settings_),
        iteration_number_(o.iteration_number_),
        spectral_fitter_(o.spectral_fitter_),
        n_polarizations_(o.n_polarizations_),
        logpoly_(o.logpoly_),
        has_logpoly_(o.has_logpoly_),
        rms_factor_(o.rms_factor_),
        record_trace_(o.record_trace_) {}

  /// Device copy (uint8) of CleanMask() for the current call, or nullptr.
  const uint8_t* DeviceCleanMask(gpu::Session& s, size_t width, size_t height);

  /// PerformSpectralFit (deconvolution_algorithm.cc:29-46) on the host, for
  /// the loops that gather a component's values on the host.
  void PerformSpectralFit(float* values, size_t x, size_t y) const;
  /// The same fit as an n_images x n_images device matrix for the device
  /// loops (rdl_subminor_params / rdl_hogbom_params d_spectral); nullptr
  /// when the fit leaves values unchanged.
  const float* DeviceSpectralMap(gpu::Session& s, size_t n_images);
  /// The log-polynomial fit's description for the device loops
  /// (rdl_subminor_params / rdl_hogbom_params logpoly), or nullptr for the
  /// other modes (which DeviceSpectralMap covers).
  const rdl_logpoly* LogPolyFit() const { return has_logpoly_ ? &logpoly_ : nullptr; }
  /// Device copy of RmsFactorImage() on session s, or nullptr.
  const float* DeviceRmsFactor(gpu::Session& s, size_t width, size_t height);
  /// The peak-search input: d_image itself, or d_image x the RMS factor in
  /// d_scratch (generic_clean.cc:258-264, multiscale_algorithm.cc:707-713).
  const float* RmsWeighted(gpu::Session& s, const float* d_image, float* d_scratch,
                           size_t width, size_t height);

 private:
  struct {
    float threshold = 0.0;
    float major_iteration_threshold = 0.0;
    float minor_loop_gain = 0.1;
    float major_loop_gain = 1.0;
    float clean_border_ratio = 0.05;
    size_t max_iterations = 500;
    float divergence_limit = 4.0;
    bool allow_negative_components = true;
    bool stop_on_negative_component = false;
    OptimizationAlgorithm component_optimization_algorithm =
        OptimizationAlgorithm::kClean;
    const bool* clean_mask = nullptr;
  } settings_;
  size_t iteration_number_ = 0;
  // device copies are bound to the worker session that made them: the
  // subimage a ParallelDeconvolution algorithm runs can move to another
  // worker (stream, GPU) between major iterations
  std::shared_ptr<gpu::Buffer> mask_buffer_;
  gpu::Session* mask_session_ = nullptr;
  std::shared_ptr<const schaapcommon::fitters::SpectralFitter> spectral_fitter_;
  size_t n_polarizations_ = 1;
  rdl_logpoly logpoly_{};
  bool has_logpoly_ = false;
  std::shared_ptr<gpu::Buffer> spectral_map_;
  size_t spectral_map_images_ = 0;
  gpu::Session* spectral_map_session_ = nullptr;
  bool spectral_map_identity_ = false;
  std::shared_ptr<const std::vector<float>> rms_factor_;
  bool record_trace_ = false;
  std::shared_ptr<gpu::Buffer> rms_device_;
  gpu::Session* rms_device_session_ = nullptr;
};

}  // namespace radler::algorithms
