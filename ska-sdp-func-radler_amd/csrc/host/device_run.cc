#include "device_run.h"

#include <stdexcept>

#include "generic_clean.h"
#include "image_accessors.h"
#include "iuwt_deconvolution.h"
#include "multiscale_algorithm.h"

namespace radler {

namespace {
// An accessor over a host buffer that DeviceRun keeps alive.
class VectorAccessor final : public aocommon::ImageAccessor {
 public:
  VectorAccessor(std::vector<float>& v, size_t w, size_t h) : v_(v), w_(w), h_(h) {}
  size_t Width() const override { return w_; }
  size_t Height() const override { return h_; }
  void Load(float* data) const override { std::copy(v_.begin(), v_.end(), data); }
  void Store(const float* data) override { std::copy_n(data, w_ * h_, v_.begin()); }

 private:
  std::vector<float>& v_;
  size_t w_, h_;
};
}  // namespace

DeviceRun::DeviceRun(const Settings& settings, const float* psf,
                     const float* residual, size_t n_channels,
                     const std::vector<double>& weights, double beam_size,
                     bool record_trace)
    : settings_(settings) {
  const size_t w = settings.trimmed_image_width, h = settings.trimmed_image_height;
  const size_t n = w * h;
  const int device =
      settings.gpu_device >= 0 ? settings.gpu_device : gpu::Session::DefaultDevice();
  session_ = gpu::Session::ForDevice(device);
  table_ = std::make_unique<WorkTable>(std::vector<PsfOffset>{}, n_channels,
                                       n_channels);
  host_psfs_.resize(3 * n_channels);
  for (size_t c = 0; c != n_channels; ++c) {
    host_psfs_[3 * c].assign(psf + c * n, psf + (c + 1) * n);
    host_psfs_[3 * c + 1].assign(residual + c * n, residual + (c + 1) * n);
    host_psfs_[3 * c + 2].assign(n, 0.0f);
    auto e = std::make_unique<WorkTableEntry>();
    e->original_channel_index = c;
    e->image_weight = weights.empty() ? 1.0 : weights[c];
    e->band_start_frequency = e->band_end_frequency = 1.0e8 + 1.0e7 * c;
    e->psf_accessors.emplace_back(
        std::make_unique<VectorAccessor>(host_psfs_[3 * c], w, h));
    e->residual_accessor =
        std::make_unique<VectorAccessor>(host_psfs_[3 * c + 1], w, h);
    e->model_accessor = std::make_unique<VectorAccessor>(host_psfs_[3 * c + 2], w, h);
    table_->AddEntry(std::move(e));
  }
  gpu::Session& s = *session_;
  residual_ = std::make_unique<ImageSet>(*table_, settings.squared_joins,
                                         settings.linked_polarizations, w, h, s);
  model_ = std::make_unique<ImageSet>(*residual_, w, h);
  initial_ = std::make_unique<ImageSet>(*residual_, w, h);
  initial_->LoadAndAverage(true);
  psfs_ = initial_->LoadAndAveragePsfs();

  std::unique_ptr<algorithms::DeconvolutionAlgorithm> algorithm;
  if (settings.algorithm_type == AlgorithmType::kGenericClean)
    algorithm = std::make_unique<algorithms::GenericClean>(
        settings.generic.use_sub_minor_optimization);
  else if (settings.algorithm_type == AlgorithmType::kMultiscale)
    algorithm = std::make_unique<algorithms::MultiScaleAlgorithm>(
        settings_.multiscale, beam_size, settings.pixel_scale.x,
        settings.pixel_scale.y, false);
  else if (settings.algorithm_type == AlgorithmType::kIuwt)
    algorithm = std::make_unique<algorithms::IuwtDeconvolution>();
  else
    throw std::runtime_error("DeviceRun: unsupported algorithm");
  algorithm->SetRecordTrace(record_trace);  // Trace(): the parity tests' component traces
  algorithm->SetMaxIterations(settings.minor_iteration_count);
  algorithm->SetThreshold(settings.absolute_threshold);
  algorithm->SetMinorLoopGain(settings.minor_loop_gain);
  algorithm->SetMajorLoopGain(settings.major_loop_gain);
  algorithm->SetCleanBorderRatio(settings.border_ratio);
  algorithm->SetDivergenceLimit(settings.divergence_limit);
  algorithm->SetAllowNegativeComponents(settings.allow_negative_components);
  algorithm->SetStopOnNegativeComponents(settings.stop_on_negative_components);
  algorithm->SetComponentOptimizationAlgorithm(settings.component_optimization_algorithm);
  {  // Radler::CreateSpectralFitter (radler.cc:318-331); channel c sits at
     // 100 MHz + c x 10 MHz
    using schaapcommon::fitters::SpectralFittingMode;
    const SpectralFittingMode mode = settings.spectral_fitting.mode;
    if (mode == SpectralFittingMode::kForcedTerms)
      throw std::runtime_error(
          "DeviceRun: forced-term spectral fitting is not available");
    std::vector<double> frequencies;
    std::vector<float> channel_weights;
    if (mode != SpectralFittingMode::kNoFitting)
      ImageSet::CalculateDeconvolutionFrequencies(*table_, frequencies, channel_weights);
    algorithm->SetSpectralFitter(
        std::make_unique<schaapcommon::fitters::SpectralFitter>(
            mode, settings.spectral_fitting.terms, std::move(frequencies),
            std::move(channel_weights)),
        1);
  }
  parallel_ = std::make_unique<algorithms::ParallelDeconvolution>(settings_);
  parallel_->SetAlgorithm(std::move(algorithm));
  Restore();
  s.Sync();
}

DeviceRun::~DeviceRun() = default;

void DeviceRun::Restore() {
  residual_->CopyFrom(*initial_);
  model_->Fill(0.0f);
  for (size_t i = 0; i != parallel_->SubImageCount(); ++i)
    parallel_->Algorithm(i).SetIterationNumber(0);
}

algorithms::ParallelDeconvolutionResult DeviceRun::Execute() {
  std::vector<size_t> before(parallel_->SubImageCount());
  for (size_t i = 0; i != before.size(); ++i)
    before[i] = parallel_->Algorithm(i).IterationNumber();
  auto r = parallel_->ExecuteMajorIteration(*residual_, *model_, psfs_, {},
                                            settings_.major_loop_gain);
  last_iterations_ = 0;
  for (size_t i = 0; i != before.size(); ++i)
    last_iterations_ += parallel_->Algorithm(i).IterationNumber() - before[i];
  return r;
}

std::vector<float> DeviceRun::Residual() const {
  std::vector<float> out(residual_->Size() * residual_->PlaneSize());
  session_->D2H(out.data(), residual_->Base(), out.size() * sizeof(float));
  return out;
}

std::vector<float> DeviceRun::Model() const {
  std::vector<float> out(model_->Size() * model_->PlaneSize());
  session_->D2H(out.data(), model_->Base(), out.size() * sizeof(float));
  return out;
}

const std::vector<uint32_t>& DeviceRun::Trace(size_t index) const {
  static const std::vector<uint32_t> empty;
  if (index >= parallel_->SubImageCount()) return empty;
  const algorithms::DeconvolutionAlgorithm& a = parallel_->Algorithm(index);
  if (auto* m = dynamic_cast<const algorithms::MultiScaleAlgorithm*>(&a))
    return m->LastTrace();
  if (auto* g = dynamic_cast<const algorithms::GenericClean*>(&a))
    return g->LastTrace();
  return empty;
}

std::vector<algorithms::IuwtDeconvolution::Step> DeviceRun::IuwtSteps(size_t index) const {
  const auto* a =
      dynamic_cast<const algorithms::IuwtDeconvolution*>(&parallel_->Algorithm(index));
  if (!a) throw std::runtime_error("DeviceRun: not an IUWT run");
  return a->Steps();
}

}  // namespace radler
