// Line references are to the reference's cpp/radler.cc.
#include "radler.h"

#include "host_profile.h"

#include <cmath>
#include <stdexcept>

#include "device.h"
#include "generic_clean.h"
#include "image_accessors.h"
#include "image_set.h"
#include "logger.h"
#include "iuwt_deconvolution.h"
#include "multiscale_algorithm.h"
#include "parallel_deconvolution.h"
#include "rms_image.h"

namespace radler {

namespace {
[[noreturn]] void Unsupported(const char* what) {
  throw std::runtime_error(std::string(what) +
                           " is not available in the MI355X build of Radler");
}
}  // namespace

Radler::Radler(const Settings& settings, std::unique_ptr<WorkTable> table,
               double beam_size)
    : Radler(settings, beam_size) {
  InitializeDeconvolutionAlgorithm(std::move(table));
}

Radler::Radler(const Settings& settings, const aocommon::Image& psf_image,
               aocommon::Image& residual_image, aocommon::Image& model_image,
               double beam_size, aocommon::PolarizationEnum polarization)
    : Radler(settings, beam_size) {
  // :52-91
  if (psf_image.Width() != settings.trimmed_image_width ||
      psf_image.Height() != settings.trimmed_image_height)
    throw std::runtime_error("Mismatch in PSF image size");
  if (residual_image.Width() != settings.trimmed_image_width ||
      residual_image.Height() != settings.trimmed_image_height)
    throw std::runtime_error("Mismatch in residual image size");
  if (model_image.Width() != settings.trimmed_image_width ||
      model_image.Height() != settings.trimmed_image_height)
    throw std::runtime_error("Mismatch in model image size");
  auto table = std::make_unique<WorkTable>(std::vector<PsfOffset>{}, 1, 1);
  auto e = std::make_unique<WorkTableEntry>();
  e->polarization = polarization;
  e->image_weight = 1.0;
  e->psf_accessors.emplace_back(
      std::make_unique<utils::LoadOnlyImageAccessor>(psf_image));
  e->residual_accessor =
      std::make_unique<utils::LoadAndStoreImageAccessor>(residual_image);
  e->model_accessor =
      std::make_unique<utils::LoadAndStoreImageAccessor>(model_image);
  table->AddEntry(std::move(e));
  InitializeDeconvolutionAlgorithm(std::move(table));
}

Radler::Radler(const Settings& settings, double beam_size)
    : settings_(settings),
      image_width_(settings.trimmed_image_width),
      image_height_(settings.trimmed_image_height),
      pixel_scale_x_(settings.pixel_scale.x),
      pixel_scale_y_(settings.pixel_scale.y),
      beam_size_(beam_size) {
  // :93-117
  if (settings.spectral_fitting.mode ==
          schaapcommon::fitters::SpectralFittingMode::kForcedTerms &&
      settings.spectral_fitting.forced_filename.empty())
    throw std::runtime_error(
        "Forced fitting filename is required when forced fitting is enabled.");
  if (settings.parallel.grid_width == 0)
    throw std::runtime_error("parallel.grid_width must be larger than zero");
  if (settings.parallel.grid_height == 0)
    throw std::runtime_error("parallel.grid_height must be larger than zero");
  if (settings.parallel.max_threads == 0)
    throw std::runtime_error("parallel.max_threads must be larger than zero");
  parallel_deconvolution_ =
      std::make_unique<algorithms::ParallelDeconvolution>(settings_);
}

Radler::~Radler() { FreeDeconvolutionAlgorithms(); }

ComponentList Radler::GetComponentList() const {
  // ParallelDeconvolution::GetComponentList (parallel_deconvolution.cc:185-210)
  if (settings_.algorithm_type == AlgorithmType::kMultiscale)
    return parallel_deconvolution_->GetMultiscaleComponentList();
  ImageSet model_set(*table_, settings_.squared_joins,
                     settings_.linked_polarizations, image_width_,
                     image_height_, DeviceSession());
  model_set.LoadAndAverage(false);
  ComponentList list(image_width_, image_height_, model_set);
  list.MergeDuplicates();
  return list;
}

const algorithms::DeconvolutionAlgorithm& Radler::MaxScaleCountAlgorithm()
    const {
  return parallel_deconvolution_->MaxScaleCountAlgorithm();
}

void Radler::Perform(bool& another_iteration_required,
                     size_t major_iteration_number) {  // :130-316
  if (!table_) throw std::runtime_error("Radler: not initialized");
  prof::Section prof_total("perform.total");
  table_->ValidatePsfs();
  log::Info() << " == Deconvolving (" << major_iteration_number << ") ==\n";
  gpu::Session& s = DeviceSession();
  ImageSet residual_set(*table_, settings_.squared_joins,
                        settings_.linked_polarizations, image_width_,
                        image_height_, s);
  ImageSet model_set(*table_, settings_.squared_joins,
                     settings_.linked_polarizations, image_width_,
                     image_height_, s);
  {
    prof::Section p("perform.load");
    residual_set.LoadAndAverage(true);
    model_set.LoadAndAverage(false);
  }

  const bool auto_mask_is_enabled =
      settings_.auto_mask_sigma || settings_.absolute_auto_mask_threshold;
  const bool local_rms = settings_.local_rms.method != LocalRmsMethod::kNone;
  if (!settings_.local_rms.image.empty())
    Unsupported("A local-RMS image file (FITS input)");
  const size_t n_px = image_width_ * image_height_;
  gpu::Buffer integrated;
  double median = 0.0, stddev = 0.0;
  if (settings_.auto_threshold_sigma || auto_mask_is_enabled || local_rms) {
    // integrated.MedianAndStdDevFromMAD() (:162-166) on the device
    integrated = gpu::Buffer(s, n_px * sizeof(float));
    residual_set.GetLinearIntegrated(integrated.F());
    float med = 0.0f, mad = 0.0f;
    gpu::Check(rdl_median(s.Handle(), integrated.F(), n_px, 0, 0.0f, &med), "rdl_median");
    gpu::Check(rdl_median(s.Handle(), integrated.F(), n_px, 1, med, &mad), "rdl_median");
    median = med;
    stddev = double(mad) * 1.48260221850560;
    log::Info() << "Estimated standard deviation of background noise: "
                << stddev << '\n';
  }
  if (auto_mask_is_enabled && auto_mask_is_finished_) {
    // :172-185: once the auto-mask is complete a more aggressive gain is
    // used, and the RMS background no longer
    parallel_deconvolution_->SetMinorLoopGain(
        std::min(1.0, settings_.minor_loop_gain * 2.0));
    parallel_deconvolution_->SetRmsFactorImage(nullptr, image_width_);
    // component optimisation only once the mask is complete (:180-185)
    if (settings_.component_optimization_algorithm != OptimizationAlgorithm::kClean)
      parallel_deconvolution_->SetComponentOptimization(
          settings_.component_optimization_algorithm);
  } else {
    parallel_deconvolution_->SetMinorLoopGain(settings_.minor_loop_gain);
    if (local_rms) {  // :196-216
      gpu::Buffer rms(s, n_px * sizeof(float));
      if (settings_.local_rms.method == LocalRmsMethod::kRmsWindow)
        math::rms_image::Make(s, rms.F(), integrated.F(), image_width_, image_height_,
                              settings_.local_rms.window, beam_size_, beam_size_, 0.0,
                              pixel_scale_x_, pixel_scale_y_);
      else
        math::rms_image::MakeWithNegativityLimit(
            s, rms.F(), integrated.F(), image_width_, image_height_,
            settings_.local_rms.window, beam_size_, beam_size_, 0.0, pixel_scale_x_,
            pixel_scale_y_);
      stddev = math::rms_image::MakeRmsFactorImage(s, rms.F(), n_px,
                                                   settings_.local_rms.strength);
      log::Info() << "Lowest RMS in image: " << stddev << '\n';
      auto factor = std::make_shared<std::vector<float>>(n_px);
      s.D2H(factor->data(), rms.F(), n_px * sizeof(float));
      parallel_deconvolution_->SetRmsFactorImage(std::move(factor), image_width_);
    }
  }
  // :228-243
  const double threshold_bias = settings_.squared_joins ? median : 0.0;
  if (auto_mask_is_enabled && !auto_mask_is_finished_) {
    const double combined_auto_mask_threshold =
        std::max(stddev * settings_.auto_mask_sigma.value_or(0.0) + threshold_bias,
                 settings_.absolute_auto_mask_threshold.value_or(0.0));
    parallel_deconvolution_->SetThreshold(
        std::max(combined_auto_mask_threshold, settings_.absolute_threshold));
  } else if (settings_.auto_threshold_sigma) {
    parallel_deconvolution_->SetThreshold(
        std::max(stddev * (*settings_.auto_threshold_sigma) + threshold_bias,
                 settings_.absolute_threshold));
  }

  // :249-275: multiscale tracks per-scale masks until the auto-mask
  // threshold is reached, then cleans inside them; the other algorithms get
  // the scale-independent mask of the model's non-zero pixels
  if (settings_.algorithm_type == AlgorithmType::kMultiscale) {
    if (auto_mask_is_enabled)
      parallel_deconvolution_->SetAutoMaskMode(!auto_mask_is_finished_,
                                               auto_mask_is_finished_);
  } else if (auto_mask_is_enabled && auto_mask_is_finished_) {
    if (auto_mask_.empty()) {
      auto_mask_.assign(image_width_ * image_height_, 0);
      std::vector<float> plane(image_width_ * image_height_);
      for (size_t i = 0; i != model_set.Size(); ++i) {
        s.D2H(plane.data(), model_set.Data(i), plane.size() * sizeof(float));
        for (size_t p = 0; p != plane.size(); ++p)
          if (std::isfinite(plane[p]) && plane[p] != 0.0f) auto_mask_[p] = 1;
      }
    }
    parallel_deconvolution_->SetCleanMask(reinterpret_cast<const bool*>(auto_mask_.data()));
  }

  std::vector<gpu::Planes> psf_images;
  {
    prof::Section p("perform.load_psfs");
    psf_images = residual_set.LoadAndAveragePsfs();
  }
  algorithms::ParallelDeconvolutionResult result;
  {
    prof::Section p("perform.execute");
    result = parallel_deconvolution_->ExecuteMajorIteration(
        residual_set, model_set, psf_images, table_->PsfOffsets(),
        settings_.major_loop_gain);
  }
  another_iteration_required = result.another_iteration_required;

  if (!another_iteration_required && auto_mask_is_enabled && !auto_mask_is_finished_) {
    log::Info() << "Auto-masking threshold reached; continuing next major "
                   "iteration with deeper threshold and mask.\n";
    auto_mask_is_finished_ = true;
    another_iteration_required = true;
    auto_mask_finishing_iteration_ = major_iteration_number;
  }
  if (another_iteration_required && settings_.major_iteration_count != 0 &&
      major_iteration_number >= settings_.major_iteration_count) {
    another_iteration_required = false;
    log::Info() << "Maximum number of major iterations was reached: not "
                   "continuing deconvolution.\n";
  }
  if (another_iteration_required && auto_mask_is_finished_ &&
      major_iteration_number - auto_mask_finishing_iteration_ >=
          settings_.major_auto_mask_iteration_count) {
    another_iteration_required = false;
    log::Info() << "Performed "
                << major_iteration_number - auto_mask_finishing_iteration_
                << " major iterations after reaching the auto-mask threshold: "
                   "not continuing deconvolution.\n";
  }
  if (another_iteration_required && settings_.minor_iteration_count != 0 &&
      parallel_deconvolution_->FirstAlgorithm().IterationNumber() >=
          settings_.minor_iteration_count) {
    another_iteration_required = false;
    log::Info() << "Maximum number of minor deconvolution iterations was "
                   "reached: not continuing deconvolution.\n";
  }
  prof::Section prof_store("perform.store");
  residual_set.AssignAndStoreResidual();
  const algorithms::DeconvolutionAlgorithm& first =
      parallel_deconvolution_->FirstAlgorithm();
  model_set.InterpolateAndStoreModel(first.HasSpectralFitter() ? &first.Fitter()
                                                               : nullptr);
}

std::unique_ptr<schaapcommon::fitters::SpectralFitter>
Radler::CreateSpectralFitter() const {  // :318-331
  std::vector<double> channel_frequencies;
  std::vector<float> channel_weights;
  if (settings_.spectral_fitting.mode !=
      schaapcommon::fitters::SpectralFittingMode::kNoFitting)
    ImageSet::CalculateDeconvolutionFrequencies(*table_, channel_frequencies,
                                                channel_weights);
  return std::make_unique<schaapcommon::fitters::SpectralFitter>(
      settings_.spectral_fitting.mode, settings_.spectral_fitting.terms,
      std::move(channel_frequencies), std::move(channel_weights));
}

void Radler::InitializeDeconvolutionAlgorithm(
    std::unique_ptr<WorkTable> table) {  // :333-395
  FreeDeconvolutionAlgorithms();
  table_ = std::move(table);
  if (table_->OriginalGroups().empty()) throw std::runtime_error("Nothing to clean");
  if (!std::isfinite(beam_size_)) {
    log::Warn() << "No proper beam size available in deconvolution!\n";
    beam_size_ = 0.0;
  }
  if (settings_.spectral_fitting.mode ==
      schaapcommon::fitters::SpectralFittingMode::kForcedTerms)
    Unsupported("Forced-term spectral fitting (a FITS spectral-term cube)");
  if (!settings_.fits_mask.empty() || !settings_.casa_mask.empty() ||
      settings_.horizon_mask_distance)
    Unsupported("Mask files / horizon masks");
  std::unique_ptr<algorithms::DeconvolutionAlgorithm> algorithm;
  switch (settings_.algorithm_type) {
    case AlgorithmType::kGenericClean:
      algorithm = std::make_unique<algorithms::GenericClean>(
          settings_.generic.use_sub_minor_optimization);
      break;
    case AlgorithmType::kMultiscale:
      algorithm = std::make_unique<algorithms::MultiScaleAlgorithm>(
          settings_.multiscale, beam_size_, pixel_scale_x_, pixel_scale_y_,
          settings_.save_source_list);
      break;
    case AlgorithmType::kIuwt:
      algorithm = std::make_unique<algorithms::IuwtDeconvolution>();
      break;
    case AlgorithmType::kAdaptiveScalePixel:
      Unsupported("The adaptive scale pixel algorithm");
    case AlgorithmType::kMoreSane:
      Unsupported("MoreSane");
    case AlgorithmType::kPython:
      Unsupported("Python deconvolution");
  }
  algorithm->SetMaxIterations(settings_.minor_iteration_count);
  algorithm->SetThreshold(settings_.absolute_threshold);
  algorithm->SetMinorLoopGain(settings_.minor_loop_gain);
  algorithm->SetMajorLoopGain(settings_.major_loop_gain);
  algorithm->SetCleanBorderRatio(settings_.border_ratio);
  algorithm->SetDivergenceLimit(settings_.divergence_limit);
  algorithm->SetAllowNegativeComponents(settings_.allow_negative_components);
  algorithm->SetStopOnNegativeComponents(settings_.stop_on_negative_components);
  algorithm->SetSpectralFitter(CreateSpectralFitter(),
                               table_->OriginalGroups().front().size());
  parallel_deconvolution_->SetAlgorithm(std::move(algorithm));
}

void Radler::FreeDeconvolutionAlgorithms() {
  parallel_deconvolution_->FreeDeconvolutionAlgorithms();
  table_.reset();
}

void Radler::SetCommunicator(std::shared_ptr<Communicator> comm) {
  parallel_deconvolution_->SetCommunicator(std::move(comm));
}

gpu::Session& Radler::DeviceSession() const {
  // The device is opened on first use, so constructing a Radler (argument
  // validation) needs no GPU; Perform() fails loudly without one.
  if (!session_) {
    const int device = settings_.gpu_device >= 0 ? settings_.gpu_device
                                                 : gpu::Session::DefaultDevice();
    session_ = gpu::Session::ForDevice(device);
  }
  return *session_;
}

bool Radler::IsInitialized() const {
  return parallel_deconvolution_->IsInitialized();
}

size_t Radler::IterationNumber() const {
  return parallel_deconvolution_->FirstAlgorithm().IterationNumber();
}

}  // namespace radler
