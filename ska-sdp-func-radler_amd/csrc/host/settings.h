// radler::Settings — every field and default of the reference's
// cpp/settings.h:132-534 (defaults pinned by python/test/test_settings.py),
// plus one optional GPU field that defaults to reference behaviour.
#pragma once

#include <optional>
#include <set>
#include <string>
#include <vector>

#include "aocommon_compat.h"

namespace radler {

enum class LocalRmsMethod { kNone, kRmsWindow, kRmsAndMinimumWindow };

enum class AlgorithmType {
  kGenericClean,
  kAdaptiveScalePixel,
  kIuwt,
  kMoreSane,
  kMultiscale,
  kPython
};

enum class MultiscaleShape { kTaperedQuadraticShape, kGaussianShape };

enum class OptimizationAlgorithm {
  kClean,
  kLinearEquationSolver,
  kGradientDescent,
  kRegularizedGradientDescent
};

struct Settings {
  size_t trimmed_image_width = 0;
  size_t trimmed_image_height = 0;
  size_t channels_out = 1;
  struct PixelScale {
    double x = 0.0;
    double y = 0.0;
  } pixel_scale;
  size_t thread_count = aocommon::system::ProcessorCount();
  std::string prefix_name = "wsclean";
  std::set<aocommon::PolarizationEnum> linked_polarizations;
  struct Parallel {
    size_t grid_width = 1;
    size_t grid_height = 1;
    size_t max_threads = aocommon::system::ProcessorCount();
  } parallel;
  double absolute_threshold = 0.0;
  double minor_loop_gain = 0.1;
  double major_loop_gain = 1.0;
  std::optional<double> auto_threshold_sigma = std::nullopt;
  std::optional<double> auto_mask_sigma = std::nullopt;
  std::optional<double> absolute_auto_mask_threshold;
  bool save_source_list = false;
  size_t minor_iteration_count = 0;
  size_t major_iteration_count = 12;
  size_t major_auto_mask_iteration_count = 2;
  bool allow_negative_components = true;
  bool stop_on_negative_components = false;
  bool squared_joins = false;
  std::vector<float> spectral_correction;
  double spectral_correction_frequency = 0.0;
  double border_ratio = 0.0;
  std::string fits_mask;
  std::string casa_mask;
  double divergence_limit = 4.0;
  std::optional<double> horizon_mask_distance = std::nullopt;
  std::string horizon_mask_filename;
  OptimizationAlgorithm component_optimization_algorithm =
      OptimizationAlgorithm::kClean;
  struct LocalRms {
    LocalRmsMethod method = LocalRmsMethod::kNone;
    double window = 25.0;
    std::string image;
    double strength = 1.0;
  } local_rms;
  struct SpectralFitting {
    schaapcommon::fitters::SpectralFittingMode mode =
        schaapcommon::fitters::SpectralFittingMode::kNoFitting;
    size_t terms = 0;
    std::string forced_filename;
  } spectral_fitting;
  AlgorithmType algorithm_type = AlgorithmType::kGenericClean;
  struct Python {
    std::string filename;
  } python;
  struct MoreSane {
    std::string location;
    std::string arguments;
    std::vector<double> sigma_levels;
  } more_sane;
  struct Multiscale {
    bool fast_sub_minor_loop = true;
    double sub_minor_loop_gain = 0.2;
    double scale_bias = 0.6;
    size_t max_scales = 0;
    double convolution_padding = 1.1;
    std::vector<double> scale_list;
    MultiscaleShape shape = MultiscaleShape::kTaperedQuadraticShape;
  } multiscale;
  struct Generic {
    bool use_sub_minor_optimization = true;
  } generic;

  // MI355X build only: HIP device for this Radler instance; -1 selects
  // $RADLER_DEVICE, else $LOCAL_RANK, else device 0.
  int gpu_device = -1;
};

}  // namespace radler
