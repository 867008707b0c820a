// radler::Radler — the public entry point (reference: cpp/radler.{h,cc}),
// same constructors, Perform() contract and accessors. Image data is
// uploaded to the GPU after ImageSet::LoadAndAverage and written back through
// the WorkTable accessors at the end of Perform(), as the reference's
// residual/model stores do.
#pragma once

#include <memory>

#include "aocommon_compat.h"
#include "component_list.h"
#include "settings.h"
#include "spectral_fitter.h"
#include "work_table.h"
#include "work_table_entry.h"

namespace radler {
namespace algorithms {
class ParallelDeconvolution;
class DeconvolutionAlgorithm;
}  // namespace algorithms
namespace gpu {
class Session;
}
class Communicator;

class Radler {
 public:
  Radler(const Settings& settings, std::unique_ptr<WorkTable> table,
         double beam_size);
  /// Single channel, single polarization (radler.h:42-46). Keep the image
  /// buffers alive while this object is used.
  Radler(const Settings& settings, const aocommon::Image& psf_image,
         aocommon::Image& residual_image, aocommon::Image& model_image,
         double beam_size,
         aocommon::PolarizationEnum polarization =
             aocommon::PolarizationEnum::StokesI);
  ~Radler();

  ComponentList GetComponentList() const;
  const algorithms::DeconvolutionAlgorithm& MaxScaleCountAlgorithm() const;
  void Perform(bool& another_iteration_required, size_t major_iteration_number);
  void FreeDeconvolutionAlgorithms();
  std::unique_ptr<schaapcommon::fitters::SpectralFitter> CreateSpectralFitter()
      const;
  bool IsInitialized() const;
  size_t IterationNumber() const;

  // MI355X build only: the device session (bench / tests) and the
  // parallel-deconvolution object.
  gpu::Session& DeviceSession() const;
  algorithms::ParallelDeconvolution& Parallel() const {
    return *parallel_deconvolution_;
  }
  /// MI355X build: share the subimages of gridded runs (settings.parallel
  /// grid > 1x1) with the other ranks of a process-per-GPU job; every rank
  /// calls Perform with the same inputs and gets the same result.
  void SetCommunicator(std::shared_ptr<Communicator> comm);

 private:
  Radler(const Settings& settings, double beam_size);
  void InitializeDeconvolutionAlgorithm(std::unique_ptr<WorkTable> table);

  const Settings settings_;
  std::unique_ptr<WorkTable> table_;
  mutable std::shared_ptr<gpu::Session> session_;
  std::unique_ptr<algorithms::ParallelDeconvolution> parallel_deconvolution_;
  size_t image_width_ = 0;
  size_t image_height_ = 0;
  double pixel_scale_x_ = 0.0;
  double pixel_scale_y_ = 0.0;
  double beam_size_ = 0.0;
  // auto-masking state across major iterations (cpp/radler.h:111-114)
  bool auto_mask_is_finished_ = false;
  size_t auto_mask_finishing_iteration_ = 0;
  std::vector<uint8_t> auto_mask_;  // scale-independent mask (non-multiscale)
};

}  // namespace radler
