// Host driver of the device sub-minor loop (reference:
// cpp/algorithms/subminor_loop.{h,cc}). Run() = findPeakPositions + MakeSets
// + the iteration loop, all device-side (rdl_subminor_run);
// CorrectResidualDirty() = padded FFT convolution of the sub-minor model with
// the PSF, subtracted from the residual.
#pragma once

#include <map>
#include <vector>

#include "component_list.h"
#include "device.h"
#include "image_set.h"

namespace radler::algorithms {

class SubMinorLoop {
 public:
  SubMinorLoop(gpu::Session& s, size_t width, size_t height,
               size_t padded_width, size_t padded_height);
  ~SubMinorLoop();
  SubMinorLoop(const SubMinorLoop&) = delete;
  SubMinorLoop& operator=(const SubMinorLoop&) = delete;

  void SetThreshold(float threshold) { threshold_ = threshold; }
  void SetIterationInfo(size_t current, size_t max) {
    current_iteration_ = current;
    max_iterations_ = max;
  }
  void SetGain(float gain) { gain_ = gain; }
  void SetAllowNegativeComponents(bool v) { allow_negative_ = v; }
  void SetStopOnNegativeComponent(bool v) { stop_on_negative_ = v; }
  void SetCleanBorders(size_t h, size_t v) {
    horizontal_border_ = h;
    vertical_border_ = v;
  }
  void SetMask(const uint8_t* d_mask) { d_mask_ = d_mask; }
  /// _parentAlgorithm->PerformSpectralFit (subminor_loop.cc:76) as a device
  /// matrix (DeconvolutionAlgorithm::DeviceSpectralMap), nullptr = none.
  void SetSpectralMap(const float* d_map) { d_spectral_ = d_map; }
  /// The same fit when it is log-polynomial (non-linear: no matrix);
  /// nullptr = none.
  void SetLogPolyFit(const rdl_logpoly* fit) { logpoly_ = fit; }
  /// SetRmsFactorImage (subminor_loop.h:162-164): the full-image device
  /// factor plane, nullptr = none.
  void SetRmsFactor(const float* d_rms) { d_rms_ = d_rms; }
  /// subminor_loop.cc:220-228 on the device (byte mask, W x H).
  void UpdateAutoMask(uint8_t* d_mask);
  void SetDivergenceLimit(float v) { divergence_limit_ = v; }
  void SetTrace(std::vector<uint32_t>* trace) { trace_ = trace; }

  struct RunResult {
    bool diverging;
    bool has_peak;
    float peak;
  };
  RunResult Run(ImageSet& convolved_residual,
                const gpu::Planes& twice_convolved_psfs);
  /// Run() in two halves (rdl_subminor_launch / _collect): Launch selects and
  /// starts the loop and returns whether it found a component (NSelected()
  /// is final); the selection's model may be used (corrections, model
  /// updates) before Collect, which waits for the loop and returns Run()'s
  /// result. No trace.
  bool Launch(ImageSet& convolved_residual, const gpu::Planes& twice_convolved_psfs);
  RunResult Collect();

  /// subminor_loop.cc:195-218. `psf_key` identifies the PSF so its padded
  /// spectrum is computed once per loop object.
  void CorrectResidualDirty(size_t image_index, float* d_residual,
                            const float* d_single_convolved_psf,
                            size_t psf_key);
  /// The same with a caller-cached padded PSF spectrum (MakePaddedPsfSpectrum).
  void CorrectResidualDirtyWithSpectrum(size_t image_index, float* d_residual,
                                        const void* d_psf_spectrum);
  static std::shared_ptr<gpu::Buffer> MakePaddedPsfSpectrum(
      gpu::Session& s, const float* d_psf, size_t width, size_t height,
      size_t padded_width, size_t padded_height, bool f64 = true);
  /// CorrectResidualDirty's transforms are float64 unless RDL_CORR_F32=1.
  static bool CorrectionF64();
  /// The padded PSF spectrum as CorrectResidualDirty(WithSpectrum) reads it:
  /// MakePaddedPsfSpectrum's float64 spectrum, or its float narrowing when
  /// CorrectionKernelF32() (RDL_CORR_KERNEL=f32) and the LDS engine runs the
  /// correction.
  static std::shared_ptr<gpu::Buffer> MakeCorrectionPsfSpectrum(
      gpu::Session& s, const float* d_psf, size_t width, size_t height,
      size_t padded_width, size_t padded_height);
  static bool CorrectionKernelF32();

  /// GetFullIndividualModel (subminor_loop.cc:186-193) into a zeroed W x H.
  void GetFullIndividualModel(size_t image_index, float* d_dest);
  /// model += GetFullIndividualModel(...) (generic_clean.cc:145-148).
  void AddIndividualModel(size_t image_index, float* d_model);
  /// model += GetFullIndividualModel(...) convolved with an odd n x n shape
  /// kernel (circular), by direct stamping.
  void AddShapeModel(size_t image_index, const float* d_kernel, size_t n,
                     float* d_model);
  /// Selected positions and per-image model values (UpdateComponentList,
  /// UpdateAutoMask inputs).
  void GetSelection(std::vector<uint32_t>& positions,
                    std::vector<float>& models) const;
  /// subminor_loop.cc:230-246: every selected pixel with a non-zero model
  /// value in any image joins `list` at `scale_index`.
  void UpdateComponentList(ComponentList& list, size_t scale_index) const;

  size_t CurrentIteration() const { return current_iteration_; }
  float FluxCleaned() const { return flux_cleaned_; }
  size_t NSelected() const { return n_selected_; }
  size_t NImages() const { return n_images_; }

 private:
  gpu::Session& s_;
  rdl_subminor* h_ = nullptr;
  size_t width_, height_, padded_width_, padded_height_;
  float threshold_ = 0.0f, gain_ = 0.0f, divergence_limit_ = 0.0f;
  size_t horizontal_border_ = 0, vertical_border_ = 0;
  size_t current_iteration_ = 0, max_iterations_ = 0;
  bool allow_negative_ = true, stop_on_negative_ = false;
  const uint8_t* d_mask_ = nullptr;
  const float* d_spectral_ = nullptr;
  const rdl_logpoly* logpoly_ = nullptr;
  const float* d_rms_ = nullptr;
  float flux_cleaned_ = 0.0f;
  size_t n_selected_ = 0, n_images_ = 0;
  bool launched_has_peak_ = false;  // Launch found a component (Collect pending)
  std::vector<uint32_t>* trace_ = nullptr;
  std::map<size_t, std::shared_ptr<gpu::Buffer>> psf_spectra_;
};

}  // namespace radler::algorithms
