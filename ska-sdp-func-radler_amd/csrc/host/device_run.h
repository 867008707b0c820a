// A Radler major iteration with the image set already resident in HBM — what
// bench.py times (inputs in HBM when the timed region starts) and what the
// multi-GPU driver shards. It runs exactly the Perform() path
// (ParallelDeconvolution -> DeconvolutionAlgorithm) minus the accessor
// loads/stores, which DeviceRun does once up front.
#pragma once

#include <memory>
#include <vector>

#include "image_set.h"
#include "iuwt_deconvolution.h"
#include "parallel_deconvolution.h"
#include "settings.h"
#include "work_table.h"

namespace radler {

class DeviceRun {
 public:
  /// psf, residual: n_images planes (one per deconvolution channel x pol,
  /// all polarizations Stokes I when n_images > 1 means channels) of
  /// width x height floats in host memory; weights per channel (may be empty).
  /// record_trace: keep every algorithm's component trace (Trace(); the
  /// parity tests); off, the run is Perform()'s, which records none.
  DeviceRun(const Settings& settings, const float* psf, const float* residual,
            size_t n_channels, const std::vector<double>& weights,
            double beam_size, bool record_trace = true);
  ~DeviceRun();

  /// Restore the residual to its initial state and zero the model (device
  /// copies, stream ordered).
  void Restore();
  /// One ParallelDeconvolution major iteration (Perform()'s hot path).
  algorithms::ParallelDeconvolutionResult Execute();
  /// Minor iterations performed by the last Execute() (sum over subimages).
  size_t LastIterations() const { return last_iterations_; }
  std::vector<float> Residual() const;
  std::vector<float> Model() const;
  /// Component trace (x, y, scale triples) of subimage `index`'s algorithm.
  const std::vector<uint32_t>& Trace(size_t index = 0) const;
  /// Outer-loop steps of the last IUWT major iteration (subimage `index`).
  std::vector<algorithms::IuwtDeconvolution::Step> IuwtSteps(size_t index = 0) const;
  /// Tiles of the last Execute (empty for a 1x1 grid).
  const std::vector<int>& CleanOwners() const { return parallel_->CleanOwners(); }
  const std::vector<algorithms::SubImage>& SubImages() const {
    return parallel_->SubImages();
  }
  gpu::Session& Session() { return *session_; }
  std::shared_ptr<gpu::Session> SharedSession() { return session_; }
  /// Process-per-GPU split of gridded runs (ParallelDeconvolution).
  void SetCommunicator(std::shared_ptr<Communicator> comm) {
    parallel_->SetCommunicator(std::move(comm));
  }
  /// ParallelDeconvolution::SetRmsFactorImage (an empty vector clears it).
  void SetRmsFactorImage(std::vector<float> factor) {
    parallel_->SetRmsFactorImage(
        factor.empty() ? nullptr
                       : std::make_shared<const std::vector<float>>(std::move(factor)),
        settings_.trimmed_image_width);
  }
  void Sync() { session_->Sync(); }

 private:
  Settings settings_;
  std::shared_ptr<gpu::Session> session_;
  std::vector<std::vector<float>> host_psfs_;
  std::unique_ptr<WorkTable> table_;
  std::unique_ptr<ImageSet> residual_, model_, initial_;
  std::vector<gpu::Planes> psfs_;
  std::unique_ptr<algorithms::ParallelDeconvolution> parallel_;
  size_t last_iterations_ = 0;
};

}  // namespace radler
