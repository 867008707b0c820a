// radler::algorithms::ParallelDeconvolution (reference:
// cpp/algorithms/parallel_deconvolution.{h,cc}). One subimage runs the
// algorithm on the whole device-resident image set; a grid splits the image
// into subimages (Dijkstra minimum-flux boundaries), finds the global start
// peak, and deconvolves every subimage on the device.
#pragma once

#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <vector>

#include "communicator.h"
#include "component_list.h"
#include "deconvolution_algorithm.h"
#include "device.h"
#include "psf_offset.h"
#include "settings.h"

namespace radler::algorithms {

/// One tile of the grid (parallel_deconvolution.h SubImage).
struct SubImage {
  size_t index = 0, x = 0, y = 0, width = 0, height = 0;
  std::vector<bool> mask, boundary_mask;
  double peak = 0.0;
  bool reached_major_threshold = false;
};

struct ParallelDeconvolutionResult {
  bool another_iteration_required = false;
  std::optional<float> start_peak;
  std::optional<float> end_peak;
};

class ParallelDeconvolution {
 public:
  explicit ParallelDeconvolution(const Settings& settings);
  ~ParallelDeconvolution();

  DeconvolutionAlgorithm& FirstAlgorithm() { return *algorithms_.front(); }
  const DeconvolutionAlgorithm& FirstAlgorithm() const {
    return *algorithms_.front();
  }
  const DeconvolutionAlgorithm& MaxScaleCountAlgorithm() const;
  void SetAlgorithm(std::unique_ptr<DeconvolutionAlgorithm> algorithm);
  void SetThreshold(double threshold);
  void SetMinorLoopGain(double gain);
  void SetCleanMask(const bool* mask);
  /// GetComponentList for multiscale (parallel_deconvolution.cc:184-196);
  /// with a process-per-GPU split each rank holds its own subimages'.
  ComponentList GetMultiscaleComponentList() const;
  /// parallel_deconvolution.cc:271-276
  void SetComponentOptimization(OptimizationAlgorithm algorithm) {
    for (auto& a : algorithms_) a->SetComponentOptimizationAlgorithm(algorithm);
  }
  /// parallel_deconvolution.cc:244-250: the single algorithm takes it as
  /// is; gridded runs trim each subimage's box (:332-337) and drop it after
  /// the run (:421-423). nullptr clears it.
  void SetRmsFactorImage(std::shared_ptr<const std::vector<float>> image, size_t width);
  /// Auto-masking (parallel_deconvolution.cc:260-268): passed to the
  /// multiscale algorithms; gridded runs keep full-image per-scale masks and
  /// hand each subimage its box (:359-390), merging it back inside the
  /// boundary mask after a converging run (:425-462).
  void SetAutoMaskMode(bool track_per_scale_masks, bool use_per_scale_masks);
  bool IsInitialized() const { return !algorithms_.empty(); }
  size_t SubImageCount() const { return algorithms_.size(); }
  DeconvolutionAlgorithm& Algorithm(size_t i) { return *algorithms_[i]; }
  const DeconvolutionAlgorithm& Algorithm(size_t i) const { return *algorithms_[i]; }

  ParallelDeconvolutionResult ExecuteMajorIteration(
      ImageSet& data_image, ImageSet& model_image,
      const std::vector<gpu::Planes>& psf_images,
      const std::vector<PsfOffset>& psf_offsets, double major_loop_gain);

  /// Tiles of the last ExecuteParallelRun (empty for a 1x1 grid).
  const std::vector<SubImage>& SubImages() const { return subimages_; }
  /// Process-per-GPU: the rank that cleaned each subimage in the last major
  /// iteration (empty without a communicator).
  const std::vector<int>& CleanOwners() const { return clean_owners_; }

  void FreeDeconvolutionAlgorithms() {
    algorithms_.clear();
    workers_.clear();
    worker_main_device_ = -1;
    mask_ = nullptr;
  }
  /// Share the subimages of gridded runs with the other ranks of a
  /// process-per-GPU job (a size-1 communicator runs them all here, in the
  /// same snapshot order). Every rank must call Perform with the same inputs.
  void SetCommunicator(std::shared_ptr<Communicator> comm) { comm_ = std::move(comm); }
  const std::shared_ptr<Communicator>& GetCommunicator() const { return comm_; }
  /// Worker streams of the concurrent subimage pool (0 until a gridded run
  /// with settings.parallel.max_threads > 1).
  size_t WorkerCount() const { return workers_.size(); }

 private:
  ParallelDeconvolutionResult ExecuteSingleThreadedRun(
      ImageSet& data_image, ImageSet& model_image,
      const std::vector<gpu::Planes>& psf_images,
      const std::vector<PsfOffset>& psf_offsets, double major_loop_gain);
  ParallelDeconvolutionResult ExecuteParallelRun(
      ImageSet& data_image, ImageSet& model_image,
      const std::vector<gpu::Planes>& psf_images,
      const std::vector<PsfOffset>& psf_offsets, double major_loop_gain);

  void RunSubImage(SubImage& sub, ImageSet& data_image, const ImageSet& model_image,
                   ImageSet& result_model, const gpu::Planes& psfs,
                   double major_iteration_threshold, bool find_peak_only);
  /// Runs the subimage's algorithm; returns whether it converged.
  bool DeconvolveSubImage(SubImage& sub, ImageSet& sub_data, ImageSet& sub_model,
                          const gpu::Planes& sub_psfs,
                          double major_iteration_threshold, bool find_peak_only);
  /// Per-subimage result of a concurrent pass (device planes on the main
  /// device, valid during the call): the residual box, the model box to add
  /// (the initial one when it diverged) and whether it converged.
  using SubImageSink = std::function<void(size_t index, const float* d_data,
                                          const float* d_model, bool converging)>;
  /// Runs the subimages (those with run[i] != 0 when `run` is given) on the
  /// worker pool; merges the results in subimage order, or hands each to
  /// `sink` in subimage order instead.
  void RunSubImagesConcurrently(ImageSet& data_image, const ImageSet& model_image,
                                ImageSet& result_model,
                                const std::vector<gpu::Planes>& psf_images,
                                const std::vector<size_t>& psf_indices,
                                double major_iteration_threshold,
                                bool find_peak_only,
                                const std::vector<char>* run = nullptr,
                                const SubImageSink& sink = nullptr);
  /// Process-per-GPU split: this rank deconvolves the subimages it owns
  /// (SubImageOwner) from the pass-start residual, then every subimage's
  /// boxes are broadcast by their owner and merged by all ranks in subimage
  /// order. Returns the global start peak for the find-peak pass.
  double RunSubImagesDistributed(ImageSet& data_image, const ImageSet& model_image,
                                 ImageSet& result_model,
                                 const std::vector<gpu::Planes>& psf_images,
                                 const std::vector<size_t>& psf_indices,
                                 double major_iteration_threshold, bool find_peak_only);
  void EnsureWorkers(gpu::Session& main, size_t n);
  /// the subimage's box of the full-image scale masks into its algorithm
  void LoadScaleMasks(const SubImage& sub, size_t width);
  /// the algorithm's scale masks of `sub` (subimage-sized, one per scale)
  std::vector<std::vector<uint8_t>> SubImageScaleMasks(const SubImage& sub);
  /// merge subimage-sized scale masks into the full-image ones (boundary mask)
  void StoreScaleMasks(const SubImage& sub, size_t width, size_t height,
                       const std::vector<std::vector<uint8_t>>& sub_masks);
  static std::vector<int> PoolDevices(int main_device);

  // worker sessions (one stream each) outlive the algorithms, whose cached
  // transforms and scratch live on them
  std::vector<std::shared_ptr<gpu::Session>> workers_;
  // process-per-GPU: the cleaning pass's subimage owners (LptOwners over the
  // find-peak pass's estimates), identical on every rank
  std::vector<int> clean_owners_;
  int worker_main_device_ = -1;
  std::vector<std::unique_ptr<DeconvolutionAlgorithm>> algorithms_;
  std::vector<SubImage> subimages_;
  const Settings& settings_;
  const bool* mask_ = nullptr;
  std::shared_ptr<const std::vector<float>> rms_image_;  // full image (gridded)
  std::unique_ptr<ComponentList> component_list_;        // gridded multiscale
  size_t rms_width_ = 0;
  std::shared_ptr<Communicator> comm_;
  bool track_masks_ = false, use_masks_ = false;
  std::vector<std::vector<uint8_t>> scale_masks_;  // full image, per scale
  std::mutex masks_mutex_;
};

/// Subimage geometry of the grid (parallel_deconvolution.cc:57-166).
std::vector<SubImage> MakeSubImages(const std::vector<float>& image, size_t width,
                                    size_t height, const bool* user_mask,
                                    const std::vector<PsfOffset>& psf_offsets,
                                    const Settings& settings,
                                    std::vector<size_t>& psf_indices);

/// parallel_deconvolution.cc:34-55 (first index on equal distance).
size_t NearestPsfIndex(const std::vector<PsfOffset>& psf_offsets, size_t x,
                       size_t y) noexcept;

}  // namespace radler::algorithms
