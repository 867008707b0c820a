// Line references are to the reference's
// cpp/algorithms/parallel_deconvolution.cc.
#include "parallel_deconvolution.h"

#include <algorithm>
#include <stdexcept>

#include "logger.h"
#include "multiscale_algorithm.h"

namespace radler::algorithms {

size_t NearestPsfIndex(const std::vector<PsfOffset>& psf_offsets, size_t x,
                       size_t y) noexcept {
  if (psf_offsets.empty()) return 0;
  auto distance = [x, y](const PsfOffset& p) {
    const ssize_t dx = ssize_t(p.x) - ssize_t(x);
    const ssize_t dy = ssize_t(p.y) - ssize_t(y);
    return size_t(dx * dx) + size_t(dy * dy);
  };
  return std::min_element(psf_offsets.begin(), psf_offsets.end(),
                          [&](const PsfOffset& a, const PsfOffset& b) {
                            return distance(a) < distance(b);
                          }) -
         psf_offsets.begin();
}

ParallelDeconvolution::ParallelDeconvolution(const Settings& settings)
    : settings_(settings) {}

ParallelDeconvolution::~ParallelDeconvolution() = default;

const DeconvolutionAlgorithm& ParallelDeconvolution::MaxScaleCountAlgorithm()
    const {
  if (settings_.algorithm_type == AlgorithmType::kMultiscale) {
    const auto* best =
        static_cast<const MultiScaleAlgorithm*>(algorithms_.front().get());
    for (size_t i = 1; i != algorithms_.size(); ++i) {
      const auto* a = static_cast<const MultiScaleAlgorithm*>(algorithms_[i].get());
      if (a->ScaleCount() > best->ScaleCount()) best = a;
    }
    return *best;
  }
  return FirstAlgorithm();
}

void ParallelDeconvolution::SetAlgorithm(
    std::unique_ptr<DeconvolutionAlgorithm> algorithm) {  // :227-242
  algorithms_.resize(settings_.parallel.grid_width *
                     settings_.parallel.grid_height);
  algorithms_.front() = std::move(algorithm);
  for (size_t i = 1; i != algorithms_.size(); ++i)
    algorithms_[i] = algorithms_.front()->Clone();
}

void ParallelDeconvolution::SetThreshold(double threshold) {
  for (auto& a : algorithms_) a->SetThreshold(threshold);
}

void ParallelDeconvolution::SetMinorLoopGain(double gain) {
  for (auto& a : algorithms_) a->SetMinorLoopGain(gain);
}

void ParallelDeconvolution::SetCleanMask(const bool* mask) {
  if (algorithms_.size() == 1)
    algorithms_.front()->SetCleanMask(mask);
  else
    mask_ = mask;
}

ParallelDeconvolutionResult ParallelDeconvolution::ExecuteMajorIteration(
    ImageSet& data_image, ImageSet& model_image,
    const std::vector<gpu::Planes>& psf_images,
    const std::vector<PsfOffset>& psf_offsets, double major_loop_gain) {
  if (algorithms_.size() == 1)
    return ExecuteSingleThreadedRun(data_image, model_image, psf_images,
                                    psf_offsets, major_loop_gain);
  return ExecuteParallelRun(data_image, model_image, psf_images, psf_offsets,
                            major_loop_gain);
}

ParallelDeconvolutionResult ParallelDeconvolution::ExecuteSingleThreadedRun(
    ImageSet& data_image, ImageSet& model_image,
    const std::vector<gpu::Planes>& psf_images,
    const std::vector<PsfOffset>& psf_offsets, double major_loop_gain) {
  // :510-553
  DeconvolutionAlgorithm& algorithm = *algorithms_.front();
  const size_t psf_index = NearestPsfIndex(
      psf_offsets, model_image.Width() / 2, model_image.Height() / 2);
  const gpu::Planes& psfs = psf_images[psf_index];
  algorithm.SetMajorLoopGain(major_loop_gain);
  DeconvolutionResult result;
  if (psfs.width == data_image.Width() && psfs.height == data_image.Height()) {
    result = algorithm.ExecuteMajorIteration(data_image, model_image, psfs);
  } else {
    // DD-PSFs smaller than the image: Image::Untrim to the image size
    if (psfs.width > data_image.Width() || psfs.height > data_image.Height())
      throw std::runtime_error("PSF larger than the image");
    gpu::Session& s = data_image.Session();
    gpu::Planes resized = gpu::Planes::Make(s, data_image.Width(),
                                            data_image.Height(), psfs.count);
    for (size_t i = 0; i != psfs.count; ++i)
      gpu::Check(rdl_untrim(s.Handle(), resized.Plane(i),
                            uint32_t(data_image.Width()),
                            uint32_t(data_image.Height()), psfs.Plane(i),
                            uint32_t(psfs.width), uint32_t(psfs.height)),
                 "rdl_untrim");
    result = algorithm.ExecuteMajorIteration(data_image, model_image, resized);
  }
  ParallelDeconvolutionResult global;
  global.another_iteration_required = result.another_iteration_required;
  global.start_peak = result.starting_peak_value;
  global.end_peak = result.final_peak_value;
  return global;
}

ParallelDeconvolutionResult ParallelDeconvolution::ExecuteParallelRun(
    ImageSet&, ImageSet&, const std::vector<gpu::Planes>&,
    const std::vector<PsfOffset>&, double) {
  throw std::runtime_error(
      "parallel.grid_width/height > 1: subimage tiling not built yet");
}

}  // namespace radler::algorithms
