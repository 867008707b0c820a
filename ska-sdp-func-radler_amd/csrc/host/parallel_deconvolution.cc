// Line references are to the reference's
// cpp/algorithms/parallel_deconvolution.cc.
#include "parallel_deconvolution.h"

#include <algorithm>
#include <stdexcept>

#include <cmath>

#include "dijkstra_splitter.h"
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

// MakeSubImages (parallel_deconvolution.cc:57-166): Dijkstra dividers through
// the integrated image, then per grid cell the overlap of its vertical and
// horizontal areas; the subimage mask is that overlap, ANDed with the user
// clean mask when there is one.
std::vector<SubImage> MakeSubImages(const std::vector<float>& image, size_t width,
                                    size_t height, const bool* user_mask,
                                    const std::vector<PsfOffset>& psf_offsets,
                                    const Settings& settings,
                                    std::vector<size_t>& psf_indices) {
  const size_t gw = settings.parallel.grid_width, gh = settings.parallel.grid_height;
  const size_t avg_w = width / gw, avg_h = height / gh;
  math::DijkstraSplitter splitter(width, height);
  std::vector<float> dividing(width * height, 0.0f);
  std::vector<char> scratch_store(width * height);
  bool* scratch = reinterpret_cast<bool*>(scratch_store.data());
  for (size_t d = 1; d < gw; ++d) {
    const size_t mid = width * d / gw;
    splitter.DivideVertically(image.data(), dividing.data(), mid - avg_w / 4,
                              mid + avg_w / 4);
  }
  struct Column {
    std::vector<char> mask;
    size_t x = 0, width = 0;
  };
  std::vector<Column> columns(gw);
  for (size_t d = 0; d != gw; ++d) {
    Column& c = columns[d];
    splitter.FloodVerticalArea(dividing.data(), d * width / gw + avg_w / 2, scratch,
                               c.x, c.width);
    c.mask.resize(c.width * height);
    for (size_t y = 0; y != height; ++y)
      std::copy_n(scratch_store.data() + y * width + c.x, c.width,
                  c.mask.data() + y * c.width);
  }
  std::fill(dividing.begin(), dividing.end(), 0.0f);
  for (size_t d = 1; d < gh; ++d) {
    const size_t mid = height * d / gh;
    splitter.DivideHorizontally(image.data(), dividing.data(), mid - avg_h / 4,
                                mid + avg_h / 4);
  }
  std::vector<char> bounding_store(width * height, 0);
  bool* bounding = reinterpret_cast<bool*>(bounding_store.data());
  std::vector<SubImage> subs;
  for (size_t gy = 0; gy != gh; ++gy) {
    size_t area_y, area_h;
    splitter.FloodHorizontalArea(dividing.data(), gy * height / gh + avg_h / 2,
                                 scratch, area_y, area_h);
    for (size_t gx = 0; gx != gw; ++gx) {
      SubImage sub;
      sub.index = subs.size();
      const Column& c = columns[gx];
      splitter.GetBoundingMask(reinterpret_cast<const bool*>(c.mask.data()), c.x,
                               c.width, scratch, bounding, sub.x, sub.y, sub.width,
                               sub.height);
      sub.mask.resize(sub.width * sub.height);
      for (size_t y = 0; y != sub.height; ++y)
        for (size_t x = 0; x != sub.width; ++x)
          sub.mask[y * sub.width + x] =
              bounding_store[(y + sub.y) * width + x + sub.x] != 0;
      sub.boundary_mask = sub.mask;
      if (user_mask)
        for (size_t y = 0; y != sub.height; ++y)
          for (size_t x = 0; x != sub.width; ++x)
            sub.mask[y * sub.width + x] =
                sub.mask[y * sub.width + x] &&
                user_mask[(y + sub.y) * width + x + sub.x];
      psf_indices.push_back(NearestPsfIndex(psf_offsets, sub.x + sub.width / 2,
                                            sub.y + sub.height / 2));
      subs.push_back(std::move(sub));
    }
  }
  return subs;
}

void ParallelDeconvolution::RunSubImage(SubImage& sub, ImageSet& data_image,
                                        const ImageSet& model_image,
                                        ImageSet& result_model,
                                        const gpu::Planes& psfs,
                                        double major_iteration_threshold,
                                        bool find_peak_only) {
  // parallel_deconvolution.cc:300-484 on the device: the subimage's planes
  // are box copies of the full image set's planes
  gpu::Session& s = data_image.Session();
  const size_t W = data_image.Width(), H = data_image.Height();
  const size_t sw = sub.width, sh = sub.height, n = sw * sh;
  const uint32_t uw = uint32_t(sw), uh = uint32_t(sh);
  gpu::Buffer boundary(s, n);
  {
    std::vector<uint8_t> b(n);
    for (size_t i = 0; i != n; ++i) b[i] = sub.boundary_mask[i] ? 1 : 0;
    s.H2D(boundary.Ptr(), b.data(), n);
  }
  const uint8_t* d_boundary = static_cast<const uint8_t*>(boundary.Ptr());
  ImageSet sub_data(data_image, sw, sh);
  ImageSet sub_model(model_image, sw, sh);
  for (size_t i = 0; i != data_image.Size(); ++i) {
    gpu::Check(rdl_box(s.Handle(), sub_data.Data(i), uw, 0, 0, data_image.Data(i),
                       uint32_t(W), uint32_t(sub.x), uint32_t(sub.y), uw, uh,
                       nullptr, RDL_BOX_COPY),
               "rdl_box");  // ImageSet::Trim
    gpu::Check(rdl_box(s.Handle(), sub_model.Data(i), uw, 0, 0, model_image.Data(i),
                       uint32_t(W), uint32_t(sub.x), uint32_t(sub.y), uw, uh,
                       d_boundary, RDL_BOX_COPY_ZERO),
               "rdl_box");  // ImageSet::TrimMasked
  }
  ImageSet initial_model(sub_model, sw, sh);
  initial_model.CopyFrom(sub_model);
  // Image::Resize of the PSFs to the subimage: centred trim (PSFs are never
  // smaller than a subimage here)
  if (psfs.width < sw || psfs.height < sh)
    throw std::runtime_error("PSF smaller than a subimage");
  gpu::Planes sub_psfs = gpu::Planes::Make(s, sw, sh, psfs.count);
  for (size_t i = 0; i != psfs.count; ++i)
    gpu::Check(rdl_box(s.Handle(), sub_psfs.Plane(i), uw, 0, 0, psfs.Plane(i),
                       uint32_t(psfs.width), uint32_t((psfs.width - sw) / 2),
                       uint32_t((psfs.height - sh) / 2), uw, uh, nullptr,
                       RDL_BOX_COPY),
               "rdl_box");
  DeconvolutionAlgorithm& alg = *algorithms_[sub.index];
  std::vector<char> mask_copy(sub.mask.begin(), sub.mask.end());
  alg.SetCleanMask(reinterpret_cast<const bool*>(mask_copy.data()));
  const size_t max_n_iter = alg.MaxIterations();
  if (find_peak_only)
    alg.SetMaxIterations(0);
  else
    alg.SetMajorIterationThreshold(float(major_iteration_threshold));
  const double peak_at_start = std::fabs(sub.peak);
  const DeconvolutionResult result =
      alg.ExecuteMajorIteration(sub_data, sub_model, sub_psfs);
  alg.SetCleanMask(nullptr);
  sub.peak = result.final_peak_value;
  sub.reached_major_threshold = result.another_iteration_required;
  const bool converging =
      (settings_.divergence_limit == 0.0 ||
       std::fabs(sub.peak) <= peak_at_start * settings_.divergence_limit) &&
      std::isfinite(sub.peak) && !result.is_diverging;
  if (!converging && !find_peak_only) {
    log::Warn() << "Peak of sub-image " << sub.index << " increased from "
                << peak_at_start << " to " << sub.peak
                << " and deconvolution probably diverged: resetting.\n";
    sub.reached_major_threshold = false;
  }
  if (find_peak_only) {
    alg.SetMaxIterations(max_n_iter);
    return;
  }
  const ImageSet& model_out = converging ? sub_model : initial_model;
  for (size_t i = 0; i != data_image.Size(); ++i) {
    if (converging)  // ImageSet::CopyMasked
      gpu::Check(rdl_box(s.Handle(), data_image.Data(i), uint32_t(W),
                         uint32_t(sub.x), uint32_t(sub.y), sub_data.Data(i), uw, 0,
                         0, uw, uh, d_boundary, RDL_BOX_COPY_MASKED),
                 "rdl_box");
    gpu::Check(rdl_box(s.Handle(), result_model.Data(i), uint32_t(W),
                       uint32_t(sub.x), uint32_t(sub.y), model_out.Data(i), uw, 0, 0,
                       uw, uh, nullptr, RDL_BOX_ADD),
               "rdl_box");  // ImageSet::AddSubImage
  }
  s.Sync();
}

ParallelDeconvolutionResult ParallelDeconvolution::ExecuteParallelRun(
    ImageSet& data_image, ImageSet& model_image,
    const std::vector<gpu::Planes>& psf_images,
    const std::vector<PsfOffset>& psf_offsets, double major_loop_gain) {
  // parallel_deconvolution.cc:556-654; subimages run one after another in
  // index order on this session's device
  gpu::Session& s = data_image.Session();
  const size_t width = data_image.Width(), height = data_image.Height();
  std::vector<float> image(width * height);
  {
    gpu::Buffer integrated(s, width * height * sizeof(float));
    data_image.GetLinearIntegrated(integrated.F());
    s.D2H(image.data(), integrated.Ptr(), image.size() * sizeof(float));
  }
  std::vector<size_t> psf_indices;
  subimages_ = MakeSubImages(image, width, height, mask_, psf_offsets, settings_,
                             psf_indices);
  ImageSet result_model(model_image, width, height);
  result_model.Fill(0.0f);
  for (SubImage& sub : subimages_)
    RunSubImage(sub, data_image, model_image, result_model,
                psf_images[psf_indices[sub.index]], 0.0, true);
  double start_peak = 0.0;
  for (const SubImage& sub : subimages_)
    if (sub.peak > start_peak) start_peak = sub.peak;
  const double threshold = start_peak * (1.0 - major_loop_gain);
  log::Info() << "Maximum start peak over " << subimages_.size()
              << " subimages: " << start_peak << '\n';
  for (SubImage& sub : subimages_)
    RunSubImage(sub, data_image, model_image, result_model,
                psf_images[psf_indices[sub.index]], threshold, false);
  model_image.CopyFrom(result_model);

  ParallelDeconvolutionResult result;
  result.start_peak = float(start_peak);
  size_t finished = 0;
  bool reached_max = false;
  double end_peak = 0.0;
  for (const SubImage& sub : subimages_) {
    if (!sub.reached_major_threshold) ++finished;
    if (algorithms_[sub.index]->IterationNumber() >=
        algorithms_[sub.index]->MaxIterations())
      reached_max = true;
    end_peak = std::max(end_peak, sub.peak);
  }
  result.end_peak = float(end_peak);
  result.another_iteration_required = finished != subimages_.size() && !reached_max;
  log::Info() << finished << " / " << subimages_.size() << " sub-images finished\n";
  return result;
}

}  // namespace radler::algorithms
