// Line references are to the reference's
// cpp/algorithms/parallel_deconvolution.cc.
#include "parallel_deconvolution.h"

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cmath>
#include <cstdlib>
#include <exception>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <new>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>

#include "dijkstra_splitter.h"
#include "host_profile.h"
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

void ParallelDeconvolution::SetAutoMaskMode(bool track_per_scale_masks,
                                            bool use_per_scale_masks) {
  track_masks_ = track_per_scale_masks;
  use_masks_ = use_per_scale_masks;
  for (auto& a : algorithms_)
    if (auto* ms = dynamic_cast<MultiScaleAlgorithm*>(a.get()))
      ms->SetAutoMaskMode(track_per_scale_masks, use_per_scale_masks);
}

void ParallelDeconvolution::LoadScaleMasks(const SubImage& sub, size_t width) {
  if (!use_masks_ && !track_masks_) return;
  auto* ms = dynamic_cast<MultiScaleAlgorithm*>(algorithms_[sub.index].get());
  if (!ms) return;
  const std::lock_guard<std::mutex> lock(masks_mutex_);
  if (scale_masks_.empty()) return;
  ms->SetScaleMaskCount(std::max(ms->GetScaleMaskCount(), scale_masks_.size()));
  for (size_t i = 0; i != ms->GetScaleMaskCount(); ++i) {
    std::vector<uint8_t>& m = ms->GetScaleMask(i);
    m.assign(sub.width * sub.height, 0);
    if (i >= scale_masks_.size()) continue;
    // scale mask box AND the subimage's clean mask (:376-386)
    for (size_t y = 0; y != sub.height; ++y)
      for (size_t x = 0; x != sub.width; ++x) {
        const size_t p = y * sub.width + x;
        m[p] = (scale_masks_[i][(sub.y + y) * width + sub.x + x] && sub.mask[p]) ? 1 : 0;
      }
  }
}

std::vector<std::vector<uint8_t>> ParallelDeconvolution::SubImageScaleMasks(
    const SubImage& sub) {
  std::vector<std::vector<uint8_t>> out;
  auto* ms = dynamic_cast<MultiScaleAlgorithm*>(algorithms_[sub.index].get());
  if (!ms) return out;
  for (size_t i = 0; i != ms->ScaleCount() && i != ms->GetScaleMaskCount(); ++i)
    out.push_back(ms->GetScaleMask(i));
  return out;
}

void ParallelDeconvolution::StoreScaleMasks(
    const SubImage& sub, size_t width, size_t height,
    const std::vector<std::vector<uint8_t>>& sub_masks) {
  const std::lock_guard<std::mutex> lock(masks_mutex_);
  if (scale_masks_.empty())
    scale_masks_.assign(sub_masks.size(), std::vector<uint8_t>(width * height, 0));
  for (size_t i = 0; i != sub_masks.size() && i != scale_masks_.size(); ++i)
    for (size_t y = 0; y != sub.height; ++y)
      for (size_t x = 0; x != sub.width; ++x) {
        const size_t p = y * sub.width + x;
        if (sub.boundary_mask[p])
          scale_masks_[i][(sub.y + y) * width + sub.x + x] = sub_masks[i][p];
      }
}

void ParallelDeconvolution::SetRmsFactorImage(
    std::shared_ptr<const std::vector<float>> image, size_t width) {
  if (algorithms_.size() == 1) {
    algorithms_.front()->SetRmsFactorImage(std::move(image));
  } else {
    rms_image_ = std::move(image);
    rms_width_ = width;
  }
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
  // one image set over the ranks: joined channels are shared by channel
  // (MultiScaleAlgorithm::SetChannelShard)
  algorithm.SetChannelShard(comm_ && comm_->Size() > 1 ? comm_.get() : nullptr);
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

namespace {

// Run f(0..n-1) on up to `threads` host threads (work items claimed in order).
template <typename F>
void ParallelFor(size_t n, size_t threads, F&& f) {
  threads = std::max<size_t>(1, std::min(threads, n));
  if (threads == 1) {
    for (size_t i = 0; i != n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::exception_ptr> errors(threads);
  std::vector<std::thread> pool;
  for (size_t t = 0; t != threads; ++t)
    pool.emplace_back([&, t] {
      try {
        for (size_t i = next++; i < n; i = next++) f(i);
      } catch (...) {
        errors[t] = std::current_exception();
      }
    });
  for (std::thread& th : pool) th.join();
  for (std::exception_ptr& e : errors)
    if (e) std::rethrow_exception(e);
}

size_t HostThreads() {
  const size_t hw = std::thread::hardware_concurrency();
  return std::max<size_t>(1, std::min<size_t>(hw ? hw : 1, 16));
}

}  // namespace

// MakeSubImages (parallel_deconvolution.cc:57-166): Dijkstra dividers through
// the integrated image, then per grid cell the overlap of its vertical and
// horizontal areas; the subimage mask is that overlap, ANDed with the user
// clean mask when there is one.
//
// Same result as DijkstraSplitter's FloodVerticalArea / FloodHorizontalArea /
// GetBoundingMask sequence (the reference's), computed as intervals: every
// row of a vertical area is one run [left, right) of columns (the flood walks
// outwards from the area's centre column over zeros, plus the divider pixels
// on its left), and every column of a horizontal area one run [top, bottom)
// of rows, so the overlap of a cell needs no full-image masks. The dividers
// are independent searches in disjoint bands (each writes only its band) and
// run concurrently, as do the cells.
std::vector<SubImage> MakeSubImages(const std::vector<float>& image, size_t width,
                                    size_t height, const bool* user_mask,
                                    const std::vector<PsfOffset>& psf_offsets,
                                    const Settings& settings,
                                    std::vector<size_t>& psf_indices) {
  const size_t gw = settings.parallel.grid_width, gh = settings.parallel.grid_height;
  const size_t avg_w = width / gw, avg_h = height / gh;
  math::DijkstraSplitter splitter(width, height);
  // the divider planes: zero pages from calloc (the searches write only
  // their bands and the floods mostly read zeros; value-initialised vectors
  // wrote 2 x 4 bytes per pixel first, ~0.1 s of the split at 8192^2)
  struct FreeDeleter {
    void operator()(float* p) const { std::free(p); }
  };
  auto zero_plane = [&] {
    std::unique_ptr<float, FreeDeleter> p(static_cast<float*>(std::calloc(width * height, sizeof(float))));
    if (!p) throw std::bad_alloc();
    return p;
  };
  std::unique_ptr<float, FreeDeleter> dividing_v = zero_plane(), dividing_h = zero_plane();
  {
    prof::Section p("split.divide");
    const size_t n_div = (gw - 1) + (gh - 1);
    ParallelFor(n_div, HostThreads(), [&](size_t k) {
      if (k + 1 < gw) {
        const size_t mid = width * (k + 1) / gw;
        splitter.DivideVertically(image.data(), dividing_v.get(), mid - avg_w / 4,
                                  mid + avg_w / 4);
      } else {
        const size_t mid = height * (k + 2 - gw) / gh;
        splitter.DivideHorizontally(image.data(), dividing_h.get(), mid - avg_h / 4,
                                    mid + avg_h / 4);
      }
    });
  }
  prof::Section p_masks("split.masks");
  // FloodVerticalArea per grid column: [left, right) per row
  struct Runs {
    std::vector<uint32_t> lo, hi;
    size_t start = 0, extent = 0;  // x, width (or y, height) of the area
  };
  std::vector<Runs> columns(gw), rows(gh);
  ParallelFor(gw + gh, HostThreads(), [&](size_t k) {
    const bool vertical = k < gw;
    const size_t d = vertical ? k : k - gw;
    const size_t n = vertical ? height : width;        // runs
    const size_t len = vertical ? width : height;      // along a run
    const size_t stride = vertical ? 1 : width;        // step along a run
    const size_t across = vertical ? width : 1;        // step between runs
    const float* div = vertical ? dividing_v.get() : dividing_h.get();
    const size_t centre = vertical ? d * width / gw + avg_w / 2
                                   : d * height / gh + avg_h / 2;
    Runs& r = vertical ? columns[d] : rows[d];
    r.lo.resize(n);
    r.hi.resize(n);
    size_t first = len, last = 0;
    for (size_t j = 0; j != n; ++j) {
      const float* line = div + j * across;
      int64_t i = int64_t(centre);
      for (; i >= 0 && line[i * stride] == 0.0f; --i) {
      }
      for (; i >= 0 && line[i * stride] != 0.0f; --i) {
      }
      const size_t lo = size_t(i + 1);
      size_t hi = centre + 1;
      for (; hi < len && line[hi * stride] == 0.0f; ++hi) {
      }
      r.lo[j] = uint32_t(lo);
      r.hi[j] = uint32_t(hi);
      first = std::min(first, lo);
      last = std::max(last, hi);
    }
    r.start = first;
    r.extent = last < first ? 0 : last - first;
  });
  dividing_v.reset();
  dividing_h.reset();

  // GetBoundingMask per cell: inside(x, y) = x in column run of row y and
  // y in row-area run of column x
  std::vector<SubImage> subs(gw * gh);
  ParallelFor(gw * gh, HostThreads(), [&](size_t index) {
    const size_t gy = index / gw, gx = index % gw;
    const Runs& col = columns[gx];
    const Runs& row = rows[gy];
    auto inside = [&](size_t x, size_t y) {
      return x >= col.lo[y] && x < col.hi[y] && y >= row.lo[x] && y < row.hi[x];
    };
    // rows that can hold the cell: the row area's extent over the column's x range
    size_t y_from = height, y_to = 0;
    for (size_t x = col.start; x < col.start + col.extent; ++x) {
      y_from = std::min<size_t>(y_from, row.lo[x]);
      y_to = std::max<size_t>(y_to, row.hi[x]);
    }
    size_t x_lo = col.extent + col.start, y_lo = height, x_hi = 0, y_hi = 0;
    for (size_t y = y_from; y < y_to; ++y)
      for (size_t x = col.lo[y]; x < col.hi[y]; ++x)
        if (y >= row.lo[x] && y < row.hi[x]) {
          x_lo = std::min(x_lo, x);
          x_hi = std::max(x_hi, x);
          y_lo = std::min(y_lo, y);
          y_hi = y;
        }
    SubImage& sub = subs[index];
    sub.index = index;
    size_t sw = 0, sh = 0;
    if (x_hi >= x_lo) {
      sw = x_hi + 1 - x_lo;
      sh = y_hi + 1 - y_lo;
    }
    // even images keep even subimages: one more column/row (to the left/top
    // when the right/bottom edge would leave the image), masked out
    // (dijkstra_splitter.cc GetBoundingMask)
    size_t ext_col = SIZE_MAX, ext_row = SIZE_MAX;
    if (width % 2 == 0 && sw % 2 != 0) {
      ++sw;
      ext_col = sw + x_lo >= width ? --x_lo : x_lo + sw - 1;
    }
    if (height % 2 == 0 && sh % 2 != 0) {
      ++sh;
      ext_row = sh + y_lo >= height ? --y_lo : y_lo + sh - 1;
    }
    sub.x = x_lo;
    sub.y = y_lo;
    sub.width = sw;
    sub.height = sh;
    sub.mask.assign(sw * sh, false);
    for (size_t y = 0; y != sh; ++y) {
      const size_t gy_ = y + y_lo;
      if (gy_ == ext_row) continue;
      const size_t from = std::max<size_t>(col.lo[gy_], x_lo);
      const size_t to = std::min<size_t>(col.hi[gy_], x_lo + sw);
      for (size_t gx_ = from; gx_ < to; ++gx_)
        if (gx_ != ext_col && inside(gx_, gy_)) sub.mask[y * sw + gx_ - x_lo] = true;
    }
    sub.boundary_mask = sub.mask;
    if (user_mask)
      for (size_t y = 0; y != sh; ++y)
        for (size_t x = 0; x != sw; ++x)
          sub.mask[y * sw + x] =
              sub.mask[y * sw + x] && user_mask[(y + sub.y) * width + x + sub.x];
  });
  for (const SubImage& sub : subs)
    psf_indices.push_back(NearestPsfIndex(psf_offsets, sub.x + sub.width / 2,
                                          sub.y + sub.height / 2));
  return subs;
}

namespace {

std::vector<uint8_t> MaskBytes(const std::vector<bool>& mask) {
  std::vector<uint8_t> b(mask.size());
  for (size_t i = 0; i != mask.size(); ++i) b[i] = mask[i] ? 1 : 0;
  return b;
}

// ImageSet::Trim / TrimMasked of the data and model planes and the centred
// Image::Resize of the PSFs into contiguous subimage planes, as box copies
// ordered on `ops` (parallel_deconvolution.cc:300-357)
void TrimSubImage(gpu::Session& ops, const SubImage& sub, const ImageSet& data_image,
                  const ImageSet& model_image, const gpu::Planes& psfs,
                  float* d_data, float* d_model, float* d_psfs,
                  const uint8_t* d_boundary) {
  prof::Section prof_section("par.trim");
  const size_t W = data_image.Width();
  const uint32_t uw = uint32_t(sub.width), uh = uint32_t(sub.height);
  const size_t n = sub.width * sub.height;
  for (size_t i = 0; i != data_image.Size(); ++i) {
    gpu::Check(rdl_box(ops.Handle(), d_data + i * n, uw, 0, 0, data_image.Data(i),
                       uint32_t(W), uint32_t(sub.x), uint32_t(sub.y), uw, uh,
                       nullptr, RDL_BOX_COPY),
               "rdl_box");  // ImageSet::Trim
    gpu::Check(rdl_box(ops.Handle(), d_model + i * n, uw, 0, 0, model_image.Data(i),
                       uint32_t(W), uint32_t(sub.x), uint32_t(sub.y), uw, uh,
                       d_boundary, RDL_BOX_COPY_ZERO),
               "rdl_box");  // ImageSet::TrimMasked
  }
  // Image::Resize (:323-330), centred per axis: a PSF larger than the
  // subimage is cropped, a smaller one (a fine DD-PSF grid) zero-padded
  const size_t cw = std::min(psfs.width, sub.width), ch = std::min(psfs.height, sub.height);
  const size_t src_x = (psfs.width - cw) / 2, src_y = (psfs.height - ch) / 2;
  const size_t dst_x = (sub.width - cw) / 2, dst_y = (sub.height - ch) / 2;
  if (cw != sub.width || ch != sub.height) ops.Zero(d_psfs, psfs.count * n * sizeof(float));
  for (size_t i = 0; i != psfs.count; ++i)
    gpu::Check(rdl_box(ops.Handle(), d_psfs + i * n, uw, uint32_t(dst_x), uint32_t(dst_y),
                       psfs.Plane(i), uint32_t(psfs.width), uint32_t(src_x),
                       uint32_t(src_y), uint32_t(cw), uint32_t(ch), nullptr, RDL_BOX_COPY),
               "rdl_box");
}

// ImageSet::CopyMasked of the residual (only when the subimage converged) and
// ImageSet::AddSubImage of the model (parallel_deconvolution.cc:458-484)
void MergeSubImage(gpu::Session& ops, const SubImage& sub, ImageSet& data_image,
                   ImageSet& result_model, const float* d_data,
                   const float* d_model, const uint8_t* d_boundary,
                   bool converging) {
  prof::Section prof_section("par.merge");
  const size_t W = data_image.Width();
  const uint32_t uw = uint32_t(sub.width), uh = uint32_t(sub.height);
  const size_t n = sub.width * sub.height;
  for (size_t i = 0; i != data_image.Size(); ++i) {
    if (converging)
      gpu::Check(rdl_box(ops.Handle(), data_image.Data(i), uint32_t(W),
                         uint32_t(sub.x), uint32_t(sub.y), d_data + i * n, uw, 0, 0,
                         uw, uh, d_boundary, RDL_BOX_COPY_MASKED),
                 "rdl_box");
    gpu::Check(rdl_box(ops.Handle(), result_model.Data(i), uint32_t(W),
                       uint32_t(sub.x), uint32_t(sub.y), d_model + i * n, uw, 0, 0,
                       uw, uh, nullptr, RDL_BOX_ADD),
               "rdl_box");
  }
}

}  // namespace

bool ParallelDeconvolution::DeconvolveSubImage(SubImage& sub, ImageSet& sub_data,
                                               ImageSet& sub_model,
                                               const gpu::Planes& sub_psfs,
                                               double major_iteration_threshold,
                                               bool find_peak_only) {
  // parallel_deconvolution.cc:363-456
  DeconvolutionAlgorithm& alg = *algorithms_[sub.index];
  std::vector<char> mask_copy(sub.mask.begin(), sub.mask.end());
  alg.SetCleanMask(reinterpret_cast<const bool*>(mask_copy.data()));
  if (rms_image_) {  // rms_image_.TrimBox (:332-337)
    auto sub_rms = std::make_shared<std::vector<float>>(sub.width * sub.height);
    for (size_t y = 0; y != sub.height; ++y)
      std::copy_n(rms_image_->data() + (sub.y + y) * rms_width_ + sub.x, sub.width,
                  sub_rms->data() + y * sub.width);
    alg.SetRmsFactorImage(std::move(sub_rms));
  }
  const size_t max_n_iter = alg.MaxIterations();
  if (find_peak_only)
    alg.SetMaxIterations(0);
  else
    alg.SetMajorIterationThreshold(float(major_iteration_threshold));
  const double peak_at_start = std::fabs(sub.peak);
  const DeconvolutionResult result =
      alg.ExecuteMajorIteration(sub_data, sub_model, sub_psfs);
  alg.SetCleanMask(nullptr);
  if (rms_image_) alg.SetRmsFactorImage(nullptr);  // :421-423
  sub.peak = result.final_peak_value;
  sub.reached_major_threshold = result.another_iteration_required;
  const bool converging =
      (settings_.divergence_limit == 0.0 ||
       std::fabs(sub.peak) <= peak_at_start * settings_.divergence_limit) &&
      std::isfinite(sub.peak) && !result.is_diverging;
  if (find_peak_only) {
    alg.SetMaxIterations(max_n_iter);
  } else if (!converging) {
    log::Warn() << "Peak of sub-image " << sub.index << " increased from "
                << peak_at_start << " to " << sub.peak
                << " and deconvolution probably diverged: resetting.\n";
    sub.reached_major_threshold = false;
  }
  // :464-479: a converging multiscale subimage's components join the
  // full-image list at the subimage offset
  if (!find_peak_only && settings_.save_source_list && algorithms_.size() > 1 &&
      settings_.algorithm_type == AlgorithmType::kMultiscale) {
    auto& ms = static_cast<MultiScaleAlgorithm&>(alg);
    if (converging && ms.HasComponentList()) {
      const std::lock_guard<std::mutex> lock(masks_mutex_);
      if (!component_list_)
        component_list_ = std::make_unique<ComponentList>(
            settings_.trimmed_image_width, settings_.trimmed_image_height,
            ms.ScaleCount(), sub_data.Size());
      component_list_->Add(ms.GetComponentList(), int(sub.x), int(sub.y));
    }
    ms.ClearComponentList();
  }
  return converging;
}

ComponentList ParallelDeconvolution::GetMultiscaleComponentList() const {
  // :184-196: the single algorithm's list, or the merged subimage lists
  ComponentList list;
  if (algorithms_.size() == 1) {
    const auto& ms = static_cast<const MultiScaleAlgorithm&>(*algorithms_.front());
    if (ms.HasComponentList()) list = ms.GetComponentList();
  } else if (component_list_) {
    list = *component_list_;
  }
  list.MergeDuplicates();
  return list;
}

void ParallelDeconvolution::RunSubImage(SubImage& sub, ImageSet& data_image,
                                        const ImageSet& model_image,
                                        ImageSet& result_model,
                                        const gpu::Planes& psfs,
                                        double major_iteration_threshold,
                                        bool find_peak_only) {
  // parallel_deconvolution.cc:300-484 on the device: the subimage's planes
  // are box copies of the full image set's planes
  prof::Section prof_section(find_peak_only ? "par.run_subimage_findpeak"
                                             : "par.run_subimage_clean");
  gpu::Session& s = data_image.Session();
  const size_t sw = sub.width, sh = sub.height, n = sw * sh;
  gpu::Buffer boundary(s, n);
  s.H2D(boundary.Ptr(), MaskBytes(sub.boundary_mask).data(), n);
  const uint8_t* d_boundary = static_cast<const uint8_t*>(boundary.Ptr());
  ImageSet sub_data(data_image, sw, sh);
  ImageSet sub_model(model_image, sw, sh);
  gpu::Planes sub_psfs = gpu::Planes::Make(s, sw, sh, psfs.count);
  TrimSubImage(s, sub, data_image, model_image, psfs, sub_data.Base(),
               sub_model.Base(), sub_psfs.Base(), d_boundary);
  ImageSet initial_model(sub_model, sw, sh);
  initial_model.CopyFrom(sub_model);
  LoadScaleMasks(sub, data_image.Width());
  const bool converging = DeconvolveSubImage(
      sub, sub_data, sub_model, sub_psfs, major_iteration_threshold, find_peak_only);
  if (find_peak_only) return;
  if (track_masks_ && converging)
    StoreScaleMasks(sub, data_image.Width(), data_image.Height(), SubImageScaleMasks(sub));
  MergeSubImage(s, sub, data_image, result_model, sub_data.Base(),
                converging ? sub_model.Base() : initial_model.Base(), d_boundary,
                converging);
  s.Sync();
}

std::vector<int> ParallelDeconvolution::PoolDevices(int main_device) {
  // RADLER_DEVICES="0,1,2,3" spreads the subimage workers over those GPUs;
  // by default they share the device of the image set
  std::vector<int> devices;
  if (const char* env = std::getenv("RADLER_DEVICES")) {
    int count = 0;
    gpu::Check(rdl_device_count(&count), "rdl_device_count");
    std::string list(env);
    size_t pos = 0;
    while (pos < list.size()) {
      size_t end = list.find(',', pos);
      if (end == std::string::npos) end = list.size();
      const std::string item = list.substr(pos, end - pos);
      if (!item.empty()) {
        const int d = std::stoi(item);
        if (d < 0 || d >= count)
          throw std::runtime_error("RADLER_DEVICES names device " + item +
                                   ", which does not exist");
        devices.push_back(d);
      }
      pos = end + 1;
    }
  }
  if (devices.empty()) devices.push_back(main_device);
  return devices;
}

void ParallelDeconvolution::EnsureWorkers(gpu::Session& main, size_t n) {
  if (workers_.size() == n && worker_main_device_ == main.Device()) return;
  if (!workers_.empty())
    throw std::runtime_error(
        "ParallelDeconvolution: the subimage worker pool cannot change between "
        "major iterations");
  const std::vector<int> devices = PoolDevices(main.Device());
  std::map<int, size_t> per_device;
  for (size_t w = 0; w != n; ++w) {
    const int d = devices[w % devices.size()];
    workers_.push_back(gpu::Session::Worker(d, per_device[d]));
    ++per_device[d];
  }
  for (auto& w : workers_) w->SetConcurrency(per_device[w->Device()]);
  worker_main_device_ = main.Device();
  main.Bind();
}

void ParallelDeconvolution::RunSubImagesConcurrently(
    ImageSet& data_image, const ImageSet& model_image, ImageSet& result_model,
    const std::vector<gpu::Planes>& psf_images,
    const std::vector<size_t>& psf_indices, double major_iteration_threshold,
    bool find_peak_only, const std::vector<char>* run, const SubImageSink& sink) {
  // The reference runs RunSubImage on settings.parallel.max_threads threads
  // (parallel_deconvolution.cc:583-616), each trimming from the shared
  // residual and copying back under a mutex. Here every subimage trims from
  // the residual as it was when the pass started and the copy-backs are
  // applied afterwards in subimage order: the schedule the reference takes
  // when all its threads trim before the first one finishes, made
  // deterministic. Boundary masks are disjoint and the model additions
  // outside them add zeros, so the merged result does not depend on the
  // number of workers or devices.
  gpu::Session& s = data_image.Session();
  const int main_device = s.Device();
  const size_t n_sub = subimages_.size(), W = workers_.size();
  const size_t n_img = data_image.Size();
  // RADLER_POOL_STAGING=1 routes same-device workers through the staging
  // buffers and peer copies a worker on another GPU uses (exercised by the
  // one-GPU tests)
  const char* staging_env = std::getenv("RADLER_POOL_STAGING");
  const bool force_staging = staging_env && staging_env[0] == '1';
  struct Slot {
    gpu::Session* ws = nullptr;
    bool remote = false;
    // main-device staging of a remote worker's planes (data | model | psfs)
    std::unique_ptr<gpu::Buffer> stage;
    std::unique_ptr<gpu::Buffer> boundary;  // on the main device
    std::unique_ptr<ImageSet> data, model, initial;
    gpu::Planes psfs;
    bool converging = false;
  };
  std::vector<Slot> slots(n_sub);
  std::vector<size_t> todo;  // the subimages this call runs, in index order
  for (size_t i = 0; i != n_sub; ++i)
    if (!run || (*run)[i]) todo.push_back(i);
  // The subimages' assignment to the pool's workers (on the main device):
  //   0: fixed round robin (subimage k on worker k mod W);
  //   1: one queue, the costliest first (the longest-processing-time rule:
  //      the cleaning pass's estimate from the start peaks, as the ranks'
  //      LptOwners; the find-peak pass by area);
  //   2: one queue in index order (first free worker takes the next).
  // Default: 1 for image sets of several images (joined channels), 0 for
  // one image; RADLER_POOL_QUEUE overrides. Measured with the stream pool
  // (r06, bench_legs.py, one job): 8 x 4096^2 joined split 8 x 8 — 0: 4.61-
  // 4.63 s, 1: 3.91-4.08 s, 2: 4.15-4.38 s; 8192^2 split 8 x 8 — 0: 4.03-
  // 4.08 s, 1: 4.17-4.23 s, 2: 4.17-4.46 s. Workers on other GPUs always
  // keep the fixed assignment (their planes are staged on the main device
  // before the pass). The result does not depend on the assignment (the
  // snapshot schedule; tests/test_tiling.py::test_concurrent_pool_queue).
  const char* queue_env = std::getenv("RADLER_POOL_QUEUE");
  const int queue_mode =
      queue_env ? std::atoi(queue_env) : (data_image.Size() > 1 ? 1 : 0);
  bool all_local = !force_staging && queue_mode >= 1 && queue_mode <= 3;
  for (size_t w = 0; w != W; ++w) all_local = all_local && workers_[w]->Device() == main_device;
  // 3: the cost order dealt round robin (worker w: the w-th, (w + W)-th, ...
  // costliest), a fixed assignment (measured: joined split 4.29-4.32 s, the
  // 8192^2 split 4.12-4.41 s; neither default improves)
  const bool dynamic = all_local && queue_mode != 3;
  std::vector<size_t> order = todo;
  if (all_local && queue_mode != 2) {
    const double thr = std::max<double>(algorithms_.front()->Threshold(), 1e-30);
    std::vector<double> cost(n_sub, 0.0);
    for (const size_t i : todo) {
      const SubImage& sub = subimages_[i];
      const double above = find_peak_only ? 1.0 : std::max(std::fabs(sub.peak), thr) / thr;
      cost[i] = double(sub.width * sub.height) * (1.0 + std::log2(above));
    }
    std::stable_sort(order.begin(), order.end(),
                     [&](size_t a, size_t b) { return cost[a] > cost[b]; });
  }
  for (size_t k = 0; k != todo.size(); ++k) {
    const size_t i = todo[k];
    Slot& slot = slots[i];
    const SubImage& sub = subimages_[i];
    const size_t n = sub.width * sub.height;
    const gpu::Planes& psfs = psf_images[psf_indices[i]];
    slot.ws = workers_[k % W].get();
    slot.remote = force_staging || slot.ws->Device() != main_device;
    slot.boundary = std::make_unique<gpu::Buffer>(s, n);
    s.H2D(slot.boundary->Ptr(), MaskBytes(sub.boundary_mask).data(), n);
    if (slot.remote) {
      slot.stage = std::make_unique<gpu::Buffer>(
          s, (2 * n_img + psfs.count) * n * sizeof(float));
      float* base = slot.stage->F();
      TrimSubImage(s, sub, data_image, model_image, psfs, base, base + n_img * n,
                   base + 2 * n_img * n,
                   static_cast<const uint8_t*>(slot.boundary->Ptr()));
    }
  }
  s.Sync();

  std::vector<std::exception_ptr> errors(W);
  std::atomic<size_t> next{0};
  std::atomic<bool> failed{false};
  auto work = [&](size_t w) {
    try {
      gpu::Session& ws = *workers_[w];
      ws.Bind();
      for (size_t k = dynamic ? next.fetch_add(1) : w; k < todo.size() && !failed;
           k = dynamic ? next.fetch_add(1) : k + W) {
        const size_t i = all_local ? order[k] : todo[k];
        Slot& slot = slots[i];
        slot.ws = &ws;
        SubImage& sub = subimages_[i];
        const size_t sw = sub.width, sh = sub.height, n = sw * sh;
        const gpu::Planes& psfs = psf_images[psf_indices[i]];
        slot.data = std::make_unique<ImageSet>(data_image, sw, sh, ws);
        slot.model = std::make_unique<ImageSet>(model_image, sw, sh, ws);
        slot.psfs = gpu::Planes::Make(ws, sw, sh, psfs.count);
        if (slot.remote) {
          const float* base = slot.stage->F();
          ws.Peer(slot.data->Base(), ws.Device(), base, main_device,
                  n_img * n * sizeof(float));
          ws.Peer(slot.model->Base(), ws.Device(), base + n_img * n, main_device,
                  n_img * n * sizeof(float));
          ws.Peer(slot.psfs.Base(), ws.Device(), base + 2 * n_img * n, main_device,
                  psfs.count * n * sizeof(float));
        } else {
          TrimSubImage(ws, sub, data_image, model_image, psfs, slot.data->Base(),
                       slot.model->Base(), slot.psfs.Base(),
                       static_cast<const uint8_t*>(slot.boundary->Ptr()));
        }
        if (!find_peak_only) {
          slot.initial = std::make_unique<ImageSet>(*slot.model, sw, sh);
          slot.initial->CopyFrom(*slot.model);
        }
        LoadScaleMasks(sub, data_image.Width());
        slot.converging = DeconvolveSubImage(sub, *slot.data, *slot.model,
                                             slot.psfs, major_iteration_threshold,
                                             find_peak_only);
        // boundary masks are disjoint: merging in any order gives one result
        if (track_masks_ && slot.converging && !find_peak_only)
          StoreScaleMasks(sub, data_image.Width(), data_image.Height(),
                          SubImageScaleMasks(sub));
        if (slot.remote && !find_peak_only) {
          float* base = slot.stage->F();
          const ImageSet& model_out = slot.converging ? *slot.model : *slot.initial;
          ws.Peer(base, main_device, slot.data->Base(), ws.Device(),
                  n_img * n * sizeof(float));
          ws.Peer(base + n_img * n, main_device, model_out.Base(), ws.Device(),
                  n_img * n * sizeof(float));
        }
        ws.Sync();
        if (find_peak_only || slot.remote) {
          slot.data.reset();
          slot.model.reset();
          slot.initial.reset();
          slot.psfs = gpu::Planes();
        }
      }
      ws.Sync();
    } catch (...) {
      errors[w] = std::current_exception();
      failed = true;
    }
  };
  std::vector<std::thread> threads;
  threads.reserve(W);
  for (size_t w = 0; w != W; ++w) threads.emplace_back(work, w);
  for (std::thread& t : threads) t.join();
  s.Bind();
  for (std::exception_ptr& e : errors)
    if (e) std::rethrow_exception(e);
  if (find_peak_only) return;

  for (const size_t i : todo) {
    Slot& slot = slots[i];
    const SubImage& sub = subimages_[i];
    const size_t n = sub.width * sub.height;
    const float* d_data;
    const float* d_model;
    if (slot.remote) {
      d_data = slot.stage->F();
      d_model = d_data + n_img * n;
    } else {
      d_data = slot.data->Base();
      d_model = (slot.converging ? slot.model : slot.initial)->Base();
    }
    if (sink)
      sink(i, d_data, d_model, slot.converging);
    else
      MergeSubImage(s, sub, data_image, result_model, d_data, d_model,
                    static_cast<const uint8_t*>(slot.boundary->Ptr()),
                    slot.converging);
  }
  s.Sync();
}

double ParallelDeconvolution::RunSubImagesDistributed(
    ImageSet& data_image, const ImageSet& model_image, ImageSet& result_model,
    const std::vector<gpu::Planes>& psf_images,
    const std::vector<size_t>& psf_indices, double major_iteration_threshold,
    bool find_peak_only) {
  // The reference's threads (parallel_deconvolution.cc:583-616) become ranks:
  // subimage i runs on rank SubImageOwner(i). Every owned subimage trims from
  // the residual as it was when the pass started (the snapshot schedule of
  // RunSubImagesConcurrently), so the merged result is the same for any
  // number of ranks, and equal to the one-process pool's.
  gpu::Session& s = data_image.Session();
  Communicator& comm = *comm_;
  const int rank = comm.Rank(), n_ranks = comm.Size();
  const size_t n_sub = subimages_.size(), n_img = data_image.Size();
  // per subimage: a 64-byte record, then the residual and model planes
  struct Record {
    double peak;
    uint64_t iteration_number;
    uint32_t reached_major_threshold;
    uint32_t converging;
    uint32_t n_mask_scales;  // tracked auto-masks that follow (second broadcast)
    uint32_t pad[9];
  };
  static_assert(sizeof(Record) == 64, "record layout");
  constexpr size_t kHeaderFloats = sizeof(Record) / sizeof(float);
  std::vector<std::unique_ptr<gpu::Buffer>> packs(n_sub);
  std::vector<std::vector<std::vector<uint8_t>>> mask_sets(n_sub);
  const bool lpt = !find_peak_only && clean_owners_.size() == n_sub;
  auto owner_of = [&](size_t i) {
    return lpt ? clean_owners_[i] : SubImageOwner(i, n_ranks);
  };
  // a packed result: the record, then the residual and model boxes
  auto pack_result = [&](size_t i, const float* d_data, const float* d_model,
                         bool converging) {
    SubImage& sub = subimages_[i];
    const size_t n = sub.width * sub.height;
    auto pack = std::make_unique<gpu::Buffer>(
        s, (kHeaderFloats + 2 * n_img * n) * sizeof(float));
    Record rec{};
    rec.peak = sub.peak;
    rec.iteration_number = algorithms_[i]->IterationNumber();
    rec.reached_major_threshold = sub.reached_major_threshold ? 1u : 0u;
    rec.converging = converging ? 1u : 0u;
    if (track_masks_ && converging) {
      mask_sets[i] = SubImageScaleMasks(sub);
      rec.n_mask_scales = uint32_t(mask_sets[i].size());
    }
    s.H2D(pack->Ptr(), &rec, sizeof(rec));
    float* base = pack->F() + kHeaderFloats;
    s.D2D(base, d_data, n_img * n * sizeof(float));
    s.D2D(base + n_img * n, d_model, n_img * n * sizeof(float));
    packs[i] = std::move(pack);
  };
  if (!workers_.empty()) {
    // this rank's subimages on its worker pool (concurrent streams)
    std::vector<char> mine(n_sub, 0);
    for (size_t i = 0; i != n_sub; ++i) mine[i] = owner_of(i) == rank ? 1 : 0;
    RunSubImagesConcurrently(data_image, model_image, result_model, psf_images,
                             psf_indices, major_iteration_threshold, find_peak_only,
                             &mine, pack_result);
  }
  for (size_t i = 0; i != n_sub && workers_.empty(); ++i) {
    if (owner_of(i) != rank) continue;
    SubImage& sub = subimages_[i];
    const size_t sw = sub.width, sh = sub.height, n = sw * sh;
    const gpu::Planes& psfs = psf_images[psf_indices[i]];
    gpu::Buffer boundary(s, n);
    s.H2D(boundary.Ptr(), MaskBytes(sub.boundary_mask).data(), n);
    ImageSet sub_data(data_image, sw, sh);
    ImageSet sub_model(model_image, sw, sh);
    gpu::Planes sub_psfs = gpu::Planes::Make(s, sw, sh, psfs.count);
    TrimSubImage(s, sub, data_image, model_image, psfs, sub_data.Base(),
                 sub_model.Base(), sub_psfs.Base(),
                 static_cast<const uint8_t*>(boundary.Ptr()));
    std::unique_ptr<ImageSet> initial;
    if (!find_peak_only) {
      initial = std::make_unique<ImageSet>(sub_model, sw, sh);
      initial->CopyFrom(sub_model);
    }
    LoadScaleMasks(sub, data_image.Width());
    const bool converging = DeconvolveSubImage(sub, sub_data, sub_model, sub_psfs,
                                               major_iteration_threshold,
                                               find_peak_only);
    if (find_peak_only) continue;
    pack_result(i, sub_data.Base(), (converging ? sub_model : *initial).Base(),
                converging);
  }
  s.Sync();
  if (find_peak_only) {
    // every rank gets every subimage's start peak (one RCCL allreduce(max)
    // of n_sub floats, the owners' entries against lowest()): the global
    // start peak (:592-599, signed, from 0.0) and the cost estimates of the
    // cleaning pass's ownership
    std::vector<float> peaks(n_sub, std::numeric_limits<float>::lowest());
    for (size_t i = 0; i != n_sub; ++i)
      if (SubImageOwner(i, n_ranks) == rank) peaks[i] = float(subimages_[i].peak);
    comm.AllreduceMax(s, peaks.data(), n_sub);
    double start_peak = 0.0;
    std::vector<double> costs(n_sub);
    const double thr = std::max<double>(algorithms_.front()->Threshold(), 1e-30);
    for (size_t i = 0; i != n_sub; ++i) {
      SubImage& sub = subimages_[i];
      sub.peak = peaks[i];
      if (sub.peak > start_peak) start_peak = sub.peak;
      // cleaning work grows with the subimage area and with how far its
      // peak lies above the threshold (components ~ log(peak/threshold)
      // per CLEANed source at a fixed gain)
      const double above = std::max(std::fabs(sub.peak), thr) / thr;
      costs[i] = double(sub.width * sub.height) * (1.0 + std::log2(above));
    }
    clean_owners_ = LptOwners(costs, n_ranks);
    return start_peak;
  }

  // copy-back (:458-484) in subimage order, identical on every rank
  std::unique_ptr<gpu::Buffer> staging;
  for (size_t i = 0; i != n_sub; ++i) {
    SubImage& sub = subimages_[i];
    const size_t n = sub.width * sub.height;
    const size_t bytes = (kHeaderFloats + 2 * n_img * n) * sizeof(float);
    const int owner = owner_of(i);
    gpu::Buffer* pack = packs[i].get();
    if (owner != rank) {
      if (!staging || staging->Bytes() < bytes)
        staging = std::make_unique<gpu::Buffer>(s, bytes);
      pack = staging.get();
    }
    comm.Broadcast(s, pack->Ptr(), bytes, owner);
    Record rec{};
    s.D2H(&rec, pack->Ptr(), sizeof(rec));
    if (owner != rank) {
      sub.peak = rec.peak;
      sub.reached_major_threshold = rec.reached_major_threshold != 0;
      algorithms_[i]->SetIterationNumber(size_t(rec.iteration_number));
    }
    gpu::Buffer boundary(s, n);
    s.H2D(boundary.Ptr(), MaskBytes(sub.boundary_mask).data(), n);
    const float* base = pack->F() + kHeaderFloats;
    MergeSubImage(s, sub, data_image, result_model, base, base + n_img * n,
                  static_cast<const uint8_t*>(boundary.Ptr()), rec.converging != 0);
    s.Sync();  // the staging buffer is reused by the next broadcast
    if (rec.n_mask_scales > 0) {  // the owner's tracked scale masks
      const size_t mb = size_t(rec.n_mask_scales) * n;
      gpu::Buffer dm(s, mb);
      if (owner == rank)
        for (size_t m = 0; m != rec.n_mask_scales; ++m)
          s.H2D(static_cast<uint8_t*>(dm.Ptr()) + m * n, mask_sets[i][m].data(), n);
      comm.Broadcast(s, dm.Ptr(), mb, owner);
      std::vector<std::vector<uint8_t>> masks(rec.n_mask_scales, std::vector<uint8_t>(n));
      for (size_t m = 0; m != rec.n_mask_scales; ++m)
        s.D2H(masks[m].data(), static_cast<const uint8_t*>(dm.Ptr()) + m * n, n);
      StoreScaleMasks(sub, data_image.Width(), data_image.Height(), masks);
    }
  }
  return 0.0;
}

ParallelDeconvolutionResult ParallelDeconvolution::ExecuteParallelRun(
    ImageSet& data_image, ImageSet& model_image,
    const std::vector<gpu::Planes>& psf_images,
    const std::vector<PsfOffset>& psf_offsets, double major_loop_gain) {
  // parallel_deconvolution.cc:556-654. One worker: subimages run one after
  // another in index order, each seeing the copy-backs of the ones before
  // (the reference with one thread). More workers (settings.parallel
  // .max_threads): subimages run concurrently on their own streams / GPUs,
  // see RunSubImagesConcurrently.
  gpu::Session& s = data_image.Session();
  const size_t width = data_image.Width(), height = data_image.Height();
  std::vector<float> image(width * height);
  {
    gpu::Buffer integrated(s, width * height * sizeof(float));
    data_image.GetLinearIntegrated(integrated.F());
    s.D2H(image.data(), integrated.Ptr(), image.size() * sizeof(float));
  }
  std::vector<size_t> psf_indices;
  {
    prof::Section prof_split("par.split");
    subimages_ = MakeSubImages(image, width, height, mask_, psf_offsets, settings_,
                               psf_indices);
  }
  ImageSet result_model(model_image, width, height);
  result_model.Fill(0.0f);
  // settings.parallel.max_threads subimages in flight (:583-616), at most
  // kMaxStreams streams per GPU: beyond that the streams only share the
  // hardware queues (Settings' default is the host's processor count)
  constexpr size_t kMaxStreams = 16;
  const size_t n_workers =
      std::min<size_t>(std::min<size_t>(std::max<size_t>(settings_.parallel.max_threads, 1),
                                        kMaxStreams * PoolDevices(s.Device()).size()),
                       subimages_.size());
  const bool distributed = comm_ != nullptr;
  const bool concurrent = !distributed && n_workers > 1;
  // with a communicator each rank runs its own subimages on a pool of its own
  const size_t rank_workers =
      distributed ? std::min<size_t>(n_workers, (subimages_.size() + comm_->Size() - 1) /
                                                    size_t(comm_->Size()))
                  : n_workers;
  if (rank_workers > 1) EnsureWorkers(s, rank_workers);
  double start_peak = 0.0;
  // (the passes' wall clock: the part of a major iteration that the ranks
  // split; bench.py's Amdahl estimate)
  std::optional<prof::Section> pass(std::in_place, "par.findpeak_pass");
  if (distributed) {
    start_peak = RunSubImagesDistributed(data_image, model_image, result_model,
                                         psf_images, psf_indices, 0.0, true);
  } else {
    if (concurrent)
      RunSubImagesConcurrently(data_image, model_image, result_model, psf_images,
                               psf_indices, 0.0, true);
    else
      for (SubImage& sub : subimages_)
        RunSubImage(sub, data_image, model_image, result_model,
                    psf_images[psf_indices[sub.index]], 0.0, true);
    for (const SubImage& sub : subimages_)
      if (sub.peak > start_peak) start_peak = sub.peak;
  }
  const double threshold = start_peak * (1.0 - major_loop_gain);
  log::Info() << "Maximum start peak over " << subimages_.size()
              << " subimages: " << start_peak << '\n';
  pass.emplace("par.clean_pass");
  if (distributed)
    RunSubImagesDistributed(data_image, model_image, result_model, psf_images,
                            psf_indices, threshold, false);
  else if (concurrent)
    RunSubImagesConcurrently(data_image, model_image, result_model, psf_images,
                             psf_indices, threshold, false);
  else
    for (SubImage& sub : subimages_)
      RunSubImage(sub, data_image, model_image, result_model,
                  psf_images[psf_indices[sub.index]], threshold, false);
  pass.reset();
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
