// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Restatement of ParallelDeconvolution's subimage tiling
// (cpp/algorithms/parallel_deconvolution.cc:57-166, 300-654) and the Dijkstra
// minimum-flux splitter (cpp/math/dijkstra_splitter.{h,cc}) for the parity
// tests of the device tiling. Subimages run in index order (the reference's
// RecursiveFor with one thread; with several threads its result depends on
// the schedule, because a subimage's trimmed residual includes neighbours'
// pixels outside its boundary mask).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <queue>
#include <stdexcept>

#include "oracle.h"
#include "tiling.h"
#include "iuwt_algorithm.h"

namespace oracle {

namespace {

// One shortest-path search through a band of the image, written once for both
// directions: `along` is the axis the path crosses (rows for a vertical
// divider), `across` the band axis. Pixel (a, c) = (along, across).
struct BandView {
  const float* image;
  size_t width;
  bool vertical;  // true: along = y, across = x
  size_t Index(size_t along, size_t across) const {
    return vertical ? along * width + across : across * width + along;
  }
};

struct Step {
  float distance;
  size_t to_along, to_across, from_along, from_across;
  // std::priority_queue is a max-heap; reversing the comparison gives the
  // smallest distance first (dijkstra_splitter.h:24-29)
  bool operator<(const Step& o) const { return distance > o.distance; }
};

// DivideVertically / DivideHorizontally (dijkstra_splitter.cc:32-136):
// output gets 1 on the path and 0 elsewhere in the band [c1, c2).
void DivideBand(const BandView& v, size_t n_along, size_t c1, size_t c2,
                float* output) {
  std::priority_queue<Step> queue;
  for (size_t c = c1; c != c2; ++c) queue.push(Step{0.0f, 0, c, 0, c});
  const size_t band = c2 - c1;
  std::vector<std::pair<size_t, size_t>> came_from(band * n_along);
  for (size_t a = 0; a != n_along; ++a)
    for (size_t c = c1; c != c2; ++c)
      output[v.Index(a, c)] = std::numeric_limits<float>::max();
  Step s{};
  while (!queue.empty()) {
    s = queue.top();
    queue.pop();
    const size_t a = s.to_along, c = s.to_across;
    if (a == n_along) break;
    const size_t idx = v.Index(a, c);
    const float d = s.distance + std::fabs(v.image[idx]);
    if (d < output[idx]) {
      output[idx] = d;
      came_from[(c - c1) + a * band] = {s.from_along, s.from_across};
      Step next{d, 0, 0, a, c};
      auto push = [&](size_t na, size_t nc) {
        next.to_along = na;
        next.to_across = nc;
        queue.push(next);
      };
      // neighbour order of the reference: lower side (diagonal, then level),
      // straight on, upper side (diagonal, then level)
      if (c > c1) {
        push(a + 1, c - 1);
        push(a, c - 1);
      }
      push(a + 1, c);
      if (c + 1 < c2) {
        push(a + 1, c + 1);
        push(a, c + 1);
      }
    }
  }
  for (size_t a = 0; a != n_along; ++a)
    for (size_t c = c1; c != c2; ++c) output[v.Index(a, c)] = 0.0f;
  size_t pa = s.from_along, pc = s.from_across;
  while (pa > 0) {
    output[v.Index(pa, pc)] = 1.0f;
    const auto prev = came_from[(pc - c1) + pa * band];
    pa = prev.first;
    pc = prev.second;
  }
  output[v.Index(0, pc)] = 1.0f;
}

// FloodVerticalArea / FloodHorizontalArea (dijkstra_splitter.cc:138-208):
// from `start` walk down the band axis to (and through) the lower border,
// and up to the upper border, in every line along the other axis.
void FloodArea(const float* division, size_t width, size_t height, bool vertical,
               size_t start, bool* mask, size_t& low, size_t& extent) {
  std::fill(mask, mask + width * height, false);
  const size_t n_lines = vertical ? height : width;
  const size_t n_across = vertical ? width : height;
  auto at = [&](size_t line, int64_t c) -> size_t {
    return vertical ? line * width + size_t(c) : size_t(c) * width + line;
  };
  low = n_across;
  size_t high = 0;
  for (size_t line = 0; line != n_lines; ++line) {
    int64_t c = int64_t(start);
    while (c >= 0 && division[at(line, c)] == 0.0f) {
      mask[at(line, c)] = true;
      --c;
    }
    while (c >= 0 && division[at(line, c)] != 0.0f) {
      mask[at(line, c)] = true;
      --c;
    }
    low = std::min<size_t>(low, size_t(c + 1));
    c = int64_t(start) + 1;
    while (size_t(c) < n_across && division[at(line, c)] == 0.0f) {
      mask[at(line, c)] = true;
      ++c;
    }
    high = std::max<size_t>(high, size_t(c));
  }
  extent = high < low ? 0 : high - low;
}

// GetBoundingMask (dijkstra_splitter.cc:210-285)
void BoundingMask(size_t width, size_t height, const bool* vmask, size_t vx,
                  size_t vwidth, const bool* hmask, bool* mask, size_t& sx,
                  size_t& sy, size_t& sw, size_t& sh) {
  sx = vwidth + vx;
  sy = height;
  size_t sx2 = 0, sy2 = 0;
  for (size_t y = 0; y != height; ++y)
    for (size_t x = 0; x != vwidth; ++x) {
      const size_t hx = x + vx;
      const bool in = vmask[y * vwidth + x] && hmask[y * width + hx];
      mask[y * width + hx] = in;
      if (in) {
        sx = std::min(sx, hx);
        sy = std::min(sy, y);
        sx2 = std::max(sx2, hx);
        sy2 = y;
      }
    }
  if (sx2 < sx) {
    sw = sh = 0;
  } else {
    sw = sx2 + 1 - sx;
    sh = sy2 + 1 - sy;
  }
  if (width % 2 == 0 && sw % 2 != 0) {  // keep even sizes even
    ++sw;
    const size_t col = (sw + sx >= width) ? --sx : sx + sw - 1;
    for (size_t y = sy; y != sy + sh; ++y) mask[col + y * width] = false;
  }
  if (height % 2 == 0 && sh % 2 != 0) {
    ++sh;
    const size_t row = (sh + sy >= height) ? --sy : sy + sh - 1;
    std::fill_n(&mask[row * width + sx], sw, false);
  }
}

template <typename T>
void CopyBox(T* dest, size_t bx, size_t by, size_t bw, size_t bh, const T* src,
             size_t src_width) {
  for (size_t y = 0; y != bh; ++y)
    std::copy_n(src + (by + y) * src_width + bx, bw, dest + y * bw);
}

}  // namespace

std::vector<SubImage> MakeSubImages(const float* image, size_t width,
                                    size_t height, const bool* user_mask,
                                    size_t grid_w, size_t grid_h) {
  // parallel_deconvolution.cc:69-166
  const size_t avg_w = width / grid_w, avg_h = height / grid_h;
  std::vector<float> dividing(width * height, 0.0f);
  std::vector<unsigned char> scratch_store(width * height);
  bool* scratch = reinterpret_cast<bool*>(scratch_store.data());
  const BandView vview{image, width, true}, hview{image, width, false};

  for (size_t d = 1; d < grid_w; ++d) {
    const size_t mid = width * d / grid_w;
    DivideBand(vview, height, mid - avg_w / 4, mid + avg_w / 4, dividing.data());
  }
  struct Area {
    std::vector<unsigned char> mask;
    size_t x, width;
  };
  std::vector<Area> areas(grid_w);
  for (size_t d = 0; d != grid_w; ++d) {
    const size_t mid_x = d * width / grid_w + avg_w / 2;
    Area& area = areas[d];
    FloodArea(dividing.data(), width, height, true, mid_x, scratch, area.x,
              area.width);
    area.mask.resize(area.width * height);
    CopyBox(area.mask.data(), area.x, 0, area.width, height,
            reinterpret_cast<unsigned char*>(scratch), width);
  }

  std::fill(dividing.begin(), dividing.end(), 0.0f);
  for (size_t d = 1; d < grid_h; ++d) {
    const size_t mid = height * d / grid_h;
    DivideBand(hview, width, mid - avg_h / 4, mid + avg_h / 4, dividing.data());
  }

  std::vector<unsigned char> bounding_store(width * height, 0);
  bool* bounding = reinterpret_cast<bool*>(bounding_store.data());
  std::vector<SubImage> subs;
  for (size_t gy = 0; gy != grid_h; ++gy) {
    const size_t mid_y = gy * height / grid_h + avg_h / 2;
    size_t hy, hh;
    FloodArea(dividing.data(), width, height, false, mid_y, scratch, hy, hh);
    for (size_t gx = 0; gx != grid_w; ++gx) {
      SubImage s;
      s.index = subs.size();
      const Area& area = areas[gx];
      BoundingMask(width, height, reinterpret_cast<const bool*>(area.mask.data()),
                   area.x, area.width, scratch, bounding, s.x, s.y, s.width,
                   s.height);
      s.mask.resize(s.width * s.height);
      CopyBox(s.mask.data(), s.x, s.y, s.width, s.height, bounding_store.data(),
              width);
      s.boundary_mask = s.mask;
      if (user_mask) {
        std::vector<unsigned char> um(s.width * s.height);
        CopyBox(um.data(), s.x, s.y, s.width, s.height,
                reinterpret_cast<const unsigned char*>(user_mask), width);
        for (size_t i = 0; i != um.size(); ++i) s.mask[i] = s.mask[i] && um[i];
      }
      subs.push_back(std::move(s));
    }
  }
  return subs;
}

// aocommon::Image::Trim to a centred window (Image::Resize to a smaller size;
// parity unpinned for DD-PSF grids coarser than the subimages)
static void ResizePsf(const float* psf, size_t w, size_t h, size_t nw, size_t nh,
                      float* out) {
  if (nw > w || nh > h) throw std::runtime_error("PSF smaller than subimage");
  CopyBox(out, (w - nw) / 2, (h - nh) / 2, nw, nh, psf, w);
}

ParallelResult ParallelRun(std::vector<TiledAlgorithm>& algorithms,
                           size_t grid_w, size_t grid_h, const SetDesc& desc,
                           ImageSet& data, ImageSet& model,
                           const std::vector<const float*>& psfs,
                           double major_loop_gain, double divergence_limit,
                           const bool* user_mask, std::vector<SubImage>* out_subs,
                           std::vector<std::vector<Component>>* traces,
                           bool snapshot, ParallelMasks* masks) {
  // snapshot == false: subimages run one after another, each trimming the
  // residual left by the ones before (the reference with one thread).
  // snapshot == true: every subimage of a pass trims the residual as it was
  // when the pass started (the reference's multi-threaded run when all
  // threads trim before the first copy-back, parallel_deconvolution.cc:
  // 583-616, 300-357 and 458-484).
  const size_t width = data.width, height = data.height;
  const size_t n_img = data.Size();
  std::vector<float> integrated(width * height);
  GetLinearIntegrated(data, integrated.data());
  std::vector<SubImage> subs =
      MakeSubImages(integrated.data(), width, height, user_mask, grid_w, grid_h);
  if (traces) traces->assign(subs.size(), {});

  std::vector<std::vector<float>> result_model(n_img,
                                               std::vector<float>(width * height, 0.0f));

  std::vector<std::vector<float>> snapshot_store;
  std::vector<const float*> source(data.images.begin(), data.images.end());

  // RunSubImage (parallel_deconvolution.cc:300-484)
  auto run = [&](SubImage& s, double major_threshold, bool find_peak_only) {
    TiledAlgorithm& alg = algorithms[s.index];
    const size_t sw = s.width, sh = s.height, n = sw * sh;
    std::vector<float> sub_data(n_img * n), sub_model(n_img * n);
    for (size_t i = 0; i != n_img; ++i) {
      CopyBox(&sub_data[i * n], s.x, s.y, sw, sh, source[i], width);
      CopyBox(&sub_model[i * n], s.x, s.y, sw, sh, model.images[i], width);
      for (size_t p = 0; p != n; ++p)
        if (!s.boundary_mask[p]) sub_model[i * n + p] = 0.0f;  // TrimMasked
    }
    const std::vector<float> initial_model = sub_model;
    std::vector<float> sub_psf_store(psfs.size() * n);
    std::vector<const float*> sub_psfs;
    for (size_t c = 0; c != psfs.size(); ++c) {
      ResizePsf(psfs[c], width, height, sw, sh, &sub_psf_store[c * n]);
      sub_psfs.push_back(&sub_psf_store[c * n]);
    }
    std::vector<unsigned char> mask_copy = s.mask;
    alg.settings.clean_mask = reinterpret_cast<const bool*>(mask_copy.data());
    std::vector<float> sub_rms;
    if (masks && !masks->rms_factor.empty()) {  // rms_image_.TrimBox (:332-337)
      sub_rms.resize(n);
      CopyBox(sub_rms.data(), s.x, s.y, sw, sh, masks->rms_factor.data(), width);
      alg.settings.rms_factor = sub_rms.data();
    }
    const size_t max_iter = alg.settings.max_iterations;
    if (find_peak_only)
      alg.settings.max_iterations = 0;
    else
      alg.settings.major_iteration_threshold = float(major_threshold);
    const double peak_at_start = std::fabs(s.peak);

    ImageSet sd, sm;
    sd.desc = sm.desc = &desc;
    sd.width = sm.width = sw;
    sd.height = sm.height = sh;
    for (size_t i = 0; i != n_img; ++i) {
      sd.images.push_back(&sub_data[i * n]);
      sm.images.push_back(&sub_model[i * n]);
    }
    const bool ms_masks = masks && (masks->track || masks->use) && alg.kind == 1;
    if (ms_masks) {  // :359-390
      if (!alg.ms) alg.ms = std::make_unique<MultiScale>(alg.settings);
      alg.ms->track_scale_masks = masks->track;
      alg.ms->use_scale_masks = masks->use;
      if (!masks->scale_masks.empty()) {
        auto& own = alg.ms->scale_masks;
        own.resize(std::max(own.size(), masks->scale_masks.size()));
        for (size_t i = 0; i != own.size(); ++i) {
          own[i].assign(n, 0);
          if (i >= masks->scale_masks.size()) continue;
          for (size_t y = 0; y != sh; ++y)
            for (size_t x = 0; x != sw; ++x)
              own[i][y * sw + x] =
                  masks->scale_masks[i][(y + s.y) * width + x + s.x] && s.mask[y * sw + x];
        }
      }
    }
    std::vector<Component> tr;
    Result r = alg.Execute(sd, sm, sub_psfs, &tr);
    if (traces && !find_peak_only) (*traces)[s.index] = tr;
    if (!find_peak_only && alg.ms) s.end_margin = alg.ms->end_margin;
    s.peak = r.final_peak;
    s.reached_major_threshold = r.another_iteration_required;
    const bool converging =
        (divergence_limit == 0.0 ||
         std::fabs(s.peak) <= peak_at_start * divergence_limit) &&
        std::isfinite(s.peak) && !r.is_diverging;
    if (!converging && !find_peak_only) s.reached_major_threshold = false;
    alg.settings.clean_mask = nullptr;
    alg.settings.rms_factor = nullptr;  // :421-423
    if (ms_masks && masks->track && converging && !find_peak_only) {  // :425-462
      const size_t n_scales = alg.ms->Scales().size();
      if (masks->scale_masks.empty())
        masks->scale_masks.assign(n_scales, std::vector<unsigned char>(width * height, 0));
      for (size_t i = 0; i != n_scales && i != masks->scale_masks.size(); ++i)
        for (size_t y = 0; y != sh; ++y)
          for (size_t x = 0; x != sw; ++x)
            if (s.boundary_mask[y * sw + x])
              masks->scale_masks[i][(y + s.y) * width + x + s.x] =
                  alg.ms->scale_masks[i][y * sw + x];
    }
    if (find_peak_only) {
      alg.settings.max_iterations = max_iter;
      return;
    }
    if (converging) {  // ImageSet::CopyMasked
      for (size_t i = 0; i != n_img; ++i)
        for (size_t y = 0; y != sh; ++y)
          for (size_t x = 0; x != sw; ++x)
            if (s.boundary_mask[y * sw + x])
              data.images[i][(y + s.y) * width + x + s.x] = sub_data[i * n + y * sw + x];
    } else {
      sub_model = initial_model;
    }
    for (size_t i = 0; i != n_img; ++i)  // ImageSet::AddSubImage
      for (size_t y = 0; y != sh; ++y)
        for (size_t x = 0; x != sw; ++x)
          result_model[i][(y + s.y) * width + x + s.x] += sub_model[i * n + y * sw + x];
  };

  for (SubImage& s : subs) run(s, 0.0, true);
  double start_peak = 0.0;
  for (const SubImage& s : subs)
    if (s.peak > start_peak) start_peak = s.peak;
  const double threshold = start_peak * (1.0 - major_loop_gain);
  if (snapshot) {
    snapshot_store.reserve(n_img);
    for (size_t i = 0; i != n_img; ++i) {
      snapshot_store.emplace_back(data.images[i], data.images[i] + width * height);
      source[i] = snapshot_store.back().data();
    }
  }
  for (SubImage& s : subs) run(s, threshold, false);
  for (size_t i = 0; i != n_img; ++i)
    std::copy(result_model[i].begin(), result_model[i].end(), model.images[i]);

  ParallelResult res;
  res.start_peak = start_peak;
  size_t finished = 0;
  bool max_iter = false;
  double end_peak = 0.0;
  for (const SubImage& s : subs) {
    if (!s.reached_major_threshold) ++finished;
    if (algorithms[s.index].iteration_number >= algorithms[s.index].settings.max_iterations)
      max_iter = true;
    end_peak = std::max(end_peak, double(s.peak));
  }
  res.end_peak = end_peak;
  res.another_iteration_required = finished != subs.size() && !max_iter;
  if (out_subs) *out_subs = subs;
  return res;
}

Result TiledAlgorithm::Execute(ImageSet& data, ImageSet& model,
                               const std::vector<const float*>& psfs,
                               std::vector<Component>* trace) {
  if (kind == 0)
    return GenericCleanExecute(settings, iteration_number, data, model, psfs, trace);
  if (kind == 2) {  // IuwtDeconvolution (iuwt_deconvolution.h:22-39)
    IuwtAlgoSettings is;
    is.minor_loop_gain = settings.minor_loop_gain;
    is.major_loop_gain = settings.major_loop_gain;
    is.clean_border = settings.clean_border_ratio;
    is.allow_negative = settings.allow_negative;
    is.mask = settings.clean_mask;
    is.absolute_threshold = settings.threshold;
    Result r;
    bool another = false;
    r.final_peak = IuwtExecute(is, iteration_number, settings.max_iterations, data, model,
                               psfs, another, nullptr);
    r.another_iteration_required = another;
    return r;
  }
  if (!ms) ms = std::make_unique<MultiScale>(settings);
  ms->Settings() = settings;
  if (ms->Settings().beam_size_in_pixels <= 0.0) ms->Settings().beam_size_in_pixels = 1.0;
  ms->iteration_number = iteration_number;
  Result r = ms->Execute(data, model, psfs, trace);
  iteration_number = ms->iteration_number;
  return r;
}

}  // namespace oracle
