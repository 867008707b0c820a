// Device-resident ImageSet; see image_set.h. Line references are to the
// reference's cpp/image_set.cc.
#include "image_set.h"

#include <cassert>
#include <cmath>
#include <stdexcept>

namespace radler {

ImageSet::ImageSet(const WorkTable& table, bool squared_joins,
                   const std::set<aocommon::PolarizationEnum>& linked_polarizations,
                   size_t width, size_t height, gpu::Session& session)
    : table_(table),
      session_(&session),
      width_(width),
      height_(height),
      square_joined_channels_(squared_joins),
      linked_polarizations_(linked_polarizations) {
  // image_set.cc:41-63
  n_pol_ = table.OriginalGroups().front().size();
  n_images_ = n_pol_ * NDeconvolutionChannels();
  if (n_images_ < 1) throw std::runtime_error("ImageSet: no images");
  if (n_images_ > RDL_MAX_IMAGES)
    throw std::runtime_error("ImageSet: more than 64 joined images");
  planes_ = gpu::Planes::Make(session, width, height, n_images_);
  image_index_to_psf_index_.resize(n_images_);
  InitializePolFactor();
  InitializeIndices();
  std::vector<double> frequencies;
  CalculateDeconvolutionFrequencies(table, frequencies, weights_);
}

ImageSet::ImageSet(const ImageSet& like, size_t width, size_t height)
    : ImageSet(like.table_, like.square_joined_channels_,
               like.linked_polarizations_, width, height, *like.session_) {}

ImageSet::ImageSet(const ImageSet& like, size_t width, size_t height,
                   gpu::Session& session)
    : ImageSet(like.table_, like.square_joined_channels_,
               like.linked_polarizations_, width, height, session) {}

void ImageSet::InitializePolFactor() {  // image_set.h:298-324
  const WorkTable::Group& first = table_.OriginalGroups().front();
  std::set<aocommon::PolarizationEnum> pols;
  bool all_stokes_without_i = true;
  for (const WorkTableEntry* e : first) {
    if (linked_polarizations_.empty() ||
        linked_polarizations_.count(e->polarization) != 0) {
      if (!aocommon::Polarization::IsStokes(e->polarization) ||
          e->polarization == aocommon::PolarizationEnum::StokesI)
        all_stokes_without_i = false;
      pols.insert(e->polarization);
    }
  }
  const bool is_dual =
      pols.size() == 2 && aocommon::Polarization::HasDualPolarization(pols);
  const bool is_full =
      pols.size() == 4 &&
      (aocommon::Polarization::HasFullLinearPolarization(pols) ||
       aocommon::Polarization::HasFullCircularPolarization(pols));
  if (all_stokes_without_i)
    polarization_normalization_factor_ = 1.0 / pols.size();
  else if (is_dual || is_full)
    polarization_normalization_factor_ = 0.5;
  else
    polarization_normalization_factor_ = 1.0;
}

void ImageSet::InitializeIndices() {  // image_set.cc:69-96
  entry_index_to_image_index_.reserve(table_.Size());
  size_t image_index = 0;
  for (const std::vector<size_t>& group : table_.DeconvolutionGroups()) {
    const size_t start = image_index;
    for (const size_t original_index : group) {
      image_index = start;
      for (const WorkTableEntry* e : table_.OriginalGroups()[original_index]) {
        if (e->index != entry_index_to_image_index_.size())
          throw std::runtime_error("ImageSet: unexpected work table order");
        entry_index_to_image_index_.push_back(image_index);
        ++image_index;
      }
    }
  }
  for (size_t ch = 0; ch != NDeconvolutionChannels(); ++ch)
    for (const WorkTableEntry* e : table_.FirstOriginalGroup(ch))
      image_index_to_psf_index_[entry_index_to_image_index_[e->index]] = ch;
}

void ImageSet::CalculateDeconvolutionFrequencies(
    const WorkTable& table, std::vector<double>& frequencies,
    std::vector<float>& weights) {  // image_set.cc:464-497
  const size_t n_in = table.OriginalGroups().size();
  const size_t n_out = table.DeconvolutionGroups().size();
  frequencies.assign(n_out, 0.0);
  weights.assign(n_out, 0.0);
  std::vector<double> unweighted(n_out, 0.0);
  std::vector<size_t> counts(n_out, 0);
  for (size_t i = 0; i != n_in; ++i) {
    const WorkTableEntry& e = *table.OriginalGroups()[i].front();
    const double freq = e.CentralFrequency();
    const double weight = e.image_weight;
    const size_t ch = i * n_out / n_in;
    frequencies[ch] += freq * weight;
    weights[ch] += weight;
    unweighted[ch] += freq;
    ++counts[ch];
  }
  for (size_t i = 0; i != n_out; ++i) {
    if (weights[i] > 0.0)
      frequencies[i] /= weights[i];
    else
      frequencies[i] = unweighted[i] / counts[i];
  }
}

rdl_integration ImageSet::Integration(bool square) const {
  rdl_integration g{};
  g.n_images = uint32_t(n_images_);
  g.n_pol = uint32_t(n_pol_);
  g.n_channels = uint32_t(NDeconvolutionChannels());
  // joined polarizations, in the order of the first channel group
  const WorkTable::Group& first = table_.OriginalGroups().front();
  g.pol_mask = 0;
  for (size_t p = 0; p != first.size(); ++p)
    if (linked_polarizations_.empty() ||
        linked_polarizations_.count(first[p]->polarization) != 0)
      g.pol_mask |= 1u << p;
  double weight_sum = 0.0;
  for (size_t ch = 0; ch != NDeconvolutionChannels(); ++ch) {
    const float w = weights_[ch];
    if (w != 0.0f) weight_sum += w;
    for (size_t p = 0; p != n_pol_; ++p) g.weights[ch * n_pol_ + p] = w;
  }
  const float pnf = polarization_normalization_factor_;
  if (square_joined_channels_) {  // image_set.cc:429-455
    g.mode = RDL_INTEGRATE_SQUARED_JOINS;
    g.copy_fast_path = 0;
    g.factor = weight_sum > 0.0 ? float(std::sqrt(pnf / weight_sum)) : 0.0f;
  } else if (!square) {  // image_set.cc:423-462
    g.mode = RDL_INTEGRATE_LINEAR;
    g.copy_fast_path =
        table_.DeconvolutionGroups().size() == 1 && first.size() == 1;
    g.factor = weight_sum > 0.0 ? float(pnf / weight_sum) : 0.0f;
  } else {  // image_set.cc:309-386
    g.mode = RDL_INTEGRATE_SQUARE;
    if (NDeconvolutionChannels() == 1) {
      g.copy_fast_path = first.size() == 1;
      g.factor = std::sqrt(pnf);
    } else {
      g.copy_fast_path = 0;
      g.factor = float(double(std::sqrt(pnf)) / weight_sum);
    }
  }
  return g;
}

void ImageSet::GetLinearIntegrated(float* d_dest) const {
  const rdl_integration g = Integration(false);
  gpu::Check(rdl_integrate(session_->Handle(), &g, Base(), PlaneSize(), d_dest),
             "rdl_integrate");
}

void ImageSet::GetSquareIntegrated(float* d_dest) const {
  const rdl_integration g = Integration(true);
  gpu::Check(rdl_integrate(session_->Handle(), &g, Base(), PlaneSize(), d_dest),
             "rdl_integrate");
}

void ImageSet::GetIntegratedPsf(float* d_dest, const gpu::Planes& psfs) const {
  // image_set.cc:499-530
  const size_t n = psfs.PlaneSize();
  rdl_session* s = session_->Handle();
  if (NDeconvolutionChannels() == 1) {
    session_->D2D(d_dest, psfs.Plane(0), n * sizeof(float));
    return;
  }
  bool is_first = true;
  double weight_sum = 0.0;
  for (size_t ch = 0; ch != NDeconvolutionChannels(); ++ch) {
    const double w = weights_[ch];
    if (w != 0.0) {
      weight_sum += w;
      gpu::Check(rdl_axpy(s, d_dest, psfs.Plane(ch), n, float(w), is_first ? 1 : 0),
                 "rdl_axpy");
      is_first = false;
    }
  }
  const double factor = weight_sum == 0.0 ? 0.0 : 1.0 / weight_sum;
  gpu::Check(rdl_scale(s, d_dest, n, float(factor)), "rdl_scale");
}

void ImageSet::LoadAndAverage(bool use_residual_images) {
  // image_set.cc:105-140: sum of weight*image per deconvolution channel and
  // polarization, then *= 1/sum(weights). Accessor loads go through the
  // session's page-locked staging buffer; the arithmetic runs on the device.
  rdl_session* s = session_->Handle();
  planes_.buffer->Zero();
  const size_t n = PlaneSize();
  float* host = static_cast<float*>(session_->PinnedStaging(n * sizeof(float)));
  gpu::Buffer& staging = session_->Scratch(gpu::Session::kStaging, n * sizeof(float));
  std::vector<double> averaged_weights(n_images_, 0.0);
  size_t image_index = 0;
  for (const std::vector<size_t>& group : table_.DeconvolutionGroups()) {
    const size_t start = image_index;
    for (const size_t original_index : group) {
      image_index = start;
      for (const WorkTableEntry* e : table_.OriginalGroups()[original_index]) {
        const std::unique_ptr<aocommon::ImageAccessor>& acc_ptr =
            use_residual_images ? e->residual_accessor : e->model_accessor;
        // the reference's test accessor throws std::logic_error on use
        // (cpp/test/imageaccessor.h, test_image_set.cc:478)
        if (!acc_ptr)
          throw std::logic_error(use_residual_images
                                     ? "ImageSet: entry has no residual accessor"
                                     : "ImageSet: entry has no model accessor");
        const aocommon::ImageAccessor& acc = *acc_ptr;
        if (acc.Width() != width_ || acc.Height() != height_)
          throw std::runtime_error("ImageSet: accessor size mismatch");
        acc.Load(host);
        if (e->image_weight != 0.0) {
          session_->H2D(staging.Ptr(), host, n * sizeof(float));
          // AddWithFactor into a zeroed plane
          gpu::Check(rdl_axpy(s, Data(image_index), staging.F(), n,
                              float(e->image_weight), 0),
                     "rdl_axpy");
          averaged_weights[image_index] += e->image_weight;
        }
        ++image_index;
      }
    }
  }
  for (size_t i = 0; i != n_images_; ++i)
    gpu::Check(rdl_scale(s, Data(i), n, float(1.0 / averaged_weights[i])),
               "rdl_scale");
  session_->Sync();
}

std::vector<gpu::Planes> ImageSet::LoadAndAveragePsfs() const {
  // image_set.cc:142-207 (weights applied in double, as the reference does)
  std::vector<gpu::Planes> result;
  const auto& first_psfs = table_.Front().psf_accessors;
  rdl_session* s = session_->Handle();
  for (size_t psf_index = 0; psf_index != first_psfs.size(); ++psf_index) {
    const size_t pw = first_psfs[psf_index]->Width();
    const size_t ph = first_psfs[psf_index]->Height();
    const size_t n = pw * ph;
    gpu::Planes planes =
        gpu::Planes::Make(*session_, pw, ph, NDeconvolutionChannels());
    planes.buffer->Zero();
    float* host = static_cast<float*>(session_->PinnedStaging(n * sizeof(float)));
    gpu::Buffer& staging = session_->Scratch(gpu::Session::kStaging, n * sizeof(float));
    std::vector<double> averaged(NDeconvolutionChannels(), 0.0);
    for (size_t g = 0; g != NOriginalChannels(); ++g) {
      const size_t ch = (g * NDeconvolutionChannels()) / NOriginalChannels();
      const WorkTableEntry& e = *table_.OriginalGroups()[g].front();
      const aocommon::ImageAccessor& acc = *e.psf_accessors[psf_index];
      acc.Load(host);
      session_->H2D(staging.Ptr(), host, n * sizeof(float));
      gpu::Check(rdl_axpy_f64(s, planes.Plane(ch), staging.F(), n,
                              e.image_weight, 0),
                 "rdl_axpy_f64");
      averaged[ch] += e.image_weight;
    }
    for (size_t ch = 0; ch != NDeconvolutionChannels(); ++ch) {
      const double f = averaged[ch] == 0.0 ? 0.0 : 1.0 / averaged[ch];
      gpu::Check(rdl_axpy_f64(s, planes.Plane(ch), nullptr, n, f, 1),
                 "rdl_axpy_f64");
    }
    session_->Sync();
    result.push_back(std::move(planes));
  }
  return result;
}

void ImageSet::AssignAndStoreResidual() {  // image_set.cc:290-307
  float* host = static_cast<float*>(session_->PinnedStaging(PlaneSize() * sizeof(float)));
  size_t image_index = 0;
  for (const std::vector<size_t>& group : table_.DeconvolutionGroups()) {
    const size_t start = image_index;
    for (const size_t original_index : group) {
      image_index = start;
      for (const WorkTableEntry* e : table_.OriginalGroups()[original_index]) {
        session_->D2H(host, Data(image_index), PlaneSize() * sizeof(float));
        e->residual_accessor->Store(host);
        ++image_index;
      }
    }
  }
}

void ImageSet::InterpolateAndStoreModel(
    const schaapcommon::fitters::SpectralFitter* fitter) {
  // image_set.cc:209-288
  float* host = static_cast<float*>(session_->PinnedStaging(PlaneSize() * sizeof(float)));
  if (NDeconvolutionChannels() == NOriginalChannels()) {
    size_t image_index = 0;
    for (const WorkTableEntry& e : table_) {
      session_->D2H(host, Data(image_index), PlaneSize() * sizeof(float));
      e.model_accessor->Store(host);
      ++image_index;
    }
    return;
  }
  rdl_logpoly lp;
  if (fitter && MakeLogPoly(*fitter, &lp)) {
    // the non-linear fit per non-zero pixel (image_set.cc:238-268), evaluated
    // at every original channel of the polarization (:270-285)
    if (lp.n_channels != NDeconvolutionChannels())
      throw std::runtime_error(
          "InterpolateAndStoreModel: the fitter's channels do not match the image set");
    const size_t n_orig = NOriginalChannels();
    const size_t chunk = std::min<size_t>(n_orig, RDL_MAX_IMAGES);
    gpu::Buffer out(*session_, chunk * PlaneSize() * sizeof(float));
    for (size_t p = 0; p != n_pol_; ++p) {
      for (size_t g0 = 0; g0 < n_orig; g0 += chunk) {
        const size_t n_out = std::min(chunk, n_orig - g0);
        std::vector<double> out_lg;
        for (size_t g = g0; g != g0 + n_out; ++g)
          out_lg.push_back(std::log10(table_.OriginalGroups()[g][p]->CentralFrequency() /
                                      fitter->ReferenceFrequency()));
        gpu::Check(rdl_logpoly_interpolate(session_->Handle(), Data(p), n_pol_ * PlaneSize(),
                                           PlaneSize(), &lp, out_lg.data(), uint32_t(n_out),
                                           out.F(), PlaneSize()),
                   "rdl_logpoly_interpolate");
        for (size_t g = g0; g != g0 + n_out; ++g) {
          session_->D2H(host, out.F() + (g - g0) * PlaneSize(), PlaneSize() * sizeof(float));
          table_.OriginalGroups()[g][p]->model_accessor->Store(host);
        }
      }
    }
    return;
  }
  const SpectralMaps maps = fitter ? MakeSpectralMaps(*fitter) : SpectralMaps{};
  if (maps.Empty()) {
    // kNoFitting (schaapcommon's fitter would evaluate nothing here; parity
    // unpinned): the deconvolution channel's model as it is
    for (size_t g = 0; g != NOriginalChannels(); ++g) {
      const size_t ch = (g * NDeconvolutionChannels()) / NOriginalChannels();
      const WorkTable::Group& group = table_.OriginalGroups()[g];
      for (size_t p = 0; p != group.size(); ++p) {
        session_->D2H(host, Data(ch * n_pol_ + p), PlaneSize() * sizeof(float));
        group[p]->model_accessor->Store(host);
      }
    }
    return;
  }
  if (maps.n_channels != NDeconvolutionChannels())
    throw std::runtime_error(
        "InterpolateAndStoreModel: the fitter's channels do not match the image set");
  const size_t n_orig = NOriginalChannels();
  const size_t chunk = std::min<size_t>(n_orig, RDL_MAX_IMAGES);
  gpu::Buffer out(*session_, chunk * PlaneSize() * sizeof(float));
  for (size_t p = 0; p != n_pol_; ++p) {
    for (size_t g0 = 0; g0 < n_orig; g0 += chunk) {
      const size_t n_out = std::min(chunk, n_orig - g0);
      std::vector<float> coef;
      coef.reserve(n_out * maps.n_channels);
      for (size_t g = g0; g != g0 + n_out; ++g) {
        const std::vector<double> row =
            maps.EvaluateAt(table_.OriginalGroups()[g][p]->CentralFrequency());
        for (double c : row) coef.push_back(float(c));
      }
      gpu::Check(rdl_spectral_interpolate(session_->Handle(), Data(p),
                                          n_pol_ * PlaneSize(),
                                          uint32_t(maps.n_channels), coef.data(),
                                          uint32_t(n_out), out.F(), PlaneSize()),
                 "rdl_spectral_interpolate");
      for (size_t g = g0; g != g0 + n_out; ++g) {
        session_->D2H(host, out.F() + (g - g0) * PlaneSize(),
                      PlaneSize() * sizeof(float));
        table_.OriginalGroups()[g][p]->model_accessor->Store(host);
      }
    }
  }
}

void ImageSet::Fill(float value) {
  if (value != 0.0f)
    throw std::runtime_error("ImageSet::Fill supports 0 only");
  planes_.buffer->Zero();
}

void ImageSet::CopyFrom(const ImageSet& other) {
  if (other.PlaneSize() != PlaneSize() || other.Size() != Size())
    throw std::runtime_error("ImageSet::CopyFrom: size mismatch");
  session_->D2D(Base(), other.Base(), Size() * PlaneSize() * sizeof(float));
}

void ImageSet::SetPlanes(gpu::Planes planes) {
  if (planes.count != n_images_)
    throw std::runtime_error("ImageSet::SetPlanes: wrong image count");
  planes_ = std::move(planes);
  width_ = planes_.width;
  height_ = planes_.height;
}

}  // namespace radler
