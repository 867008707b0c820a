#include "subminor.h"

#include <cstdlib>
#include <string>

#include <stdexcept>

namespace radler::algorithms {

SubMinorLoop::SubMinorLoop(gpu::Session& s, size_t width, size_t height,
                           size_t padded_width, size_t padded_height)
    : s_(s),
      width_(width),
      height_(height),
      padded_width_(padded_width),
      padded_height_(padded_height) {
  h_ = s.SharedSubminor();
}

SubMinorLoop::~SubMinorLoop() {
  // a launched loop whose result was never read (an exception between
  // Launch and Collect): read it, so the session's shared handle is free
  if (launched_has_peak_) {
    rdl_subminor_result r{};
    (void)rdl_subminor_collect(h_, &r);
  }
}

namespace {
rdl_subminor_params MakeParams(const ImageSet& residual) {
  rdl_subminor_params p{};
  p.width = uint32_t(residual.Width());
  p.height = uint32_t(residual.Height());
  p.n_images = uint32_t(residual.Size());
  p.n_pol = uint32_t(residual.NPolarizations());
  p.integ = residual.Integration(false);  // GetLinearIntegrated
  return p;
}
}  // namespace

bool SubMinorLoop::Launch(ImageSet& residual, const gpu::Planes& psfs) {
  rdl_subminor_params p = MakeParams(residual);
  p.width = uint32_t(width_);
  p.height = uint32_t(height_);
  p.h_border = uint32_t(horizontal_border_);
  p.v_border = uint32_t(vertical_border_);
  p.allow_negative = allow_negative_;
  p.stop_on_negative = stop_on_negative_;
  p.threshold = threshold_;
  p.gain = gain_;
  p.divergence_limit = divergence_limit_;
  p.iteration_start = current_iteration_;
  p.max_iterations = max_iterations_;
  p.d_mask = d_mask_;
  p.d_spectral = d_spectral_;
  p.logpoly = logpoly_;
  p.d_rms = d_rms_;
  n_images_ = residual.Size();
  rdl_subminor_result r{};
  gpu::Check(rdl_subminor_launch(h_, residual.Base(), psfs.Base(), &p, &r),
             "rdl_subminor_launch");
  n_selected_ = r.n_selected;
  launched_has_peak_ = r.has_peak != 0;
  return launched_has_peak_;
}

SubMinorLoop::RunResult SubMinorLoop::Collect() {
  if (!launched_has_peak_) return {false, false, 0.0f};
  launched_has_peak_ = false;
  rdl_subminor_result r{};
  gpu::Check(rdl_subminor_collect(h_, &r), "rdl_subminor_collect");
  current_iteration_ = r.iteration;
  flux_cleaned_ += r.flux_cleaned;
  return {r.diverging != 0, true, r.peak};
}

SubMinorLoop::RunResult SubMinorLoop::Run(ImageSet& residual,
                                          const gpu::Planes& psfs) {
  rdl_subminor_params p{};
  p.width = uint32_t(width_);
  p.height = uint32_t(height_);
  p.n_images = uint32_t(residual.Size());
  p.n_pol = uint32_t(residual.NPolarizations());
  p.integ = residual.Integration(false);  // GetLinearIntegrated
  p.h_border = uint32_t(horizontal_border_);
  p.v_border = uint32_t(vertical_border_);
  p.allow_negative = allow_negative_;
  p.stop_on_negative = stop_on_negative_;
  p.threshold = threshold_;
  p.gain = gain_;
  p.divergence_limit = divergence_limit_;
  p.iteration_start = current_iteration_;
  p.max_iterations = max_iterations_;
  p.d_mask = d_mask_;
  p.d_spectral = d_spectral_;
  p.logpoly = logpoly_;
  p.d_rms = d_rms_;
  n_images_ = residual.Size();
  uint64_t cap = 0;
  if (trace_) {
    cap = max_iterations_ > current_iteration_ ? max_iterations_ - current_iteration_ : 0;
    cap = std::min<uint64_t>(cap, uint64_t(1) << 22);
  }
  // grow-only per-thread trace buffer: a fresh (zeroed, page-faulting) 32 MB
  // vector per outer iteration cost milliseconds of host time while the GPU
  // idled; the device writes only the components it cleans
  thread_local std::vector<uint32_t> tr;
  if (tr.size() < 2 * cap) tr.resize(2 * cap);
  rdl_subminor_result r;
  gpu::Check(rdl_subminor_run(h_, residual.Base(), psfs.Base(), &p, &r,
                              cap ? tr.data() : nullptr, cap),
             "rdl_subminor_run");
  n_selected_ = r.n_selected;
  const size_t done = r.iteration - current_iteration_;
  current_iteration_ = r.iteration;
  flux_cleaned_ += r.flux_cleaned;
  if (trace_ && cap)
    trace_->insert(trace_->end(), tr.begin(),
                   tr.begin() + 2 * std::min<uint64_t>(done, cap));
  return {r.diverging != 0, r.has_peak != 0, r.peak};
}

std::shared_ptr<gpu::Buffer> SubMinorLoop::MakePaddedPsfSpectrum(
    gpu::Session& s, const float* d_psf, size_t width, size_t height,
    size_t pw, size_t ph, bool f64) {
  // float64 transforms by default: see rdl_fft_create_f64 / DESIGN.md
  gpu::Fft& fft = s.GetFft(pw, ph, f64);
  auto spectrum = std::make_shared<gpu::Buffer>(s, fft.SpectrumBytes());
  if (fft.UsesLds()) {
    // Image::Untrim + PrepareConvolutionKernel (subminor_loop.cc:199-202)
    gpu::Buffer kernel(s, pw * ph * sizeof(float));
    gpu::Check(rdl_prepare_psf_kernel(s.Handle(), kernel.F(), uint32_t(pw),
                                      uint32_t(ph), d_psf, uint32_t(width),
                                      uint32_t(height)),
               "rdl_prepare_psf_kernel");
    if (fft.SplitColumns())
      fft.Forward(kernel.F(), spectrum->Ptr());
    else
      fft.ForwardColumnMajor(kernel.F(), spectrum->Ptr());
  } else {
    gpu::Buffer kernel(s, pw * ph * sizeof(double));
    gpu::Check(rdl_prepare_psf_kernel_f64(s.Handle(), kernel.D(), uint32_t(pw),
                                          uint32_t(ph), d_psf, uint32_t(width),
                                          uint32_t(height)),
               "rdl_prepare_psf_kernel_f64");
    if (f64) {
      fft.Forward64(kernel.D(), spectrum->Ptr());
    } else {
      gpu::Check(rdl_prepare_psf_kernel(s.Handle(), kernel.F(), uint32_t(pw), uint32_t(ph),
                                        d_psf, uint32_t(width), uint32_t(height)),
                 "rdl_prepare_psf_kernel");
      fft.Forward(kernel.F(), spectrum->Ptr());
    }
  }
  s.Sync();
  return spectrum;
}

bool SubMinorLoop::CorrectionF64() {
  // RDL_CORR_F32=1: CorrectResidualDirty's padded convolution in float32, the
  // reference's precision (FFTW float, subminor_loop.cc:210) -- a comparison
  // switch (DESIGN.md §4 "Residual correction precision")
  static const bool f64 = [] {
    const char* e = std::getenv("RDL_CORR_F32");
    return !(e && e[0] == '1');
  }();
  return f64;
}

bool SubMinorLoop::CorrectionKernelF32() {
  const char* e = std::getenv("RDL_CORR_KERNEL");
  return e && std::string(e) == "f32";
}

std::shared_ptr<gpu::Buffer> SubMinorLoop::MakeCorrectionPsfSpectrum(
    gpu::Session& s, const float* d_psf, size_t width, size_t height, size_t pw, size_t ph) {
  auto spectrum = MakePaddedPsfSpectrum(s, d_psf, width, height, pw, ph, CorrectionF64());
  gpu::Fft& fft = s.GetFft(pw, ph, CorrectionF64());
  if (!CorrectionKernelF32() || !fft.ConvColumnsD()) return spectrum;
  const size_t n = fft.SpectrumBytes() / 16;
  auto narrow = std::make_shared<gpu::Buffer>(s, n * 8);
  gpu::Check(rdl_complex_narrow(s.Handle(), narrow->Ptr(), spectrum->Ptr(), n),
             "rdl_complex_narrow");
  s.Sync();
  return narrow;
}

void SubMinorLoop::CorrectResidualDirty(size_t image_index, float* d_residual,
                                        const float* d_psf, size_t psf_key) {
  auto it = psf_spectra_.find(psf_key);
  if (it == psf_spectra_.end())
    it = psf_spectra_
             .emplace(psf_key, MakeCorrectionPsfSpectrum(s_, d_psf, width_, height_,
                                                         padded_width_,
                                                         padded_height_))
             .first;
  CorrectResidualDirtyWithSpectrum(image_index, d_residual, it->second->Ptr());
}

void SubMinorLoop::CorrectResidualDirtyWithSpectrum(size_t image_index,
                                                    float* d_residual,
                                                    const void* d_spectrum) {
  gpu::Fft& fft = s_.GetFft(padded_width_, padded_height_, CorrectionF64());
  const uint32_t ox = uint32_t((padded_width_ - width_) / 2);
  const uint32_t oy = uint32_t((padded_height_ - height_) / 2);
  if (fft.UsesLds()) {
    // GetFullIndividualModel into a W x H plane; Untrim, Convolve, Trim and
    // the subtraction run inside the three transform passes
    gpu::Buffer& model = s_.Scratch(gpu::Session::kCorrectionModel,
                                    width_ * height_ * sizeof(float));
    gpu::Buffer& work =
        s_.Scratch(gpu::Session::kCorrectionSpectrum, fft.ConvolveSubtractBytes());
    gpu::Buffer& rows = s_.Scratch(gpu::Session::kCorrectionRows, padded_height_);
    // the model holds a few hundred components per outer iteration: the
    // transform skips its empty rows (exactly zero, so nothing changes), and
    // only the rows it reads are zeroed before the components are stored
    gpu::Check(rdl_subminor_model_rows(h_, uint32_t(image_index),
                                       static_cast<uint8_t*>(rows.Ptr()),
                                       uint32_t(padded_height_), oy),
               "rdl_subminor_model_rows");
    gpu::Check(rdl_subminor_model_masked(h_, uint32_t(image_index), model.F(),
                                         uint32_t(width_), uint32_t(height_),
                                         static_cast<const uint8_t*>(rows.Ptr()), oy),
               "rdl_subminor_model_masked");
    fft.ConvolveSubtract(model.F(), width_, height_, ox, oy, d_spectrum, work.Ptr(),
                         d_residual, static_cast<const uint8_t*>(rows.Ptr()),
                         !fft.SplitColumns(), CorrectionKernelF32() && fft.ConvColumnsD());
    return;
  }
  if (!fft.IsF64()) {  // rocFFT float (RDL_CORR_F32=1 at a size the LDS engine lacks)
    gpu::Buffer& padded = s_.Scratch(gpu::Session::kCorrectionSpectrum,
                                     padded_width_ * padded_height_ * sizeof(float));
    gpu::Check(rdl_subminor_model(h_, uint32_t(image_index), padded.F(),
                                  uint32_t(padded_width_), uint32_t(padded_height_), ox, oy, 0),
               "rdl_subminor_model");
    fft.Convolve(padded.F(), d_spectrum);
    gpu::Check(rdl_trim_subtract(s_.Handle(), d_residual, uint32_t(width_), uint32_t(height_),
                                 padded.F(), uint32_t(padded_width_),
                                 uint32_t(padded_height_)),
               "rdl_trim_subtract");
    return;
  }
  gpu::Buffer& padded_ = s_.Scratch(gpu::Session::kCorrectionSpectrum,
                                    padded_width_ * padded_height_ * sizeof(double));
  // GetFullIndividualModel + Image::Untrim, fused scatter into a zero plane
  gpu::Check(rdl_subminor_model_f64(h_, uint32_t(image_index), padded_.D(),
                                    uint32_t(padded_width_),
                                    uint32_t(padded_height_), ox, oy),
             "rdl_subminor_model_f64");
  fft.Convolve64(padded_.D(), d_spectrum);
  // Image::Trim (to float) + residual -= (subminor_loop.cc:214-217)
  gpu::Check(rdl_trim_subtract_f64(s_.Handle(), d_residual, uint32_t(width_),
                                   uint32_t(height_), padded_.D(),
                                   uint32_t(padded_width_),
                                   uint32_t(padded_height_)),
             "rdl_trim_subtract_f64");
}

void SubMinorLoop::GetFullIndividualModel(size_t image_index, float* d_dest) {
  gpu::Check(rdl_subminor_model(h_, uint32_t(image_index), d_dest,
                                uint32_t(width_), uint32_t(height_), 0, 0, 0),
             "rdl_subminor_model");
}

void SubMinorLoop::AddIndividualModel(size_t image_index, float* d_model) {
  gpu::Check(rdl_subminor_model(h_, uint32_t(image_index), d_model,
                                uint32_t(width_), uint32_t(height_), 0, 0, 1),
             "rdl_subminor_model");
}

void SubMinorLoop::AddShapeModel(size_t image_index, const float* d_kernel,
                                 size_t n, float* d_model) {
  gpu::Check(rdl_subminor_add_shape_model(h_, uint32_t(image_index), d_kernel,
                                          uint32_t(n), d_model, uint32_t(width_),
                                          uint32_t(height_)),
             "rdl_subminor_add_shape_model");
}

void SubMinorLoop::UpdateAutoMask(uint8_t* d_mask) {
  gpu::Check(rdl_subminor_update_mask(h_, d_mask), "rdl_subminor_update_mask");
}

void SubMinorLoop::UpdateComponentList(ComponentList& list,
                                       size_t scale_index) const {
  std::vector<uint32_t> positions;
  std::vector<float> models;
  GetSelection(positions, models);
  const size_t n = positions.size();
  std::vector<float> values(n_images_);
  for (size_t px = 0; px != n; ++px) {
    bool non_zero = false;
    for (size_t i = 0; i != n_images_; ++i) {
      values[i] = models[i * n + px];
      non_zero = non_zero || values[i] != 0.0f;
    }
    if (non_zero)
      list.Add(positions[px] & 0xffffu, positions[px] >> 16, scale_index, values.data());
  }
}

void SubMinorLoop::GetSelection(std::vector<uint32_t>& positions,
                                std::vector<float>& models) const {
  positions.resize(n_selected_);
  models.resize(n_selected_ * n_images_);
  gpu::Check(rdl_subminor_get(h_, positions.data(), models.data(), n_selected_),
             "rdl_subminor_get");
}

}  // namespace radler::algorithms
