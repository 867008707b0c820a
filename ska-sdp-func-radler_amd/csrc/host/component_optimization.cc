#include "component_optimization.h"

#include <cmath>

#include "multiscale_transforms.h"
#include "subminor.h"

namespace radler::math {

void PaddedConvolveSubtract(gpu::Session& s, const float* d_src, float* d_dst,
                            size_t width, size_t height, size_t padded_width,
                            size_t padded_height, const void* d_psf_spectrum) {
  gpu::Fft& fft = s.GetFft(padded_width, padded_height, true);
  const size_t ox = (padded_width - width) / 2, oy = (padded_height - height) / 2;
  if (fft.UsesLds()) {
    gpu::Buffer work(s, fft.SpectrumBytes());
    fft.ConvolveSubtract(d_src, width, height, ox, oy, d_psf_spectrum, work.Ptr(), d_dst,
                         nullptr, !fft.SplitColumns());
    return;
  }
  const size_t pn = padded_width * padded_height;
  gpu::Buffer padded(s, pn * sizeof(float)), padded64(s, pn * sizeof(double));
  gpu::Check(rdl_untrim(s.Handle(), padded.F(), uint32_t(padded_width),
                        uint32_t(padded_height), d_src, uint32_t(width), uint32_t(height)),
             "rdl_untrim");
  gpu::Check(rdl_convert(s.Handle(), padded.F(), padded64.D(), pn, 1), "rdl_convert");
  fft.Convolve64(padded64.D(), d_psf_spectrum);
  gpu::Check(rdl_trim_subtract_f64(s.Handle(), d_dst, uint32_t(width), uint32_t(height),
                                   padded64.D(), uint32_t(padded_width),
                                   uint32_t(padded_height)),
             "rdl_trim_subtract_f64");
}

void GradientDescent(gpu::Session& s, float* d_model, const float* d_image,
                     const float* d_psf, size_t width, size_t height,
                     size_t padded_width, size_t padded_height) {
  const size_t n = width * height;
  const size_t bytes = n * sizeof(float);
  const std::shared_ptr<gpu::Buffer> spectrum =
      algorithms::SubMinorLoop::MakePaddedPsfSpectrum(s, d_psf, width, height,
                                                       padded_width, padded_height);
  // planes: the component values, their step (the derivatives), the residual
  // and two convolution outputs
  gpu::Buffer values(s, bytes), step(s, bytes), residual(s, bytes), conv(s, bytes);
  values.Zero();
  for (size_t iteration = 0; iteration != 4; ++iteration) {  // :282-302
    s.D2D(residual.Ptr(), d_image, bytes);
    if (iteration != 0)  // ConvolveModel<true>
      PaddedConvolveSubtract(s, values.F(), residual.F(), width, height, padded_width,
                             padded_height, spectrum->Ptr());
    // CalculateDerivatives: conv(residual) at the components; conv holds
    // -conv(residual) (0 - ...)
    conv.Zero();
    PaddedConvolveSubtract(s, residual.F(), conv.F(), width, height, padded_width,
                           padded_height, spectrum->Ptr());
    gpu::Check(rdl_masked_copy(s.Handle(), d_model, conv.F(), step.F(), n, -1.0f),
               "rdl_masked_copy");
    // ConvolveModel<false> into a zero direction image: conv = -direction
    conv.Zero();
    PaddedConvolveSubtract(s, step.F(), conv.F(), width, height, padded_width,
                           padded_height, spectrum->Ptr());
    // ApplyLineSearch (:154-177): step = sum(dir*res) / sum(dir^2)
    double neg_numerator = 0.0, divisor = 0.0;
    gpu::Check(rdl_dot_pair(s.Handle(), conv.F(), residual.F(), n, &neg_numerator, &divisor),
               "rdl_dot_pair");
    if (float(divisor) != 0.0f) {
      const float lambda = float(-neg_numerator) / float(divisor);
      if (std::isfinite(lambda))  // values += derivative * step
        gpu::Check(rdl_axpy(s.Handle(), values.F(), step.F(), n, lambda, 0), "rdl_axpy");
    }
  }
  gpu::Check(rdl_masked_add(s.Handle(), d_model, values.F(), n), "rdl_masked_add");
}

}  // namespace radler::math

namespace radler::math {

void RunFullComponentFitter(gpu::Session& s, float* d_residual, float* d_model,
                            const float* d_psf, size_t width, size_t height,
                            const std::vector<float>& scales,
                            const std::vector<std::vector<std::pair<size_t, size_t>>>& lists,
                            algorithms::multiscale::MultiScaleTransforms& transforms,
                            size_t padded_width, size_t padded_height) {
  const size_t n = width * height, bytes = n * sizeof(float), n_scales = scales.size();
  std::vector<std::shared_ptr<gpu::Buffer>> spectra;
  std::vector<gpu::Buffer> mask, values, step;
  for (size_t sc = 0; sc != n_scales; ++sc) {
    // the PSF convolved by the scale's shape (:845-853) and its padded spectrum
    gpu::Buffer convolved(s, bytes);
    s.D2D(convolved.Ptr(), d_psf, bytes);
    transforms.Transform(convolved.F(), scales[sc]);
    spectra.push_back(algorithms::SubMinorLoop::MakePaddedPsfSpectrum(
        s, convolved.F(), width, height, padded_width, padded_height));
    // a 1.0 at every component position of the scale
    std::vector<float> m(n, 0.0f);
    for (const auto& p : lists[sc]) m[p.second * width + p.first] = 1.0f;
    mask.emplace_back(s, bytes);
    s.H2D(mask.back().Ptr(), m.data(), bytes);
    values.emplace_back(s, bytes);
    values.back().Zero();
    step.emplace_back(s, bytes);
  }
  gpu::Buffer residual(s, bytes), conv(s, bytes), direction(s, bytes);
  for (size_t iteration = 0; iteration != 10; ++iteration) {  // :347-386
    s.D2D(residual.Ptr(), d_residual, bytes);
    if (iteration != 0)
      for (size_t sc = 0; sc != n_scales; ++sc)
        PaddedConvolveSubtract(s, values[sc].F(), residual.F(), width, height,
                               padded_width, padded_height, spectra[sc]->Ptr());
    direction.Zero();  // holds -(direction image)
    for (size_t sc = 0; sc != n_scales; ++sc) {
      conv.Zero();
      PaddedConvolveSubtract(s, residual.F(), conv.F(), width, height, padded_width,
                             padded_height, spectra[sc]->Ptr());
      gpu::Check(rdl_masked_copy(s.Handle(), mask[sc].F(), conv.F(), step[sc].F(), n, -1.0f),
                 "rdl_masked_copy");
      PaddedConvolveSubtract(s, step[sc].F(), direction.F(), width, height, padded_width,
                             padded_height, spectra[sc]->Ptr());
    }
    double neg_numerator = 0.0, divisor = 0.0;
    gpu::Check(rdl_dot_pair(s.Handle(), direction.F(), residual.F(), n, &neg_numerator,
                            &divisor),
               "rdl_dot_pair");
    if (float(divisor) != 0.0f) {
      const float lambda = float(-neg_numerator) / float(divisor);
      if (std::isfinite(lambda))
        for (size_t sc = 0; sc != n_scales; ++sc)
          gpu::Check(rdl_axpy(s.Handle(), values[sc].F(), step[sc].F(), n, lambda, 0),
                     "rdl_axpy");
    }
  }
  const std::shared_ptr<gpu::Buffer> psf_spectrum =
      algorithms::SubMinorLoop::MakePaddedPsfSpectrum(s, d_psf, width, height,
                                                       padded_width, padded_height);
  for (size_t sc = 0; sc != n_scales; ++sc) {  // :898-911
    transforms.Transform(values[sc].F(), scales[sc]);
    gpu::Check(rdl_add(s.Handle(), d_model, values[sc].F(), n), "rdl_add");
  }
  for (size_t sc = 0; sc != n_scales; ++sc)
    PaddedConvolveSubtract(s, values[sc].F(), d_residual, width, height, padded_width,
                           padded_height, psf_spectrum->Ptr());
}

}  // namespace radler::math
