#include "component_optimization.h"

#include <cmath>
#include <stdexcept>

#include "multiscale_transforms.h"
#include "spectral_fitter.h"
#include "subminor.h"

namespace radler::math {

void PaddedConvolveSubtract(gpu::Session& s, const float* d_src, float* d_dst,
                            size_t width, size_t height, size_t padded_width,
                            size_t padded_height, const void* d_psf_spectrum) {
  gpu::Fft& fft = s.GetFft(padded_width, padded_height, true);
  const size_t ox = (padded_width - width) / 2, oy = (padded_height - height) / 2;
  if (fft.UsesLds()) {
    gpu::Buffer work(s, fft.ConvolveSubtractBytes());
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

std::vector<gpu::Buffer> GradientDescentWithVariablePsf(
    gpu::Session& s, const std::vector<std::vector<std::pair<size_t, size_t>>>& lists,
    const float* d_image, const std::vector<std::shared_ptr<gpu::Buffer>>& psf_spectra,
    size_t width, size_t height, size_t padded_width, size_t padded_height) {
  const size_t n = width * height, bytes = n * sizeof(float), n_psfs = lists.size();
  std::vector<gpu::Buffer> mask, values, step;
  for (size_t p = 0; p != n_psfs; ++p) {
    // a 1.0 at every component position of the PSF's list
    std::vector<float> m(n, 0.0f);
    for (const auto& c : lists[p]) m[c.second * width + c.first] = 1.0f;
    mask.emplace_back(s, bytes);
    s.H2D(mask.back().Ptr(), m.data(), bytes);
    values.emplace_back(s, bytes);
    values.back().Zero();
    step.emplace_back(s, bytes);
  }
  gpu::Buffer residual(s, bytes), conv(s, bytes), direction(s, bytes);
  for (size_t iteration = 0; iteration != 10; ++iteration) {  // :347-386
    s.D2D(residual.Ptr(), d_image, bytes);
    if (iteration != 0)
      for (size_t p = 0; p != n_psfs; ++p)
        PaddedConvolveSubtract(s, values[p].F(), residual.F(), width, height,
                               padded_width, padded_height, psf_spectra[p]->Ptr());
    direction.Zero();  // holds -(direction image)
    for (size_t p = 0; p != n_psfs; ++p) {
      conv.Zero();
      PaddedConvolveSubtract(s, residual.F(), conv.F(), width, height, padded_width,
                             padded_height, psf_spectra[p]->Ptr());
      gpu::Check(rdl_masked_copy(s.Handle(), mask[p].F(), conv.F(), step[p].F(), n, -1.0f),
                 "rdl_masked_copy");
      PaddedConvolveSubtract(s, step[p].F(), direction.F(), width, height, padded_width,
                             padded_height, psf_spectra[p]->Ptr());
    }
    double neg_numerator = 0.0, divisor = 0.0;
    gpu::Check(rdl_dot_pair(s.Handle(), direction.F(), residual.F(), n, &neg_numerator,
                            &divisor),
               "rdl_dot_pair");
    if (float(divisor) != 0.0f) {
      const float lambda = float(-neg_numerator) / float(divisor);
      if (std::isfinite(lambda))
        for (size_t p = 0; p != n_psfs; ++p)
          gpu::Check(rdl_axpy(s.Handle(), values[p].F(), step[p].F(), n, lambda, 0),
                     "rdl_axpy");
    }
  }
  return values;
}

void RunFullComponentFitter(gpu::Session& s, float* d_residual, float* d_model,
                            const float* d_psf, size_t width, size_t height,
                            const std::vector<float>& scales,
                            const std::vector<std::vector<std::pair<size_t, size_t>>>& lists,
                            algorithms::multiscale::MultiScaleTransforms& transforms,
                            size_t padded_width, size_t padded_height) {
  const size_t n = width * height, bytes = n * sizeof(float), n_scales = scales.size();
  std::vector<std::shared_ptr<gpu::Buffer>> spectra;
  for (size_t sc = 0; sc != n_scales; ++sc) {
    // the PSF convolved by the scale's shape (:845-853) and its padded spectrum
    gpu::Buffer convolved(s, bytes);
    s.D2D(convolved.Ptr(), d_psf, bytes);
    transforms.Transform(convolved.F(), scales[sc]);
    spectra.push_back(algorithms::SubMinorLoop::MakePaddedPsfSpectrum(
        s, convolved.F(), width, height, padded_width, padded_height));
  }
  std::vector<gpu::Buffer> values = GradientDescentWithVariablePsf(
      s, lists, d_residual, spectra, width, height, padded_width, padded_height);
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

void LinearComponentSolve(gpu::Session& s, float* d_model, const float* d_image,
                          const float* d_psf, size_t width, size_t height) {
  // component_optimization.cc:181-263. The system is n_active x n_active (one
  // equation per active pixel): the model's non-zero pixels are read back,
  // the PSF and image values at the pairwise offsets gathered on the host
  // and solved by least squares (the reference: gsl_multifit_linear, an SVD
  // whose singular values below DBL_EPSILON * max are dropped).
  const size_t n = width * height;
  std::vector<float> model(n), image(n), psf(n);
  s.D2H(model.data(), d_model, n * sizeof(float));
  s.D2H(image.data(), d_image, n * sizeof(float));
  s.D2H(psf.data(), d_psf, n * sizeof(float));
  std::vector<std::pair<size_t, size_t>> active;  // GetActivePositions (:20-32)
  for (size_t y = 0; y != height; ++y)
    for (size_t x = 0; x != width; ++x)
      if (model[y * width + x] != 0.0f) active.emplace_back(x, y);
  const size_t n_active = active.size();
  if (n_active == 0) return;
  std::vector<double> x_matrix(n_active * n_active), y(n_active);
  for (size_t i = 0; i != n_active; ++i) {  // :204-208 (the index uses the height)
    const size_t idx = active[i].first + active[i].second * height;
    // the reference's index reads past its image when width < height; that
    // is undefined behaviour there, an error here
    if (idx >= n)
      throw std::runtime_error(
          "LinearComponentSolve: component index x + y * height outside the image "
          "(width < height, as the reference indexes)");
    y[i] = image[idx];
  }
  const size_t mid_x = width + width / 2, mid_y = height + height / 2;
  for (size_t i = 0; i != n_active; ++i)
    for (size_t j = 0; j != n_active; ++j) {
      const size_t psf_x = (active[i].first + mid_x - active[j].first) % width;
      const size_t psf_y = (active[i].second + mid_y - active[j].second) % height;
      x_matrix[i * n_active + j] = psf[psf_x + psf_y * width];
    }
  const std::vector<double> pinv = PseudoInverse(std::move(x_matrix), n_active, n_active);
  for (size_t p = 0; p != n_active; ++p) {
    double c = 0.0;
    for (size_t i = 0; i != n_active; ++i) c += pinv[p * n_active + i] * y[i];
    model[active[p].first + active[p].second * width] += float(c);
  }
  s.H2D(d_model, model.data(), n * sizeof(float));
}

}  // namespace radler::math
