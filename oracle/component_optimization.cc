// TEST INFRASTRUCTURE — see component_optimization.h.
#include "component_optimization.h"

#include <cmath>
#include <utility>
#include <vector>

#include "fft.h"
#include "oracle.h"

namespace oracle {

void PaddedConvolution(float* image, const float* psf, size_t width, size_t height,
                       size_t padded_width, size_t padded_height) {
  const size_t pn = padded_width * padded_height;
  std::vector<float> a(pn), b(pn), kernel(pn);
  Untrim(a.data(), padded_width, padded_height, psf, width, height);
  PrepareConvolutionKernel(kernel.data(), a.data(), padded_width, padded_height);
  Untrim(b.data(), padded_width, padded_height, image, width, height);
  ConvolveCircular(b.data(), kernel.data(), padded_width, padded_height);
  Trim(image, width, height, b.data(), padded_width, padded_height);
}

namespace {
using Positions = std::vector<std::pair<size_t, size_t>>;

// ConvolveModel (component_optimization.cc:48-98), FFT branch
template <bool Subtract>
void ConvolveModel(float* result, const Positions& components, const float* psf,
                   const float* values, size_t w, size_t h, size_t pw, size_t ph) {
  std::vector<float> scratch(w * h, 0.0f);
  for (size_t i = 0; i != components.size(); ++i)
    scratch[components[i].second * w + components[i].first] += values[i];
  PaddedConvolution(scratch.data(), psf, w, h, pw, ph);
  for (size_t i = 0; i != w * h; ++i) {
    if constexpr (Subtract)
      result[i] -= scratch[i];
    else
      result[i] += scratch[i];
  }
}
}  // namespace

void GradientDescent(float* model, const float* image, const float* psf,
                     size_t width, size_t height, size_t padded_width,
                     size_t padded_height) {
  Positions components;  // GetActivePositions (:20-32)
  for (size_t y = 0; y != height; ++y)
    for (size_t x = 0; x != width; ++x)
      if (model[y * width + x] != 0.0) components.emplace_back(x, y);
  if (components.empty()) return;
  const size_t n = width * height;
  std::vector<float> model_step(components.size()), model_values(components.size(), 0.0f);
  std::vector<float> derivative_image(n), residual(n), times_psf(n);
  for (size_t iteration = 0; iteration != 4; ++iteration) {  // :282-302
    residual.assign(image, image + n);
    if (iteration != 0)
      ConvolveModel<true>(residual.data(), components, psf, model_values.data(), width,
                          height, padded_width, padded_height);
    // CalculateDerivatives (:100-152)
    times_psf = residual;
    PaddedConvolution(times_psf.data(), psf, width, height, padded_width, padded_height);
    for (size_t i = 0; i != components.size(); ++i)
      model_step[i] = times_psf[components[i].first + components[i].second * width];
    std::fill(derivative_image.begin(), derivative_image.end(), 0.0f);
    ConvolveModel<false>(derivative_image.data(), components, psf, model_step.data(),
                         width, height, padded_width, padded_height);
    // ApplyLineSearch (:154-177): float sums in pixel order
    float numerator = 0.0f, divisor = 0.0f;
    for (size_t i = 0; i != n; ++i) {
      numerator += derivative_image[i] * residual[i];
      divisor += derivative_image[i] * derivative_image[i];
    }
    if (divisor != 0.0f) {
      const float step = numerator / divisor;
      if (std::isfinite(step))
        for (size_t i = 0; i != components.size(); ++i)
          model_values[i] += model_step[i] * step;
    }
  }
  for (size_t i = 0; i != components.size(); ++i)  // :307-321
    model[components[i].first + components[i].second * width] += model_values[i];
}

}  // namespace oracle

namespace oracle {

std::vector<std::vector<float>> GradientDescentWithVariablePsf(
    const std::vector<std::vector<std::pair<size_t, size_t>>>& components_per_psf,
    const float* image, const std::vector<std::vector<float>>& psfs, size_t width,
    size_t height, size_t padded_width, size_t padded_height) {
  const size_t n = width * height;
  size_t count = 0;
  for (const auto& c : components_per_psf) count += c.size();
  std::vector<float> model_step(count), model_values(count, 0.0f);
  std::vector<float> derivative_image(n), residual(n), times_psf(n);
  for (size_t iteration = 0; iteration != 10; ++iteration) {  // :347-386
    residual.assign(image, image + n);
    if (iteration != 0) {
      size_t parameter = 0;
      for (size_t p = 0; p != psfs.size(); ++p) {
        ConvolveModel<true>(residual.data(), components_per_psf[p], psfs[p].data(),
                            &model_values[parameter], width, height, padded_width,
                            padded_height);
        parameter += components_per_psf[p].size();
      }
    }
    size_t parameter = 0;
    std::fill(derivative_image.begin(), derivative_image.end(), 0.0f);
    for (size_t p = 0; p != psfs.size(); ++p) {
      const auto& components = components_per_psf[p];
      times_psf = residual;
      PaddedConvolution(times_psf.data(), psfs[p].data(), width, height, padded_width,
                        padded_height);
      for (size_t i = 0; i != components.size(); ++i)
        model_step[parameter + i] =
            times_psf[components[i].first + components[i].second * width];
      ConvolveModel<false>(derivative_image.data(), components, psfs[p].data(),
                           &model_step[parameter], width, height, padded_width,
                           padded_height);
      parameter += components.size();
    }
    float numerator = 0.0f, divisor = 0.0f;  // ApplyLineSearch
    for (size_t i = 0; i != n; ++i) {
      numerator += derivative_image[i] * residual[i];
      divisor += derivative_image[i] * derivative_image[i];
    }
    if (divisor != 0.0f) {
      const float step = numerator / divisor;
      if (std::isfinite(step))
        for (size_t i = 0; i != count; ++i) model_values[i] += model_step[i] * step;
    }
  }
  std::vector<std::vector<float>> result(psfs.size(), std::vector<float>(n, 0.0f));
  size_t parameter = 0;
  for (size_t p = 0; p != psfs.size(); ++p) {
    for (size_t i = 0; i != components_per_psf[p].size(); ++i) {
      const auto& pos = components_per_psf[p][i];
      result[p][pos.second * width + pos.first] += model_values[parameter + i];
    }
    parameter += components_per_psf[p].size();
  }
  return result;
}

void RunFullComponentFitter(float* residual, float* model, const float* psf, size_t width,
                            size_t height, const std::vector<float>& scales,
                            const std::vector<std::vector<std::pair<size_t, size_t>>>& lists,
                            double convolution_padding, int shape) {
  const size_t n = width * height;
  std::vector<std::vector<float>> convolved_psfs;
  for (float scale : scales) {  // :845-853
    convolved_psfs.emplace_back(psf, psf + n);
    std::vector<float*> l{convolved_psfs.back().data()};
    MsTransform(l, width, height, scale, Shape(shape));
  }
  const size_t pw = GetConvolutionSize(scales.back(), width, convolution_padding);
  const size_t ph = GetConvolutionSize(scales.back(), height, convolution_padding);
  std::vector<std::vector<float>> delta = GradientDescentWithVariablePsf(
      lists, residual, convolved_psfs, width, height, pw, ph);
  for (size_t s = 0; s != scales.size(); ++s) {  // :898-904
    std::vector<float*> l{delta[s].data()};
    MsTransform(l, width, height, scales[s], Shape(shape));
    for (size_t i = 0; i != n; ++i) model[i] += delta[s][i];
  }
  for (size_t s = 0; s != scales.size(); ++s) {  // :906-911
    PaddedConvolution(delta[s].data(), psf, width, height, pw, ph);
    for (size_t i = 0; i != n; ++i) residual[i] -= delta[s][i];
  }
}

void LinearComponentSolve(float* model, const float* image, const float* psf,
                          size_t width, size_t height) {
  Positions active;  // GetActivePositions (:20-32)
  for (size_t y = 0; y != height; ++y)
    for (size_t x = 0; x != width; ++x)
      if (model[y * width + x] != 0.0) active.emplace_back(x, y);
  const size_t n = active.size();
  if (n == 0) return;
  // X (n x n) and y (:203-227)
  std::vector<long double> a(n * n), v(n * n, 0.0L), rhs(n);
  for (size_t i = 0; i != n; ++i) rhs[i] = image[active[i].first + active[i].second * height];
  const size_t mid_x = width + width / 2, mid_y = height + height / 2;
  for (size_t i = 0; i != n; ++i)
    for (size_t j = 0; j != n; ++j) {
      const size_t psf_x = (active[i].first + mid_x - active[j].first) % width;
      const size_t psf_y = (active[i].second + mid_y - active[j].second) % height;
      a[i * n + j] = psf[psf_x + psf_y * width];
    }
  // one-sided Jacobi SVD: A V = U S
  for (size_t j = 0; j != n; ++j) v[j * n + j] = 1.0L;
  for (int sweep = 0; sweep != 100; ++sweep) {
    bool rotated = false;
    for (size_t j = 0; j + 1 < n; ++j)
      for (size_t k = j + 1; k != n; ++k) {
        long double alpha = 0, beta = 0, gamma = 0;
        for (size_t i = 0; i != n; ++i) {
          alpha += a[i * n + j] * a[i * n + j];
          beta += a[i * n + k] * a[i * n + k];
          gamma += a[i * n + j] * a[i * n + k];
        }
        if (gamma == 0 || std::fabs(gamma) <= 1e-19L * std::sqrt(alpha * beta)) continue;
        rotated = true;
        const long double zeta = (beta - alpha) / (2 * gamma);
        const long double t =
            (zeta >= 0 ? 1.0L : -1.0L) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const long double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (size_t i = 0; i != n; ++i) {
          const long double x = a[i * n + j], y = a[i * n + k];
          a[i * n + j] = c * x - s * y;
          a[i * n + k] = s * x + c * y;
          const long double p = v[i * n + j], q = v[i * n + k];
          v[i * n + j] = c * p - s * q;
          v[i * n + k] = s * p + c * q;
        }
      }
    if (!rotated) break;
  }
  std::vector<long double> sigma(n);
  long double sigma_max = 0;
  for (size_t k = 0; k != n; ++k) {
    long double n2 = 0;
    for (size_t i = 0; i != n; ++i) n2 += a[i * n + k] * a[i * n + k];
    sigma[k] = std::sqrt(n2);
    sigma_max = std::max(sigma_max, sigma[k]);
  }
  // c = V S^-1 U^T y, with U_k = A_k / sigma_k
  std::vector<long double> c(n, 0.0L);
  for (size_t k = 0; k != n; ++k) {
    if (!(sigma[k] > 2.220446049250313e-16L * sigma_max)) continue;
    long double uty = 0;
    for (size_t i = 0; i != n; ++i) uty += a[i * n + k] * rhs[i];
    uty /= sigma[k] * sigma[k];
    for (size_t j = 0; j != n; ++j) c[j] += v[j * n + k] * uty;
  }
  for (size_t p = 0; p != n; ++p)  // model += LinearComponentSolve(...) (:262)
    model[active[p].first + active[p].second * width] += float(double(c[p]));
}

}  // namespace oracle
