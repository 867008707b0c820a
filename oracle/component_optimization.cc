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
