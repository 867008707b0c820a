// TEST INFRASTRUCTURE — CPU oracle, used only by tests/, smoke() and the
// bench's cpu_baseline; never by the product.
//
// radler::math::GradientDescent (cpp/math/component_optimization.cc:20-177,
// 265-321) with schaapcommon::math::PaddedConvolution restated (Untrim image
// and PSF to the padded size, centre the PSF at the origin, circular FFT
// convolution, Trim), as GenericClean's RunComponentOptimization calls it
// (cpp/algorithms/generic_clean.cc:26-48: padded size 2W x 2H, FFT
// convolution).
#pragma once

#include <cstddef>
#include <utility>
#include <vector>

namespace oracle {

// schaapcommon::math::PaddedConvolution
void PaddedConvolution(float* image, const float* psf, size_t width, size_t height,
                       size_t padded_width, size_t padded_height);

// model += the gradient-descent update of its non-zero components
void GradientDescent(float* model, const float* image, const float* psf,
                     size_t width, size_t height, size_t padded_width,
                     size_t padded_height);

}  // namespace oracle

namespace oracle {

// component_optimization.cc:181-263: model += the least-squares solution of
// the n_active x n_active system (one equation per component pixel; the
// reference's gsl_multifit_linear, restated as an SVD pseudo-inverse in long
// double with singular values below DBL_EPSILON * max dropped). The
// reference's image index `x + y * height` (:206) is kept.
void LinearComponentSolve(float* model, const float* image, const float* psf,
                          size_t width, size_t height);

// component_optimization.cc:323-402: all scales' components fitted together,
// each scale with its own (scale-convolved) PSF; returns one delta image of
// component values per scale.
std::vector<std::vector<float>> GradientDescentWithVariablePsf(
    const std::vector<std::vector<std::pair<size_t, size_t>>>& components_per_psf,
    const float* image, const std::vector<std::vector<float>>& psfs, size_t width,
    size_t height, size_t padded_width, size_t padded_height);

// MultiScaleAlgorithm::RunFullComponentFitter for one image
// (multiscale_algorithm.cc:837-914, component-list bookkeeping aside):
// residual and model updated in place.
void RunFullComponentFitter(float* residual, float* model, const float* psf, size_t width,
                            size_t height, const std::vector<float>& scales,
                            const std::vector<std::vector<std::pair<size_t, size_t>>>& lists,
                            double convolution_padding, int shape);

}  // namespace oracle
