// radler::math component optimisation (cpp/math/component_optimization.h)
// on the device: GenericClean's kGradientDescent (generic_clean.cc:26-48).
#pragma once

#include <cstddef>
#include <memory>
#include <utility>
#include <vector>

#include "device.h"

namespace radler::math {

/// schaapcommon::math::PaddedConvolution as dst -= Trim(conv(Untrim(src)))
/// with a padded PSF spectrum (SubMinorLoop::MakePaddedPsfSpectrum).
void PaddedConvolveSubtract(gpu::Session& s, const float* d_src, float* d_dst,
                            size_t width, size_t height, size_t padded_width,
                            size_t padded_height, const void* d_psf_spectrum);

/// component_optimization.cc:265-321 with FFT convolutions: d_model's
/// non-zero pixels are the components; d_model += the four-iteration
/// gradient-descent update fitting d_image (the residual) with d_psf.
void GradientDescent(gpu::Session& s, float* d_model, const float* d_image,
                     const float* d_psf, size_t width, size_t height,
                     size_t padded_width, size_t padded_height);

}  // namespace radler::math

namespace radler::algorithms::multiscale {
class MultiScaleTransforms;
}

namespace radler::math {

/// component_optimization.cc:323-402 (FFT convolutions): every list's
/// components fitted together, list p with the PSF whose padded spectrum is
/// psf_spectra[p] (SubMinorLoop::MakePaddedPsfSpectrum); returns one plane
/// of component values per list (the deltas).
std::vector<gpu::Buffer> GradientDescentWithVariablePsf(
    gpu::Session& s, const std::vector<std::vector<std::pair<size_t, size_t>>>& lists,
    const float* d_image, const std::vector<std::shared_ptr<gpu::Buffer>>& psf_spectra,
    size_t width, size_t height, size_t padded_width, size_t padded_height);

/// component_optimization.cc:181-263 (LinearComponentSolve(model, image,
/// psf)): d_model += the least-squares fit of its non-zero components to
/// d_image, one equation per component pixel.
void LinearComponentSolve(gpu::Session& s, float* d_model, const float* d_image,
                          const float* d_psf, size_t width, size_t height);

/// MultiScaleAlgorithm::RunFullComponentFitter for one image
/// (multiscale_algorithm.cc:837-914) with GradientDescentWithVariablePsf
/// (component_optimization.cc:323-402): lists[s] are the scale-s component
/// positions; every scale is fitted with the PSF convolved by its shape, the
/// updates are shape-transformed into the model and convolved out of the
/// residual (padded to the largest scale's convolution size).
void RunFullComponentFitter(gpu::Session& s, float* d_residual, float* d_model,
                            const float* d_psf, size_t width, size_t height,
                            const std::vector<float>& scales,
                            const std::vector<std::vector<std::pair<size_t, size_t>>>& lists,
                            algorithms::multiscale::MultiScaleTransforms& transforms,
                            size_t padded_width, size_t padded_height);

}  // namespace radler::math
