// radler::math component optimisation (cpp/math/component_optimization.h)
// on the device: GenericClean's kGradientDescent (generic_clean.cc:26-48).
#pragma once

#include <cstddef>

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
