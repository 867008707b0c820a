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

namespace oracle {

// schaapcommon::math::PaddedConvolution
void PaddedConvolution(float* image, const float* psf, size_t width, size_t height,
                       size_t padded_width, size_t padded_height);

// model += the gradient-descent update of its non-zero components
void GradientDescent(float* model, const float* image, const float* psf,
                     size_t width, size_t height, size_t padded_width,
                     size_t padded_height);

}  // namespace oracle
