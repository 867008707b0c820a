// radler::math::rms_image (cpp/math/rms_image.{h,cc}) on the device: the
// local-RMS image Radler::Perform builds from the integrated residual
// (cpp/radler.cc:196-216) and the factor image every peak search multiplies
// in. Images are device planes of the session.
#pragma once

#include <cstddef>

#include "device.h"

namespace radler::math::rms_image {

/// rms_image.cc:16-33: sqrt(window-Gaussian-weighted mean of input^2). The
/// window is schaapcommon::math::RestoreImage's Gaussian (peak 1, FWHM
/// beam x window_size, truncated to an even box of ceil(40 sigma) pixels, at
/// most the smaller image side), convolved circularly through the FFT engine.
void Make(gpu::Session& s, float* d_rms_output, const float* d_input, size_t width,
          size_t height, double window_size, long double beam_major,
          long double beam_minor, long double beam_pa, long double pixel_scale_l,
          long double pixel_scale_m);

/// rms_image.cc:35-68 (d_scratch: 3 x width x height floats).
void SlidingMinimum(gpu::Session& s, float* d_output, const float* d_input,
                    float* d_scratch, size_t width, size_t height, size_t window_size);

/// rms_image.cc:77-93: Make, then max(rms, 0.3 x |sliding minimum|).
void MakeWithNegativityLimit(gpu::Session& s, float* d_rms_output, const float* d_input,
                             size_t width, size_t height, double window_size,
                             long double beam_major, long double beam_minor,
                             long double beam_pa, long double pixel_scale_l,
                             long double pixel_scale_m);

/// rms_image.cc:95-125 in place; returns the lowest RMS.
double MakeRmsFactorImage(gpu::Session& s, float* d_rms_image, size_t n,
                          double local_rms_strength);

}  // namespace radler::math::rms_image
