// TEST INFRASTRUCTURE — CPU oracle, used only by tests/, smoke() and the
// bench's cpu_baseline; never by the product.
//
// radler::math::rms_image (cpp/math/rms_image.cc:16-125) and the
// schaapcommon::math::RestoreImage it calls (the schaapcommon submodule is not
// vendored in /root/reference; restated: an elliptical Gaussian of peak 1,
// FWHM axes beam_major / beam_minor, truncated to an even bounding box of
// ceil(40 sigma_max / pixel scale) pixels (at most the smaller image side),
// circularly FFT-convolved and added). Radler calls it with a circular beam
// and position angle 0, so the rotation convention is not observable there.
#pragma once

#include <cstddef>

namespace oracle {

void RestoreImage(float* image, const float* model, size_t width, size_t height,
                  long double beam_major, long double beam_minor,
                  long double beam_pa, long double pixel_scale_l,
                  long double pixel_scale_m);

// rms_image.cc:16-33
void RmsImageMake(float* rms_out, const float* input, size_t width, size_t height,
                  double window_size, long double beam_major, long double beam_minor,
                  long double beam_pa, long double pixel_scale_l,
                  long double pixel_scale_m);
// rms_image.cc:35-68
void SlidingMinimum(float* output, const float* input, size_t width,
                    size_t height, size_t window_size);
// rms_image.cc:77-93
void RmsImageMakeWithNegativityLimit(float* rms_out, const float* input,
                                     size_t width, size_t height,
                                     double window_size, long double beam_major,
                                     long double beam_minor, long double beam_pa,
                                     long double pixel_scale_l,
                                     long double pixel_scale_m);
// rms_image.cc:95-125; returns the lowest RMS (throws on a negative one)
double MakeRmsFactorImage(float* rms_image, size_t n, double local_rms_strength);

}  // namespace oracle
