#include "rms_image.h"

#include <algorithm>
#include <cmath>

namespace radler::math::rms_image {

void Make(gpu::Session& s, float* d_rms_output, const float* d_input, size_t width,
          size_t height, double window_size, long double beam_major,
          long double beam_minor, long double beam_pa, long double pixel_scale_l,
          long double pixel_scale_m) {
  const size_t n = width * height;
  // Image::Square, then RestoreImage into a zero image (0 + x == x)
  gpu::Check(rdl_square(s.Handle(), d_input, d_rms_output, n), "rdl_square");
  const long double bmaj = beam_major * window_size, bmin = beam_minor * window_size;
  if (bmaj != 0.0L || bmin != 0.0L) {
    const long double fwhm_to_sigma = 1.0L / (2.0L * sqrtl(2.0L * logl(2.0L)));
    const long double sigma_major = bmaj * fwhm_to_sigma;
    const long double sigma_minor = bmin * fwhm_to_sigma;
    const long double angle = beam_pa + 0.5L * M_PI;  // from North
    const double sigma_max = double(std::max(fabsl(sigma_major * cosl(angle)),
                                             fabsl(sigma_major * sinl(angle))));
    const size_t min_dim = std::min(width, height);
    size_t box = std::min<size_t>(
        size_t(std::ceil(sigma_max * 40.0 /
                         double(std::min(pixel_scale_l, pixel_scale_m)))),
        min_dim);
    if (box % 2 != 0) ++box;
    if (box > min_dim) box = min_dim;
    // float64 FFT convolution of the float squares and the float kernel,
    // rounded to float once: a float32 transform's rounding (relative to the
    // brightest squares) swamps the faint regions whose RMS sets the factor
    gpu::Fft& fft = s.GetFft(width, height, true);
    gpu::Buffer placed(s, n * sizeof(float));
    gpu::Check(rdl_place_gaussian(s.Handle(), placed.F(), uint32_t(width),
                                  uint32_t(height), uint32_t(box), double(pixel_scale_l),
                                  double(pixel_scale_m), double(sigma_major),
                                  double(sigma_minor), double(angle)),
               "rdl_place_gaussian");
    gpu::Buffer spectrum(s, fft.SpectrumBytes());
    if (fft.UsesLds()) {  // float in/out, float64 transforms
      fft.Forward(placed.F(), spectrum.Ptr());
      fft.Convolve(d_rms_output, spectrum.Ptr());
    } else {  // rocFFT double
      gpu::Buffer placed64(s, n * sizeof(double)), squares64(s, n * sizeof(double));
      gpu::Check(rdl_convert(s.Handle(), placed.F(), placed64.D(), n, 1), "rdl_convert");
      gpu::Check(rdl_convert(s.Handle(), d_rms_output, squares64.D(), n, 1), "rdl_convert");
      fft.Forward64(placed64.D(), spectrum.Ptr());
      fft.Convolve64(squares64.D(), spectrum.Ptr());
      gpu::Check(rdl_convert(s.Handle(), squares64.D(), d_rms_output, n, 0), "rdl_convert");
    }
  }
  const double root = std::sqrt(2.0 * M_PI);
  const long double sigma_maj = beam_major / (2.0L * sqrtl(2.0L * logl(2.0L)));
  const long double sigma_min = beam_minor / (2.0L * sqrtl(2.0L * logl(2.0L)));
  const double norm = 1.0 / double(root * sigma_maj / pixel_scale_l * window_size * root *
                                   sigma_min / pixel_scale_l * window_size);
  gpu::Check(rdl_rms_finish(s.Handle(), d_rms_output, n, norm), "rdl_rms_finish");
}

void SlidingMinimum(gpu::Session& s, float* d_output, const float* d_input,
                    float* d_scratch, size_t width, size_t height, size_t window_size) {
  gpu::Check(rdl_sliding_min(s.Handle(), d_input, d_output, d_scratch, uint32_t(width),
                             uint32_t(height), window_size),
             "rdl_sliding_min");
}

void MakeWithNegativityLimit(gpu::Session& s, float* d_rms_output, const float* d_input,
                             size_t width, size_t height, double window_size,
                             long double beam_major, long double beam_minor,
                             long double beam_pa, long double pixel_scale_l,
                             long double pixel_scale_m) {
  Make(s, d_rms_output, d_input, width, height, window_size, beam_major, beam_minor,
       beam_pa, pixel_scale_l, pixel_scale_m);
  const size_t n = width * height;
  gpu::Buffer minimum(s, n * sizeof(float)), scratch(s, 3 * n * sizeof(float));
  const long double beam_in_pixels = std::max(beam_major / pixel_scale_l, 1.0L);
  SlidingMinimum(s, minimum.F(), d_input, scratch.F(), width, height,
                 size_t(window_size * beam_in_pixels));
  gpu::Check(rdl_rms_negativity_limit(s.Handle(), d_rms_output, minimum.F(), n),
             "rdl_rms_negativity_limit");
}

double MakeRmsFactorImage(gpu::Session& s, float* d_rms_image, size_t n,
                          double local_rms_strength) {
  double lowest = 0.0;
  gpu::Check(rdl_rms_factor(s.Handle(), d_rms_image, n, local_rms_strength, &lowest),
             "rdl_rms_factor");
  return lowest;
}

}  // namespace radler::math::rms_image
