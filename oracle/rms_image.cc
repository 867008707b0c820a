// TEST INFRASTRUCTURE — see rms_image.h.
#include "rms_image.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <vector>

#include "fft.h"
#include "oracle.h"

namespace oracle {

void RestoreImage(float* image, const float* model, size_t width, size_t height,
                  long double beam_major, long double beam_minor,
                  long double beam_pa, long double pixel_scale_l,
                  long double pixel_scale_m) {
  const size_t n_px = width * height;
  if (beam_major == 0.0L && beam_minor == 0.0L) {
    for (size_t i = 0; i != n_px; ++i) image[i] += model[i];
    return;
  }
  const long double fwhm_to_sigma = 1.0L / (2.0L * sqrtl(2.0L * logl(2.0L)));
  const long double sigma_major = beam_major * fwhm_to_sigma;
  const long double sigma_minor = beam_minor * fwhm_to_sigma;
  // position angle from North: the major axis along angle + pi/2
  const long double angle = beam_pa + 0.5L * M_PI;
  const long double c = cosl(angle), s = sinl(angle);
  const double sigma_max =
      double(std::max(fabsl(sigma_major * c), fabsl(sigma_major * s)));
  const size_t min_dim = std::min(width, height);
  size_t box = std::min<size_t>(
      size_t(std::ceil(sigma_max * 40.0 / double(std::min(pixel_scale_l, pixel_scale_m)))),
      min_dim);
  if (box % 2 != 0) ++box;
  if (box > min_dim) box = min_dim;
  std::vector<float> kernel(box * box);
  for (size_t y = 0; y != box; ++y) {
    for (size_t x = 0; x != box; ++x) {
      const long double l = (long double)(ptrdiff_t(box / 2) - ptrdiff_t(x)) * pixel_scale_l;
      const long double m = (long double)(ptrdiff_t(y) - ptrdiff_t(box / 2)) * pixel_scale_m;
      const long double lt = (l * c + m * s) / sigma_major;
      const long double mt = (-l * s + m * c) / sigma_minor;
      kernel[y * box + x] = float(expl(-0.5L * (lt * lt + mt * mt)));
    }
  }
  std::vector<float> placed(n_px, 0.0f);
  PrepareSmallConvolutionKernel(placed.data(), width, height, kernel.data(), box);
  std::vector<float> convolved(model, model + n_px);
  ConvolveCircular(convolved.data(), placed.data(), width, height);
  for (size_t i = 0; i != n_px; ++i) image[i] += convolved[i];
}

void RmsImageMake(float* rms_out, const float* input, size_t width, size_t height,
                  double window_size, long double beam_major, long double beam_minor,
                  long double beam_pa, long double pixel_scale_l,
                  long double pixel_scale_m) {
  const size_t n = width * height;
  std::vector<float> image(input, input + n);
  for (float& v : image) v = v * v;  // Image::Square
  std::fill_n(rms_out, n, 0.0f);
  RestoreImage(rms_out, image.data(), width, height, beam_major * window_size,
               beam_minor * window_size, beam_pa, pixel_scale_l, pixel_scale_m);
  const double s = std::sqrt(2.0 * M_PI);
  const long double sigma_maj = beam_major / (2.0L * sqrtl(2.0L * logl(2.0L)));
  const long double sigma_min = beam_minor / (2.0L * sqrtl(2.0L * logl(2.0L)));
  const double norm = 1.0 / double(s * sigma_maj / pixel_scale_l * window_size * s *
                                   sigma_min / pixel_scale_l * window_size);
  for (size_t i = 0; i != n; ++i) rms_out[i] = float(std::sqrt(rms_out[i] * norm));
}

void SlidingMinimum(float* output, const float* input, size_t width,
                    size_t height, size_t window_size) {
  std::vector<float> temp(width * height);
  const size_t half = window_size / 2;
  for (size_t y = 0; y != height; ++y) {
    const float* in_row = &input[y * width];
    for (size_t x = 0; x != width; ++x) {
      const size_t left = std::max(x, half) - half;
      const size_t right = std::min(x, width - half) + half;
      temp[y * width + x] = *std::min_element(in_row + left, in_row + right);
    }
  }
  std::vector<float> vals;
  for (size_t x = 0; x != width; ++x) {
    for (size_t y = 0; y != height; ++y) {
      const size_t top = std::max(y, half) - half;
      const size_t bottom = std::min(y, height - half) + half;
      vals.clear();
      for (size_t wy = top; wy != bottom; ++wy) vals.push_back(temp[wy * width + x]);
      output[y * width + x] = *std::min_element(vals.begin(), vals.end());
    }
  }
}

void RmsImageMakeWithNegativityLimit(float* rms_out, const float* input,
                                     size_t width, size_t height,
                                     double window_size, long double beam_major,
                                     long double beam_minor, long double beam_pa,
                                     long double pixel_scale_l,
                                     long double pixel_scale_m) {
  RmsImageMake(rms_out, input, width, height, window_size, beam_major, beam_minor,
               beam_pa, pixel_scale_l, pixel_scale_m);
  std::vector<float> sliding_minimum(width * height);
  const long double beam_in_pixels = std::max(beam_major / pixel_scale_l, 1.0L);
  SlidingMinimum(sliding_minimum.data(), input, width, height,
                 size_t(window_size * beam_in_pixels));
  for (size_t i = 0; i != width * height; ++i)
    rms_out[i] = std::max<float>(rms_out[i],
                                 std::abs(sliding_minimum[i]) * (1.5 / 5.0));
}

double MakeRmsFactorImage(float* rms_image, size_t n, double local_rms_strength) {
  const double stddev = *std::min_element(rms_image, rms_image + n);
  if (stddev < 0.0)
    throw std::runtime_error(
        "RMS image can only contain values >= 0, but contains values < 0.0");
  if (local_rms_strength == 1.0) {
    for (size_t i = 0; i != n; ++i)
      if (rms_image[i] != 0.0) rms_image[i] = stddev / rms_image[i];
  } else if (local_rms_strength == 0.0) {
    std::fill_n(rms_image, n, 1.0f);
  } else {
    for (size_t i = 0; i != n; ++i)
      if (rms_image[i] != 0.0)
        rms_image[i] = std::pow(stddev / rms_image[i], local_rms_strength);
  }
  return stddev;
}

}  // namespace oracle
