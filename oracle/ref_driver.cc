// ORACLE / TEST INFRASTRUCTURE ONLY. Thin extern "C" driver around the
// reference's own compilable pieces (never copied: included / linked from
// /root/reference/cpp where they lie).
#include <cstddef>
#include <cstdint>

#include "algorithms/simple_clean.h"
#include "utils/fft_size_calculations.h"

extern "C" {
void ref_partial_subtract(float* image, const float* psf, uint64_t w,
                          uint64_t h, uint64_t x, uint64_t y, float factor,
                          uint64_t start_y, uint64_t end_y) {
  radler::algorithms::simple_clean::PartialSubtractImage(
      image, psf, w, h, x, y, factor, start_y, end_y);
}
uint64_t ref_good_fft_size(uint64_t n) {
  return radler::utils::CalculateGoodFFTSize(n);
}
uint64_t ref_convolution_size(double scale, uint64_t n, double padding) {
  return radler::utils::GetConvolutionSize(scale, n, padding);
}
}
