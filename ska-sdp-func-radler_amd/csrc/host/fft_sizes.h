// FFT size selection (reference: cpp/utils/fft_size_calculations.h:15-50):
// smallest even 2^a 3^b 5^c 7^d >= n, and the multiscale padded size.
#pragma once

#include <cmath>
#include <cstddef>

namespace radler::utils {

inline size_t CalculateGoodFFTSize(size_t minimum_size) {
  size_t best = 2 * minimum_size;
  for (size_t f2 = 2; f2 < best; f2 *= 2)
    for (size_t f3 = f2; f3 < best; f3 *= 3)
      for (size_t f5 = f3; f5 < best; f5 *= 5)
        for (size_t f7 = f5; f7 < best; f7 *= 7)
          if (f7 >= minimum_size) best = f7;
  return best;
}

inline size_t GetConvolutionSize(double scale, size_t original_size,
                                 double padding) {
  return CalculateGoodFFTSize(
      size_t(std::ceil(padding * (scale * 1.5 + original_size))));
}

}  // namespace radler::utils
