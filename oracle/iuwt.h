// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
// IUWT à-trous decomposition restatement (see iuwt.cc).
#pragma once

#include <cstddef>
#include <vector>

namespace oracle {

void IuwtHorizontal(float* output, const float* image, size_t width,
                    size_t height, int scale);
void IuwtVertical(float* output, const float* image, size_t width, size_t height,
                  int scale);
// coeffs: n_scales + 1 planes (the last is the approximation, empty when
// !include_largest). input may equal scratch (aliased reference calls).
void IuwtDecompose(const float* input, float* scratch, size_t w, size_t h,
                   size_t n_scales, std::vector<std::vector<float>>& coeffs,
                   bool include_largest);
void IuwtRecompose(const std::vector<std::vector<float>>& coeffs, size_t w,
                   size_t h, size_t n_scales, bool include_largest, float* output);

}  // namespace oracle
