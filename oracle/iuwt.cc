// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// IuwtDecomposition restated (cpp/algorithms/iuwt/iuwt_decomposition.cc:9-237,
// iuwt_decomposition.h:94-146, 200-276): B3-spline à-trous transform with
// spacing 2^(s+1)-1 and zero boundaries.
//
// FMA: the reference's -O3 -march=native build contracts a tap sum
// t_0 + t_1 + ... + t_k (t_j = x_j * h_j, in source order) into
//   fma(x_k, h_k, ... fma(x_2, h_2, fma(x_0, h_0, x_1 * h_1)))
// and `o += x * v` into fma(x, v, o). Established by compiling the same
// expression shapes with g++ -O3 -march=x86-64-v3 (oracle/probes/iuwt_fma_*.cc, `make -C oracle probe`).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "iuwt.h"

namespace oracle {

namespace {

const float kH[5] = {1.0 / 16.0, 4.0 / 16.0, 6.0 / 16.0, 4.0 / 16.0, 1.0 / 16.0};

// sum in the given tap order, contracted as the reference build does
inline float Taps(const float* x, const int* order, int n) {
  float acc = x[order[1]] * kH[order[1]];
  acc = std::fmaf(x[order[0]], kH[order[0]], acc);
  for (int i = 2; i < n; ++i) acc = std::fmaf(x[order[i]], kH[order[i]], acc);
  return acc;
}

}  // namespace

// convolveHorizontalFast (iuwt_decomposition.cc:84-131); rows are processed
// left to right, so output == image reproduces the reference's in-place
// (aliased) behaviour.
void IuwtHorizontal(float* output, const float* image, size_t width,
                    size_t height, int scale) {
  const int d = (1 << scale) - 1;
  const int64_t w = int64_t(width);
  static const int r1[3] = {2, 3, 4}, r2[4] = {2, 1, 3, 4}, r3[5] = {2, 1, 0, 3, 4},
                   r4[4] = {2, 1, 0, 3}, r5[3] = {2, 1, 0};
  for (size_t y = 0; y != height; ++y) {
    float* out = output + y * width;
    const float* in = image + y * width;
    for (int64_t x = 0; x != w; ++x) {
      float t[5];
      for (int k = 0; k != 5; ++k) {
        const int64_t xx = x + int64_t(d) * (k - 2);
        t[k] = (xx >= 0 && xx < w) ? in[xx] : 0.0f;
      }
      float v;
      if (x < d)
        v = Taps(t, r1, 3);
      else if (x < 2 * d)
        v = Taps(t, r2, 4);
      else if (x < w - 2 * d)
        v = Taps(t, r3, 5);
      else if (x < w - d)
        v = Taps(t, r4, 4);
      else
        v = Taps(t, r5, 3);
      out[x] = v;
    }
  }
}

// convolveVerticalPartialFast (iuwt_decomposition.cc:172-235)
void IuwtVertical(float* output, const float* image, size_t width, size_t height,
                  int scale) {
  const int d = (1 << scale) - 1;
  const int64_t h = int64_t(height);
  static const int r1[3] = {2, 3, 4}, r2[4] = {1, 2, 3, 4}, r3[5] = {0, 1, 2, 3, 4},
                   r4[4] = {0, 1, 2, 3}, r5[3] = {0, 1, 2};
  for (int64_t y = 0; y != h; ++y) {
    for (size_t x = 0; x != width; ++x) {
      float t[5];
      for (int k = 0; k != 5; ++k) {
        const int64_t yy = y + int64_t(d) * (k - 2);
        t[k] = (yy >= 0 && yy < h) ? image[yy * width + x] : 0.0f;
      }
      float v;
      if (y < d)
        v = Taps(t, r1, 3);
      else if (y < 2 * d)
        v = Taps(t, r2, 4);
      else if (y < h - 2 * d)
        v = Taps(t, r3, 5);
      else if (y < h - d)
        v = Taps(t, r4, 4);
      else
        v = Taps(t, r5, 3);
      output[y * width + x] = v;
    }
  }
}

static void ConvolveMT(float* output, const float* image, float* scratch,
                       size_t w, size_t h, int scale) {
  IuwtHorizontal(scratch, image, w, h, scale);
  IuwtVertical(output, scratch, w, h, scale);
}

void IuwtDecompose(const float* input, float* scratch, size_t w, size_t h,
                   size_t n_scales, std::vector<std::vector<float>>& coeffs,
                   bool include_largest) {
  // DecomposeMt (iuwt_decomposition.cc:9-54); `input` may equal `scratch`
  const size_t n = w * h;
  coeffs.assign(n_scales + 1, std::vector<float>());
  std::vector<float>& i1 = coeffs.back();
  i1.assign(n, 0.0f);
  coeffs[0].assign(n, 0.0f);
  ConvolveMT(i1.data(), input, scratch, w, h, 1);
  ConvolveMT(coeffs[0].data(), i1.data(), scratch, w, h, 1);
  for (size_t i = 0; i != n; ++i) coeffs[0][i] = input[i] - coeffs[0][i];
  std::vector<float> i0(i1);
  for (size_t s = 1; s < n_scales; ++s) {
    coeffs[s].assign(n, 0.0f);
    ConvolveMT(i1.data(), i0.data(), scratch, w, h, int(s) + 1);
    ConvolveMT(coeffs[s].data(), i1.data(), scratch, w, h, int(s) + 1);
    for (size_t i = 0; i != n; ++i) coeffs[s][i] = i0[i] - coeffs[s][i];
    if (s + 1 != n_scales) i0 = i1;
  }
  if (!include_largest) coeffs.back().clear();
}

// IuwtDecomposition::convolve (iuwt_decomposition.h:243-261): zeroed
// accumulators, one full pass per tap h0..h4, horizontal then vertical
static void ConvolveAccumulate(float* output, const float* image, size_t w,
                               size_t h, int scale) {
  std::vector<float> scratch(w * h, 0.0f);
  const int d = (1 << scale) - 1;
  for (int k = 0; k != 5; ++k) {
    const int64_t dist = int64_t(d) * (k - 2);
    const int64_t lo = std::max<int64_t>(0, -dist), hi = std::min<int64_t>(w, w - dist);
    for (size_t y = 0; y != h; ++y)
      for (int64_t x = lo; x < hi; ++x)
        scratch[y * w + x] = std::fmaf(image[y * w + x + dist], kH[k], scratch[y * w + x]);
  }
  std::fill(output, output + w * h, 0.0f);
  for (int k = 0; k != 5; ++k) {
    const int64_t dist = int64_t(d) * (k - 2);
    const int64_t lo = std::max<int64_t>(0, -dist), hi = std::min<int64_t>(h, h - dist);
    for (int64_t y = lo; y < hi; ++y)
      for (size_t x = 0; x != w; ++x)
        output[y * w + x] = std::fmaf(scratch[(y + dist) * w + x], kH[k], output[y * w + x]);
  }
}

void IuwtRecompose(const std::vector<std::vector<float>>& coeffs, size_t w,
                   size_t h, size_t n_scales, bool include_largest, float* output) {
  // Recompose (iuwt_decomposition.h:121-146)
  const size_t n = w * h;
  bool is_zero;
  if (include_largest) {
    std::copy_n(coeffs[n_scales].data(), n, output);
    is_zero = false;
  } else {
    std::fill(output, output + n, 0.0f);
    is_zero = true;
  }
  std::vector<float> tmp(n);
  for (int s = int(n_scales) - 1; s != -1; --s) {
    if (is_zero) {
      std::copy_n(coeffs[s].data(), n, output);
      is_zero = false;
    } else {
      ConvolveAccumulate(tmp.data(), output, w, h, s + 1);
      for (size_t i = 0; i != n; ++i) output[i] = tmp[i] + coeffs[s][i];
    }
  }
}

}  // namespace oracle
