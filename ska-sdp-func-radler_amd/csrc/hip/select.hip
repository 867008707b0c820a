// Exact order statistics by 4-pass 8-bit radix select over the float total
// order: the median / MAD behind aocommon Image::MedianAndStdDevFromMAD
// (called from Radler::Perform, cpp/radler.cc:162-166). 4 B/px per pass.
#include <cmath>
#include <cstring>

#include "rdl_internal.h"

namespace rdl {

__device__ __forceinline__ uint32_t OrderKey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void RadixHist(const float* v, size_t n,
                                                 int use_center, float center,
                                                 uint32_t prefix,
                                                 uint32_t prefix_mask,
                                                 int shift,
                                                 unsigned long long* hist) {
  __shared__ unsigned int lh[256];
  lh[threadIdx.x] = 0;
  __syncthreads();
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const float x = use_center ? fabsf(v[i] - center) : v[i];
    const uint32_t k = OrderKey(x);
    if ((k & prefix_mask) == prefix) atomicAdd(&lh[(k >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (lh[threadIdx.x])
    atomicAdd(&hist[threadIdx.x], (unsigned long long)lh[threadIdx.x]);
}

int SelectKth(rdl_session* s, const float* d_values, size_t n, int use_center,
              float center, uint64_t k, float* out) {
  RDL_TRY(s->EnsureScratch(s->radix, 256 * sizeof(unsigned long long)));
  auto* hist = static_cast<unsigned long long*>(s->radix.ptr);
  auto* h_hist = static_cast<unsigned long long*>(s->h_small);
  uint32_t prefix = 0, mask = 0;
  const unsigned grid = unsigned(std::min<size_t>(2048, DivUp(n, 256)));
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    RDL_HIP_CHECK(hipMemsetAsync(hist, 0, 256 * sizeof(unsigned long long),
                                 s->stream));
    {
      ScopedTiming t(s, "radix_select", double(n) * 4.0);
      RadixHist<<<grid, 256, 0, s->stream>>>(d_values, n, use_center, center,
                                             prefix, mask, shift, hist);
    }
    RDL_HIP_CHECK(hipGetLastError());
    RDL_HIP_CHECK(hipMemcpyAsync(h_hist, hist, 256 * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, s->stream));
    RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
    uint64_t cum = 0;
    uint32_t b = 0;
    for (; b < 256; ++b) {
      if (cum + h_hist[b] > k) break;
      cum += h_hist[b];
    }
    if (b == 256) {
      SetError("radix select: rank out of range");
      return RDL_ERR_ARG;
    }
    k -= cum;
    prefix |= b << shift;
    mask |= 0xffu << shift;
  }
  const uint32_t u = (prefix & 0x80000000u) ? (prefix & 0x7fffffffu) : ~prefix;
  float f;
  std::memcpy(&f, &u, sizeof(f));
  *out = f;
  return RDL_OK;
}

}  // namespace rdl

extern "C" int rdl_median(rdl_session* s, const float* d_values, size_t n,
                          int use_center, float center, float* out) {
  RDL_ARG_CHECK(s && d_values && out, "NULL argument");
  if (n == 0) {
    *out = std::nanf("");
    return RDL_OK;
  }
  if (n % 2 == 1) return rdl::SelectKth(s, d_values, n, use_center, center, n / 2, out);
  float lo, hi;
  RDL_TRY(rdl::SelectKth(s, d_values, n, use_center, center, n / 2 - 1, &lo));
  RDL_TRY(rdl::SelectKth(s, d_values, n, use_center, center, n / 2, &hi));
  *out = 0.5f * (lo + hi);
  return RDL_OK;
}

/* k-th smallest of values (or of |values - center|), exact
 * (std::nth_element at k; IuwtDeconvolutionAlgorithm::Mad selects k = n/2). */
extern "C" int rdl_select_kth(rdl_session* s, const float* d_values, size_t n,
                              int use_center, float center, size_t k, float* out) {
  RDL_ARG_CHECK(s && d_values && out, "NULL argument");
  RDL_ARG_CHECK(k < n, "k out of range");
  return rdl::SelectKth(s, d_values, n, use_center, center, k, out);
}
