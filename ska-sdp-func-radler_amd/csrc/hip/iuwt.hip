// IUWT à-trous B3-spline decomposition and recomposition (IuwtDecomposition,
// cpp/algorithms/iuwt/iuwt_decomposition.cc:9-237, .h:94-146, 243-261).
//
// Separable 5-tap filter h = (1, 4, 6, 4, 1)/16 with spacing d = 2^(s+1)-1 and
// zero boundaries. Each output pixel is computed by one thread with the
// reference's tap order per boundary region and its FMA contraction
// (t0 + t1 + ... -> fma(x_k, h_k, ... fma(x_0, h_0, x_1*h_1)); see
// oracle/iuwt.cc), so results are bit-identical to the reference build.
// Decompose(x, x, ..) — input used as its own scratch, as the reference's IUWT
// deconvolution does — makes the first horizontal pass a recursive in-place row
// filter; that case runs one thread per row, left to right.
#include "rdl_internal.h"

namespace rdl {

__device__ __forceinline__ float IuwtTap(int k) {
  return k == 2 ? 6.0f / 16.0f : (k == 1 || k == 3) ? 4.0f / 16.0f : 1.0f / 16.0f;
}

// taps in `order` (first two: x[o0]*h + x[o1]*h contracted as fma(x0, h0, x1*h1))
template <int N>
__device__ __forceinline__ float TapSum(const float* t, const int (&order)[N]) {
  float acc = t[order[1]] * IuwtTap(order[1]);
  acc = __builtin_fmaf(t[order[0]], IuwtTap(order[0]), acc);
#pragma unroll
  for (int i = 2; i < N; ++i) acc = __builtin_fmaf(t[order[i]], IuwtTap(order[i]), acc);
  return acc;
}

// convolveHorizontalFast regions (iuwt_decomposition.cc:84-131)
__device__ __forceinline__ float HorizontalValue(const float* t, int64_t x,
                                                 int64_t w, int d) {
  if (x < d) return TapSum<3>(t, {2, 3, 4});
  if (x < 2 * d) return TapSum<4>(t, {2, 1, 3, 4});
  if (x < w - 2 * d) return TapSum<5>(t, {2, 1, 0, 3, 4});
  if (x < w - d) return TapSum<4>(t, {2, 1, 0, 3});
  return TapSum<3>(t, {2, 1, 0});
}

// convolveVerticalPartialFast regions (iuwt_decomposition.cc:172-235)
__device__ __forceinline__ float VerticalValue(const float* t, int64_t y,
                                               int64_t h, int d) {
  if (y < d) return TapSum<3>(t, {2, 3, 4});
  if (y < 2 * d) return TapSum<4>(t, {1, 2, 3, 4});
  if (y < h - 2 * d) return TapSum<5>(t, {0, 1, 2, 3, 4});
  if (y < h - d) return TapSum<4>(t, {0, 1, 2, 3});
  return TapSum<3>(t, {0, 1, 2});
}

// The dispatcher deals workgroups round-robin over the 8 XCDs; a workgroup's
// row comes from its XCD's contiguous band of rows, so the vertical taps
// (rows y +- d, y +- 2d) another workgroup of the same XCD read moments
// earlier are still in that XCD's L2.
__device__ __forceinline__ int64_t XcdBandRow(uint32_t block, uint32_t h) {
  const uint32_t band = (h + 7u) / 8u;
  return int64_t((block % 8u) * band + block / 8u);
}
inline unsigned XcdBandBlocks(uint32_t h) { return 8u * ((h + 7u) / 8u); }

__global__ __launch_bounds__(256) void IuwtHorizontalKernel(float* out,
                                                            const float* in,
                                                            uint32_t w, uint32_t h,
                                                            int d) {
  const size_t n = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const int64_t x = int64_t(i % w);
    const float* row = in + (i - size_t(x));
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = x + int64_t(d) * (k - 2);
      t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
    }
    out[i] = HorizontalValue(t, x, int64_t(w), d);
  }
}

// in-place (aliased) variant: one thread per row, left to right
__global__ __launch_bounds__(64) void IuwtHorizontalInPlaceKernel(float* data,
                                                                  uint32_t w,
                                                                  uint32_t h, int d) {
  const uint32_t y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= h) return;
  float* row = data + size_t(y) * w;
  for (int64_t x = 0; x < int64_t(w); ++x) {
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = x + int64_t(d) * (k - 2);
      t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
    }
    row[x] = HorizontalValue(t, x, int64_t(w), d);
  }
}

// out = V(in), or with lhs: out = lhs - V(in) (differenceMT fused)
__global__ __launch_bounds__(256) void IuwtVerticalKernel(float* out,
                                                          const float* in,
                                                          const float* lhs,
                                                          uint32_t w, uint32_t h,
                                                          int d) {
  // one row per workgroup, rows in XCD bands (XcdBandRow)
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  for (uint32_t x = threadIdx.x; x < w; x += blockDim.x) {
    const size_t i = size_t(y) * w + x;
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      t[k] = (yy >= 0 && yy < int64_t(h)) ? in[size_t(yy) * w + x] : 0.0f;
    }
    const float v = VerticalValue(t, y, int64_t(h), d);
    out[i] = lhs ? lhs[i] - v : v;
  }
}

// IuwtDecomposition::convolve (.h:243-261) per pixel: accumulators start at 0
// and take the taps h0..h4 in order where in range, each as fma(x, h, acc)
__global__ __launch_bounds__(256) void IuwtAccumulateH(float* out, const float* in,
                                                       uint32_t w, uint32_t h,
                                                       int d) {
  const size_t n = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const int64_t x = int64_t(i % w);
    const float* row = in + (i - size_t(x));
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = x + int64_t(d) * (k - 2);
      if (xx >= 0 && xx < int64_t(w)) acc = __builtin_fmaf(row[xx], IuwtTap(k), acc);
    }
    out[i] = acc;
  }
}

// vertical accumulate, then + coefficients (Recompose, .h:138-142)
__global__ __launch_bounds__(256) void IuwtAccumulateVAdd(float* out,
                                                          const float* in,
                                                          const float* add,
                                                          uint32_t w, uint32_t h,
                                                          int d) {
  // one row per workgroup, rows in XCD bands (XcdBandRow)
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  for (uint32_t x = threadIdx.x; x < w; x += blockDim.x) {
    const size_t i = size_t(y) * w + x;
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      if (yy >= 0 && yy < int64_t(h))
        acc = __builtin_fmaf(in[size_t(yy) * w + x], IuwtTap(k), acc);
    }
    out[i] = acc + add[i];
  }
}

// ---- fused row kernels (r06). Each block owns image rows; a row of the
// intermediate lives in LDS between the vertical and horizontal filters, so
// the intermediates of the four passes per scale do not all reach HBM. Every
// value is computed by the same per-pixel operations as the kernels above
// (VerticalValue / HorizontalValue / the Recompose accumulations), so the
// outputs are bit-identical.
//
// DecomposeRows (one scale, spacing d; DecomposeMt's i1 = V(H(a)) and the
// scratch = H(i1) of iuwt_decomposition.cc:9-54): row y of i1 = V_d(s1) from
// rows y + k d of s1 = H_d(a), kept in LDS, then s2 = H_d(i1) for this
// scale's difference pass and, when d_next > 0, s1' = H_d_next(i1), the
// next scale's first pass (a_{s+1} = i1).
__global__ __launch_bounds__(256) void IuwtDecomposeRows(float* __restrict__ i1,
                                                         float* __restrict__ s2,
                                                         float* __restrict__ s1_next,
                                                         const float* __restrict__ s1,
                                                         uint32_t w, uint32_t h, int d,
                                                         int d_next) {
  extern __shared__ float row[];
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  // the vertical filter four pixels (one float4 per tap row) at a time, all
  // five tap rows' loads issued before the sums (w % 4 == 0: the launcher)
  const float4* s1v = reinterpret_cast<const float4*>(s1);
  float4* i1v = reinterpret_cast<float4*>(i1);
  const uint32_t w4 = w / 4;
  // (restrict pointers and unrolling: every tap row's load of the next
  // float4s issues before this one's sums and stores)
#pragma unroll 4
  for (uint32_t x4 = threadIdx.x; x4 < w4; x4 += blockDim.x) {
    float4 t4[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      t4[k] = (yy >= 0 && yy < int64_t(h)) ? s1v[size_t(yy) * w4 + x4]
                                            : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    float4 v;
    {
      float t[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].x;
      v.x = VerticalValue(t, y, int64_t(h), d);
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].y;
      v.y = VerticalValue(t, y, int64_t(h), d);
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].z;
      v.z = VerticalValue(t, y, int64_t(h), d);
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].w;
      v.w = VerticalValue(t, y, int64_t(h), d);
    }
    reinterpret_cast<float4*>(row)[x4] = v;
    i1v[size_t(y) * w4 + x4] = v;
  }
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < w; x += blockDim.x) {
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = int64_t(x) + int64_t(d) * (k - 2);
      t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
    }
    s2[size_t(y) * w + x] = HorizontalValue(t, x, int64_t(w), d);
    if (d_next > 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int64_t xx = int64_t(x) + int64_t(d_next) * (k - 2);
        t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
      }
      s1_next[size_t(y) * w + x] = HorizontalValue(t, x, int64_t(w), d_next);
    }
  }
}

// out = lhs - V_d(in), four pixels per thread (w % 4 == 0): the difference
// pass of the fused decomposition, one float4 per tap row in flight
__global__ __launch_bounds__(256) void IuwtVerticalDiff4(float* __restrict__ out,
                                                         const float* __restrict__ in,
                                                         const float* __restrict__ lhs,
                                                         uint32_t w, uint32_t h, int d) {
  // one row per workgroup, rows in XCD bands (XcdBandRow)
  const uint32_t w4 = w / 4;
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  const float4* inv = reinterpret_cast<const float4*>(in);
#pragma unroll 4
  for (uint32_t x4 = threadIdx.x; x4 < w4; x4 += blockDim.x) {
    const size_t i = size_t(y) * w4 + x4;
    float4 t4[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      t4[k] = (yy >= 0 && yy < int64_t(h)) ? inv[size_t(yy) * w4 + x4]
                                            : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    const float4 l = reinterpret_cast<const float4*>(lhs)[i];
    float t[5];
    float4 o;
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].x;
    o.x = l.x - VerticalValue(t, y, int64_t(h), d);
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].y;
    o.y = l.y - VerticalValue(t, y, int64_t(h), d);
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].z;
    o.z = l.z - VerticalValue(t, y, int64_t(h), d);
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].w;
    o.w = l.w - VerticalValue(t, y, int64_t(h), d);
    reinterpret_cast<float4*>(out)[i] = o;
  }
}

// RDL_IUWT_FUSED=0: the four-pass kernels for every call (comparison)
inline bool IuwtFusedOn() {
  const char* e = std::getenv("RDL_IUWT_FUSED");
  return !(e && e[0] == '0');
}
// rows of at most this many floats go through LDS (one row per block: 64 KiB
// at most)
constexpr uint32_t kIuwtFusedMaxWidth = 16384;

inline unsigned IuwtGrid(size_t n) {
  return unsigned(std::min<size_t>(16384, std::max<size_t>(1, (n + 255) / 256)));
}

int Horizontal(rdl_session* s, float* out, const float* in, uint32_t w, uint32_t h,
               int d) {
  ScopedTiming t(s, "iuwt", double(w) * h * 8.0);
  if (out == in) {
    IuwtHorizontalInPlaceKernel<<<DivUp(h, 64), 64, 0, s->stream>>>(out, w, h, d);
  } else {
    IuwtHorizontalKernel<<<IuwtGrid(size_t(w) * h), 256, 0, s->stream>>>(out, in, w,
                                                                          h, d);
  }
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int Vertical(rdl_session* s, float* out, const float* in, const float* lhs,
             uint32_t w, uint32_t h, int d) {
  ScopedTiming t(s, "iuwt", double(w) * h * (lhs ? 12.0 : 8.0));
  IuwtVerticalKernel<<<XcdBandBlocks(h), 256, 0, s->stream>>>(out, in, lhs, w, h, d);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // namespace rdl

extern "C" {

int rdl_iuwt_decompose(rdl_session* s, float* d_input, float* d_scratch,
                       uint32_t width, uint32_t height, uint32_t n_scales,
                       float* d_coeffs, int include_largest) {
  RDL_ARG_CHECK(s && d_input && d_scratch && d_coeffs, "NULL argument");
  RDL_ARG_CHECK(n_scales >= 1 && n_scales <= 24, "n_scales out of range");
  RDL_ARG_CHECK(width >= 1 && height >= 1, "bad size");
  // DecomposeMt (iuwt_decomposition.cc:9-54)
  const size_t n = size_t(width) * height;
  if (d_input != d_scratch && width <= rdl::kIuwtFusedMaxWidth && width % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(d_input) | reinterpret_cast<uintptr_t>(d_coeffs)) % 16 == 0 &&
      rdl::IuwtFusedOn()) {
    // fused: per scale one row kernel (i1, s2 = H(i1), next scale's H(i1))
    // and the difference pass; the approximation planes alternate between
    // the largest-scale plane and a scratch plane (no copy), arranged so the
    // last one lands in the largest-scale plane as the four-pass form leaves
    // it. The caller's scratch is not written (not aliased: nothing reads it).
    RDL_TRY(s->EnsureScratch(s->iuwt, 4 * n * sizeof(float)));
    float* big = d_coeffs + size_t(n_scales) * n;
    float* spare = static_cast<float*>(s->iuwt.ptr);
    float* s1[2] = {spare + n, spare + 2 * n};
    float* s2 = spare + 3 * n;
    RDL_TRY(rdl::Horizontal(s, s1[0], d_input, width, height, 1));
    const float* a = d_input;
    for (uint32_t sc = 0; sc < n_scales; ++sc) {
      const int d = (1 << (sc + 1)) - 1;
      const int d_next = sc + 1 < n_scales ? (1 << (sc + 2)) - 1 : 0;
      float* i1 = ((n_scales - 1 - sc) % 2 == 0) ? big : spare;
      {
        rdl::ScopedTiming t(s, "iuwt", double(n) * (d_next ? 16.0 : 12.0));
        rdl::IuwtDecomposeRows<<<rdl::XcdBandBlocks(height), 256, width * sizeof(float),
                                 s->stream>>>(
            i1, s2, s1[(sc + 1) & 1u], s1[sc & 1u], width, height, d, d_next);
        RDL_HIP_CHECK(hipGetLastError());
      }
      {
        rdl::ScopedTiming t(s, "iuwt", double(n) * 12.0);
        rdl::IuwtVerticalDiff4<<<rdl::XcdBandBlocks(height), 256, 0, s->stream>>>(
            d_coeffs + size_t(sc) * n, s2, a, width, height, d);
        RDL_HIP_CHECK(hipGetLastError());
      }
      a = i1;
    }
    if (!include_largest)
      RDL_HIP_CHECK(hipMemsetAsync(big, 0, n * sizeof(float), s->stream));
    return RDL_OK;
  }
  RDL_TRY(s->EnsureScratch(s->iuwt, n * sizeof(float)));
  float* i0 = static_cast<float*>(s->iuwt.ptr);
  float* i1 = d_coeffs + size_t(n_scales) * n;  // the largest scale aliases i1
  RDL_TRY(rdl::Horizontal(s, d_scratch, d_input, width, height, 1));
  RDL_TRY(rdl::Vertical(s, i1, d_scratch, nullptr, width, height, 1));
  RDL_TRY(rdl::Horizontal(s, d_scratch, i1, width, height, 1));
  // coefficients0 = input - V(...); `input` has become the scratch when aliased
  RDL_TRY(rdl::Vertical(s, d_coeffs, d_scratch, d_input, width, height, 1));
  RDL_HIP_CHECK(hipMemcpyAsync(i0, i1, n * sizeof(float), hipMemcpyDeviceToDevice,
                               s->stream));
  for (uint32_t sc = 1; sc < n_scales; ++sc) {
    const int d = (1 << (sc + 1)) - 1;
    float* coef = d_coeffs + size_t(sc) * n;
    RDL_TRY(rdl::Horizontal(s, d_scratch, i0, width, height, d));
    RDL_TRY(rdl::Vertical(s, i1, d_scratch, nullptr, width, height, d));
    RDL_TRY(rdl::Horizontal(s, d_scratch, i1, width, height, d));
    RDL_TRY(rdl::Vertical(s, coef, d_scratch, i0, width, height, d));
    if (sc + 1 != n_scales)
      RDL_HIP_CHECK(hipMemcpyAsync(i0, i1, n * sizeof(float),
                                   hipMemcpyDeviceToDevice, s->stream));
  }
  if (!include_largest)
    RDL_HIP_CHECK(hipMemsetAsync(i1, 0, n * sizeof(float), s->stream));
  return RDL_OK;
}

int rdl_iuwt_recompose(rdl_session* s, const float* d_coeffs, uint32_t width,
                       uint32_t height, uint32_t n_scales, int include_largest,
                       float* d_out) {
  RDL_ARG_CHECK(s && d_coeffs && d_out, "NULL argument");
  RDL_ARG_CHECK(n_scales >= 1 && n_scales <= 24, "n_scales out of range");
  // Recompose (iuwt_decomposition.h:121-146)
  const size_t n = size_t(width) * height;
  RDL_TRY(s->EnsureScratch(s->iuwt, n * sizeof(float)));
  float* tmp = static_cast<float*>(s->iuwt.ptr);
  int sc = int(n_scales) - 1;
  if (include_largest) {
    RDL_HIP_CHECK(hipMemcpyAsync(d_out, d_coeffs + size_t(n_scales) * n,
                                 n * sizeof(float), hipMemcpyDeviceToDevice,
                                 s->stream));
  } else {
    RDL_HIP_CHECK(hipMemcpyAsync(d_out, d_coeffs + size_t(sc) * n, n * sizeof(float),
                                 hipMemcpyDeviceToDevice, s->stream));
    --sc;
  }
  for (; sc >= 0; --sc) {
    const int d = (1 << (sc + 1)) - 1;
    {
      rdl::ScopedTiming t(s, "iuwt", double(n) * 20.0);
      rdl::IuwtAccumulateH<<<rdl::IuwtGrid(n), 256, 0, s->stream>>>(tmp, d_out, width,
                                                                  height, d);
      rdl::IuwtAccumulateVAdd<<<rdl::XcdBandBlocks(height), 256, 0, s->stream>>>(
          d_out, tmp, d_coeffs + size_t(sc) * n, width, height, d);
    }
    RDL_HIP_CHECK(hipGetLastError());
  }
  return RDL_OK;
}

}  // extern "C"
