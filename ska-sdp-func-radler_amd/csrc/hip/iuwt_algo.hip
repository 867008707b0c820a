// Device pieces of IuwtDeconvolutionAlgorithm
// (cpp/algorithms/iuwt_deconvolution_algorithm.cc) that are not the IUWT
// transform itself (iuwt.hip) or a convolution (lds_fft.hip / fftconv.hip):
// the structure selection and masking, GetMaxAbs, the conjugate-gradient dot
// products and SNR sums, the bounding-box scan and precision conversions.
// All are single streaming passes (HBM-bound, 4-8 B/px); reductions
// accumulate in double.
#include <cfloat>

#include "rdl_internal.h"

namespace rdl {

namespace {
unsigned Grid256(size_t n) {
  return unsigned(std::max<size_t>(1, std::min<size_t>(4096, (n + 255) / 256)));
}
}  // namespace

// ---- GetMaxAbs: strict '>' from numeric_limits<float>::lowest(), first
// index on ties (iuwt_deconvolution_algorithm.cc:112-167). Key: monotonic
// image of the float order in the high word (0 = does not qualify), ~index
// in the low word.
__device__ __forceinline__ uint64_t MaxAbsKey(float v, bool allow_negative,
                                              uint32_t index) {
  if (allow_negative) v = fabsf(v);
  if (!(v > -FLT_MAX)) return 0ull;  // NaN, -inf and lowest() itself
  uint32_t u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return (uint64_t(u) << 32) | uint64_t(0xffffffffu - index);
}

struct MaxAbsArgs {
  const float* data;
  const uint8_t* mask;
  uint32_t width, xs, xe, ys, ye;
  int allow_negative;
};

__global__ __launch_bounds__(256) void MaxAbsPartial(MaxAbsArgs a, uint64_t* partials) {
  __shared__ uint64_t lds[16];
  uint64_t best = 0;
  const uint32_t bw = a.xe - a.xs;
  const uint64_t total = uint64_t(bw) * (a.ye - a.ys);
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < total;
       i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t y = a.ys + uint32_t(i / bw), x = a.xs + uint32_t(i % bw);
    const size_t idx = size_t(y) * a.width + x;
    if (a.mask && !a.mask[idx]) continue;
    const uint64_t k = MaxAbsKey(a.data[idx], a.allow_negative != 0, uint32_t(idx));
    best = k > best ? k : best;
  }
  best = BlockMaxU64(best, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = best;
}

__global__ __launch_bounds__(1024) void MaxAbsFinal(const uint64_t* partials, uint32_t n,
                                                    const float* data, uint32_t width,
                                                    uint32_t height, int allow_negative,
                                                    float* out_value, uint32_t* out_xy) {
  __shared__ uint64_t lds[16];
  uint64_t best = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    best = partials[i] > best ? partials[i] : best;
  best = BlockMaxU64(best, lds);
  if (threadIdx.x == 0) {
    if (best == 0) {
      *out_value = -FLT_MAX;
      out_xy[0] = width;
      out_xy[1] = height;
    } else {
      const uint32_t idx = 0xffffffffu - uint32_t(best & 0xffffffffu);
      const float v = data[idx];
      *out_value = allow_negative ? fabsf(v) : v;
      out_xy[0] = idx % width;
      out_xy[1] = idx / width;
    }
  }
}

// ---- SelectStructures result and ApplyMask (image_analysis.cc:9-15,
// 227-259; iuwt_decomposition.h:284-291)
__device__ __forceinline__ bool ExceedsThreshold(float v, float t) {
  return t >= 0.0f ? v > t : (v < t || v > -t);
}

struct SelectArgs {
  const float* coeffs;
  const uint8_t* prior;
  uint8_t* mask;
  uint32_t width, height, min_scale, end_scale, xs, xe, ys, ye;
  float thr[32];
};

__global__ __launch_bounds__(256) void IuwtSelectKernel(SelectArgs a,
                                                        unsigned long long* area) {
  const size_t plane = size_t(a.width) * a.height;
  const size_t total = plane * a.end_scale;
  uint32_t count = 0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t s = uint32_t(i / plane);
    const size_t p = i - size_t(s) * plane;
    const uint32_t y = uint32_t(p / a.width), x = uint32_t(p - size_t(y) * a.width);
    const bool in = s >= a.min_scale && x >= a.xs && x < a.xe && y >= a.ys && y < a.ye &&
                    (a.prior == nullptr || a.prior[p] != 0) &&
                    ExceedsThreshold(a.coeffs[i], a.thr[s]);
    a.mask[i] = in ? 1 : 0;
    count += in ? 1u : 0u;
  }
  // wave sum, one atomic per wave
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) count += __shfl_xor(count, off, 64);
  if ((threadIdx.x & 63) == 0 && count) atomicAdd(area, (unsigned long long)count);
}

__global__ __launch_bounds__(256) void IuwtApplyMaskKernel(float* coeffs, const uint8_t* mask,
                                                           size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    if (!mask[i]) coeffs[i] = 0.0f;
}

// ---- dot products / SNR sums in double
template <int K>
__global__ __launch_bounds__(256) void SumsPartial(const float* a, const float* b, size_t n,
                                                   int mode, double* partials) {
  __shared__ double lds[4][K];
  double acc[K] = {};
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const double x = a[i], y = b[i];
    if (mode == 0) {
      acc[0] += x * y;  // dot
    } else {           // SNR: sum m^2, sum (m - n)^2 (a = noisy, b = model)
      acc[0] += y * y;
      const double d = double(b[i] - a[i]);
      acc[K - 1] += d * d;
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[k] += __shfl_xor(acc[k], off, 64);
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < K; ++k) lds[threadIdx.x >> 6][k] = acc[k];
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 0; k < K; ++k) {
      double s = 0.0;
      for (unsigned w = 0; w < blockDim.x / 64; ++w) s += lds[w][k];
      partials[blockIdx.x * K + k] = s;
    }
}

__global__ void SumsFinal(const double* partials, uint32_t n_blocks, int k, double* out) {
  if (threadIdx.x < uint32_t(k)) {
    double s = 0.0;
    for (uint32_t b = 0; b < n_blocks; ++b) s += partials[b * k + threadIdx.x];
    out[threadIdx.x] = s;
  }
}

// ---- BoundingBox (iuwt_deconvolution_algorithm.cc:180-214): max |v| of the
// image, then per row the first and last x with |v| > m * 0.01 (double
// compare, like the reference)
__global__ __launch_bounds__(256) void AbsMaxPartial(const float* v, size_t n,
                                                     float* partials) {
  __shared__ float lds[4];
  float m = 0.0f;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    m = fmaxf(m, fabsf(v[i]));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (unsigned w = 1; w < blockDim.x / 64; ++w) m = fmaxf(m, lds[w]);
    partials[blockIdx.x] = m;
  }
}

__global__ __launch_bounds__(256) void BBoxRows(const float* v, uint32_t width,
                                                const float* partials, uint32_t n_partials,
                                                int32_t* first, int32_t* last) {
  __shared__ int lo, hi;
  float m = 0.0f;
  for (uint32_t i = 0; i < n_partials; ++i) m = fmaxf(m, partials[i]);
  const double thr = double(m) * 0.01;
  if (threadIdx.x == 0) {
    lo = int(width);
    hi = -1;
  }
  __syncthreads();
  const float* row = v + size_t(blockIdx.x) * width;
  int my_lo = int(width), my_hi = -1;
  for (uint32_t x = threadIdx.x; x < width; x += blockDim.x)
    if (double(fabsf(row[x])) > thr) {
      my_lo = min(my_lo, int(x));
      my_hi = max(my_hi, int(x));
    }
  if (my_hi >= 0) {
    atomicMin(&lo, my_lo);
    atomicMax(&hi, my_hi);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    first[blockIdx.x] = hi >= 0 ? lo : -1;
    last[blockIdx.x] = hi;
  }
}

__global__ __launch_bounds__(256) void ConvertKernel(const void* src, void* dst, size_t n,
                                                     int to_f64) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    if (to_f64)
      static_cast<double*>(dst)[i] = double(static_cast<const float*>(src)[i]);
    else
      static_cast<float*>(dst)[i] = float(static_cast<const double*>(src)[i]);
  }
}

}  // namespace rdl

extern "C" {

int rdl_max_abs(rdl_session* s, const float* d_data, uint32_t width, uint32_t height,
                uint32_t x_border, uint32_t y_border, int allow_negative,
                const uint8_t* d_mask, rdl_peak* out) {
  RDL_ARG_CHECK(s && d_data && out, "NULL argument");
  RDL_ARG_CHECK(2ull * x_border <= width && 2ull * y_border <= height, "border too wide");
  rdl::MaxAbsArgs a{d_data, d_mask, width, x_border, width - x_border, y_border,
                    height - y_border, allow_negative};
  const size_t total = size_t(a.xe - a.xs) * (a.ye - a.ys);
  const uint32_t blocks = uint32_t(std::max<size_t>(1, std::min<size_t>(1024, rdl::DivUp(total, 256))));
  RDL_TRY(s->EnsureScratch(s->partials, blocks * sizeof(uint64_t)));
  uint64_t* partials = static_cast<uint64_t*>(s->partials.ptr);
  float* d_val = static_cast<float*>(s->d_small);
  uint32_t* d_xy = reinterpret_cast<uint32_t*>(static_cast<char*>(s->d_small) + 16);
  {
    rdl::ScopedTiming t(s, "find_peak", double(total) * (d_mask ? 5.0 : 4.0));
    rdl::MaxAbsPartial<<<blocks, 256, 0, s->stream>>>(a, partials);
    rdl::MaxAbsFinal<<<1, 1024, 0, s->stream>>>(partials, blocks, d_data, width, height,
                                                allow_negative, d_val, d_xy);
  }
  RDL_HIP_CHECK(hipGetLastError());
  float v = 0.0f;
  uint32_t xy[2] = {0, 0};
  const rdl::SmallRead r[2] = {{&v, d_val, sizeof(v)}, {xy, d_xy, sizeof(xy)}};
  RDL_TRY(rdl::ReadSmall(s, r, 2));
  out->value = v;
  out->x = xy[0];
  out->y = xy[1];
  out->found = xy[0] < width ? 1 : 0;
  return RDL_OK;
}

int rdl_iuwt_select(rdl_session* s, const float* d_coeffs, uint32_t width, uint32_t height,
                    uint32_t min_scale, uint32_t end_scale, const float* h_thresholds,
                    uint32_t x_border, uint32_t y_border, const uint8_t* d_prior,
                    uint8_t* d_mask, uint64_t* area) {
  RDL_ARG_CHECK(s && d_coeffs && h_thresholds && d_mask, "NULL argument");
  RDL_ARG_CHECK(end_scale >= 1 && end_scale <= 32 && min_scale <= end_scale,
                "scale range must satisfy min <= end <= 32");
  RDL_ARG_CHECK(2ull * x_border <= width && 2ull * y_border <= height, "border too wide");
  rdl::SelectArgs a{};
  a.coeffs = d_coeffs;
  a.prior = d_prior;
  a.mask = d_mask;
  a.width = width;
  a.height = height;
  a.min_scale = min_scale;
  a.end_scale = end_scale;
  a.xs = x_border;
  a.xe = width - x_border;
  a.ys = y_border;
  a.ye = height - y_border;
  for (uint32_t i = 0; i < end_scale; ++i) a.thr[i] = h_thresholds[i];
  const size_t total = size_t(width) * height * end_scale;
  unsigned long long* d_area = static_cast<unsigned long long*>(s->d_small);
  RDL_HIP_CHECK(hipMemsetAsync(d_area, 0, sizeof(*d_area), s->stream));
  {
    rdl::ScopedTiming t(s, "iuwt", double(total) * 5.0);
    rdl::IuwtSelectKernel<<<rdl::Grid256(total), 256, 0, s->stream>>>(a, d_area);
  }
  RDL_HIP_CHECK(hipGetLastError());
  unsigned long long n = 0;
  const rdl::SmallRead r{&n, d_area, sizeof(n)};
  RDL_TRY(rdl::ReadSmall(s, &r, 1));
  if (area) *area = n;
  return RDL_OK;
}

int rdl_iuwt_apply_mask(rdl_session* s, float* d_coeffs, const uint8_t* d_mask,
                        uint32_t width, uint32_t height, uint32_t n_scales) {
  RDL_ARG_CHECK(s && d_coeffs && d_mask, "NULL argument");
  const size_t n = size_t(width) * height * n_scales;
  if (n == 0) return RDL_OK;
  {
    rdl::ScopedTiming t(s, "iuwt", double(n) * 9.0);
    rdl::IuwtApplyMaskKernel<<<rdl::Grid256(n), 256, 0, s->stream>>>(d_coeffs, d_mask, n);
  }
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

static int Sums(rdl_session* s, const float* a, const float* b, size_t n, int mode,
                double* out) {
  RDL_ARG_CHECK(s && a && b && out, "NULL argument");
  const int k = mode == 0 ? 1 : 2;
  if (n == 0) {
    for (int i = 0; i < k; ++i) out[i] = 0.0;
    return RDL_OK;
  }
  const uint32_t blocks = std::min<uint32_t>(1024, rdl::DivUp(n, 256));
  RDL_TRY(s->EnsureScratch(s->partials, size_t(blocks) * k * sizeof(double)));
  double* partials = static_cast<double*>(s->partials.ptr);
  double* d_out = static_cast<double*>(s->d_small);
  {
    rdl::ScopedTiming t(s, "dot", double(n) * 8.0);
    if (k == 1)
      rdl::SumsPartial<1><<<blocks, 256, 0, s->stream>>>(a, b, n, mode, partials);
    else
      rdl::SumsPartial<2><<<blocks, 256, 0, s->stream>>>(a, b, n, mode, partials);
    rdl::SumsFinal<<<1, 64, 0, s->stream>>>(partials, blocks, k, d_out);
  }
  RDL_HIP_CHECK(hipGetLastError());
  const rdl::SmallRead r{out, d_out, sizeof(double) * k};
  return rdl::ReadSmall(s, &r, 1);
}

int rdl_dot(rdl_session* s, const float* d_a, const float* d_b, size_t n, double* out) {
  return Sums(s, d_a, d_b, n, 0, out);
}

int rdl_iuwt_snr_sums(rdl_session* s, const float* d_noisy, const float* d_model, size_t n,
                      double* model_sum, double* noise_sum) {
  RDL_ARG_CHECK(model_sum && noise_sum, "NULL argument");
  double out[2];
  RDL_TRY(Sums(s, d_noisy, d_model, n, 1, out));
  *model_sum = out[0];
  *noise_sum = out[1];
  return RDL_OK;
}

int rdl_bbox_rows(rdl_session* s, const float* d_image, uint32_t width, uint32_t height,
                  int32_t* h_first, int32_t* h_last) {
  RDL_ARG_CHECK(s && d_image && h_first && h_last, "NULL argument");
  const size_t n = size_t(width) * height;
  const uint32_t blocks = std::min<uint32_t>(1024, rdl::DivUp(n, 256));
  const size_t rows_bytes = size_t(height) * sizeof(int32_t);
  RDL_TRY(s->EnsureScratch(s->partials, blocks * sizeof(float) + 2 * rows_bytes + 64));
  char* base = static_cast<char*>(s->partials.ptr);
  float* partials = reinterpret_cast<float*>(base);
  int32_t* d_first = reinterpret_cast<int32_t*>(base + (blocks * sizeof(float) + 15) / 16 * 16);
  int32_t* d_last = d_first + height;
  {
    rdl::ScopedTiming t(s, "iuwt", double(n) * 8.0);
    rdl::AbsMaxPartial<<<blocks, 256, 0, s->stream>>>(d_image, n, partials);
    rdl::BBoxRows<<<height, 256, 0, s->stream>>>(d_image, width, partials, blocks, d_first,
                                                 d_last);
  }
  RDL_HIP_CHECK(hipGetLastError());
  RDL_HIP_CHECK(hipMemcpyAsync(h_first, d_first, rows_bytes, hipMemcpyDeviceToHost, s->stream));
  RDL_HIP_CHECK(hipMemcpyAsync(h_last, d_last, rows_bytes, hipMemcpyDeviceToHost, s->stream));
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

int rdl_convert(rdl_session* s, const void* d_src, void* d_dst, size_t n, int to_f64) {
  RDL_ARG_CHECK(s && d_src && d_dst, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ConvertKernel<<<rdl::Grid256(n), 256, 0, s->stream>>>(d_src, d_dst, n, to_f64);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // extern "C"
