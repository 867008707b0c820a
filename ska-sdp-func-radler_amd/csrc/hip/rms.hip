// Local-RMS images: radler::math::rms_image
// (cpp/math/rms_image.cc:16-125) on the device. The Gaussian window
// convolution runs through the FFT engine (host: csrc/host/rms_image.cc);
// these are the streaming steps around it — squaring, the placed Gaussian
// kernel, sqrt(x * norm), the separable sliding minimum (van Herk /
// Gil-Werman: three reads per pixel whatever the window), the negativity
// limit and the factor conversion — plus the elementwise product the peak
// searches use. All HBM-bound.
#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>

#include "rdl_internal.h"

namespace rdl {
namespace {

constexpr unsigned kThreads = 256;
inline unsigned Grid(size_t n) {
  return unsigned(std::min<size_t>((n + kThreads - 1) / kThreads, 8192));
}

__global__ __launch_bounds__(256) void SquareKernel(const float* src, float* dst,
                                                    size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    dst[i] = src[i] * src[i];
}

__global__ __launch_bounds__(256) void MultiplyKernel(float* dst, const float* a,
                                                      const float* b, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    dst[i] = a[i] * b[i];
}

__global__ __launch_bounds__(256) void FinishKernel(float* d, size_t n, double norm) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    d[i] = float(sqrt(double(d[i]) * norm));
}

// box x box Gaussian of peak 1 wrapped so its centre (box/2, box/2) sits at
// the origin of a w x h plane (PrepareSmallConvolutionKernel placement).
__global__ __launch_bounds__(256) void PlaceGaussianKernel(
    float* dest, uint32_t w, uint32_t h, uint32_t box, double pl, double pm,
    double c, double s, double inv_major, double inv_minor) {
  const size_t n = size_t(box) * box;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = uint32_t(i % box), y = uint32_t(i / box);
    const double l = double(int64_t(box / 2) - int64_t(x)) * pl;
    const double m = double(int64_t(y) - int64_t(box / 2)) * pm;
    const double lt = (l * c + m * s) * inv_major;
    const double mt = (-l * s + m * c) * inv_minor;
    const uint32_t px = (x + w - box / 2) % w, py = (y + h - box / 2) % h;
    dest[size_t(py) * w + px] = float(exp(-0.5 * (lt * lt + mt * mt)));
  }
}

// Prefix and suffix minima within blocks of L consecutive elements of each
// line (lines of `len` elements, `stride` apart between elements): thread
// (line, block) scans its block.
__global__ __launch_bounds__(256) void BlockScanKernel(const float* in, float* pre,
                                                       float* suf, uint32_t n_lines,
                                                       uint32_t len, size_t line_step,
                                                       size_t elem_step, uint32_t L) {
  const uint32_t n_blocks = (len + L - 1) / L;
  const size_t total = size_t(n_lines) * n_blocks;
  for (size_t t = blockIdx.x * size_t(blockDim.x) + threadIdx.x; t < total;
       t += size_t(gridDim.x) * blockDim.x) {
    // adjacent threads take adjacent lines (coalesced when lines are columns)
    const uint32_t line = uint32_t(t % n_lines), blk = uint32_t(t / n_lines);
    const uint32_t b0 = blk * L, b1 = min(len, b0 + L);
    const size_t base = size_t(line) * line_step;
    float acc = FLT_MAX;
    bool first = true;
    for (uint32_t k = b0; k < b1; ++k) {
      const float v = in[base + size_t(k) * elem_step];
      acc = first ? v : (v < acc ? v : acc);
      first = false;
      pre[base + size_t(k) * elem_step] = acc;
    }
    first = true;
    for (uint32_t k = b1; k-- > b0;) {
      const float v = in[base + size_t(k) * elem_step];
      acc = first ? v : (v < acc ? v : acc);
      first = false;
      suf[base + size_t(k) * elem_step] = acc;
    }
  }
}

// out[k] = min over [max(k, half) - half, min(k, len - half) + half) of the
// line (rms_image.cc:44-46), from the block scans with L = 2 * half.
__global__ __launch_bounds__(256) void WindowMinKernel(const float* pre, const float* suf,
                                                       float* out, uint32_t n_lines,
                                                       uint32_t len, size_t line_step,
                                                       size_t elem_step, uint32_t half) {
  const uint32_t L = 2 * half;
  const size_t total = size_t(n_lines) * len;
  for (size_t t = blockIdx.x * size_t(blockDim.x) + threadIdx.x; t < total;
       t += size_t(gridDim.x) * blockDim.x) {
    uint32_t line, k;
    if (elem_step == 1) {
      line = uint32_t(t / len);
      k = uint32_t(t % len);
    } else {
      line = uint32_t(t % n_lines);
      k = uint32_t(t / n_lines);
    }
    const uint32_t a = max(k, half) - half;
    const uint32_t e = min(k, len - half) + half;  // exclusive
    const size_t base = size_t(line) * line_step;
    const float x = suf[base + size_t(a) * elem_step];
    const float y = pre[base + size_t(e - 1) * elem_step];
    float r;
    if (a / L != (e - 1) / L)
      r = y < x ? y : x;  // two blocks: suffix of the first, prefix of the second
    else
      r = (a % L == 0) ? y : x;  // one block: the window starts it or ends it
    out[base + size_t(k) * elem_step] = r;
  }
}

__global__ __launch_bounds__(256) void NegativityLimitKernel(float* rms, const float* mn,
                                                             size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const float lim = float(double(fabsf(mn[i])) * (1.5 / 5.0));
    rms[i] = rms[i] < lim ? lim : rms[i];  // std::max<float>(rms, lim)
  }
}

__device__ __forceinline__ uint32_t OrderedBits(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void MinKernel(const float* d, size_t n,
                                                 uint32_t* out) {
  uint32_t best = 0xffffffffu;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const float v = d[i];
    if (v == v) best = min(best, OrderedBits(v));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) best = min(best, uint32_t(__shfl_xor(int(best), off, 64)));
  if ((threadIdx.x & 63) == 0) atomicMin(out, best);
}

__global__ __launch_bounds__(256) void FactorKernel(float* d, size_t n, double stddev,
                                                    double strength) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const float v = d[i];
    if (strength == 0.0)
      d[i] = 1.0f;
    else if (v != 0.0f)
      d[i] = strength == 1.0 ? float(stddev / double(v))
                             : float(pow(stddev / double(v), strength));
  }
}

}  // namespace
}  // namespace rdl

extern "C" {

int rdl_square(rdl_session* s, const float* d_src, float* d_dst, size_t n) {
  RDL_ARG_CHECK(s && d_src && d_dst, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "rms_elementwise", 8.0 * double(n));
  rdl::SquareKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_src, d_dst, n);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_multiply(rdl_session* s, float* d_dst, const float* d_a, const float* d_b,
                 size_t n) {
  RDL_ARG_CHECK(s && d_dst && d_a && d_b, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "rms_elementwise", 12.0 * double(n));
  rdl::MultiplyKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_dst, d_a, d_b, n);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_rms_finish(rdl_session* s, float* d, size_t n, double norm) {
  RDL_ARG_CHECK(s && d, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "rms_elementwise", 8.0 * double(n));
  rdl::FinishKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d, n, norm);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_place_gaussian(rdl_session* s, float* d_dest, uint32_t width, uint32_t height,
                       uint32_t box, double pixel_scale_l, double pixel_scale_m,
                       double sigma_major, double sigma_minor, double angle) {
  RDL_ARG_CHECK(s && d_dest, "NULL argument");
  RDL_ARG_CHECK(box >= 1 && box <= width && box <= height, "box larger than the plane");
  RDL_ARG_CHECK(sigma_major > 0.0 && sigma_minor > 0.0, "sigma must be positive");
  RDL_HIP_CHECK(hipMemsetAsync(d_dest, 0, size_t(width) * height * sizeof(float),
                               s->stream));
  const size_t n = size_t(box) * box;
  rdl::PlaceGaussianKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(
      d_dest, width, height, box, pixel_scale_l, pixel_scale_m, std::cos(angle),
      std::sin(angle), 1.0 / sigma_major, 1.0 / sigma_minor);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_sliding_min(rdl_session* s, const float* d_in, float* d_out, float* d_scratch,
                    uint32_t width, uint32_t height, uint64_t window) {
  RDL_ARG_CHECK(s && d_in && d_out && d_scratch, "NULL argument");
  RDL_ARG_CHECK(d_out != d_in, "output must not alias the input");
  const uint32_t half = uint32_t(std::min<uint64_t>(window / 2, 0xffffffffu));
  RDL_ARG_CHECK(half >= 1, "window must be at least 2 pixels");
  RDL_ARG_CHECK(half <= width && half <= height, "window larger than the image");
  const size_t n = size_t(width) * height;
  float* tmp = d_scratch;            // the row pass' result
  float* pre = d_scratch + n;
  float* suf = d_scratch + 2 * n;
  const uint32_t L = 2 * half;
  rdl::ScopedTiming t(s, "sliding_min", 28.0 * double(n));
  // rows (rms_image.cc:40-50)
  {
    const size_t lines = height, blocks = (width + L - 1) / L;
    rdl::BlockScanKernel<<<rdl::Grid(lines * blocks), rdl::kThreads, 0, s->stream>>>(
        d_in, pre, suf, height, width, width, 1, L);
    rdl::WindowMinKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(
        pre, suf, tmp, height, width, width, 1, half);
  }
  // columns (:52-66)
  {
    const size_t blocks = (height + L - 1) / L;
    rdl::BlockScanKernel<<<rdl::Grid(size_t(width) * blocks), rdl::kThreads, 0,
                           s->stream>>>(tmp, pre, suf, width, height, 1, width, L);
    rdl::WindowMinKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(
        pre, suf, d_out, width, height, 1, width, half);
  }
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_rms_negativity_limit(rdl_session* s, float* d_rms, const float* d_min, size_t n) {
  RDL_ARG_CHECK(s && d_rms && d_min, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "rms_elementwise", 12.0 * double(n));
  rdl::NegativityLimitKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_rms, d_min,
                                                                            n);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_rms_factor(rdl_session* s, float* d_rms, size_t n, double strength,
                   double* lowest_rms) {
  RDL_ARG_CHECK(s && d_rms && lowest_rms && n > 0, "bad argument");
  RDL_TRY(s->EnsureScratch(s->partials, 256));
  uint32_t* d_min = static_cast<uint32_t*>(s->partials.ptr);
  RDL_HIP_CHECK(hipMemsetAsync(d_min, 0xff, sizeof(uint32_t), s->stream));
  rdl::MinKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_rms, n, d_min);
  RDL_HIP_CHECK(hipGetLastError());
  uint32_t key = 0;
  {
    const rdl::SmallRead r{&key, d_min, sizeof(key)};
    RDL_TRY(rdl::ReadSmall(s, &r, 1));
  }
  const uint32_t u = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
  float mn;
  std::memcpy(&mn, &u, sizeof(mn));
  if (key == 0xffffffffu) mn = std::numeric_limits<float>::quiet_NaN();
  *lowest_rms = double(mn);
  if (mn < 0.0f) {
    rdl::SetError("RMS image can only contain values >= 0, but contains values < 0.0");
    return RDL_ERR_ARG;
  }
  rdl::ScopedTiming t(s, "rms_elementwise", 8.0 * double(n));
  rdl::FactorKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_rms, n, double(mn),
                                                                   strength);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // extern "C"
