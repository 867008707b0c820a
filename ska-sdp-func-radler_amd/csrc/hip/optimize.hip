// Component optimisation: the streaming steps of
// math::GradientDescent (cpp/math/component_optimization.cc:100-177,
// 265-321) on whole planes. The component list is the model's non-zero
// pixels, so a plane that is zero off the components replaces the list: the
// derivative gather, the line-search sums and the value updates are masked
// elementwise passes around the padded FFT convolutions (host:
// csrc/host/component_optimization.cc). HBM-bound.
#include <algorithm>

#include "rdl_internal.h"

namespace rdl {
namespace {

constexpr unsigned kThreads = 256;
inline unsigned Grid(size_t n) {
  return unsigned(std::min<size_t>((n + kThreads - 1) / kThreads, 8192));
}

// out = model != 0 ? sign * t : 0
__global__ __launch_bounds__(256) void MaskedCopyKernel(const float* model, const float* t,
                                                        float* out, size_t n, float sign) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    out[i] = model[i] != 0.0f ? sign * t[i] : 0.0f;
}

// model[i] += v[i] where model[i] != 0
__global__ __launch_bounds__(256) void MaskedAddKernel(float* model, const float* v,
                                                       size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    if (model[i] != 0.0f) model[i] += v[i];
}

// Fixed-order two-stage dot products (reproducible: no atomics). Stage 1:
// block b writes partials[2b] = its sum of a*b, partials[2b+1] = its sum of
// a*a (double), over a fixed grid-stride partition; stage 2: one block sums
// the partials in a fixed tree.
constexpr uint32_t kDotBlocks = 1024;

__global__ __launch_bounds__(256) void DotPairPartials(const float* a, const float* b,
                                                       size_t n, double* partials) {
  __shared__ double lds[2][4];
  double ab = 0.0, aa = 0.0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const double x = a[i];
    ab += x * double(b[i]);
    aa += x * x;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    ab += __shfl_xor(ab, off, 64);
    aa += __shfl_xor(aa, off, 64);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    lds[0][wave] = ab;
    lds[1][wave] = aa;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = (lds[0][0] + lds[0][1]) + (lds[0][2] + lds[0][3]);
    partials[2 * blockIdx.x + 1] = (lds[1][0] + lds[1][1]) + (lds[1][2] + lds[1][3]);
  }
}

__global__ __launch_bounds__(1024) void DotPairFinal(const double* partials, uint32_t n_blocks,
                                                     double* sums) {
  __shared__ double lds[2][1024];
  const uint32_t t = threadIdx.x;
  lds[0][t] = t < n_blocks ? partials[2 * t] : 0.0;
  lds[1][t] = t < n_blocks ? partials[2 * t + 1] : 0.0;
  __syncthreads();
  for (uint32_t half = 512; half > 0; half >>= 1) {
    if (t < half) {
      lds[0][t] += lds[0][t + half];
      lds[1][t] += lds[1][t + half];
    }
    __syncthreads();
  }
  if (t == 0) {
    sums[0] = lds[0][0];
    sums[1] = lds[1][0];
  }
}

}  // namespace
}  // namespace rdl

extern "C" {

int rdl_masked_copy(rdl_session* s, const float* d_model, const float* d_src, float* d_dst,
                    size_t n, float sign) {
  RDL_ARG_CHECK(s && d_model && d_src && d_dst, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "component_optimization", 12.0 * double(n));
  rdl::MaskedCopyKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_model, d_src, d_dst,
                                                                       n, sign);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_masked_add(rdl_session* s, float* d_model, const float* d_values, size_t n) {
  RDL_ARG_CHECK(s && d_model && d_values, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "component_optimization", 12.0 * double(n));
  rdl::MaskedAddKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_model, d_values, n);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_dot_pair(rdl_session* s, const float* d_a, const float* d_b, size_t n,
                 double* ab, double* aa) {
  RDL_ARG_CHECK(s && d_a && d_b && ab && aa, "NULL argument");
  RDL_TRY(s->EnsureScratch(s->partials, (2 * rdl::kDotBlocks + 2) * sizeof(double)));
  double* d_partials = static_cast<double*>(s->partials.ptr);
  double* d_sums = d_partials + 2 * rdl::kDotBlocks;
  RDL_HIP_CHECK(hipMemsetAsync(d_sums, 0, 2 * sizeof(double), s->stream));
  if (n > 0) {
    rdl::ScopedTiming t(s, "component_optimization", 8.0 * double(n));
    const uint32_t blocks = std::min<uint32_t>(rdl::kDotBlocks, rdl::DivUp(n, 256));
    rdl::DotPairPartials<<<blocks, 256, 0, s->stream>>>(d_a, d_b, n, d_partials);
    rdl::DotPairFinal<<<1, 1024, 0, s->stream>>>(d_partials, blocks, d_sums);
    RDL_HIP_CHECK(hipGetLastError());
  }
  double h[2] = {0.0, 0.0};
  const rdl::SmallRead r{h, d_sums, sizeof(h)};
  RDL_TRY(rdl::ReadSmall(s, &r, 1));
  *ab = h[0];
  *aa = h[1];
  return RDL_OK;
}

}  // extern "C"
