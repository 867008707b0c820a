// Component optimisation: the streaming steps of
// math::GradientDescent (cpp/math/component_optimization.cc:100-177,
// 265-321) on whole planes. The component list is the model's non-zero
// pixels, so a plane that is zero off the components replaces the list: the
// derivative gather, the line-search sums and the value updates are masked
// elementwise passes around the padded FFT convolutions (host:
// csrc/host/component_optimization.cc). HBM-bound.
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

// sums[0] += sum a*b, sums[1] += sum a*a (double)
__global__ __launch_bounds__(256) void DotPairKernel(const float* a, const float* b, size_t n,
                                                     double* sums) {
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
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&sums[0], ab);
    atomicAdd(&sums[1], aa);
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
  RDL_TRY(s->EnsureScratch(s->partials, 256));
  double* d_sums = static_cast<double*>(s->partials.ptr);
  RDL_HIP_CHECK(hipMemsetAsync(d_sums, 0, 2 * sizeof(double), s->stream));
  if (n > 0) {
    rdl::ScopedTiming t(s, "component_optimization", 8.0 * double(n));
    rdl::DotPairKernel<<<rdl::Grid(n), rdl::kThreads, 0, s->stream>>>(d_a, d_b, n, d_sums);
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
