// Spectral interpolation of the model:
// ImageSet::InterpolateAndStoreModel (cpp/image_set.cc:209-288) with a
// polynomial fitter. Per pixel the reference fits terms over the
// deconvolution channels and evaluates them at every original channel's
// frequency; with fixed frequencies and weights that is one n_out x n_in
// linear map, so this is a single HBM pass: read the n_in channel values of
// a pixel once, write its n_out interpolated values. Bound: HBM,
// 4 * (n_in + n_out) bytes per pixel.
#include "rdl_internal.h"

namespace rdl {

template <int NI>
__global__ __launch_bounds__(256) void InterpolateKernel(
    const float* in, size_t in_stride, uint32_t n_in, const float* coef,
    uint32_t n_out, float* out, size_t n) {
  __shared__ float c[RDL_MAX_IMAGES * NI];
  for (uint32_t i = threadIdx.x; i < n_out * n_in; i += blockDim.x) {
    const uint32_t g = i / n_in, k = i % n_in;
    c[g * NI + k] = coef[i];
  }
  __syncthreads();
  for (size_t px = blockIdx.x * size_t(blockDim.x) + threadIdx.x; px < n;
       px += size_t(gridDim.x) * blockDim.x) {
    float v[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k)
      v[k] = k < int(n_in) ? in[size_t(k) * in_stride + px] : 0.0f;
    for (uint32_t g = 0; g < n_out; ++g) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < NI; ++k)
        if (k < int(n_in)) acc = __builtin_fmaf(c[g * NI + k], v[k], acc);
      out[size_t(g) * n + px] = acc;
    }
  }
}

}  // namespace rdl

extern "C" int rdl_spectral_interpolate(rdl_session* s, const float* d_in,
                                        size_t in_stride, uint32_t n_in,
                                        const float* h_coefficients,
                                        uint32_t n_out, float* d_out, size_t n) {
  RDL_ARG_CHECK(s && d_in && h_coefficients && d_out, "NULL argument");
  RDL_ARG_CHECK(n_in >= 1 && n_in <= RDL_MAX_IMAGES && n_out >= 1 &&
                    n_out <= RDL_MAX_IMAGES,
                "channel count out of range");
  RDL_ARG_CHECK(n_in == 1 || in_stride >= n, "input planes overlap");
  if (n == 0) return RDL_OK;
  const size_t cbytes = size_t(n_out) * n_in * sizeof(float);
  RDL_TRY(s->EnsureScratch(s->kernel, cbytes));
  float* d_c = static_cast<float*>(s->kernel.ptr);
  RDL_HIP_CHECK(hipMemcpyAsync(d_c, h_coefficients, cbytes,
                               hipMemcpyHostToDevice, s->stream));
  const unsigned grid = unsigned(std::min<size_t>((n + 255) / 256, 2048));
  rdl::ScopedTiming t(s, "spectral_interpolate",
                      double(n) * 4.0 * double(n_in + n_out));
  if (n_in <= 4)
    rdl::InterpolateKernel<4><<<grid, 256, 0, s->stream>>>(d_in, in_stride, n_in, d_c,
                                                           n_out, d_out, n);
  else if (n_in <= 16)
    rdl::InterpolateKernel<16><<<grid, 256, 0, s->stream>>>(d_in, in_stride, n_in, d_c,
                                                            n_out, d_out, n);
  else
    rdl::InterpolateKernel<RDL_MAX_IMAGES><<<grid, 256, 0, s->stream>>>(
        d_in, in_stride, n_in, d_c, n_out, d_out, n);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

// ---------------------------------------------------------- log-polynomial
// InterpolateAndStoreModel with the non-linear log-polynomial fitter
// (logpoly.h): one thread per pixel fits its channel spectrum (zero spectra
// are not fitted: cpp/image_set.cc:247-264) and evaluates the terms at every
// output frequency. Model images are mostly zero, so the fit runs on few
// pixels and the pass is HBM-bound elsewhere.
#include "logpoly.h"

namespace rdl {

__global__ __launch_bounds__(256) void LogPolyInterpolateKernel(
    const float* in, size_t in_stride, size_t n, rdl_logpoly f, const double* out_lg,
    uint32_t n_out, float* out, size_t out_stride) {
  for (size_t px = blockIdx.x * size_t(blockDim.x) + threadIdx.x; px < n;
       px += size_t(gridDim.x) * blockDim.x) {
    float v[lp::kMaxCh];
    bool zero = true;
    for (uint32_t c = 0; c < f.n_channels; ++c) {
      v[c] = in[size_t(c) * in_stride + px];
      zero = zero && v[c] == 0.0f;
    }
    float terms[lp::kMaxTerms];
    if (zero) {
      for (int k = 0; k < lp::kMaxTerms; ++k) terms[k] = 0.0f;
    } else {
      lp::Fit(f, v, terms);
    }
    for (uint32_t g = 0; g < n_out; ++g)
      out[size_t(g) * out_stride + px] =
          zero ? 0.0f : lp::Evaluate(terms, int(f.n_terms), out_lg[g]);
  }
}

}  // namespace rdl

extern "C" int rdl_logpoly_interpolate(rdl_session* s, const float* d_in, size_t in_stride,
                                       size_t n_pixels, const rdl_logpoly* fit,
                                       const double* out_lg, uint32_t n_out, float* d_out,
                                       size_t out_stride) {
  RDL_ARG_CHECK(s && d_in && fit && out_lg && d_out, "NULL argument");
  RDL_ARG_CHECK(fit->n_channels >= 1 && fit->n_channels <= RDL_LOGPOLY_MAX_CHANNELS,
                "log-polynomial fit: channel count out of range");
  RDL_ARG_CHECK(fit->n_terms >= 1 && fit->n_terms <= RDL_LOGPOLY_MAX_TERMS,
                "log-polynomial fit: term count out of range");
  RDL_ARG_CHECK(n_out >= 1 && n_out <= RDL_MAX_IMAGES, "output count out of range");
  RDL_ARG_CHECK(fit->n_channels == 1 || in_stride >= n_pixels, "input planes overlap");
  RDL_ARG_CHECK(n_out == 1 || out_stride >= n_pixels, "output planes overlap");
  if (n_pixels == 0) return RDL_OK;
  const size_t bytes = size_t(n_out) * sizeof(double);
  RDL_TRY(s->EnsureScratch(s->kernel, bytes));
  double* d_lg = static_cast<double*>(s->kernel.ptr);
  RDL_HIP_CHECK(hipMemcpyAsync(d_lg, out_lg, bytes, hipMemcpyHostToDevice, s->stream));
  const unsigned grid = unsigned(std::min<size_t>((n_pixels + 255) / 256, 8192));
  rdl::ScopedTiming t(s, "spectral_interpolate",
                      double(n_pixels) * 4.0 * double(fit->n_channels + n_out));
  rdl::LogPolyInterpolateKernel<<<grid, 256, 0, s->stream>>>(d_in, in_stride, n_pixels, *fit,
                                                              d_lg, n_out, d_out, out_stride);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}
