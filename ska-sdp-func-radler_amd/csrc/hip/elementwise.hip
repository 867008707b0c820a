// ImageSet integration and elementwise helpers (cpp/image_set.cc,
// aocommon Image arithmetic as used by the reference), plus the shape-kernel
// stamp used by the non-fast multiscale loop. All HBM-streaming, float4 wide
// where the plane size allows.
#include "rdl_internal.h"

namespace rdl {

// complex double -> complex float (the float kernel spectra of
// rdl_conv_columns_window)
__global__ __launch_bounds__(256) void NarrowComplexKernel(float2* __restrict__ dst,
                                                           const double2* __restrict__ src,
                                                           size_t n) {
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    const double2 v = src[i];
    dst[i] = make_float2(float(v.x), float(v.y));
  }
}


__global__ __launch_bounds__(256) void IntegrateKernel(rdl_integration g,
                                                       const float* images,
                                                       size_t n, float* dest) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    dest[i] = IntegratePixel(g, [&](uint32_t k) { return images[k * n + i]; });
  }
}

__global__ __launch_bounds__(256) void AxpyKernel(float* dest, const float* a,
                                                  size_t n, float alpha,
                                                  int assign) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    dest[i] = assign == 1   ? a[i] * alpha
              : assign == 2 ? dest[i] + a[i]
                            : __builtin_fmaf(a[i], alpha, dest[i]);
  }
}

__global__ __launch_bounds__(256) void AxpyF64Kernel(float* dest,
                                                     const float* a, size_t n,
                                                     double alpha, int mode) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    dest[i] = mode == 0 ? float(__builtin_fma(double(a[i]), alpha, double(dest[i])))
                        : float(double(dest[i]) * alpha);
  }
}

__global__ __launch_bounds__(256) void ScaleKernel(float* dest, size_t n,
                                                   float alpha) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x)
    dest[i] *= alpha;
}

__global__ __launch_bounds__(256) void AddKernel(float* dest, const float* a,
                                                 size_t n) {
  const size_t n4 = n / 4;
  float4* d4 = reinterpret_cast<float4*>(dest);
  const float4* a4 = reinterpret_cast<const float4*>(a);
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n4;
       i += size_t(gridDim.x) * blockDim.x) {
    float4 x = d4[i];
    const float4 y = a4[i];
    x.x += y.x;
    x.y += y.y;
    x.z += y.z;
    x.w += y.w;
    d4[i] = x;
  }
  for (size_t i = n4 * 4 + blockIdx.x * size_t(blockDim.x) + threadIdx.x;
       i < n; i += size_t(gridDim.x) * blockDim.x)
    dest[i] += a[i];
}

// multiscale_transforms.h:62-89: image[yi][xi] += kernel * gain over the
// clipped n x n window centred at (x, y); contracted to FMA by the reference.
__global__ void AddShapeKernel(float* image, uint32_t width, const float* k,
                               uint32_t n, uint32_t x, uint32_t y,
                               uint32_t left, uint32_t top, uint32_t right,
                               uint32_t bottom, float gain) {
  const uint32_t xi = left + blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t yi = top + blockIdx.y;
  if (xi >= right || yi >= bottom) return;
  const float kv = k[(yi + n / 2 - y) * n + xi + n / 2 - x];
  float& px = image[size_t(yi) * width + xi];
  px = __builtin_fmaf(kv, gain, px);
}

inline unsigned GridFor(size_t n) {
  return unsigned(std::min<size_t>(8192, std::max<size_t>(1, DivUp(n, 256))));
}

}  // namespace rdl


namespace rdl {
// Box transfer between two planes (ImageSet::Trim / TrimMasked / CopyMasked /
// AddSubImage, cpp/image_set.h:216-262, aocommon Image box helpers).
__global__ __launch_bounds__(256) void BoxKernel(float* dst, uint32_t dst_w,
                                                 uint32_t dst_x, uint32_t dst_y,
                                                 const float* src, uint32_t src_w,
                                                 uint32_t src_x, uint32_t src_y,
                                                 uint32_t w, uint32_t h,
                                                 const uint8_t* mask, int op) {
  const size_t total = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = uint32_t(i % w), y = uint32_t(i / w);
    const float v = src[size_t(y + src_y) * src_w + x + src_x];
    float& d = dst[size_t(y + dst_y) * dst_w + x + dst_x];
    const bool m = mask ? mask[i] != 0 : true;
    switch (op) {
      case RDL_BOX_COPY: d = v; break;
      case RDL_BOX_COPY_MASKED: if (m) d = v; break;
      case RDL_BOX_COPY_ZERO: d = m ? v : 0.0f; break;
      default: d += v; break;
    }
  }
}
}  // namespace rdl

extern "C" {

int rdl_integrate(rdl_session* s, const rdl_integration* integ,
                  const float* d_images, size_t n, float* d_dest) {
  RDL_ARG_CHECK(s && integ && d_images && d_dest, "NULL argument");
  RDL_ARG_CHECK(integ->n_images >= 1 && integ->n_images <= RDL_MAX_IMAGES,
                "n_images out of range");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "integrate", double(n) * 4.0 * (integ->n_images + 1));
  rdl::IntegrateKernel<<<rdl::GridFor(n), 256, 0, s->stream>>>(*integ, d_images,
                                                                n, d_dest);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_axpy(rdl_session* s, float* d_dest, const float* d_a, size_t n,
             float alpha, int assign) {
  RDL_ARG_CHECK(s && d_dest && d_a, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "axpy", double(n) * (assign ? 8.0 : 12.0));
  rdl::AxpyKernel<<<rdl::GridFor(n), 256, 0, s->stream>>>(d_dest, d_a, n, alpha,
                                                           assign);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_axpy_f64(rdl_session* s, float* d_dest, const float* d_a, size_t n,
                 double alpha, int mode) {
  RDL_ARG_CHECK(s && d_dest && (d_a || mode == 1), "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::AxpyF64Kernel<<<rdl::GridFor(n), 256, 0, s->stream>>>(d_dest, d_a, n,
                                                              alpha, mode);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_scale(rdl_session* s, float* d_dest, size_t n, float alpha) {
  RDL_ARG_CHECK(s && d_dest, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScaleKernel<<<rdl::GridFor(n), 256, 0, s->stream>>>(d_dest, n, alpha);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_add(rdl_session* s, float* d_dest, const float* d_a, size_t n) {
  RDL_ARG_CHECK(s && d_dest && d_a, "NULL argument");
  if (n == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "add", double(n) * 12.0);
  if (reinterpret_cast<uintptr_t>(d_dest) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(d_a) % 16 == 0)
    rdl::AddKernel<<<rdl::GridFor(n / 4 + 1), 256, 0, s->stream>>>(d_dest, d_a,
                                                                    n);
  else
    rdl::AxpyKernel<<<rdl::GridFor(n), 256, 0, s->stream>>>(d_dest, d_a, n,
                                                             1.0f, 2);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_add_shape_component(rdl_session* s, float* d_image, uint32_t width,
                            uint32_t height, const float* h_kernel, uint32_t n,
                            uint32_t x, uint32_t y, float gain) {
  RDL_ARG_CHECK(s && d_image && h_kernel && n > 0, "bad argument");
  RDL_ARG_CHECK(x < width && y < height, "component outside the image");
  const size_t kbytes = size_t(n) * n * sizeof(float);
  RDL_TRY(s->EnsureScratch(s->kernel, kbytes));
  float* d_k = static_cast<float*>(s->kernel.ptr);
  RDL_HIP_CHECK(hipMemcpyAsync(d_k, h_kernel, kbytes, hipMemcpyHostToDevice,
                               s->stream));
  const uint32_t left = x > n / 2 ? x - n / 2 : 0;
  const uint32_t top = y > n / 2 ? y - n / 2 : 0;
  const uint32_t right = std::min(x + (n + 1) / 2, width);
  const uint32_t bottom = std::min(y + (n + 1) / 2, height);
  if (right > left && bottom > top) {
    dim3 grid(rdl::DivUp(right - left, 64), bottom - top);
    rdl::AddShapeKernel<<<grid, 64, 0, s->stream>>>(
        d_image, width, d_k, n, x, y, left, top, right, bottom, gain);
    RDL_HIP_CHECK(hipGetLastError());
  }
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}


int rdl_box(rdl_session* s, float* d_dst, uint32_t dst_w, uint32_t dst_x,
            uint32_t dst_y, const float* d_src, uint32_t src_w, uint32_t src_x,
            uint32_t src_y, uint32_t w, uint32_t h, const uint8_t* d_mask, int op) {
  RDL_ARG_CHECK(s && d_dst && d_src, "NULL argument");
  RDL_ARG_CHECK(op >= RDL_BOX_COPY && op <= RDL_BOX_ADD, "bad box op");
  RDL_ARG_CHECK(uint64_t(dst_x) + w <= dst_w && uint64_t(src_x) + w <= src_w,
                "box outside the row");
  if (w == 0 || h == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "box", double(w) * h * (op == RDL_BOX_ADD ? 12.0 : 8.0));
  const size_t total = size_t(w) * h;
  rdl::BoxKernel<<<unsigned(std::min<size_t>(16384, (total + 255) / 256)), 256, 0,
                   s->stream>>>(d_dst, dst_w, dst_x, dst_y, d_src, src_w, src_x,
                                src_y, w, h, d_mask, op);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_complex_narrow(rdl_session* s, void* d_dst, const void* d_src, size_t n_complex) {
  RDL_ARG_CHECK(s && d_dst && d_src, "NULL argument");
  if (n_complex == 0) return RDL_OK;
  rdl::NarrowComplexKernel<<<unsigned(std::min<size_t>(16384, (n_complex + 255) / 256)), 256, 0,
                             s->stream>>>(static_cast<float2*>(d_dst),
                                          static_cast<const double2*>(d_src), n_complex);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // extern "C"
