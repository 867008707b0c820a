// FFT convolution (rocFFT) and the kernel-preparation passes that replace
// schaapcommon::math::{PrepareSmallConvolutionKernel, PrepareConvolutionKernel,
// Convolve} and aocommon Image::{Untrim, Trim} (call sites:
// cpp/algorithms/multiscale/multiscale_transforms.cc:9-21,
// cpp/algorithms/subminor_loop.cc:195-218).
//
// rocFFT is used only for the transforms themselves (real 2-D, single
// precision, not-in-place). The pointwise spectrum product, the kernel
// placement and the trim/subtract epilogue are hand-written streaming
// kernels; callers cache kernel spectra so one convolution costs one forward
// transform, one multiply pass and one inverse transform.
#include <rocfft/rocfft.h>

#include <set>

#include "rdl_internal.h"

namespace {
std::once_flag g_rocfft_once;
std::atomic<bool> g_rocfft_used{false};
}

struct rdl_fft {
  rdl_session* s = nullptr;
  uint32_t width = 0, height = 0;
  bool f64 = false;
  rocfft_plan fwd = nullptr, inv = nullptr;
  rocfft_execution_info info_fwd = nullptr, info_inv = nullptr;
  void* work = nullptr;
  size_t work_bytes = 0;
};

namespace rdl {

#define RDL_FFT_CHECK(expr)                                         \
  do {                                                              \
    rocfft_status _st = (expr);                                     \
    if (_st != rocfft_status_success) {                             \
      ::rdl::SetError(std::string(#expr) + " failed: rocfft status " + \
                      std::to_string(int(_st)));                    \
      return RDL_ERR_FFT;                                           \
    }                                                               \
  } while (0)

__global__ __launch_bounds__(256) void SpectrumMultiply(float2* dst,
                                                        const float2* a,
                                                        const float2* b,
                                                        size_t n, float scale) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const float2 x = a[i], y = b[i];
    float2 r;
    r.x = (x.x * y.x - x.y * y.y) * scale;
    r.y = (x.x * y.y + x.y * y.x) * scale;
    dst[i] = r;
  }
}

__global__ __launch_bounds__(256) void SpectrumMultiplyF64(double2* dst,
                                                           const double2* a,
                                                           const double2* b,
                                                           size_t n,
                                                           double scale) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const double2 x = a[i], y = b[i];
    double2 r;
    r.x = (x.x * y.x - x.y * y.y) * scale;
    r.y = (x.x * y.y + x.y * y.x) * scale;
    dst[i] = r;
  }
}

// Zero + wrap an n x n kernel (centre n/2) so its centre sits at the origin.
__global__ __launch_bounds__(256) void PlaceSmallKernel(float* dest,
                                                        uint32_t width,
                                                        uint32_t height,
                                                        const float* k,
                                                        uint32_t n) {
  const size_t total = size_t(n) * n;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t kx = i % n, ky = i / n;
    int64_t dx = int64_t(kx) - int64_t(n / 2);
    int64_t dy = int64_t(ky) - int64_t(n / 2);
    if (dx < 0) dx += width;
    if (dy < 0) dy += height;
    dest[size_t(dy) * width + dx] = k[i];
  }
}

// dest(x, y) of the pw x ph plane = untrimmed(sx, sy) with
// sx = (x + pw/2) % pw, sy = (y + ph/2) % ph, where untrimmed is the w x h
// image centred at offset ((pw-w)/2, (ph-h)/2) in a zero plane.
__global__ __launch_bounds__(256) void PreparePsfKernel(float* dest,
                                                        uint32_t pw,
                                                        uint32_t ph,
                                                        const float* psf,
                                                        uint32_t w, uint32_t h) {
  const uint32_t ox = (pw - w) / 2, oy = (ph - h) / 2;
  const size_t total = size_t(pw) * ph;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = i % pw, y = i / pw;
    const uint32_t sx = (x + pw / 2) % pw, sy = (y + ph / 2) % ph;
    float v = 0.0f;
    if (sx >= ox && sx < ox + w && sy >= oy && sy < oy + h)
      v = psf[size_t(sy - oy) * w + (sx - ox)];
    dest[i] = v;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void PreparePsfKernelT(T* dest, uint32_t pw,
                                                         uint32_t ph,
                                                         const float* psf,
                                                         uint32_t w, uint32_t h) {
  const uint32_t ox = (pw - w) / 2, oy = (ph - h) / 2;
  const size_t total = size_t(pw) * ph;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = i % pw, y = i / pw;
    const uint32_t sx = (x + pw / 2) % pw, sy = (y + ph / 2) % ph;
    T v = T(0);
    if (sx >= ox && sx < ox + w && sy >= oy && sy < oy + h)
      v = T(psf[size_t(sy - oy) * w + (sx - ox)]);
    dest[i] = v;
  }
}

// residual -= float(trimmed convolution): the reference trims into a float
// scratch image before subtracting (subminor_loop.cc:214-217).
__global__ __launch_bounds__(256) void TrimSubtractF64(float* residual,
                                                       uint32_t w, uint32_t h,
                                                       const double* padded,
                                                       uint32_t pw,
                                                       uint32_t ph) {
  const uint32_t ox = (pw - w) / 2, oy = (ph - h) / 2;
  const size_t total = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = i % w, y = i / w;
    residual[i] -= float(padded[size_t(y + oy) * pw + x + ox]);
  }
}

__global__ __launch_bounds__(256) void TrimSubtract(float* residual,
                                                    uint32_t w, uint32_t h,
                                                    const float* padded,
                                                    uint32_t pw, uint32_t ph) {
  const uint32_t ox = (pw - w) / 2, oy = (ph - h) / 2;
  const size_t total = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = i % w, y = i / w;
    residual[i] -= padded[size_t(y + oy) * pw + x + ox];
  }
}

__global__ __launch_bounds__(256) void UntrimKernel(float* dest, uint32_t pw,
                                                    uint32_t ph,
                                                    const float* src,
                                                    uint32_t w, uint32_t h) {
  const uint32_t ox = (pw - w) / 2, oy = (ph - h) / 2;
  const size_t total = size_t(pw) * ph;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = i % pw, y = i / pw;
    float v = 0.0f;
    if (x >= ox && x < ox + w && y >= oy && y < oy + h)
      v = src[size_t(y - oy) * w + (x - ox)];
    dest[i] = v;
  }
}

// dest (pw x ph) = the w x h image repeated periodically, shifted by (sx, sy):
// dest[y][x] = src[(y - sy) mod h][(x - sx) mod w]. A circular convolution at
// w x h with a kernel of radius r <= sx, sy equals the linear convolution of
// this plane cropped at (sx, sy) when pw >= w + 2r and ph >= h + 2r.
__global__ __launch_bounds__(256) void PeriodicExtendKernel(
    float* __restrict__ dest, uint32_t pw, uint32_t ph, const float* __restrict__ src,
    uint32_t w, uint32_t h, uint32_t sx, uint32_t sy) {
  const uint32_t x = blockIdx.x * 256 + threadIdx.x;
  const uint32_t y = blockIdx.y;
  if (x >= pw) return;
  const uint32_t sxr = sx % w, syr = sy % h;
  const uint32_t ix = (x + w - sxr) % w;
  const uint32_t iy = (y + h - syr) % h;
  dest[size_t(y) * pw + x] = src[size_t(iy) * w + ix];
}

__global__ __launch_bounds__(256) void TrimKernel(float* dest, uint32_t w,
                                                  uint32_t h, const float* src,
                                                  uint32_t pw, uint32_t ph) {
  const uint32_t ox = (pw - w) / 2, oy = (ph - h) / 2;
  const size_t total = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < total;
       i += size_t(gridDim.x) * blockDim.x) {
    const uint32_t x = i % w, y = i / w;
    dest[i] = src[size_t(y + oy) * pw + x + ox];
  }
}

inline unsigned Grid(size_t n) {
  return unsigned(std::min<size_t>(16384, std::max<size_t>(1, DivUp(n, 256))));
}

}  // namespace rdl

// every live rdl_fft (rdl_shutdown destroys their rocFFT plans)
static std::mutex g_fft_registry_mutex;
static std::set<rdl_fft*> g_fft_registry;

void rdl::ReleaseFftPlans() {
  const std::lock_guard<std::mutex> lock(g_fft_registry_mutex);
  for (rdl_fft* f : g_fft_registry) {
    if (f->fwd) rocfft_plan_destroy(f->fwd);
    if (f->inv) rocfft_plan_destroy(f->inv);
    if (f->info_fwd) rocfft_execution_info_destroy(f->info_fwd);
    if (f->info_inv) rocfft_execution_info_destroy(f->info_inv);
    f->fwd = f->inv = nullptr;
    f->info_fwd = f->info_inv = nullptr;
    f->work = nullptr;  // a tracked block: rdl_shutdown frees it
  }
  g_fft_registry.clear();
  if (g_rocfft_used.load()) rocfft_cleanup();
}

static int CreateFft(rdl_session* s, uint32_t width, uint32_t height, bool f64,
                     rdl_fft** out) {
  RDL_ARG_CHECK(s && out, "NULL argument");
  RDL_ARG_CHECK(width >= 2 && height >= 1, "bad FFT size");
  std::call_once(g_rocfft_once, [] {
    rocfft_setup();
    g_rocfft_used.store(true);
  });
  // plans are created from the subimage workers' threads; keep rocFFT's
  // plan cache single-threaded
  static std::mutex plan_mutex;
  std::lock_guard<std::mutex> lock(plan_mutex);
  RDL_HIP_CHECK(hipSetDevice(s->device));
  auto f = std::make_unique<rdl_fft>();
  f->s = s;
  f->width = width;
  f->height = height;
  f->f64 = f64;
  const rocfft_precision prec =
      f64 ? rocfft_precision_double : rocfft_precision_single;
  size_t lengths[2] = {width, height};  // fastest dimension first
  RDL_FFT_CHECK(rocfft_plan_create(&f->fwd, rocfft_placement_notinplace,
                                   rocfft_transform_type_real_forward, prec, 2,
                                   lengths, 1, nullptr));
  RDL_FFT_CHECK(rocfft_plan_create(&f->inv, rocfft_placement_notinplace,
                                   rocfft_transform_type_real_inverse, prec, 2,
                                   lengths, 1, nullptr));
  size_t w1 = 0, w2 = 0;
  RDL_FFT_CHECK(rocfft_plan_get_work_buffer_size(f->fwd, &w1));
  RDL_FFT_CHECK(rocfft_plan_get_work_buffer_size(f->inv, &w2));
  f->work_bytes = std::max(w1, w2);
  if (f->work_bytes) RDL_HIP_CHECK(rdl::DevMalloc(&f->work, f->work_bytes));
  RDL_FFT_CHECK(rocfft_execution_info_create(&f->info_fwd));
  RDL_FFT_CHECK(rocfft_execution_info_create(&f->info_inv));
  RDL_FFT_CHECK(rocfft_execution_info_set_stream(f->info_fwd, s->stream));
  RDL_FFT_CHECK(rocfft_execution_info_set_stream(f->info_inv, s->stream));
  if (f->work_bytes) {
    RDL_FFT_CHECK(
        rocfft_execution_info_set_work_buffer(f->info_fwd, f->work, f->work_bytes));
    RDL_FFT_CHECK(
        rocfft_execution_info_set_work_buffer(f->info_inv, f->work, f->work_bytes));
  }
  {
    const std::lock_guard<std::mutex> rlock(g_fft_registry_mutex);
    g_fft_registry.insert(f.get());
  }
  *out = f.release();
  return RDL_OK;
}

static int Execute(rdl_fft* f, bool forward, void* in, void* out) {
  const double real_bytes = double(f->width) * f->height * (f->f64 ? 8.0 : 4.0);
  rdl::ScopedTiming t(f->s, f->f64 ? "fft64" : "fft",
                      real_bytes + double(rdl_fft_spectrum_bytes(f)));
  void* ins[1] = {in};
  void* outs[1] = {out};
  // the session's current lane: a plan made while lane 1 was current must not
  // keep running on that lane's stream
  rocfft_execution_info info = forward ? f->info_fwd : f->info_inv;
  RDL_FFT_CHECK(rocfft_execution_info_set_stream(info, f->s->stream));
  RDL_FFT_CHECK(rocfft_execute(forward ? f->fwd : f->inv, ins, outs, info));
  return RDL_OK;
}

extern "C" {

int rdl_fft_create(rdl_session* s, uint32_t width, uint32_t height,
                   rdl_fft** out) {
  return CreateFft(s, width, height, false, out);
}

int rdl_fft_create_f64(rdl_session* s, uint32_t width, uint32_t height,
                       rdl_fft** out) {
  return CreateFft(s, width, height, true, out);
}

int rdl_fft_destroy(rdl_fft* f) {
  if (!f) return RDL_OK;
  if (rdl::ShutDown()) return RDL_OK;  // rdl_shutdown released the plans
  {
    const std::lock_guard<std::mutex> lock(g_fft_registry_mutex);
    g_fft_registry.erase(f);
  }
  (void)hipStreamSynchronize(f->s->stream);
  if (f->fwd) rocfft_plan_destroy(f->fwd);
  if (f->inv) rocfft_plan_destroy(f->inv);
  if (f->info_fwd) rocfft_execution_info_destroy(f->info_fwd);
  if (f->info_inv) rocfft_execution_info_destroy(f->info_inv);
  if (f->work) (void)rdl::DevFree(f->work);
  delete f;
  return RDL_OK;
}

size_t rdl_fft_spectrum_bytes(const rdl_fft* f) {
  return f ? size_t(f->width / 2 + 1) * f->height * 2 *
                 (f->f64 ? sizeof(double) : sizeof(float))
           : 0;
}

int rdl_fft_forward(rdl_fft* f, const float* d_in, void* d_spectrum) {
  RDL_ARG_CHECK(f && d_in && d_spectrum, "NULL argument");
  RDL_ARG_CHECK(!f->f64, "double-precision plan: use rdl_fft64_*");
  return Execute(f, true, const_cast<float*>(d_in), d_spectrum);
}

int rdl_fft_inverse(rdl_fft* f, void* d_spectrum, float* d_out) {
  RDL_ARG_CHECK(f && d_out && d_spectrum, "NULL argument");
  RDL_ARG_CHECK(!f->f64, "double-precision plan: use rdl_fft64_*");
  return Execute(f, false, d_spectrum, d_out);
}

int rdl_fft64_forward(rdl_fft* f, const double* d_in, void* d_spectrum) {
  RDL_ARG_CHECK(f && d_in && d_spectrum, "NULL argument");
  RDL_ARG_CHECK(f->f64, "single-precision plan: use rdl_fft_*");
  return Execute(f, true, const_cast<double*>(d_in), d_spectrum);
}

int rdl_fft64_inverse(rdl_fft* f, void* d_spectrum, double* d_out) {
  RDL_ARG_CHECK(f && d_out && d_spectrum, "NULL argument");
  RDL_ARG_CHECK(f->f64, "single-precision plan: use rdl_fft_*");
  return Execute(f, false, d_spectrum, d_out);
}

int rdl_fft64_convolve(rdl_fft* f, double* d_image, const void* d_kernel_spectrum,
                       void* d_work) {
  RDL_ARG_CHECK(f && d_image && d_kernel_spectrum && d_work, "NULL argument");
  RDL_TRY(rdl_fft64_forward(f, d_image, d_work));
  const size_t nc = size_t(f->width / 2 + 1) * f->height;
  {
    rdl::ScopedTiming t(f->s, "spectrum_multiply64", double(nc) * 48.0);
    rdl::SpectrumMultiplyF64<<<rdl::Grid(nc), 256, 0, f->s->stream>>>(
        static_cast<double2*>(d_work), static_cast<const double2*>(d_work),
        static_cast<const double2*>(d_kernel_spectrum), nc,
        1.0 / (double(f->width) * f->height));
    RDL_HIP_CHECK(hipGetLastError());
  }
  RDL_TRY(rdl_fft64_inverse(f, d_work, d_image));
  return RDL_OK;
}

int rdl_spectrum_multiply(rdl_session* s, void* d_dst, const void* d_a,
                          const void* d_b, size_t n_complex, float scale) {
  RDL_ARG_CHECK(s && d_dst && d_a && d_b, "NULL argument");
  if (n_complex == 0) return RDL_OK;
  rdl::ScopedTiming t(s, "spectrum_multiply", double(n_complex) * 24.0);
  rdl::SpectrumMultiply<<<rdl::Grid(n_complex), 256, 0, s->stream>>>(
      static_cast<float2*>(d_dst), static_cast<const float2*>(d_a),
      static_cast<const float2*>(d_b), n_complex, scale);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_fft_convolve(rdl_fft* f, float* d_image, const void* d_kernel_spectrum,
                     void* d_work) {
  RDL_ARG_CHECK(f && d_image && d_kernel_spectrum && d_work, "NULL argument");
  RDL_ARG_CHECK(!f->f64, "double-precision plan: use rdl_fft64_convolve");
  RDL_TRY(rdl_fft_forward(f, d_image, d_work));
  const size_t nc = size_t(f->width / 2 + 1) * f->height;
  RDL_TRY(rdl_spectrum_multiply(f->s, d_work, d_work, d_kernel_spectrum, nc,
                                1.0f / float(double(f->width) * f->height)));
  RDL_TRY(rdl_fft_inverse(f, d_work, d_image));
  return RDL_OK;
}

int rdl_prepare_small_kernel(rdl_session* s, float* d_dest, uint32_t width,
                             uint32_t height, const float* h_kernel,
                             uint32_t n) {
  RDL_ARG_CHECK(s && d_dest && h_kernel, "NULL argument");
  if (n > width || n > height) {
    rdl::SetError("Kernel size is larger than the image size");
    return RDL_ERR_ARG;
  }
  // H2D into hipMalloc'd session scratch (a pageable copy into hipMallocAsync
  // memory was observed to land incompletely above ~4 KiB on ROCm 7.2)
  const size_t kbytes = size_t(n) * n * sizeof(float);
  RDL_TRY(s->EnsureScratch(s->kernel, kbytes));
  float* d_k = static_cast<float*>(s->kernel.ptr);
  RDL_HIP_CHECK(hipMemcpyAsync(d_k, h_kernel, kbytes, hipMemcpyHostToDevice,
                               s->stream));
  RDL_HIP_CHECK(hipMemsetAsync(d_dest, 0, size_t(width) * height * sizeof(float),
                               s->stream));
  rdl::PlaceSmallKernel<<<rdl::Grid(size_t(n) * n), 256, 0, s->stream>>>(
      d_dest, width, height, d_k, n);
  RDL_HIP_CHECK(hipGetLastError());
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

int rdl_prepare_psf_kernel(rdl_session* s, float* d_dest, uint32_t pw,
                           uint32_t ph, const float* d_psf, uint32_t width,
                           uint32_t height) {
  RDL_ARG_CHECK(s && d_dest && d_psf, "NULL argument");
  RDL_ARG_CHECK(pw >= width && ph >= height, "padded size smaller than image");
  rdl::PreparePsfKernel<<<rdl::Grid(size_t(pw) * ph), 256, 0, s->stream>>>(
      d_dest, pw, ph, d_psf, width, height);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_prepare_psf_kernel_f64(rdl_session* s, double* d_dest, uint32_t pw,
                               uint32_t ph, const float* d_psf, uint32_t width,
                               uint32_t height) {
  RDL_ARG_CHECK(s && d_dest && d_psf, "NULL argument");
  RDL_ARG_CHECK(pw >= width && ph >= height, "padded size smaller than image");
  rdl::PreparePsfKernelT<double>
      <<<rdl::Grid(size_t(pw) * ph), 256, 0, s->stream>>>(d_dest, pw, ph, d_psf,
                                                           width, height);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_trim_subtract_f64(rdl_session* s, float* d_residual, uint32_t width,
                          uint32_t height, const double* d_padded, uint32_t pw,
                          uint32_t ph) {
  RDL_ARG_CHECK(s && d_residual && d_padded, "NULL argument");
  RDL_ARG_CHECK(pw >= width && ph >= height, "padded size smaller than image");
  rdl::ScopedTiming t(s, "trim_subtract", double(width) * height * 16.0);
  rdl::TrimSubtractF64<<<rdl::Grid(size_t(width) * height), 256, 0, s->stream>>>(
      d_residual, width, height, d_padded, pw, ph);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_trim_subtract(rdl_session* s, float* d_residual, uint32_t width,
                      uint32_t height, const float* d_padded, uint32_t pw,
                      uint32_t ph) {
  RDL_ARG_CHECK(s && d_residual && d_padded, "NULL argument");
  RDL_ARG_CHECK(pw >= width && ph >= height, "padded size smaller than image");
  rdl::ScopedTiming t(s, "trim_subtract", double(width) * height * 12.0);
  rdl::TrimSubtract<<<rdl::Grid(size_t(width) * height), 256, 0, s->stream>>>(
      d_residual, width, height, d_padded, pw, ph);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_untrim(rdl_session* s, float* d_dest, uint32_t pw, uint32_t ph,
               const float* d_src, uint32_t width, uint32_t height) {
  RDL_ARG_CHECK(s && d_dest && d_src, "NULL argument");
  RDL_ARG_CHECK(pw >= width && ph >= height, "padded size smaller than image");
  rdl::UntrimKernel<<<rdl::Grid(size_t(pw) * ph), 256, 0, s->stream>>>(
      d_dest, pw, ph, d_src, width, height);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_periodic_extend(rdl_session* s, float* d_dest, uint32_t pw, uint32_t ph,
                        const float* d_src, uint32_t width, uint32_t height,
                        uint32_t shift_x, uint32_t shift_y) {
  RDL_ARG_CHECK(s && d_dest && d_src, "NULL argument");
  RDL_ARG_CHECK(width > 0 && height > 0 && ph < 65536, "bad plane size");
  rdl::ScopedTiming t(s, "extend", double(pw) * ph * 8.0);
  const dim3 grid((pw + 255) / 256, ph);
  rdl::PeriodicExtendKernel<<<grid, 256, 0, s->stream>>>(d_dest, pw, ph, d_src, width,
                                                        height, shift_x, shift_y);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_trim(rdl_session* s, float* d_dest, uint32_t width, uint32_t height,
             const float* d_src, uint32_t pw, uint32_t ph) {
  RDL_ARG_CHECK(s && d_dest && d_src, "NULL argument");
  RDL_ARG_CHECK(pw >= width && ph >= height, "padded size smaller than image");
  rdl::TrimKernel<<<rdl::Grid(size_t(width) * height), 256, 0, s->stream>>>(
      d_dest, width, height, d_src, pw, ph);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // extern "C"
