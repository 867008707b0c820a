#include "device.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "host_profile.h"

namespace radler::gpu {

void Check(int rc, const char* what) {
  if (rc != RDL_OK)
    throw std::runtime_error(std::string(what) + ": " + rdl_last_error());
}

Buffer::Buffer(Session& s, size_t bytes) { Resize(s, bytes); }

Buffer::~Buffer() {
  prof::Section p("gpu.free");
  if (ptr_) rdl_free(s_->Handle(), ptr_);
}

Buffer& Buffer::operator=(Buffer&& o) noexcept {
  if (this != &o) {
    if (ptr_) rdl_free(s_->Handle(), ptr_);
    s_ = o.s_;
    ptr_ = o.ptr_;
    bytes_ = o.bytes_;
    o.ptr_ = nullptr;
    o.bytes_ = 0;
  }
  return *this;
}

void Buffer::Resize(Session& s, size_t bytes) {
  if (ptr_ && bytes <= bytes_) return;
  prof::Section p("gpu.malloc");
  if (ptr_) Check(rdl_free(s_->Handle(), ptr_), "rdl_free");
  s_ = &s;
  ptr_ = nullptr;
  bytes_ = 0;
  // 256-byte granularity keeps every plane start 16-byte aligned
  const size_t alloc = (std::max<size_t>(bytes, 16) + 255) / 256 * 256;
  Check(rdl_malloc(s.Handle(), alloc, &ptr_), "rdl_malloc");
  bytes_ = alloc;
}

void Buffer::Zero() {
  if (ptr_) Check(rdl_memset_zero(s_->Handle(), ptr_, bytes_), "rdl_memset_zero");
}

Fft::Fft(Session& s, size_t width, size_t height, bool f64)
    : s_(s), width_(width), height_(height), f64_(f64) {
  // The LDS engine wins for the float64 padded residual correction (mixed-radix
  // sizes, where rocFFT needs many transpose passes); rocFFT's single-precision
  // power-of-two kernels are faster for the scale convolutions
  // (tools/bench_fft.py). RADLER_FFT=rocfft / lds overrides.
  const char* force = std::getenv("RADLER_FFT");
  const std::string mode = force ? force : "";
  // float: the LDS engine at every size it holds (compile-time four-step
  // plans at 4096 / 8192, runtime plans elsewhere): at the subimage planes of
  // a tiled run it beat rocFFT (8192^2 split 8 x 8: 7.2 vs 8.1 s per
  // Perform) and plans in microseconds where rocFFT compiles kernels for
  // 0.2-0.3 s per size. RADLER_FFT=rocfft restores rocFFT.
  const bool want_lds = mode != "rocfft";
  // RADLER_FFT_COLUMNS=single / split overrides the column-pass choice
  const char* cols_env = std::getenv("RADLER_FFT_COLUMNS");
  const std::string cols = cols_env ? cols_env : "";
  const int strategy = cols == "single"  ? RDL_CONV_COLUMNS_SINGLE
                       : cols == "split" ? RDL_CONV_COLUMNS_SPLIT
                                         : RDL_CONV_COLUMNS_AUTO;
  if (!want_lds || rdl_conv_create_ex(s.Handle(), uint32_t(width), uint32_t(height),
                                      f64 ? 1 : 0, strategy, &conv_) != RDL_OK)
    conv_ = nullptr;
  if (conv_) {
    // the compile-time-planned column kernels read and write any layout:
    // spectra are then stored column by column (contiguous column reads)
    cm_ = (rdl_conv_fast(conv_) & RDL_CONV_FAST_COLUMNS) != 0 && !SplitColumns();
    spectrum_bytes_ = rdl_conv_spectrum_bytes(conv_);
  } else {
    conv_ = nullptr;
    if (f64)
      Check(rdl_fft_create_f64(s.Handle(), uint32_t(width), uint32_t(height), &f_),
            "rdl_fft_create_f64");
    else
      Check(rdl_fft_create(s.Handle(), uint32_t(width), uint32_t(height), &f_),
            "rdl_fft_create");
    spectrum_bytes_ = rdl_fft_spectrum_bytes(f_);
  }
  work_.Resize(s, spectrum_bytes_);
}

Fft::~Fft() {
  if (conv_) rdl_conv_destroy(conv_);
  if (f_) rdl_fft_destroy(f_);
}

void Fft::Forward(const float* d_in, void* d_spectrum) {
  if (conv_ && cm_)
    ForwardColumnMajor(d_in, d_spectrum);
  else if (conv_)
    Check(rdl_conv_forward(conv_, d_in, d_spectrum), "rdl_conv_forward");
  else
    Check(rdl_fft_forward(f_, d_in, d_spectrum), "rdl_fft_forward");
}

void Fft::Inverse(void* d_spectrum, float* d_out) {
  if (conv_)
    throw std::logic_error("Fft::Inverse: use ConvolveSpectrum with the LDS engine");
  Check(rdl_fft_inverse(f_, d_spectrum, d_out), "rdl_fft_inverse");
}

void Fft::Convolve(float* d_image, const void* d_kernel_spectrum) {
  if (conv_) {
    const double norm = 1.0 / (double(width_) * double(height_));
    Check(rdl_conv_rows_forward(conv_, d_image, uint32_t(width_), uint32_t(height_),
                                0, 0, work_.Ptr()),
          "rdl_conv_rows_forward");
    Check(rdl_conv_columns_layout(conv_, work_.Ptr(), work_.Ptr(), d_kernel_spectrum, 1,
                                  f64_ ? norm : double(float(norm)), nullptr,
                                  RDL_CONV_ROW_MAJOR, Layout(), RDL_CONV_ROW_MAJOR),
          "rdl_conv_columns_layout");
    Check(rdl_conv_rows_inverse(conv_, work_.Ptr(), d_image, uint32_t(width_),
                                uint32_t(height_), 0, 0, 0),
          "rdl_conv_rows_inverse");
  } else {
    Check(rdl_fft_convolve(f_, d_image, d_kernel_spectrum, work_.Ptr()),
          "rdl_fft_convolve");
  }
}

void Fft::ConvolveSpectrum(const void* d_spectrum, const void* d_kernel_spectrum,
                           void* d_work, float* d_out) {
  const double norm = 1.0 / (double(width_) * double(height_));
  if (conv_) {
    Check(rdl_conv_columns_layout(conv_, d_spectrum, d_work, d_kernel_spectrum, 2,
                                  f64_ ? norm : double(float(norm)), nullptr, Layout(),
                                  Layout(), RDL_CONV_ROW_MAJOR),
          "rdl_conv_columns_layout");
    Check(rdl_conv_rows_inverse(conv_, d_work, d_out, uint32_t(width_),
                                uint32_t(height_), 0, 0, 0),
          "rdl_conv_rows_inverse");
  } else {
    Check(rdl_spectrum_multiply(s_.Handle(), d_work, d_spectrum, d_kernel_spectrum,
                                ComplexCount(), float(norm)),
          "rdl_spectrum_multiply");
    Check(rdl_fft_inverse(f_, d_work, d_out), "rdl_fft_inverse");
  }
}

bool Fft::ConvolveSpectrumPeak(const void* d_spectrum, const void* d_kernel_spectrum,
                               void* d_work, float* d_out, uint32_t h_border,
                               uint32_t v_border, bool allow_negative,
                               const uint8_t* d_mask, uint32_t slot) {
  return ConvolveSpectrumWindowPeak(d_spectrum, d_kernel_spectrum, d_work, d_out, width_,
                                    height_, 0, 0, h_border, v_border, allow_negative, d_mask,
                                    slot);
}

bool Fft::ConvolveSpectrumWindowPeak(const void* d_spectrum, const void* d_kernel_spectrum,
                                     void* d_work, float* d_out, size_t out_w, size_t out_h,
                                     size_t ox, size_t oy, uint32_t h_border,
                                     uint32_t v_border, bool allow_negative,
                                     const uint8_t* d_mask, uint32_t slot) {
  if (!conv_ || !(rdl_conv_fast(conv_) & RDL_CONV_FAST_ROWS)) return false;
  const double norm = 1.0 / (double(width_) * double(height_));
  Check(rdl_conv_columns_layout(conv_, d_spectrum, d_work, d_kernel_spectrum, 2,
                                f64_ ? norm : double(float(norm)), nullptr, Layout(),
                                Layout(), RDL_CONV_ROW_MAJOR),
        "rdl_conv_columns_layout");
  Check(rdl_conv_rows_inverse_peak(conv_, d_work, d_out, uint32_t(out_w), uint32_t(out_h),
                                   uint32_t(ox), uint32_t(oy), h_border, v_border,
                                   allow_negative ? 1 : 0, d_mask, slot),
        "rdl_conv_rows_inverse_peak");
  return true;
}

bool Fft::ConvolveSpectrumWindow(const void* d_spectrum, const void* d_kernel_spectrum,
                                 void* d_work, float* d_out, size_t out_w, size_t out_h,
                                 size_t ox, size_t oy) {
  if (!conv_) return false;
  const double norm = 1.0 / (double(width_) * double(height_));
  Check(rdl_conv_columns_layout(conv_, d_spectrum, d_work, d_kernel_spectrum, 2,
                                f64_ ? norm : double(float(norm)), nullptr, Layout(),
                                Layout(), RDL_CONV_ROW_MAJOR),
        "rdl_conv_columns_layout");
  Check(rdl_conv_rows_inverse(conv_, d_work, d_out, uint32_t(out_w), uint32_t(out_h),
                              uint32_t(ox), uint32_t(oy), 0),
        "rdl_conv_rows_inverse");
  return true;
}

bool Fft::ConvolveWindow(const float* d_plane, const void* d_kernel_spectrum, float* d_out,
                         size_t out_w, size_t out_h, size_t ox, size_t oy) {
  if (!conv_) return false;
  const double norm = 1.0 / (double(width_) * double(height_));
  Check(rdl_conv_rows_forward(conv_, d_plane, uint32_t(width_), uint32_t(height_), 0, 0,
                              work_.Ptr()),
        "rdl_conv_rows_forward");
  Check(rdl_conv_columns_layout(conv_, work_.Ptr(), work_.Ptr(), d_kernel_spectrum, 1,
                                f64_ ? norm : double(float(norm)), nullptr,
                                RDL_CONV_ROW_MAJOR, Layout(), RDL_CONV_ROW_MAJOR),
        "rdl_conv_columns_layout");
  Check(rdl_conv_rows_inverse(conv_, work_.Ptr(), d_out, uint32_t(out_w), uint32_t(out_h),
                              uint32_t(ox), uint32_t(oy), 0),
        "rdl_conv_rows_inverse");
  return true;
}

bool Fft::FusedScales() const {
  return conv_ && !f64_ && (rdl_conv_fast(conv_) & RDL_CONV_FAST_TILED) &&
         (rdl_conv_fast(conv_) & RDL_CONV_FAST_ROWS);
}

size_t Fft::RealKernelBytes() const { return conv_ ? rdl_conv_real_kernel_bytes(conv_) : 0; }

void Fft::RealKernel(const float* h_shape, size_t n, void* d_kernel) {
  Check(rdl_conv_real_kernel(conv_, h_shape, uint32_t(n), d_kernel), "rdl_conv_real_kernel");
}

void Fft::ForwardHalf(const float* d_in, void* d_half) {
  Check(rdl_conv_forward_half(conv_, d_in, uint32_t(width_), uint32_t(height_), 0, 0, d_half),
        "rdl_conv_forward_half");
}

void Fft::Scales(const void* d_half, const std::vector<const void*>& d_kernels,
                 const std::vector<void*>& d_outs) {
  const double norm = 1.0 / (double(width_) * double(height_));
  // rdl_conv_scales takes at most 8 scales per launch (rdl_hip.h); a longer
  // ladder (a 1-pixel beam at 2048^2, a scale_list of 10) runs in chunks of
  // the same forward half, which the launches only read
  constexpr size_t kPerLaunch = 8;
  if (d_kernels.size() != d_outs.size())
    throw std::logic_error("Fft::Scales: one output per kernel");
  for (size_t i = 0; i < d_kernels.size(); i += kPerLaunch) {
    const size_t n = std::min(kPerLaunch, d_kernels.size() - i);
    Check(rdl_conv_scales(conv_, d_half, uint32_t(n), d_kernels.data() + i,
                          d_outs.data() + i, double(float(norm))),
          "rdl_conv_scales");
  }
}

void Fft::ScaleFinishWindowPeak(const void* d_u, void* d_work, float* d_out, size_t out_w,
                                size_t out_h, size_t ox, size_t oy, uint32_t h_border,
                                uint32_t v_border, bool allow_negative,
                                const uint8_t* d_mask, uint32_t slot) {
  Check(rdl_conv_scale_finish(conv_, d_u, d_work), "rdl_conv_scale_finish");
  Check(rdl_conv_rows_inverse_peak(conv_, d_work, d_out, uint32_t(out_w), uint32_t(out_h),
                                   uint32_t(ox), uint32_t(oy), h_border, v_border,
                                   allow_negative ? 1 : 0, d_mask, slot),
        "rdl_conv_rows_inverse_peak");
}

void Fft::ForwardColumnMajor(const float* d_in, void* d_spectrum) {
  if (!conv_) throw std::logic_error("Fft::ForwardColumnMajor needs the LDS engine");
  Check(rdl_conv_rows_forward(conv_, d_in, uint32_t(width_), uint32_t(height_), 0, 0,
                              work_.Ptr()),
        "rdl_conv_rows_forward");
  Check(rdl_conv_columns_ex(conv_, work_.Ptr(), d_spectrum, nullptr, 0, 1.0, nullptr,
                            RDL_CONV_ROW_MAJOR, RDL_CONV_COL_MAJOR),
        "rdl_conv_columns_ex");
}

void Fft::ConvolveSubtract(const float* d_image, size_t img_w, size_t img_h,
                           size_t ox, size_t oy, const void* d_kernel_spectrum,
                           void* d_work, float* d_residual,
                           const uint8_t* d_row_mask, bool kernel_col_major,
                           bool kernel_f32) {
  if (!conv_) throw std::logic_error("Fft::ConvolveSubtract needs the LDS engine");
  const double norm = 1.0 / (double(width_) * double(height_));
  Check(rdl_conv_convolve_subtract(
            conv_, d_image, uint32_t(img_w), uint32_t(img_h), uint32_t(ox), uint32_t(oy),
            d_kernel_spectrum, kernel_col_major ? RDL_CONV_COL_MAJOR : RDL_CONV_ROW_MAJOR,
            kernel_f32 ? 1 : 0, f64_ ? norm : double(float(norm)), d_row_mask, d_work,
            d_residual),
        "rdl_conv_convolve_subtract");
}

size_t Fft::ConvolveSubtractBytes() const {
  return conv_ ? rdl_conv_convolve_subtract_bytes(conv_) : spectrum_bytes_;
}

void Fft::Forward64(const double* d_in, void* d_spectrum) {
  Check(rdl_fft64_forward(f_, d_in, d_spectrum), "rdl_fft64_forward");
}

void Fft::Convolve64(double* d_image, const void* d_kernel_spectrum) {
  Check(rdl_fft64_convolve(f_, d_image, d_kernel_spectrum, work_.Ptr()),
        "rdl_fft64_convolve");
}

Session::Session(int device) : device_(device) {
  Check(rdl_session_create(device, &s_), "rdl_session_create");
}

Session::~Session() {
  ffts_.clear();
  for (Buffer& b : scratch_) b = Buffer();
  if (subminor_) rdl_subminor_destroy(subminor_);
  if (pinned_) rdl_host_free(pinned_);
  rdl_session_destroy(s_);
}

Fft& Session::GetFft(size_t width, size_t height, bool f64) {
  auto key = std::make_tuple(width, height, f64);
  auto it = ffts_.find(key);
  if (it == ffts_.end()) {
    prof::Section p("gpu.fft_plan");
    it = ffts_.emplace(key, std::make_unique<Fft>(*this, width, height, f64)).first;
  }
  return *it->second;
}

Buffer& Session::Scratch(ScratchSlot slot, size_t bytes) {
  scratch_[slot].Resize(*this, bytes);
  return scratch_[slot];
}

void* Session::PinnedStaging(size_t bytes) {
  if (bytes > pinned_bytes_) {
    prof::Section p("gpu.host_alloc");
    if (pinned_) Check(rdl_host_free(pinned_), "rdl_host_free");
    pinned_ = nullptr;
    pinned_bytes_ = 0;
    Check(rdl_host_alloc(bytes, &pinned_), "rdl_host_alloc");
    pinned_bytes_ = bytes;
  }
  return pinned_;
}

rdl_subminor* Session::SharedSubminor() {
  if (!subminor_) Check(rdl_subminor_create(s_, &subminor_), "rdl_subminor_create");
  return subminor_;
}

void Session::Sync() {
  prof::Section p("gpu.sync");
  Check(rdl_session_sync(s_), "rdl_session_sync"); }
void Session::Bind() { Check(rdl_session_bind(s_), "rdl_session_bind"); }
void Session::SetConcurrency(size_t n) {
  Check(rdl_session_set_concurrency(s_, uint32_t(n)), "rdl_session_set_concurrency");
}
void Session::Peer(void* d, int dst_device, const void* src, int src_device,
                   size_t bytes) {
  Check(rdl_memcpy_peer(s_, d, dst_device, src, src_device, bytes),
        "rdl_memcpy_peer");
}

void Session::H2D(void* d, const void* h, size_t bytes) {
  prof::Section p("gpu.h2d");
  Check(rdl_memcpy_h2d(s_, d, h, bytes), "rdl_memcpy_h2d");
}
void Session::D2H(void* h, const void* d, size_t bytes) {
  prof::Section p("gpu.d2h");
  Check(rdl_memcpy_d2h(s_, h, d, bytes), "rdl_memcpy_d2h");
}
void Session::D2D(void* d, const void* src, size_t bytes) {
  Check(rdl_memcpy_d2d(s_, d, src, bytes), "rdl_memcpy_d2d");
}
void Session::Zero(void* d, size_t bytes) {
  Check(rdl_memset_zero(s_, d, bytes), "rdl_memset_zero");
}
float Session::ReadFloat(const float* d) {
  float v;
  D2H(&v, d, sizeof(float));
  return v;
}

std::shared_ptr<Session> Session::ForDevice(int device) {
  // One session per GPU for the life of the process: its FFT plans, kernel
  // spectra scratch and sub-minor state outlive the Radler objects, so
  // consecutive Perform calls (WSClean creates a Radler per run) do not
  // re-plan or re-allocate. Intentionally never destroyed: the HIP runtime
  // releases the device at exit, after static destructors would have run.
  static std::mutex mutex;
  static auto* sessions = new std::map<int, std::shared_ptr<Session>>();
  std::lock_guard<std::mutex> lock(mutex);
  auto it = sessions->find(device);
  if (it != sessions->end()) return it->second;
  auto s = std::make_shared<Session>(device);
  (*sessions)[device] = s;
  return s;
}

std::shared_ptr<Session> Session::Worker(int device, size_t index) {
  static std::mutex mutex;
  static auto* workers = new std::map<std::pair<int, size_t>, std::shared_ptr<Session>>();
  std::lock_guard<std::mutex> lock(mutex);
  auto& w = (*workers)[{device, index}];
  if (!w) {
    w = std::make_shared<Session>(device);
    w->worker_ = true;
  }
  return w;
}

int Session::DefaultDevice() {
  for (const char* var : {"RADLER_DEVICE", "LOCAL_RANK"}) {
    if (const char* v = std::getenv(var)) {
      int count = 0;
      Check(rdl_device_count(&count), "rdl_device_count");
      const int d = std::atoi(v);
      if (count > 0) return d % count;
    }
  }
  return 0;
}

Planes Planes::Make(Session& s, size_t width, size_t height, size_t count) {
  Planes p;
  p.width = width;
  p.height = height;
  p.count = count;
  p.buffer = std::make_shared<Buffer>(s, std::max<size_t>(1, width * height * count) *
                                             sizeof(float));
  return p;
}

}  // namespace radler::gpu
