// C++ side of the boundary: RAII wrappers over the rdl_hip.h C-ABI. Every
// non-zero status becomes std::runtime_error carrying rdl_last_error(), which
// is how the reference reports failures (cpp/radler.cc:52-112).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "rdl_hip.h"

namespace radler::gpu {

void Check(int rc, const char* what);

class Session;

/// A device allocation owned by one session.
class Buffer {
 public:
  Buffer() = default;
  Buffer(Session& s, size_t bytes);
  ~Buffer();
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;
  Buffer(Buffer&& o) noexcept { *this = std::move(o); }
  Buffer& operator=(Buffer&& o) noexcept;
  void* Ptr() const { return ptr_; }
  float* F() const { return static_cast<float*>(ptr_); }
  double* D() const { return static_cast<double*>(ptr_); }
  size_t Bytes() const { return bytes_; }
  void Resize(Session& s, size_t bytes);  // grow-only, contents discarded
  void Zero();

 private:
  Session* s_ = nullptr;
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
};

/// Real 2-D FFT pair of one size. Uses the LDS-resident convolution engine
/// (rdl_conv_*) when the size allows, rocFFT (rdl_fft_*) otherwise; spectra
/// have the same layout either way (RADLER_FFT=rocfft|lds overrides the choice).
class Fft {
 public:
  Fft(Session& s, size_t width, size_t height, bool f64 = false);
  ~Fft();
  Fft(const Fft&) = delete;
  Fft& operator=(const Fft&) = delete;
  size_t Width() const { return width_; }
  size_t Height() const { return height_; }
  size_t SpectrumBytes() const { return spectrum_bytes_; }
  size_t ComplexCount() const { return size_t(width_ / 2 + 1) * height_; }
  bool IsF64() const { return f64_; }
  void Forward(const float* d_in, void* d_spectrum);
  void Inverse(void* d_spectrum, float* d_out);
  /// In-place circular convolution with a cached kernel spectrum.
  void Convolve(float* d_image, const void* d_kernel_spectrum);
  /// out = image whose spectrum is d_spectrum x d_kernel_spectrum / N
  /// (d_spectrum is preserved; d_work is spectrum-sized scratch).
  void ConvolveSpectrum(const void* d_spectrum, const void* d_kernel_spectrum,
                        void* d_work, float* d_out);
  /// ConvolveSpectrum with the image's peak search (rdl_find_peak box,
  /// mask and sign rules) fused into the last pass; the result goes to peak
  /// slot `slot` (rdl_find_peak_collect). False (nothing done) when this
  /// plan has no fused form.
  bool ConvolveSpectrumPeak(const void* d_spectrum, const void* d_kernel_spectrum,
                            void* d_work, float* d_out, uint32_t h_border,
                            uint32_t v_border, bool allow_negative, const uint8_t* d_mask,
                            uint32_t slot);
  /// LDS engine: ConvolveSpectrum / Convolve writing only the out_w x out_h
  /// window at (ox, oy) of the plane into d_out (out_w wide), and the peak
  /// form on that window; false (nothing done) without the LDS engine (or,
  /// for the peak form, without compile-time row plans).
  bool ConvolveSpectrumWindow(const void* d_spectrum, const void* d_kernel_spectrum,
                              void* d_work, float* d_out, size_t out_w, size_t out_h,
                              size_t ox, size_t oy);
  bool ConvolveSpectrumWindowPeak(const void* d_spectrum, const void* d_kernel_spectrum,
                                  void* d_work, float* d_out, size_t out_w, size_t out_h,
                                  size_t ox, size_t oy, uint32_t h_border, uint32_t v_border,
                                  bool allow_negative, const uint8_t* d_mask, uint32_t slot);
  bool ConvolveWindow(const float* d_plane, const void* d_kernel_spectrum, float* d_out,
                      size_t out_w, size_t out_h, size_t ox, size_t oy);
  /// LDS engine only: residual(window) -= Trim(conv(Untrim(image), kernel)),
  /// the image (img_w x img_h) placed at (ox, oy) in the plane.
  /// d_row_mask (plane rows, 0 = the image row is all zero) skips the empty
  /// rows; kernel_col_major reads a spectrum made by ForwardColumnMajor.
  /// d_work holds ConvolveSubtractBytes() (the float64 convolution-column
  /// plans keep its spectrum in the tiled layout: rdl_conv_convolve_subtract).
  void ConvolveSubtract(const float* d_image, size_t img_w, size_t img_h,
                        size_t ox, size_t oy, const void* d_kernel_spectrum,
                        void* d_work, float* d_residual,
                        const uint8_t* d_row_mask = nullptr,
                        bool kernel_col_major = false, bool kernel_f32 = false);
  size_t ConvolveSubtractBytes() const;
  /// LDS engine only: forward spectrum stored column by column (column k at
  /// k * height), the layout the column pass reads contiguously.
  void ForwardColumnMajor(const float* d_in, void* d_spectrum);
  /// Four-step (tiled) float plans: several scale convolutions of one image
  /// from one forward half (rdl_conv_forward_half / _real_kernel / _scales /
  /// _scale_finish; the forward spectrum is never stored).
  bool FusedScales() const;
  size_t RealKernelBytes() const;
  /// the real spectrum of a symmetric n x n kernel placed at the origin
  void RealKernel(const float* h_shape, size_t n, void* d_kernel);
  void ForwardHalf(const float* d_in, void* d_half);
  void Scales(const void* d_half, const std::vector<const void*>& d_kernels,
              const std::vector<void*>& d_outs);
  /// one scale's outer inverse step and the inverse rows with the fused peak
  /// search, writing the out_w x out_h window at (ox, oy)
  void ScaleFinishWindowPeak(const void* d_u, void* d_work, float* d_out, size_t out_w,
                             size_t out_h, size_t ox, size_t oy, uint32_t h_border,
                             uint32_t v_border, bool allow_negative, const uint8_t* d_mask,
                             uint32_t slot);
  bool UsesLds() const { return conv_ != nullptr; }
  /// LDS engine with compile-time-planned columns: Forward() stores spectra
  /// column by column, which Convolve / ConvolveSpectrum then expect.
  bool ColumnMajorSpectra() const { return cm_; }
  int Layout() const { return cm_ ? RDL_CONV_COL_MAJOR : RDL_CONV_ROW_MAJOR; }
  /// LDS engine with the split (four-step) column passes: spectra are read
  /// row-major, so ForwardColumnMajor is not used.
  bool SplitColumns() const { return conv_ && rdl_conv_columns_split(conv_); }
  /// float64 convolution columns by ff::ColumnsConvD (float kernels allowed)
  bool ConvColumnsD() const { return conv_ && (rdl_conv_fast(conv_) & RDL_CONV_FAST_CONVD); }
  /// Double-precision rocFFT plan only.
  void Forward64(const double* d_in, void* d_spectrum);
  void Convolve64(double* d_image, const void* d_kernel_spectrum);
  rdl_fft* Handle() { return f_; }

 private:
  Session& s_;
  rdl_fft* f_ = nullptr;
  rdl_conv* conv_ = nullptr;
  bool cm_ = false;  // column-major spectra (see ColumnMajorSpectra)
  size_t width_, height_, spectrum_bytes_;
  bool f64_;
  Buffer work_;
};

/// One HIP device + stream, with cached FFT plans.
class Session {
 public:
  explicit Session(int device);
  ~Session();
  Session(const Session&) = delete;
  Session& operator=(const Session&) = delete;
  rdl_session* Handle() const { return s_; }
  int Device() const { return device_; }
  /// A subimage pool's worker (Session::Worker): its streams already run
  /// concurrently with the pool's other workers.
  bool IsWorker() const { return worker_; }
  Fft& GetFft(size_t width, size_t height, bool f64 = false);
  void Sync();
  /// Make this session's device current for the calling thread.
  void Bind();
  /// `n` sessions share the device concurrently (caps cooperative grids).
  void SetConcurrency(size_t n);
  /// Copy between devices (or within one) on this session's stream.
  void Peer(void* d, int dst_device, const void* s, int src_device, size_t bytes);
  void H2D(void* d, const void* h, size_t bytes);
  void D2H(void* h, const void* d, size_t bytes);
  void D2D(void* d, const void* s, size_t bytes);
  void Zero(void* d, size_t bytes);
  float ReadFloat(const float* d);

  /// Grow-only scratch buffers that outlive the algorithm objects (a
  /// SubMinorLoop is created per outer iteration; allocating its ~1 GB of
  /// planes each time costs a hipMalloc/hipFree pair and a device sync).
  enum ScratchSlot {
    kCorrectionModel = 0,
    kCorrectionSpectrum,
    kCorrectionRows,
    kStaging,  // device side of the accessor staging (ImageSet loads)
    kNumScratch
  };
  Buffer& Scratch(ScratchSlot slot, size_t bytes);
  /// Grow-only page-locked host buffer for accessor loads/stores (one per
  /// session: the loads and stores of a Perform are sequential).
  void* PinnedStaging(size_t bytes);
  /// The session's sub-minor loop state (selection, model values), reused by
  /// consecutive SubMinorLoop objects.
  rdl_subminor* SharedSubminor();

  /// Process-wide session for a device (one per GPU, shared by the Radler
  /// objects of this process).
  static std::shared_ptr<Session> ForDevice(int device);
  /// Process-wide worker session `index` on a device (a subimage pool's
  /// streams), kept with its FFT plans across Radler objects.
  static std::shared_ptr<Session> Worker(int device, size_t index);
  /// The device a Radler instance uses when Settings::gpu_device == -1.
  static int DefaultDevice();

 private:
  rdl_session* s_ = nullptr;
  int device_;
  bool worker_ = false;
  std::map<std::tuple<size_t, size_t, bool>, std::unique_ptr<Fft>> ffts_;
  Buffer scratch_[kNumScratch];
  rdl_subminor* subminor_ = nullptr;
  void* pinned_ = nullptr;
  size_t pinned_bytes_ = 0;
};

/// A stack of `count` planes of width x height floats, contiguous.
struct Planes {
  std::shared_ptr<Buffer> buffer;
  size_t width = 0, height = 0, count = 0;
  size_t PlaneSize() const { return width * height; }
  float* Plane(size_t i) const { return buffer->F() + i * PlaneSize(); }
  float* Base() const { return buffer ? buffer->F() : nullptr; }
  static Planes Make(Session& s, size_t width, size_t height, size_t count);
};

}  // namespace radler::gpu
