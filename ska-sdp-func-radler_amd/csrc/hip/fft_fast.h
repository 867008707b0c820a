// Compile-time-planned FFT kernels (fft_fast.hip): plan lookup and launches
// used by the LDS engine's host code (lds_fft.hip) for the sizes they cover.
#pragma once

#include <cstddef>
#include <cstdint>

struct rdl_session;

namespace rdl {

constexpr size_t kFftLdsBytesFast = 160 * 1024;

/* Float transforms keep one pad element per 16 in LDS (ff::Lx): a pass's
 * butterfly outputs land R elements apart, and ds_write_b64 serves 16
 * contiguous lanes per bank cycle over 128 B, so a power-of-two stride put all
 * 16 lanes on one bank (16-way). Double plans run an odd radix first instead
 * (odd strides are conflict-free) and keep the LDS for the transform.
 * One pad per 32 (fewer 2-way read wraps) measured slower on the box:
 * rows_inverse_peak 170.6 -> 177.1 us, bench 716 -> 725 ms/step (r05). */
constexpr uint32_t kFastPadShift = 4;
inline size_t FastLdsBytes(uint32_t n, bool f64) {
  return f64 ? size_t(n) * 16 : (size_t(n) + (n >> kFastPadShift)) * 8;
}

/* radices of a compile-time plan, in pass order */
struct RadixList {
  uint8_t r[8];
  uint8_t n;
};
template <uint32_t... Rs>
constexpr RadixList MakeRadixList() {
  return RadixList{{uint8_t(Rs)...}, uint8_t(sizeof...(Rs))};
}

struct FastColumns {
  uint32_t n;  // column length
  bool f64;
  uint32_t threads;
  const void* kernel;
  RadixList radix;
  const void* kernel_kf = nullptr;  // ColumnsConvD reading a float kernel spectrum
};
struct FastRows {
  uint32_t n;  // full row length (2 x the half-length transform)
  bool f64;
  uint32_t threads;
  const void* inverse;
  const void* forward;
  RadixList radix;  // of the half-length transform
  const void* inverse_lt;  // float: LDS double twiddles, persistent (else nullptr)
  const void* forward_lt;
  const void* inverse_dma;  // float: ff::RowsInverseDma (else nullptr)
  size_t inverse_dma_lds;   // its dynamic LDS bytes
  const void* forward_dma;  // float: ff::RowsForwardDma (else nullptr)
  size_t forward_dma_lds;
};

/* float four-step column passes (column tiles of 16, see ff::TileIndex) */
struct FastSteps {
  uint32_t n, n1, n2, ga, gb;
  uint32_t threads;
  const void* step_a;
  const void* step_b;
  RadixList radix_a, radix_b;  // of the length-n1 / length-n2 transforms
  const void* step_b_scales;   // ff::ColStepBScales (forward B, x K_s, inner inverse)
  const void* step_a_inv;      // ff::ColStepAInv (outer inverse step)
};

/* The pass table of a length-n transform with these radices (ff::Pass):
 * for pass p (span NS = product of the earlier radices, M = n / (NS R)),
 * entries W_n^{k (q+1) M} at [offset_p + q NS + k], q < R - 1, k < NS;
 * float or double complex, computed in long double. hipMalloc'ed. */
int MakePassTable(uint32_t n, const RadixList& radix, bool f64, void** out,
                  hipStream_t stream);

const FastColumns* FindFastColumns(uint32_t n, bool f64);
const FastSteps* FindFastSteps(uint32_t n);
/* One four-step pass over all column tiles (pass_b: B, else A). inverse: A
 * loads conj(in x kern x scale), B stores conjugated. */
int FastStepLaunch(rdl_session* s, const FastSteps* p, bool pass_b, const void* in,
                   void* out, const void* kern, const void* tw, const void* ptw,
                   uint32_t n_cols, int inverse, float scale);
/* Several scale convolutions from one forward half (A pass output `in`):
 * per scale s, the forward B DFT, x kerns[s] (real, float tiles) x scale,
 * the inner inverse DFT and its twiddle into outs[s] (ff::ColStepBScales);
 * then per scale FastStepAInvLaunch -> the natural-order column inverse.
 * tw: the length-n table W_n^k. At most 8 scales per launch. */
int FastScalesLaunch(rdl_session* s, const FastSteps* p, const void* in, const void* tw,
                     const void* ptw_b, uint32_t n_cols, uint32_t n_scales,
                     const float* const* kerns, void* const* outs, float scale);
int FastStepAInvLaunch(rdl_session* s, const FastSteps* p, const void* in, void* out,
                       const void* ptw_a, uint32_t n_cols);
/* cos(2 pi j / n), j < n, double (long double on the host) */
int MakeCosTable(uint32_t n, void** out, hipStream_t stream);
/* the real spectrum of a symmetric n x n kernel (n odd) placed at the origin
 * of a w x h plane, float, tiled; a_scratch: (n / 2 + 1) x (w / 2 + 1) doubles */
int RealKernelLaunch(rdl_session* s, const float* shape, uint32_t n, uint32_t w, uint32_t h,
                     const void* cos_w, const void* cos_h, void* a_scratch, float* out);
/* tiled spectrum size in complex elements for a plane of `width` x `height` */
inline size_t TiledComplexCount(uint32_t width, uint32_t height) {
  return size_t((width / 2 + 1 + 15) / 16) * 16 * height;
}
const FastRows* FindFastRows(uint32_t n, bool f64);

/* mode 0 forward / 1 forward x K x s inverse / 2 x K x s inverse, one
 * spectrum column per workgroup round. Input rows: a device list (rows,
 * n_rows) or the range [row0, row0 + row_n) (other rows zero). */
int FastColumnsLaunch(rdl_session* s, const FastColumns* p, const void* in, void* out,
                      const void* kern, const void* ptw, uint32_t n_cols, uint32_t mode,
                      int in_cm, int out_cm, int kern_cm, const uint32_t* rows,
                      const uint32_t* n_rows, uint32_t row0, uint32_t row_n,
                      double scale);
/* Peak search fused into the inverse row pass (peak_finder::Find semantics,
 * rdl_find_peak): every written row's max key in the box x in [xs, xe),
 * y in [ys, ye) (and mask) goes to partials[row] (0 outside the box). */
struct RowPeak {
  uint64_t* partials;
  const uint8_t* mask;
  uint32_t xs, xe, ys, ye;
  int allow_negative;
};
/* spectrum rows oy .. oy+img_h-1 -> the img_w x img_h window at (ox, oy);
 * with `peak`, *n_partials = the peak partials written (one per row, or one
 * per workgroup for the LDS-DMA kernel) */
/* twd: MakeTwiddleBase(n) for the float plans' LDS-twiddle kernels (NULL:
 * the global pass tables) */
int FastRowsInverseLaunch(rdl_session* s, const FastRows* p, const void* spec, float* out,
                          const void* tw, const void* ptw, uint32_t height, uint32_t img_w, uint32_t img_h,
                          uint32_t ox, uint32_t oy, int subtract, int tiled = 0,
                          const RowPeak* peak = nullptr, const void* twd = nullptr,
                          uint32_t* n_partials = nullptr);
/* the window's rows (or the listed plane rows) -> spectrum rows */
int FastRowsForwardLaunch(rdl_session* s, const FastRows* p, const float* in, void* spec,
                          const void* tw, const void* ptw, uint32_t height, uint32_t img_w, uint32_t img_h,
                          uint32_t ox, uint32_t oy, const uint32_t* rows,
                          const uint32_t* n_rows, int tiled = 0, const void* twd = nullptr,
                          int all_rows = -1);
/* the two-level double twiddle base of length `base` (ff::TwdLds layout) */
int MakeTwiddleBase(uint32_t base, void** out, hipStream_t stream);
/* float64 convolution columns (mode 1: forward, x K x s, inverse; row-major
 * input and output) with LDS twiddles and a register-resident K multiply
 * (ff::ColumnsConvD); nullptr where no plan exists or RDL_FFT_CONVD=0. tw:
 * the plan's length-n table W_n^k. */
const FastColumns* FindConvColumnsD(uint32_t n);
int ConvColumnsDLaunch(rdl_session* s, const FastColumns* p, const void* in, void* out,
                       const void* kern, const void* tw, uint32_t n_cols, int kern_cm,
                       int out_cm, const uint32_t* rows, const uint32_t* n_rows, uint32_t row0,
                       uint32_t row_n, double scale, uint32_t out_row0 = 0,
                       uint32_t out_row_n = 0xffffffffu, bool kernel_f32 = false,
                       bool tiled = false);
/* ascending list of the rows whose mask byte is non-zero, and its length */
int FastCompactRows(rdl_session* s, const uint8_t* mask, uint32_t n, uint32_t* rows,
                    uint32_t* count);

}  // namespace rdl
