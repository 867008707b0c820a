// Compile-time-planned FFT kernels (fft_fast.hip): plan lookup and launches
// used by the LDS engine's host code (lds_fft.hip) for the sizes they cover.
#pragma once

#include <cstddef>
#include <cstdint>

struct rdl_session;

namespace rdl {

constexpr size_t kFftLdsBytesFast = 160 * 1024;

struct FastColumns {
  uint32_t n;  // column length
  bool f64;
  uint32_t threads;
  const void* kernel;
};
struct FastRows {
  uint32_t n;  // full row length (2 x the half-length transform)
  bool f64;
  uint32_t threads;
  const void* inverse;
  const void* forward;
};

const FastColumns* FindFastColumns(uint32_t n, bool f64);
const FastRows* FindFastRows(uint32_t n, bool f64);

/* mode 0 forward / 1 forward x K x s inverse / 2 x K x s inverse, one
 * spectrum column per workgroup round. Input rows: a device list (rows,
 * n_rows) or the range [row0, row0 + row_n) (other rows zero). */
int FastColumnsLaunch(rdl_session* s, const FastColumns* p, const void* in, void* out,
                      const void* kern, const void* tw, uint32_t n_cols, uint32_t mode,
                      int in_cm, int out_cm, int kern_cm, const uint32_t* rows,
                      const uint32_t* n_rows, uint32_t row0, uint32_t row_n,
                      double scale);
/* spectrum rows oy .. oy+img_h-1 -> the img_w x img_h window at (ox, oy) */
int FastRowsInverseLaunch(rdl_session* s, const FastRows* p, const void* spec, float* out,
                          const void* tw, uint32_t height, uint32_t img_w, uint32_t img_h,
                          uint32_t ox, uint32_t oy, int subtract);
/* the window's rows (or the listed plane rows) -> spectrum rows */
int FastRowsForwardLaunch(rdl_session* s, const FastRows* p, const float* in, void* spec,
                          const void* tw, uint32_t height, uint32_t img_w, uint32_t img_h,
                          uint32_t ox, uint32_t oy, const uint32_t* rows,
                          const uint32_t* n_rows);
/* ascending list of the rows whose mask byte is non-zero, and its length */
int FastCompactRows(rdl_session* s, const uint8_t* mask, uint32_t n, uint32_t* rows,
                    uint32_t* count);

}  // namespace rdl
