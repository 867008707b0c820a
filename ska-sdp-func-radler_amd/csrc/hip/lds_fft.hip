// LDS-resident FFT convolution engine: the multiscale scale convolutions and
// SubMinorLoop::CorrectResidualDirty (cpp/algorithms/multiscale/
// multiscale_transforms.cc:9-21, cpp/algorithms/subminor_loop.cc:195-218;
// schaapcommon::math::Convolve contract restated in oracle/oracle.cc) as
// three HBM passes instead of rocFFT's transpose-heavy plans:
//
//   rows forward   : two real rows per transform packed as z = a + i b, one
//                    complex Stockham FFT of the row length in LDS, split into
//                    the two half spectra (W/2+1 bins) -> row-major spectrum.
//                    The input is read from a w x h float image placed at an
//                    offset inside the (possibly padded) plane (Image::Untrim
//                    fused; rows outside it are zero and never loaded).
//   columns        : `count` spectrum columns per workgroup, complex FFT of the
//                    column length in LDS; optionally x kernel spectrum x 1/N
//                    and the inverse column FFT in the same pass.
//   rows inverse   : Hermitian half rows -> packed complex row -> inverse FFT
//                    in LDS -> two real rows, written (Image::Trim fused) or
//                    subtracted from the residual.
//
// Lengths must be 2^a 3^b 5^c 7^d (every CalculateGoodFFTSize output is) and
// fit in LDS (160 KiB: 20480 float / 10240 double complex); otherwise
// rdl_conv_create returns RDL_ERR_UNSUPPORTED and callers use rocFFT.
// Twiddles come from a float64 table (rounded to T for float plans).
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include "fft_dft.h"
#include "fft_fast.h"
#include "rdl_internal.h"

namespace rdl {

#ifndef RDL_FFT_THREADS
#define RDL_FFT_THREADS 1024
#endif
constexpr uint32_t kFftThreads = RDL_FFT_THREADS;
constexpr uint32_t kFftMaxPasses = 24;
constexpr size_t kFftLdsBytes = 160 * 1024;

// Complex elements one workgroup transforms at a time (count x length):
// bounds the butterflies per thread, hence registers (no spills at 512 threads).
constexpr uint32_t kMaxWgElems = 10240;
template <typename T>
constexpr uint32_t MaxElems() {
  return kMaxWgElems;
}

struct LdsPlan {
  uint32_t n;       // transform length
  uint32_t n_pass;
  uint8_t radix[kFftMaxPasses];
  const void* tw;   // n twiddles exp(-2 pi i k / n), Cx<T>
};



// ---- one Stockham pass over `count` transforms of length n held in LDS
// (in place: all butterfly inputs are read to registers before the barrier)
// Not inlined on purpose: with every radix inlined into one kernel the
// register allocator spilled 150-300 bytes per lane (scratch traffic showed
// up as 4-5x the algorithmic HBM writes); as separate functions each pass is
// allocated on its own (no spills; the call saves a few callee-saved VGPRs).
template <typename T, int R>
__device__ __attribute__((noinline)) void StockhamPass(Cx<T>* buf, uint32_t n,
                                             uint32_t count, uint32_t ns,
                                             const Cx<T>* __restrict__ tw,
                                             uint32_t tid, uint32_t stride) {
  constexpr uint32_t BPT = (MaxElems<T>() / R + kFftThreads - 1) / kFftThreads;
  const uint32_t nb = n / R;
  const uint32_t total = nb * count;
  const uint32_t m = n / (ns * R);
  Cx<T> v[BPT][R];
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t b = tid + i * kFftThreads;
    if (b < total) {
      const uint32_t t = b / nb, j = b - t * nb;
      const Cx<T>* base = buf + size_t(t) * stride;
#pragma unroll
      for (int r = 0; r < R; ++r) v[i][r] = base[j + r * nb];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t b = tid + i * kFftThreads;
    if (b < total) {
      const uint32_t t = b / nb, j = b - t * nb;
      const uint32_t k = j % ns;
      if (ns > 1) {
#pragma unroll
        for (int r = 1; r < R; ++r) v[i][r] = Mul(v[i][r], tw[k * r * m]);
      }
      Dft<T, R>::Run(v[i]);
      Cx<T>* base = buf + size_t(t) * stride;
      const uint32_t d = (j / ns) * ns * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) base[d + r * ns] = v[i][r];
    }
  }
  __syncthreads();
}

// Forward complex FFT (natural order in and out) of `count` transforms, each
// `stride` elements apart (>= n; padding keeps transposing loads off one bank).
template <typename T>
__device__ void LdsFftForward(Cx<T>* buf, const LdsPlan& p, uint32_t count,
                              uint32_t tid, uint32_t stride = 0) {
  if (stride == 0) stride = p.n;
  const Cx<T>* tw = static_cast<const Cx<T>*>(p.tw);
  uint32_t ns = 1;
  for (uint32_t q = 0; q < p.n_pass; ++q) {
    const uint32_t r = p.radix[q];
    switch (r) {
      case 16:
        if constexpr (sizeof(T) == 4) StockhamPass<T, 16>(buf, p.n, count, ns, tw, tid, stride);
        break;
      case 9:
        if constexpr (sizeof(T) == 4) StockhamPass<T, 9>(buf, p.n, count, ns, tw, tid, stride);
        break;
      case 8: StockhamPass<T, 8>(buf, p.n, count, ns, tw, tid, stride); break;
      case 4: StockhamPass<T, 4>(buf, p.n, count, ns, tw, tid, stride); break;
      case 2: StockhamPass<T, 2>(buf, p.n, count, ns, tw, tid, stride); break;
      case 3: StockhamPass<T, 3>(buf, p.n, count, ns, tw, tid, stride); break;
      case 5: StockhamPass<T, 5>(buf, p.n, count, ns, tw, tid, stride); break;
      default: StockhamPass<T, 7>(buf, p.n, count, ns, tw, tid, stride); break;
    }
    ns *= r;
  }
}

// ---------------------------------------------------------------- kernels
struct RowArgs {
  LdsPlan plan;        // row length n = plane width
  uint32_t height;     // plane rows
  uint32_t count;      // row pairs per workgroup
  uint32_t ld;         // spectrum row stride (complex) = n/2+1
  // forward input / inverse output window inside the plane
  uint32_t img_w, img_h, ox, oy;
  // forward: per plane row, 0 = known zero. A workgroup whose rows are all
  // zero neither reads nor writes (the column pass must get the same mask)
  const uint8_t* row_mask;
};

// rows forward: float image window -> half spectra (T)
template <typename T>
__global__ __launch_bounds__(kFftThreads) void RowsForward(RowArgs a,
                                                           const float* __restrict__ in,
                                                           Cx<T>* __restrict__ spec) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  const uint32_t tid = threadIdx.x;
  const uint32_t n = a.plan.n;
  const uint32_t pair0 = blockIdx.x * a.count;
  const uint32_t n_pairs = (a.height + 1) / 2;
  const uint32_t count = min(a.count, n_pairs - pair0);
  if (a.row_mask) {
    // workgroup OR through the (not yet used) dynamic LDS: the engine owns
    // all of it, so no static __shared__ flag or __syncthreads_or
    volatile uint32_t* flag = reinterpret_cast<volatile uint32_t*>(lds_raw);
    if (tid == 0) *flag = 0u;
    __syncthreads();
    const uint32_t y = 2 * pair0 + tid;
    if (tid < 2 * count && y < a.height && a.row_mask[y] != 0) *flag = 1u;
    __syncthreads();
    const bool any = *flag != 0u;
    __syncthreads();
    if (!any) return;
  }
  for (uint32_t idx = tid; idx < count * n; idx += kFftThreads) {
    const uint32_t t = idx / n, x = idx - t * n;
    const uint32_t y0 = 2 * (pair0 + t), y1 = y0 + 1;
    T va = T(0), vb = T(0);
    const int64_t ix = int64_t(x) - a.ox;
    // A masked row is zero whatever the plane holds there: the two rows of a
    // pair share one complex transform, so a stale row would leak into its
    // partner's spectrum through rounding (the partial-zeroing correction
    // model plane keeps old data in its unmarked rows).
    const bool use0 = !a.row_mask || a.row_mask[y0] != 0;
    const bool use1 = y1 < a.height && (!a.row_mask || a.row_mask[y1] != 0);
    if (ix >= 0 && ix < a.img_w) {
      const int64_t iy0 = int64_t(y0) - a.oy, iy1 = int64_t(y1) - a.oy;
      if (use0 && iy0 >= 0 && iy0 < a.img_h) va = T(in[size_t(iy0) * a.img_w + ix]);
      if (use1 && iy1 >= 0 && iy1 < a.img_h) vb = T(in[size_t(iy1) * a.img_w + ix]);
    }
    buf[idx] = {va, vb};
  }
  __syncthreads();
  LdsFftForward<T>(buf, a.plan, count, tid);
  const uint32_t nh = n / 2 + 1;
  for (uint32_t idx = tid; idx < count * nh; idx += kFftThreads) {
    const uint32_t t = idx / nh, k = idx - t * nh;
    const Cx<T> zk = buf[size_t(t) * n + k];
    const Cx<T> zc = Conj(buf[size_t(t) * n + (k == 0 ? 0 : n - k)]);
    const T h = T(0.5);
    const Cx<T> A = {h * (zk.x + zc.x), h * (zk.y + zc.y)};
    const Cx<T> B = {h * (zk.y - zc.y), -h * (zk.x - zc.x)};
    const uint32_t y0 = 2 * (pair0 + t), y1 = y0 + 1;
    spec[size_t(y0) * a.ld + k] = A;
    if (y1 < a.height) spec[size_t(y1) * a.ld + k] = B;
  }
}

// rows inverse: half spectra -> real rows; write (mode 0) or subtract
// (mode 1) the window [ox, ox+img_w) x [oy, oy+img_h) into out (img_w wide)
template <typename T>
__global__ __launch_bounds__(kFftThreads) void RowsInverse(RowArgs a,
                                                           const Cx<T>* __restrict__ spec,
                                                           float* __restrict__ out,
                                                           int subtract) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  const uint32_t tid = threadIdx.x;
  const uint32_t n = a.plan.n;
  const uint32_t pair0 = blockIdx.x * a.count;
  const uint32_t n_pairs = (a.height + 1) / 2;
  const uint32_t count = min(a.count, n_pairs - pair0);
  const uint32_t nh = n / 2 + 1;
  const bool even = (n & 1u) == 0;
  for (uint32_t idx = tid; idx < count * nh; idx += kFftThreads) {
    const uint32_t t = idx / nh, k = idx - t * nh;
    const uint32_t y0 = 2 * (pair0 + t), y1 = y0 + 1;
    Cx<T> A = spec[size_t(y0) * a.ld + k];
    Cx<T> B = y1 < a.height ? spec[size_t(y1) * a.ld + k] : Cx<T>{T(0), T(0)};
    if (k == 0 || (even && k == n / 2)) {  // C2R ignores these imaginary parts
      A.y = T(0);
      B.y = T(0);
    }
    // Z[k] = A + iB ; Z[n-k] = conj(A) + i conj(B). Stored conjugated (inverse
    // FFT = conj(FFT(conj)))
    Cx<T>* row = buf + size_t(t) * n;
    row[k] = {A.x - B.y, -(A.y + B.x)};
    if (k != 0 && !(even && k == n / 2)) row[n - k] = {A.x + B.y, -(B.x - A.y)};
  }
  __syncthreads();
  LdsFftForward<T>(buf, a.plan, count, tid);
  for (uint32_t idx = tid; idx < count * n; idx += kFftThreads) {
    const uint32_t t = idx / n, x = idx - t * n;
    const int64_t ix = int64_t(x) - a.ox;
    if (ix < 0 || ix >= a.img_w) continue;
    const Cx<T> z = buf[idx];  // conj(result): a = z.x, b = -z.y
    const uint32_t y0 = 2 * (pair0 + t), y1 = y0 + 1;
    const int64_t iy0 = int64_t(y0) - a.oy, iy1 = int64_t(y1) - a.oy;
    if (iy0 >= 0 && iy0 < a.img_h) {
      float* o = out + size_t(iy0) * a.img_w + ix;
      if (subtract)
        *o -= float(z.x);
      else
        *o = float(z.x);
    }
    if (y1 < a.height && iy1 >= 0 && iy1 < a.img_h) {
      float* o = out + size_t(iy1) * a.img_w + ix;
      if (subtract)
        *o -= float(-z.y);
      else
        *o = float(-z.y);
    }
  }
}

struct ColArgs {
  LdsPlan plan;      // column length n = plane height
  uint32_t n_cols;   // spectrum columns = width/2+1
  uint32_t count;    // columns per workgroup
  uint32_t ld;       // spectrum row stride
  uint32_t tiles_per_xcd;
  int mode;          // 0 fwd, 1 fwd*K*s+inv, 2 (already fwd) *K*s+inv
  double scale;
  const uint8_t* row_mask;  // rows known zero are not read (NULL: dense)
  uint32_t kern_cm;         // kernel spectrum column-major (column k at k*n)
  uint32_t out_cm;          // mode 0: write the spectrum column-major
};

template <typename T>
__global__ __launch_bounds__(kFftThreads) void Columns(ColArgs a,
                                                       const Cx<T>* __restrict__ in,
                                                       Cx<T>* __restrict__ out,
                                                       const Cx<T>* __restrict__ kern) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  // XCD-aware tiles: consecutive column tiles run on the same XCD so the
  // 128-byte lines they share are fetched into one L2
  const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
  const uint32_t tile = xcd * a.tiles_per_xcd + slot;
  const uint32_t k0 = tile * a.count;
  if (k0 >= a.n_cols) return;
  const uint32_t count = min(a.count, a.n_cols - k0);
  const uint32_t tid = threadIdx.x;
  const uint32_t n = a.plan.n;
  const T s = T(a.scale);
  for (uint32_t idx = tid; idx < count * n; idx += kFftThreads) {
    const uint32_t y = idx / count, j = idx - y * count;
    Cx<T> v = (a.row_mask && a.row_mask[y] == 0) ? Cx<T>{T(0), T(0)}
                                                 : in[size_t(y) * a.ld + k0 + j];
    if (a.mode == 2)
      v = Conj(Scale(Mul(v, a.kern_cm ? kern[size_t(k0 + j) * n + y]
                                      : kern[size_t(y) * a.ld + k0 + j]),
                     s));
    buf[size_t(j) * n + y] = v;
  }
  __syncthreads();
  if (a.mode != 2) LdsFftForward<T>(buf, a.plan, count, tid);
  if (a.mode == 1) {
    if (a.kern_cm) {  // contiguous kernel columns: walk each column
      for (uint32_t idx = tid; idx < count * n; idx += kFftThreads) {
        Cx<T>& v = buf[idx];  // idx = j*n + y
        v = Conj(Scale(Mul(v, kern[size_t(k0) * n + idx]), s));
      }
    } else {
      for (uint32_t idx = tid; idx < count * n; idx += kFftThreads) {
        const uint32_t y = idx / count, j = idx - y * count;
        Cx<T>& v = buf[size_t(j) * n + y];
        v = Conj(Scale(Mul(v, kern[size_t(y) * a.ld + k0 + j]), s));
      }
    }
    __syncthreads();
  }
  if (a.mode != 0) LdsFftForward<T>(buf, a.plan, count, tid);
  if (a.out_cm) {  // column-major spectrum (mode 0 only)
    for (uint32_t idx = tid; idx < count * n; idx += kFftThreads)
      out[size_t(k0) * n + idx] = buf[idx];
    return;
  }
  for (uint32_t idx = tid; idx < count * n; idx += kFftThreads) {
    const uint32_t y = idx / count, j = idx - y * count;
    const Cx<T> v = buf[size_t(j) * n + y];
    out[size_t(y) * a.ld + k0 + j] = a.mode == 0 ? v : Conj(v);
  }
}

// ------------------------------------------- split (four-step) column passes
// A column transform of length N = N1 * N2 in two coalesced passes instead of
// one strided one (with one double column per workgroup the single-pass
// column kernel touches a separate 128-byte line for every element):
//   A  : for each n2, the N1 elements at rows N2*n1 + n2 (strided rows, but
//        `cols` adjacent columns per row, so every load/store is a full
//        line): length-N1 FFT, x W_N^(n2*k1), back to rows N2*k1 + n2.
//   B  : for each k1, the N2 elements at rows N2*k1 + n2 (one contiguous
//        block of rows): length-N2 FFT -> X[k1 + N1*k2].
// The inverse runs the same passes backwards (B^-1 over the block, then A^-1
// with conj twiddles). B stores/loads the spectrum in natural row order
// (row k1 + N1*k2), so spectra keep the single-pass layout; the fused
// convolution (forward, x K x s, inverse) keeps B and B^-1 in one pass over
// the block.
struct SplitArgs {
  LdsPlan plan;        // sub-transform (N1 for A, N2 for B)
  uint32_t n, n1, n2;  // column length and its split
  uint32_t n_cols;     // spectrum columns (W/2+1)
  uint32_t ld;         // spectrum row stride
  uint32_t cols;       // adjacent columns per tile
  uint32_t groups;     // sub-columns per tile (A: n2 values, B: k1 values)
  uint32_t col_tiles;  // tiles across the columns
  uint32_t n_groups;   // A: n2, B: n1
  const void* tw_n;    // exp(-2 pi i k / N), k < N
  const uint8_t* row_mask;  // A forward: rows known zero are not read
  double scale;
  int mode;            // A: 0 forward, 1 inverse. B: 0 fwd, 1 fwd*K*s+inv, 2 *K*s+inv
};

template <typename T>
__global__ __launch_bounds__(kFftThreads) void ColumnsSplitA(SplitArgs a,
                                                             const Cx<T>* in,
                                                             Cx<T>* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  const uint32_t ct = blockIdx.x % a.col_tiles, gt = blockIdx.x / a.col_tiles;
  const uint32_t k0 = ct * a.cols, g0 = gt * a.groups;
  const uint32_t cnt = min(a.cols, a.n_cols - k0);
  const uint32_t gcnt = min(a.groups, a.n_groups - g0);
  const uint32_t tid = threadIdx.x, n1 = a.n1, n2 = a.n2, C = a.cols;
  const bool inverse = a.mode == 1;
  const Cx<T>* __restrict__ twn = static_cast<const Cx<T>*>(a.tw_n);
  const uint32_t total = n1 * gcnt * C;
  for (uint32_t idx = tid; idx < total; idx += kFftThreads) {
    const uint32_t j = idx % C, rest = idx / C;
    const uint32_t g = rest % gcnt, i1 = rest / gcnt;
    const uint32_t sub = g0 + g;
    const uint32_t row = n2 * i1 + sub;
    Cx<T> v{T(0), T(0)};
    if (j < cnt && !(a.row_mask && a.row_mask[row] == 0))
      v = in[size_t(row) * a.ld + k0 + j];
    if (inverse)  // conj(v * conj(w)) = conj(v) * w, w = W_N^(n2*k1)
      v = Mul(Conj(v), twn[(uint64_t(sub) * i1) % a.n]);
    buf[size_t(g * C + j) * (n1 + 1) + i1] = v;
  }
  __syncthreads();
  LdsFftForward<T>(buf, a.plan, gcnt * C, tid, n1 + 1);
  for (uint32_t idx = tid; idx < total; idx += kFftThreads) {
    const uint32_t j = idx % C, rest = idx / C;
    const uint32_t g = rest % gcnt, i1 = rest / gcnt;
    const uint32_t sub = g0 + g;
    Cx<T> v = buf[size_t(g * C + j) * (n1 + 1) + i1];
    v = inverse ? Conj(v) : Mul(v, twn[(uint64_t(sub) * i1) % a.n]);
    if (j < cnt) out[size_t(n2 * i1 + sub) * a.ld + k0 + j] = v;
  }
}

template <typename T>
__global__ __launch_bounds__(kFftThreads) void ColumnsSplitB(SplitArgs a,
                                                             const Cx<T>* in,
                                                             Cx<T>* out,
                                                             const Cx<T>* kern) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  const uint32_t ct = blockIdx.x % a.col_tiles, gt = blockIdx.x / a.col_tiles;
  const uint32_t k0 = ct * a.cols, g0 = gt * a.groups;
  const uint32_t cnt = min(a.cols, a.n_cols - k0);
  const uint32_t gcnt = min(a.groups, a.n_groups - g0);
  const uint32_t tid = threadIdx.x, n1 = a.n1, n2 = a.n2, C = a.cols;
  const T s = T(a.scale);
  const uint32_t total = n2 * gcnt * C;
  // mode 0/1 read the block (rows n2*k1 + i2), mode 2 the natural spectrum
  // (rows k1 + n1*k2); mode 2 starts in the conjugated domain
  for (uint32_t idx = tid; idx < total; idx += kFftThreads) {
    const uint32_t j = idx % C, rest = idx / C;
    const uint32_t g = rest % gcnt, i2 = rest / gcnt;
    const uint32_t k1 = g0 + g;
    Cx<T> v{T(0), T(0)};
    if (a.mode == 2) {
      const size_t at = size_t(k1 + n1 * i2) * a.ld + k0 + j;
      if (j < cnt) v = Conj(Scale(Mul(in[at], kern[at]), s));
    } else if (j < cnt) {
      v = in[size_t(n2 * k1 + i2) * a.ld + k0 + j];
    }
    buf[size_t(g * C + j) * (n2 + 1) + i2] = v;
  }
  __syncthreads();
  LdsFftForward<T>(buf, a.plan, gcnt * C, tid, n2 + 1);
  if (a.mode == 1) {
    for (uint32_t idx = tid; idx < total; idx += kFftThreads) {
      const uint32_t j = idx % C, rest = idx / C;
      const uint32_t g = rest % gcnt, i2 = rest / gcnt;
      const uint32_t k1 = g0 + g;
      Cx<T>& v = buf[size_t(g * C + j) * (n2 + 1) + i2];
      const Cx<T> k = j < cnt ? kern[size_t(k1 + n1 * i2) * a.ld + k0 + j]
                              : Cx<T>{T(0), T(0)};
      v = Conj(Scale(Mul(v, k), s));
    }
    __syncthreads();
    LdsFftForward<T>(buf, a.plan, gcnt * C, tid, n2 + 1);
  }
  for (uint32_t idx = tid; idx < total; idx += kFftThreads) {
    const uint32_t j = idx % C, rest = idx / C;
    const uint32_t g = rest % gcnt, i2 = rest / gcnt;
    const uint32_t k1 = g0 + g;
    const Cx<T> v = buf[size_t(g * C + j) * (n2 + 1) + i2];
    if (j >= cnt) continue;
    if (a.mode == 0)  // X[k1 + n1*k2] in natural order
      out[size_t(k1 + n1 * i2) * a.ld + k0 + j] = v;
    else  // back from the conjugated domain, block layout for A^-1
      out[size_t(n2 * k1 + i2) * a.ld + k0 + j] = Conj(v);
  }
}

// ---------------------------------------------------------------- planning
// Double plans stop at radix 8 and 3: the composite radix-16 / radix-9
// butterflies hold twice their inputs in registers, which in double spills
// past the 128 VGPRs a 1024-thread workgroup leaves each wave (the spill
// traffic showed up as 4-5x the algorithmic HBM writes).
// Odd radices run first: the first pass writes its outputs R elements apart,
// and an odd stride spreads a wave's stores over the LDS banks where a
// power-of-two one piles them on a few (ds_write_b128: 8-way at stride 8).
bool Factorize(uint32_t n, bool f64, std::vector<uint8_t>& radix) {
  radix.clear();
  uint32_t m = n;
  uint32_t twos = 0;
  while (m % 2 == 0) {
    m /= 2;
    ++twos;
  }
  for (uint32_t r : {7u, 5u})
    while (m % r == 0) {
      m /= r;
      radix.push_back(uint8_t(r));
    }
  while (!f64 && m % 9 == 0) {
    m /= 9;
    radix.push_back(9);
  }
  while (m % 3 == 0) {
    m /= 3;
    radix.push_back(3);
  }
  const uint32_t big2 = f64 ? 3 : 4;
  while (twos >= big2) {
    radix.push_back(uint8_t(1u << big2));
    twos -= big2;
  }
  if (twos == 3) radix.push_back(8);
  if (twos == 2) radix.push_back(4);
  if (twos == 1) radix.push_back(2);
  return m == 1 && radix.size() <= kFftMaxPasses;
}

}  // namespace rdl

struct rdl_conv {
  rdl_session* s = nullptr;
  uint32_t width = 0, height = 0;
  bool f64 = false;
  void* tw_row = nullptr;
  void* tw_col = nullptr;
  rdl::LdsPlan row_plan{}, col_plan{};
  uint32_t row_count = 1, col_count = 1;
  // split (four-step) column passes
  bool split = false;
  uint32_t n1 = 0, n2 = 0;
  rdl::LdsPlan plan_n1{}, plan_n2{};
  void* tw_n1 = nullptr;
  void* tw_n2 = nullptr;
  uint32_t split_cols = 0;
  // spectrum-sized, for the out-of-place B passes; one per session lane
  void* scratch_lane[2] = {nullptr, nullptr};
  void* scratch = nullptr;  // the current lane's (set by EnsureSplitScratch)
  size_t scratch_bytes[2] = {0, 0};
  // compile-time-planned kernels (fft_fast.hip) where the size has a plan
  const rdl::FastColumns* fast_cols = nullptr;
  const rdl::FastColumns* conv_cols = nullptr;  // float64 mode-1 columns (ColumnsConvD)
  const rdl::FastRows* fast_rows = nullptr;
  uint32_t* rows_list = nullptr;            // height words + the count
  const uint8_t* rows_list_mask = nullptr;  // mask the list was made from
  // float planes with four-step column plans: spectra in 16-column tiles
  const rdl::FastSteps* steps = nullptr;
  bool tiled = false;
  // pass tables of the compile-time plans (rdl::MakePassTable)
  void* ptw_row = nullptr;
  void* ptw_col = nullptr;
  void* ptw_a = nullptr;
  void* ptw_b = nullptr;
  void* twd_row = nullptr;  // float rows: two-level double twiddles of width (MakeTwiddleBase)
  // rdl_conv_real_kernel: cosine tables of width and height, stage-1 scratch
  void* cos_w = nullptr;
  void* cos_h = nullptr;
  rdl::Scratch real_a;
};

namespace {

double SpectrumBytes(const rdl_conv* c);
int EnsureSplitScratch(rdl_conv* c, size_t bytes);

int MakePlan(rdl_conv* c, uint32_t n, bool f64, rdl::LdsPlan* plan, void** tw) {
  std::vector<uint8_t> radix;
  if (!rdl::Factorize(n, f64, radix)) {
    rdl::SetError("LDS FFT: length " + std::to_string(n) + " is not 2/3/5/7-smooth");
    return RDL_ERR_UNSUPPORTED;
  }
  plan->n = n;
  plan->n_pass = uint32_t(radix.size());
  std::memset(plan->radix, 0, sizeof(plan->radix));
  for (size_t i = 0; i < radix.size(); ++i) plan->radix[i] = radix[i];
  const size_t esz = f64 ? 16 : 8;
  std::vector<unsigned char> host(size_t(n) * esz);
  for (uint32_t k = 0; k < n; ++k) {
    // exp(-2 pi i k/n) with the angle reduced to the first octant in double
    const long double ang = -2.0L * 3.14159265358979323846264338327950288L * k / n;
    const double cr = double(std::cos(ang)), ci = double(std::sin(ang));
    if (f64) {
      double v[2] = {cr, ci};
      std::memcpy(&host[k * esz], v, 16);
    } else {
      float v[2] = {float(cr), float(ci)};
      std::memcpy(&host[k * esz], v, 8);
    }
  }
  RDL_HIP_CHECK(rdl::DevMalloc(tw, host.size()));
  RDL_HIP_CHECK(rdl::UploadSync(*tw, host.data(), host.size(), c->s->stream));
  plan->tw = *tw;
  (void)c;
  return RDL_OK;
}

// the non-zero rows of `row_mask` as a device list (+ count), made once per
// rows-forward / columns pair
int CompactRowsFor(rdl_conv* c, const uint8_t* row_mask, bool reuse) {
  if (reuse && c->rows_list_mask == row_mask) return RDL_OK;
  if (!c->rows_list)
    RDL_HIP_CHECK(rdl::DevMalloc(&c->rows_list, (size_t(c->height) + 1) * sizeof(uint32_t)));
  RDL_TRY(rdl::FastCompactRows(c->s, row_mask, c->height, c->rows_list,
                               c->rows_list + c->height));
  c->rows_list_mask = row_mask;
  return RDL_OK;
}

template <typename T>
int LaunchRowsForward(rdl_conv* c, const float* in, uint32_t in_w, uint32_t in_h,
                      uint32_t ox, uint32_t oy, void* spec, const uint8_t* row_mask) {
  if (c->tiled) {
    if (row_mask) {
      rdl::SetError("LDS FFT: row masks need the row-major (float64) plans");
      return RDL_ERR_UNSUPPORTED;
    }
    return rdl::FastRowsForwardLaunch(c->s, c->fast_rows, in, spec, c->tw_row, c->ptw_row,
                                      c->height, in_w, in_h, ox, oy, nullptr, nullptr, 1,
                                      c->twd_row);
  }
  if (c->fast_rows) {
    const size_t row_bytes = size_t(c->width / 2 + 1) * sizeof(rdl::Cx<T>);
    if (row_mask) {
      RDL_TRY(CompactRowsFor(c, row_mask, false));
      return rdl::FastRowsForwardLaunch(c->s, c->fast_rows, in, spec, c->tw_row,
                                        c->ptw_row, c->height, in_w, in_h, ox, oy,
                                        c->rows_list, c->rows_list + c->height, 0,
                                        c->twd_row);
    }
    // rows outside the window are zero spectra
    char* base = static_cast<char*>(spec);
    if (oy > 0) RDL_HIP_CHECK(hipMemsetAsync(base, 0, size_t(oy) * row_bytes, c->s->stream));
    if (oy + in_h < c->height)
      RDL_HIP_CHECK(hipMemsetAsync(base + size_t(oy + in_h) * row_bytes, 0,
                                   size_t(c->height - oy - in_h) * row_bytes,
                                   c->s->stream));
    return rdl::FastRowsForwardLaunch(c->s, c->fast_rows, in, spec, c->tw_row, c->ptw_row,
                                      c->height, in_w, in_h, ox, oy, nullptr, nullptr, 0,
                                      c->twd_row);
  }
  rdl::RowArgs a{};
  a.row_mask = row_mask;
  a.plan = c->row_plan;
  a.height = c->height;
  a.count = c->row_count;
  a.ld = c->width / 2 + 1;
  a.img_w = in_w;
  a.img_h = in_h;
  a.ox = ox;
  a.oy = oy;
  const uint32_t n_pairs = (c->height + 1) / 2;
  const uint32_t grid = (n_pairs + a.count - 1) / a.count;
  const size_t lds = size_t(a.count) * c->width * sizeof(rdl::Cx<T>);
  auto k = rdl::RowsForward<T>;
  static std::atomic<uint64_t> attr_done{0};  // per instantiation and device
  RDL_TRY(rdl::SetMaxLdsOnce(reinterpret_cast<const void*>(k), int(rdl::kFftLdsBytes),
                             c->s->device, attr_done));
  k<<<grid, rdl::kFftThreads, lds, c->s->stream>>>(a, in,
                                                   static_cast<rdl::Cx<T>*>(spec));
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

template <typename T>
int LaunchRowsInverse(rdl_conv* c, const void* spec, float* out, uint32_t out_w,
                      uint32_t out_h, uint32_t ox, uint32_t oy, int subtract) {
  if (c->fast_rows)
    return rdl::FastRowsInverseLaunch(c->s, c->fast_rows, spec, out, c->tw_row, c->ptw_row,
                                      c->height, out_w, out_h, ox, oy, subtract,
                                      c->tiled ? 1 : 0, nullptr, c->twd_row);
  rdl::RowArgs a{};
  a.plan = c->row_plan;
  a.height = c->height;
  a.count = c->row_count;
  a.ld = c->width / 2 + 1;
  a.img_w = out_w;
  a.img_h = out_h;
  a.ox = ox;
  a.oy = oy;
  const uint32_t n_pairs = (c->height + 1) / 2;
  const uint32_t grid = (n_pairs + a.count - 1) / a.count;
  const size_t lds = size_t(a.count) * c->width * sizeof(rdl::Cx<T>);
  auto k = rdl::RowsInverse<T>;
  static std::atomic<uint64_t> attr_done{0};  // per instantiation and device
  RDL_TRY(rdl::SetMaxLdsOnce(reinterpret_cast<const void*>(k), int(rdl::kFftLdsBytes),
                             c->s->device, attr_done));
  k<<<grid, rdl::kFftThreads, lds, c->s->stream>>>(
      a, static_cast<const rdl::Cx<T>*>(spec), out, subtract);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

template <typename T>
int LaunchColumns(rdl_conv* c, const void* in, void* out, const void* kern,
                  int mode, double scale, const uint8_t* row_mask, int kern_cm,
                  int out_cm, int in_cm = 0, uint32_t out_row0 = 0,
                  uint32_t out_rows = 0xffffffffu) {
  if (c->tiled) {
    // four-step passes through the conv's scratch (tiled spectra; the
    // layout flags do not apply)
    if (row_mask) {
      rdl::SetError("LDS FFT: row masks need the row-major (float64) plans");
      return RDL_ERR_UNSUPPORTED;
    }
    RDL_TRY(EnsureSplitScratch(c, size_t(SpectrumBytes(c))));
    const uint32_t nc = c->width / 2 + 1;
    const float sc = float(scale);
    auto step = [&](bool b, const void* i, void* o, int inv) {
      return rdl::FastStepLaunch(c->s, c->steps, b, i, o, kern, c->tw_col,
                                 b ? c->ptw_b : c->ptw_a, nc, inv, sc);
    };
    if (mode != 2) {
      RDL_TRY(step(false, in, c->scratch, 0));
      RDL_TRY(step(true, c->scratch, out, 0));
      if (mode == 0) return RDL_OK;
      in = out;
    }
    RDL_TRY(step(false, in, c->scratch, 1));
    return step(true, c->scratch, out, 1);
  }
  if (c->fast_cols) {
    const uint32_t* rows = nullptr;
    const uint32_t* n_rows = nullptr;
    if (row_mask && mode != 2) {
      RDL_TRY(CompactRowsFor(c, row_mask, true));
      rows = c->rows_list;
      n_rows = c->rows_list + c->height;
      c->rows_list_mask = nullptr;  // the mask's contents may change next time
    }
    if (c->conv_cols && mode == 1 && !in_cm && (!out_cm || in != out))
      return rdl::ConvColumnsDLaunch(c->s, c->conv_cols, in, out, kern, c->tw_col,
                                     c->width / 2 + 1, kern_cm, out_cm, rows, n_rows, 0,
                                     c->height, scale, out_row0, out_rows);
    return rdl::FastColumnsLaunch(c->s, c->fast_cols, in, out, kern, c->ptw_col,
                                  c->width / 2 + 1, uint32_t(mode), in_cm, out_cm, kern_cm,
                                  rows, n_rows, 0, c->height, scale);
  }
  rdl::ColArgs a{};
  a.row_mask = row_mask;
  a.kern_cm = kern_cm ? 1u : 0u;
  a.out_cm = out_cm ? 1u : 0u;
  a.plan = c->col_plan;
  a.n_cols = c->width / 2 + 1;
  a.count = c->col_count;
  a.ld = a.n_cols;
  a.mode = mode;
  a.scale = scale;
  const uint32_t n_tiles = (a.n_cols + a.count - 1) / a.count;
  a.tiles_per_xcd = (n_tiles + 7) / 8;
  const uint32_t grid = 8 * a.tiles_per_xcd;
  const size_t lds = size_t(a.count) * c->height * sizeof(rdl::Cx<T>);
  auto k = rdl::Columns<T>;
  static std::atomic<uint64_t> attr_done{0};  // per instantiation and device
  RDL_TRY(rdl::SetMaxLdsOnce(reinterpret_cast<const void*>(k), int(rdl::kFftLdsBytes),
                             c->s->device, attr_done));
  k<<<grid, rdl::kFftThreads, lds, c->s->stream>>>(
      a, static_cast<const rdl::Cx<T>*>(in), static_cast<rdl::Cx<T>*>(out),
      static_cast<const rdl::Cx<T>*>(kern));
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

// one A or B pass over the whole spectrum
template <typename T>
int LaunchSplit(rdl_conv* c, bool pass_b, int mode, const void* in, void* out,
                const void* kern, double scale, const uint8_t* row_mask) {
  rdl::SplitArgs a{};
  a.plan = pass_b ? c->plan_n2 : c->plan_n1;
  a.n = c->height;
  a.n1 = c->n1;
  a.n2 = c->n2;
  a.n_cols = c->width / 2 + 1;
  a.ld = a.n_cols;
  a.cols = c->split_cols;
  const uint32_t sub_len = pass_b ? c->n2 : c->n1;
  // elements per workgroup: half the LDS for double (two workgroups per CU
  // overlap one's loads with the other's transform), the engine's maximum
  // for float; the padded stride must fit as well
  const uint32_t target = c->f64 ? rdl::kMaxWgElems / 2 : rdl::kMaxWgElems;
  a.groups = std::max<uint32_t>(1, target / (a.cols * (sub_len + 1)));
  a.n_groups = pass_b ? c->n1 : c->n2;
  a.groups = std::min(a.groups, a.n_groups);
  a.col_tiles = (a.n_cols + a.cols - 1) / a.cols;
  a.tw_n = c->col_plan.tw;
  a.row_mask = row_mask;
  a.scale = scale;
  a.mode = mode;
  const uint32_t grid = a.col_tiles * ((a.n_groups + a.groups - 1) / a.groups);
  const size_t lds = size_t(a.groups) * a.cols * (sub_len + 1) * sizeof(rdl::Cx<T>);
  if (pass_b) {
    auto k = rdl::ColumnsSplitB<T>;
    static std::atomic<uint64_t> attr_done{0};
    RDL_TRY(rdl::SetMaxLdsOnce(reinterpret_cast<const void*>(k),
                               int(rdl::kFftLdsBytes), c->s->device, attr_done));
    k<<<grid, rdl::kFftThreads, lds, c->s->stream>>>(
        a, static_cast<const rdl::Cx<T>*>(in), static_cast<rdl::Cx<T>*>(out),
        static_cast<const rdl::Cx<T>*>(kern));
  } else {
    auto k = rdl::ColumnsSplitA<T>;
    static std::atomic<uint64_t> attr_done{0};
    RDL_TRY(rdl::SetMaxLdsOnce(reinterpret_cast<const void*>(k),
                               int(rdl::kFftLdsBytes), c->s->device, attr_done));
    k<<<grid, rdl::kFftThreads, lds, c->s->stream>>>(
        a, static_cast<const rdl::Cx<T>*>(in), static_cast<rdl::Cx<T>*>(out));
  }
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int EnsureSplitScratch(rdl_conv* c, size_t bytes) {
  const int l = c->s->lane;
  c->scratch = c->scratch_lane[l];
  if (c->scratch_bytes[l] >= bytes) return RDL_OK;
  if (c->scratch) {
    RDL_HIP_CHECK(hipStreamSynchronize(c->s->home));
    if (c->s->aux) RDL_HIP_CHECK(hipStreamSynchronize(c->s->aux));
    RDL_HIP_CHECK(rdl::DevFree(c->scratch));
    c->scratch = c->scratch_lane[l] = nullptr;
    c->scratch_bytes[l] = 0;
  }
  RDL_HIP_CHECK(rdl::DevMalloc(&c->scratch, bytes));
  if (rdl::PoisonOn()) RDL_HIP_CHECK(hipMemsetAsync(c->scratch, 0xff, bytes, c->s->stream));
  c->scratch_lane[l] = c->scratch;
  c->scratch_bytes[l] = bytes;
  return RDL_OK;
}

// the column pass of any mode through the split passes (see SplitArgs)
template <typename T>
int LaunchColumnsSplit(rdl_conv* c, const void* in, void* out, const void* kern,
                       int mode, double scale, const uint8_t* row_mask) {
  const size_t bytes = size_t(c->width / 2 + 1) * c->height * sizeof(rdl::Cx<T>);
  if (mode == 0) {  // A: in -> scratch, B: scratch -> out (natural order)
    RDL_TRY(EnsureSplitScratch(c, bytes));
    RDL_TRY(LaunchSplit<T>(c, false, 0, in, c->scratch, nullptr, 1.0, row_mask));
    return LaunchSplit<T>(c, true, 0, c->scratch, out, nullptr, 1.0, nullptr);
  }
  if (mode == 1) {  // A: in -> out, B (fwd x K x s inv) and A^-1 in place
    RDL_TRY(LaunchSplit<T>(c, false, 0, in, out, nullptr, 1.0, row_mask));
    RDL_TRY(LaunchSplit<T>(c, true, 1, out, out, kern, scale, nullptr));
    return LaunchSplit<T>(c, false, 1, out, out, nullptr, 1.0, nullptr);
  }
  // mode 2: B (x K x s inv) from the natural spectrum into scratch, A^-1 -> out
  RDL_TRY(EnsureSplitScratch(c, bytes));
  RDL_TRY(LaunchSplit<T>(c, true, 2, in, c->scratch, kern, scale, nullptr));
  return LaunchSplit<T>(c, false, 1, c->scratch, out, nullptr, 1.0, nullptr);
}

template <typename T>
int LaunchColumnsAny(rdl_conv* c, const void* in, void* out, const void* kern,
                     int mode, double scale, const uint8_t* row_mask, int kern_cm,
                     int out_cm, int in_cm = 0) {
  if (c->split)
    return LaunchColumnsSplit<T>(c, in, out, kern, mode, scale, row_mask);
  return LaunchColumns<T>(c, in, out, kern, mode, scale, row_mask, kern_cm, out_cm, in_cm);
}

double SpectrumBytes(const rdl_conv* c) {
  if (c->tiled) return double(rdl::TiledComplexCount(c->width, c->height)) * 8.0;
  return double(c->width / 2 + 1) * c->height * (c->f64 ? 16.0 : 8.0);
}

}  // namespace

extern "C" {

int rdl_conv_create(rdl_session* s, uint32_t width, uint32_t height, int f64,
                    rdl_conv** out) {
  return rdl_conv_create_ex(s, width, height, f64, RDL_CONV_COLUMNS_AUTO, out);
}

int rdl_conv_columns_split(const rdl_conv* c) { return c && c->split ? 1 : 0; }

int rdl_conv_create_ex(rdl_session* s, uint32_t width, uint32_t height, int f64,
                       int columns, rdl_conv** out) {
  RDL_ARG_CHECK(s && out, "NULL argument");
  RDL_ARG_CHECK(columns >= RDL_CONV_COLUMNS_AUTO && columns <= RDL_CONV_COLUMNS_SPLIT,
                "bad column strategy");
  RDL_ARG_CHECK(width >= 2 && height >= 2, "bad size");
  *out = nullptr;
  const size_t esz = f64 ? 16 : 8;
  const size_t max_elems = std::min<size_t>(rdl::kFftLdsBytes / esz, rdl::kMaxWgElems);
  if (width > max_elems || height > max_elems) {
    rdl::SetError("LDS FFT: size exceeds LDS capacity");
    return RDL_ERR_UNSUPPORTED;
  }
  auto c = std::make_unique<rdl_conv>();
  c->s = s;
  c->width = width;
  c->height = height;
  c->f64 = f64 != 0;
  RDL_HIP_CHECK(hipSetDevice(s->device));
  RDL_TRY(MakePlan(c.get(), width, c->f64, &c->row_plan, &c->tw_row));
  RDL_TRY(MakePlan(c.get(), height, c->f64, &c->col_plan, &c->tw_col));
  // transforms per workgroup: fill ~64 KiB (float) / the LDS (double) so small
  // planes still give each workgroup enough work; never more than LDS holds
  const size_t budget = c->f64 ? rdl::kFftLdsBytes : 64 * 1024;
  c->row_count = uint32_t(std::max<size_t>(1, std::min<size_t>(budget / (width * esz), 64)));
  c->col_count = uint32_t(std::max<size_t>(1, std::min<size_t>(budget / (height * esz), 64)));
  c->row_count = std::min<uint32_t>(c->row_count, uint32_t(max_elems / width));
  c->col_count = std::min<uint32_t>(c->col_count, uint32_t(max_elems / height));
  // split columns: N = N1 * N2 with N1 the largest divisor <= sqrt(N)
  uint32_t n1 = 1;
  for (uint32_t d = 1; uint64_t(d) * d <= height; ++d)
    if (height % d == 0) n1 = d;
  const uint32_t n2 = height / n1;
  const bool can_split = n1 >= 4 && n2 >= 4;
  // AUTO keeps the single pass: measured on MI355X (tools/bench_fft.py) the
  // split passes are faster only for the shared-spectrum inverse in float
  // (8192^2: 606 vs 909 us) and slower for the fused convolutions
  const bool want_split = columns == RDL_CONV_COLUMNS_SPLIT;
  if (columns == RDL_CONV_COLUMNS_SPLIT && !can_split) {
    rdl::SetError("LDS FFT: column length " + std::to_string(height) +
                  " has no split into two factors >= 4");
    return RDL_ERR_UNSUPPORTED;
  }
  // compile-time-planned kernels for the sizes that have one
  // (RDL_FFT_FAST=0 keeps the runtime-plan kernels, for comparison)
  const char* fast_env = std::getenv("RDL_FFT_FAST");
  const bool fast_ok = !(fast_env && fast_env[0] == '0') && !want_split;
  if (fast_ok) {
    c->fast_cols = rdl::FindFastColumns(height, c->f64);
    if (c->f64) c->conv_cols = rdl::FindConvColumnsD(height);
    if (width % 2 == 0) c->fast_rows = rdl::FindFastRows(width, c->f64);
    // four-step column passes from this length up (RDL_FFT_STEPS_MIN,
    // experiments; below it the one-pass column kernel)
    static const uint32_t steps_min = [] {
      const char* e = std::getenv("RDL_FFT_STEPS_MIN");
      return e ? uint32_t(std::strtoul(e, nullptr, 10)) : 0u;
    }();
    if (!c->f64 && c->fast_rows && height >= steps_min) {
      c->steps = rdl::FindFastSteps(height);
      c->tiled = c->steps != nullptr;
    }
    if (c->fast_rows)
      RDL_TRY(rdl::MakePassTable(width / 2, c->fast_rows->radix, c->f64, &c->ptw_row, c->s->stream));
    if (c->fast_rows && c->fast_rows->inverse_lt)
      RDL_TRY(rdl::MakeTwiddleBase(width, &c->twd_row, c->s->stream));
    if (c->fast_cols)
      RDL_TRY(rdl::MakePassTable(height, c->fast_cols->radix, c->f64, &c->ptw_col, c->s->stream));
    if (c->steps) {
      RDL_TRY(rdl::MakePassTable(c->steps->n1, c->steps->radix_a, false, &c->ptw_a, c->s->stream));
      RDL_TRY(rdl::MakePassTable(c->steps->n2, c->steps->radix_b, false, &c->ptw_b, c->s->stream));
    }
  }
  if (want_split && can_split) {
    c->split = true;
    c->n1 = n1;
    c->n2 = n2;
    RDL_TRY(MakePlan(c.get(), n1, c->f64, &c->plan_n1, &c->tw_n1));
    RDL_TRY(MakePlan(c.get(), n2, c->f64, &c->plan_n2, &c->tw_n2));
    // 256-byte row segments, as many as the sub-lengths allow
    c->split_cols = std::max<uint32_t>(
        1, std::min<uint32_t>(c->f64 ? 16 : 32,
                              rdl::kMaxWgElems / (std::max(n1, n2) + 1)));
  }
  // RDL_LOG_FFT_PLANS=1: one line per plan (sizes, precision, which kernels)
  static const bool log_plans = [] {
    const char* e = std::getenv("RDL_LOG_FFT_PLANS");
    return e && e[0] == '1';
  }();
  if (log_plans)
    std::fprintf(stderr, "[fft-plan] %ux%u %s rows=%s cols=%s\n", width, height,
                 c->f64 ? "f64" : "f32", c->fast_rows ? "fast" : "runtime",
                 c->tiled ? "four-step" : c->fast_cols ? "fast" : "runtime");
  *out = c.release();
  return RDL_OK;
}

int rdl_conv_destroy(rdl_conv* c) {
  if (!c) return RDL_OK;
  if (rdl::ShutDown()) return RDL_OK;  // its blocks were released by rdl_shutdown
  (void)hipStreamSynchronize(c->s->stream);
  if (c->tw_row) (void)rdl::DevFree(c->tw_row);
  if (c->tw_col) (void)rdl::DevFree(c->tw_col);
  if (c->tw_n1) (void)rdl::DevFree(c->tw_n1);
  if (c->tw_n2) (void)rdl::DevFree(c->tw_n2);
  for (void* p : c->scratch_lane)
    if (p) (void)rdl::DevFree(p);
  if (c->rows_list) (void)rdl::DevFree(c->rows_list);
  for (void* p : {c->ptw_row, c->ptw_col, c->ptw_a, c->ptw_b, c->twd_row, c->cos_w, c->cos_h,
                  c->real_a.ptr})
    if (p) (void)rdl::DevFree(p);
  delete c;
  return RDL_OK;
}

size_t rdl_conv_spectrum_bytes(const rdl_conv* c) {
  return c ? size_t(SpectrumBytes(c)) : 0;
}

int rdl_conv_rows_forward(rdl_conv* c, const float* d_in, uint32_t in_w,
                          uint32_t in_h, uint32_t ox, uint32_t oy, void* d_spec) {
  RDL_ARG_CHECK(c && d_in && d_spec, "NULL argument");
  RDL_ARG_CHECK(uint64_t(ox) + in_w <= c->width && uint64_t(oy) + in_h <= c->height,
                "input window outside the plane");
  rdl::ScopedTiming t(c->s, c->f64 ? "conv64_rows" : "conv_rows",
                      double(in_w) * in_h * 4.0 + SpectrumBytes(c));
  return c->f64 ? LaunchRowsForward<double>(c, d_in, in_w, in_h, ox, oy, d_spec, nullptr)
                : LaunchRowsForward<float>(c, d_in, in_w, in_h, ox, oy, d_spec, nullptr);
}

int rdl_conv_rows_forward_masked(rdl_conv* c, const float* d_in, uint32_t in_w,
                                 uint32_t in_h, uint32_t ox, uint32_t oy,
                                 void* d_spec, const uint8_t* d_row_mask) {
  RDL_ARG_CHECK(c && d_in && d_spec && d_row_mask, "NULL argument");
  RDL_ARG_CHECK(uint64_t(ox) + in_w <= c->width && uint64_t(oy) + in_h <= c->height,
                "input window outside the plane");
  // bytes depend on the mask's occupancy (known only on the device): the
  // sparse family reports time and launches, not bandwidth
  rdl::ScopedTiming t(c->s, c->f64 ? "conv64_rows_sparse" : "conv_rows_sparse", 0.0);
  return c->f64 ? LaunchRowsForward<double>(c, d_in, in_w, in_h, ox, oy, d_spec,
                                            d_row_mask)
                : LaunchRowsForward<float>(c, d_in, in_w, in_h, ox, oy, d_spec,
                                           d_row_mask);
}

int rdl_conv_columns(rdl_conv* c, const void* d_in, void* d_out,
                     const void* d_kernel, int mode, double scale) {
  RDL_ARG_CHECK(c && d_in && d_out, "NULL argument");
  RDL_ARG_CHECK(mode >= 0 && mode <= 2, "mode must be 0, 1 or 2");
  RDL_ARG_CHECK(mode == 0 || d_kernel, "kernel spectrum required");
  const double sb = SpectrumBytes(c);
  rdl::ScopedTiming t(c->s, c->f64 ? "conv64_cols" : "conv_cols",
                      mode == 0 ? 2.0 * sb : 3.0 * sb);
  return c->f64 ? LaunchColumnsAny<double>(c, d_in, d_out, d_kernel, mode, scale,
                                           nullptr, 0, 0)
                : LaunchColumnsAny<float>(c, d_in, d_out, d_kernel, mode, scale,
                                          nullptr, 0, 0);
}

int rdl_conv_columns_ex(rdl_conv* c, const void* d_in, void* d_out,
                        const void* d_kernel, int mode, double scale,
                        const uint8_t* d_row_mask, int kernel_layout,
                        int out_layout) {
  RDL_ARG_CHECK(c && d_in && d_out, "NULL argument");
  RDL_ARG_CHECK(mode >= 0 && mode <= 2, "mode must be 0, 1 or 2");
  RDL_ARG_CHECK(mode == 0 || d_kernel, "kernel spectrum required");
  RDL_ARG_CHECK(out_layout == RDL_CONV_ROW_MAJOR ||
                    ((mode == 0 || (mode == 1 && c->conv_cols)) && d_out != d_in),
                "a column-major output needs mode 0 (or mode 1 with a float64 "
                "convolution-column plan) and a separate output");
  RDL_ARG_CHECK(kernel_layout == RDL_CONV_ROW_MAJOR ||
                    kernel_layout == RDL_CONV_COL_MAJOR,
                "bad kernel layout");
  RDL_ARG_CHECK(!c->split || (kernel_layout == RDL_CONV_ROW_MAJOR &&
                              out_layout == RDL_CONV_ROW_MAJOR),
                "split column plans use the row-major layout only");
  const double sb = SpectrumBytes(c);
  // with a row mask the input reads are skipped for the zero rows: count
  // the kernel read and the output write only (a lower bound)
  const char* fam = d_row_mask ? (c->f64 ? "conv64_cols_sparse" : "conv_cols_sparse")
                               : (c->f64 ? "conv64_cols" : "conv_cols");
  const double bytes = d_row_mask ? (mode == 0 ? sb : 2.0 * sb)
                                  : (mode == 0 ? 2.0 * sb : 3.0 * sb);
  rdl::ScopedTiming t(c->s, fam, bytes);
  const int kcm = kernel_layout == RDL_CONV_COL_MAJOR;
  const int ocm = out_layout == RDL_CONV_COL_MAJOR;
  return c->f64 ? LaunchColumnsAny<double>(c, d_in, d_out, d_kernel, mode, scale,
                                           d_row_mask, kcm, ocm)
                : LaunchColumnsAny<float>(c, d_in, d_out, d_kernel, mode, scale,
                                          d_row_mask, kcm, ocm);
}

int rdl_conv_columns_window(rdl_conv* c, const void* d_in, void* d_out,
                            const void* d_kernel, double scale, const uint8_t* d_row_mask,
                            int kernel_layout, uint32_t out_row0, uint32_t out_rows,
                            int kernel_f32) {
  RDL_ARG_CHECK(c && d_in && d_out && d_kernel, "NULL argument");
  RDL_ARG_CHECK(uint64_t(out_row0) + out_rows <= c->height, "output rows outside the plane");
  RDL_ARG_CHECK(kernel_layout == RDL_CONV_ROW_MAJOR || kernel_layout == RDL_CONV_COL_MAJOR,
                "bad kernel layout");
  const bool convd = c->f64 && c->conv_cols && !c->split;
  RDL_ARG_CHECK(!kernel_f32 || convd, "a float kernel needs a float64 convolution-column plan");
  if (!convd)
    return rdl_conv_columns_ex(c, d_in, d_out, d_kernel, 1, scale, d_row_mask, kernel_layout,
                               RDL_CONV_ROW_MAJOR);
  const double sb = SpectrumBytes(c);
  const double win = sb * double(out_rows) / double(c->height);
  const double kb = kernel_f32 ? 0.5 * sb : sb;
  const char* fam = d_row_mask ? "conv64_cols_sparse" : "conv64_cols";
  rdl::ScopedTiming t(c->s, fam, d_row_mask ? kb + win : kb + sb + win);
  const uint32_t* rows = nullptr;
  const uint32_t* n_rows = nullptr;
  if (d_row_mask) {
    RDL_TRY(CompactRowsFor(c, d_row_mask, true));
    rows = c->rows_list;
    n_rows = c->rows_list + c->height;
    c->rows_list_mask = nullptr;  // the mask's contents may change next time
  }
  return rdl::ConvColumnsDLaunch(c->s, c->conv_cols, d_in, d_out, d_kernel, c->tw_col,
                                 c->width / 2 + 1, kernel_layout == RDL_CONV_COL_MAJOR, 0, rows,
                                 n_rows, 0, c->height, scale, out_row0, out_rows,
                                 kernel_f32 != 0);
}

namespace {
// the float64 convolution-column plans keep the correction's spectrum in the
// tiled layout (RDL_CONV64_TILED=0: row-major, for comparison)
bool Tiled64(const rdl_conv* c) {
  static const bool on = [] {
    const char* e = std::getenv("RDL_CONV64_TILED");
    return !(e && e[0] == '0');
  }();
  return on && c->f64 && c->conv_cols && c->fast_rows && !c->split && !c->tiled;
}
}  // namespace

size_t rdl_conv_convolve_subtract_bytes(const rdl_conv* c) {
  if (!c) return 0;
  return Tiled64(c) ? rdl::TiledComplexCount(c->width, c->height) * 16
                    : size_t(SpectrumBytes(c));
}

int rdl_conv_convolve_subtract(rdl_conv* c, const float* d_image, uint32_t img_w,
                               uint32_t img_h, uint32_t ox, uint32_t oy,
                               const void* d_kernel, int kernel_layout, int kernel_f32,
                               double scale, const uint8_t* d_row_mask, void* d_work,
                               float* d_residual) {
  RDL_ARG_CHECK(c && d_image && d_kernel && d_work && d_residual, "NULL argument");
  RDL_ARG_CHECK(uint64_t(ox) + img_w <= c->width && uint64_t(oy) + img_h <= c->height,
                "image window outside the plane");
  if (!Tiled64(c)) {
    RDL_TRY(d_row_mask
                ? rdl_conv_rows_forward_masked(c, d_image, img_w, img_h, ox, oy, d_work,
                                               d_row_mask)
                : rdl_conv_rows_forward(c, d_image, img_w, img_h, ox, oy, d_work));
    RDL_TRY(rdl_conv_columns_window(c, d_work, d_work, d_kernel, scale, d_row_mask,
                                    kernel_layout, oy, img_h, kernel_f32));
    return rdl_conv_rows_inverse(c, d_work, d_residual, img_w, img_h, ox, oy, 1);
  }
  RDL_ARG_CHECK(kernel_layout == RDL_CONV_ROW_MAJOR || kernel_layout == RDL_CONV_COL_MAJOR,
                "bad kernel layout");
  // the same three passes on the tiled layout: the row passes move whole
  // 256-byte tile rows, the column pass reads and writes column c at a
  // 256-byte stride inside its tile (not a full row stride)
  const double sb = SpectrumBytes(c);
  const double win = sb * double(img_h) / double(c->height);
  const uint32_t* rows = nullptr;
  const uint32_t* n_rows = nullptr;
  {
    rdl::ScopedTiming t(c->s, d_row_mask ? "conv64_rows_sparse" : "conv64_rows",
                        d_row_mask ? 0.0 : double(img_w) * img_h * 4.0 + win);
    if (d_row_mask) {
      RDL_TRY(CompactRowsFor(c, d_row_mask, false));
      rows = c->rows_list;
      n_rows = c->rows_list + c->height;
    }
    RDL_TRY(rdl::FastRowsForwardLaunch(c->s, c->fast_rows, d_image, d_work, c->tw_row,
                                       c->ptw_row, c->height, img_w, img_h, ox, oy, rows,
                                       n_rows, 1, c->twd_row, 0));
  }
  {
    const double kb = kernel_f32 ? 0.5 * sb : sb;
    rdl::ScopedTiming t(c->s, d_row_mask ? "conv64_cols_sparse" : "conv64_cols",
                        d_row_mask ? kb + win : kb + 2.0 * win);
    // unmasked: the rows outside the window are zero (never written)
    RDL_TRY(rdl::ConvColumnsDLaunch(c->s, c->conv_cols, d_work, d_work, d_kernel, c->tw_col,
                                    c->width / 2 + 1, kernel_layout == RDL_CONV_COL_MAJOR, 0,
                                    rows, n_rows, oy, img_h, scale, oy, img_h,
                                    kernel_f32 != 0, true));
    c->rows_list_mask = nullptr;  // the mask's contents may change next time
  }
  rdl::ScopedTiming t(c->s, "conv64_rows", win + double(img_w) * img_h * 8.0);
  return rdl::FastRowsInverseLaunch(c->s, c->fast_rows, d_work, d_residual, c->tw_row,
                                    c->ptw_row, c->height, img_w, img_h, ox, oy, 1, 1, nullptr,
                                    c->twd_row);
}

int rdl_conv_columns_layout(rdl_conv* c, const void* d_in, void* d_out,
                            const void* d_kernel, int mode, double scale,
                            const uint8_t* d_row_mask, int in_layout,
                            int kernel_layout, int out_layout) {
  RDL_ARG_CHECK(c && d_in && d_out, "NULL argument");
  RDL_ARG_CHECK(mode >= 0 && mode <= 2, "mode must be 0, 1 or 2");
  RDL_ARG_CHECK(mode == 0 || d_kernel, "kernel spectrum required");
  for (int l : {in_layout, kernel_layout, out_layout})
    RDL_ARG_CHECK(l == RDL_CONV_ROW_MAJOR || l == RDL_CONV_COL_MAJOR, "bad layout");
  RDL_ARG_CHECK(c->tiled || in_layout == RDL_CONV_ROW_MAJOR || mode == 2,
                "a column-major input is a mode-2 spectrum");
  RDL_ARG_CHECK(c->tiled || in_layout == out_layout || d_out != d_in,
                "changing the layout needs a separate output");
  if (!c->fast_cols && !c->tiled) {
    if (in_layout == RDL_CONV_ROW_MAJOR && (out_layout == RDL_CONV_ROW_MAJOR || mode == 0))
      return rdl_conv_columns_ex(c, d_in, d_out, d_kernel, mode, scale, d_row_mask,
                                 kernel_layout, out_layout);
    rdl::SetError("LDS FFT: this layout needs the compile-time-planned column kernels");
    return RDL_ERR_UNSUPPORTED;
  }
  const double sb = SpectrumBytes(c);
  const char* fam = d_row_mask ? (c->f64 ? "conv64_cols_sparse" : "conv_cols_sparse")
                               : (c->f64 ? "conv64_cols" : "conv_cols");
  const double bytes = d_row_mask ? (mode == 0 ? sb : 2.0 * sb)
                                  : (mode == 0 ? 2.0 * sb : 3.0 * sb);
  rdl::ScopedTiming t(c->s, fam, bytes);
  const int icm = in_layout == RDL_CONV_COL_MAJOR;
  const int kcm = kernel_layout == RDL_CONV_COL_MAJOR;
  const int ocm = out_layout == RDL_CONV_COL_MAJOR;
  return c->f64 ? LaunchColumnsAny<double>(c, d_in, d_out, d_kernel, mode, scale,
                                           d_row_mask, kcm, ocm, icm)
                : LaunchColumnsAny<float>(c, d_in, d_out, d_kernel, mode, scale,
                                          d_row_mask, kcm, ocm, icm);
}

int rdl_conv_fast(const rdl_conv* c) {
  if (!c) return 0;
  return (c->fast_cols ? RDL_CONV_FAST_COLUMNS : 0) | (c->fast_rows ? RDL_CONV_FAST_ROWS : 0) |
         (c->tiled ? RDL_CONV_FAST_TILED : 0) |
         (c->f64 && c->conv_cols && !c->split ? RDL_CONV_FAST_CONVD : 0);
}

int rdl_conv_rows_inverse(rdl_conv* c, const void* d_spec, float* d_out,
                          uint32_t out_w, uint32_t out_h, uint32_t ox, uint32_t oy,
                          int subtract) {
  RDL_ARG_CHECK(c && d_spec && d_out, "NULL argument");
  RDL_ARG_CHECK(uint64_t(ox) + out_w <= c->width && uint64_t(oy) + out_h <= c->height,
                "output window outside the plane");
  rdl::ScopedTiming t(c->s, c->f64 ? "conv64_rows" : "conv_rows",
                      SpectrumBytes(c) + double(out_w) * out_h * (subtract ? 8.0 : 4.0));
  return c->f64 ? LaunchRowsInverse<double>(c, d_spec, d_out, out_w, out_h, ox, oy,
                                            subtract)
                : LaunchRowsInverse<float>(c, d_spec, d_out, out_w, out_h, ox, oy,
                                           subtract);
}

int rdl_conv_rows_inverse_peak(rdl_conv* c, const void* d_spec, float* d_out,
                               uint32_t out_w, uint32_t out_h, uint32_t ox, uint32_t oy,
                               uint32_t h_border, uint32_t v_border, int allow_negative,
                               const uint8_t* d_mask, uint32_t slot) {
  RDL_ARG_CHECK(c && d_spec && d_out, "NULL argument");
  RDL_ARG_CHECK(uint64_t(ox) + out_w <= c->width && uint64_t(oy) + out_h <= c->height,
                "output window outside the plane");
  RDL_ARG_CHECK(slot < RDL_PEAK_SLOTS, "peak slot out of range");
  RDL_ARG_CHECK(uint64_t(out_w) * out_h < 0xffffffffull, "image too large for 32-bit index");
  if (!c->fast_rows) {
    rdl::SetError("fused peak search needs the compile-time-planned row kernels");
    return RDL_ERR_UNSUPPORTED;
  }
  rdl_session* s = c->s;
  // the box of rdl_find_peak(start_y 0, end_y out_h) (peak_finder.cc:27-32)
  rdl::RowPeak pk{};
  pk.xs = h_border;
  pk.xe = out_w - h_border;
  pk.ys = v_border;
  pk.ye = out_h - v_border;
  if (pk.xe < pk.xs) pk.xe = pk.xs;
  if (pk.ye < pk.ys) pk.ye = pk.ys;
  if (pk.xe > out_w) pk.xe = out_w;
  if (pk.ye > out_h) pk.ye = out_h;
  pk.mask = d_mask;
  pk.allow_negative = allow_negative;
  // one partials area per peak slot: the scales' searches may run on two
  // session lanes at once
  const size_t rows = std::max<size_t>(out_h, 1);
  RDL_TRY(s->EnsureScratch(s->partials, RDL_PEAK_SLOTS * rows * sizeof(uint64_t)));
  pk.partials = static_cast<uint64_t*>(s->partials.ptr) + slot * rows;
  uint32_t n_partials = 1;
  {
    rdl::ScopedTiming t(s, "conv_rows",
                        SpectrumBytes(c) + double(out_w) * out_h * 4.0);
    if (out_h == 0)
      RDL_HIP_CHECK(hipMemsetAsync(pk.partials, 0, sizeof(uint64_t), s->stream));
    else
      RDL_TRY(rdl::FastRowsInverseLaunch(s, c->fast_rows, d_spec, d_out, c->tw_row,
                                         c->ptw_row, c->height, out_w, out_h, ox, oy, 0,
                                         c->tiled ? 1 : 0, &pk, c->twd_row, &n_partials));
  }
  return rdl::LaunchPeakFinal(s, pk.partials, std::max<uint32_t>(n_partials, 1), d_out, out_w,
                              out_h, 1, d_mask != nullptr, rdl::PeakSlot(s, slot));
}

int rdl_conv_forward(rdl_conv* c, const float* d_in, void* d_spec) {
  RDL_TRY(rdl_conv_rows_forward(c, d_in, c->width, c->height, 0, 0, d_spec));
  return rdl_conv_columns(c, d_spec, d_spec, nullptr, 0, 1.0);
}

size_t rdl_conv_real_kernel_bytes(const rdl_conv* c) {
  return c && c->tiled ? rdl::TiledComplexCount(c->width, c->height) * sizeof(float) : 0;
}

int rdl_conv_real_kernel(rdl_conv* c, const float* h_shape, uint32_t n, void* d_kernel) {
  RDL_ARG_CHECK(c && h_shape && d_kernel, "NULL argument");
  if (!c->tiled) {
    rdl::SetError("rdl_conv_real_kernel: needs a four-step (tiled) float plan");
    return RDL_ERR_UNSUPPORTED;
  }
  RDL_ARG_CHECK(n % 2 == 1 && n <= c->width && n <= c->height,
                "kernel side must be odd and fit the plane");
  for (uint32_t y = 0; y < n; ++y)  // the evaluation assumes the symmetry
    for (uint32_t x = 0; x < n; ++x) {
      const float v = h_shape[x + y * n];
      RDL_ARG_CHECK(v == h_shape[(n - 1 - x) + y * n] && v == h_shape[x + (n - 1 - y) * n],
                    "rdl_conv_real_kernel: the kernel is not symmetric in x and y");
    }
  rdl_session* s = c->s;
  if (!c->cos_w) RDL_TRY(rdl::MakeCosTable(c->width, &c->cos_w, c->s->stream));
  if (!c->cos_h) RDL_TRY(rdl::MakeCosTable(c->height, &c->cos_h, c->s->stream));
  const size_t shape_bytes = size_t(n) * n * sizeof(float);
  RDL_TRY(s->EnsureScratch(s->kernel, shape_bytes));
  RDL_HIP_CHECK(hipMemcpyAsync(s->kernel.ptr, h_shape, shape_bytes, hipMemcpyHostToDevice,
                               s->stream));
  RDL_TRY(s->EnsureScratch(c->real_a, size_t(n / 2 + 1) * (c->width / 2 + 1) * sizeof(double)));
  RDL_TRY(rdl::RealKernelLaunch(s, static_cast<const float*>(s->kernel.ptr), n, c->width,
                                c->height, c->cos_w, c->cos_h, c->real_a.ptr,
                                static_cast<float*>(d_kernel)));
  // the shape scratch is host-written next time: finish with it first
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

int rdl_conv_forward_half(rdl_conv* c, const float* d_in, uint32_t in_w, uint32_t in_h,
                          uint32_t ox, uint32_t oy, void* d_half) {
  RDL_ARG_CHECK(c && d_in && d_half, "NULL argument");
  if (!c->tiled) {
    rdl::SetError("rdl_conv_forward_half: needs a four-step (tiled) float plan");
    return RDL_ERR_UNSUPPORTED;
  }
  const double sb = SpectrumBytes(c);
  // rows into the lane's scratch, A from there into d_half (A is not
  // in-place safe: rows n2 + N2 n1 -> k1 N2 + n2)
  RDL_TRY(EnsureSplitScratch(c, size_t(sb)));
  void* rows = c->scratch;
  RDL_TRY(rdl_conv_rows_forward(c, d_in, in_w, in_h, ox, oy, rows));
  // algorithmic bytes (the one-pass minimum of the column work, counted per
  // iteration as 2 sb for the forward columns + 2.5 sb per scale: spectrum
  // read, real kernel read, result write), attributed to the three launches
  // as A 1 sb, B* 1 + 1.5 sb per scale, A* 1 sb; the four-step passes move
  // 2, 1 + 1.5 per scale and 2 (the intermediates): PMC shows the ratio
  rdl::ScopedTiming t(c->s, "conv_cols", sb);
  return rdl::FastStepLaunch(c->s, c->steps, false, rows, d_half, nullptr, c->tw_col, c->ptw_a,
                             c->width / 2 + 1, 0, 1.0f);
}

int rdl_conv_scales(rdl_conv* c, const void* d_half, uint32_t n_scales,
                    const void* const* d_kernels, void* const* d_outs, double scale) {
  RDL_ARG_CHECK(c && d_half && (n_scales == 0 || (d_kernels && d_outs)), "NULL argument");
  if (!c->tiled) {
    rdl::SetError("rdl_conv_scales: needs a four-step (tiled) float plan");
    return RDL_ERR_UNSUPPORTED;
  }
  for (uint32_t i = 0; i < n_scales; ++i)
    RDL_ARG_CHECK(d_kernels[i] && d_outs[i] && d_outs[i] != d_half, "bad kernel / output");
  const double sb = SpectrumBytes(c);
  // algorithmic (see rdl_conv_forward_half): the forward columns' write, and
  // per scale the spectrum and real-kernel reads
  rdl::ScopedTiming t(c->s, "conv_cols", sb + n_scales * 1.5 * sb);
  return rdl::FastScalesLaunch(c->s, c->steps, d_half, c->tw_col, c->ptw_b, c->width / 2 + 1,
                               n_scales, reinterpret_cast<const float* const*>(d_kernels),
                               d_outs, float(scale));
}

int rdl_conv_scale_finish(rdl_conv* c, const void* d_in, void* d_out) {
  RDL_ARG_CHECK(c && d_in && d_out && d_in != d_out, "NULL or aliased argument");
  if (!c->tiled) {
    rdl::SetError("rdl_conv_scale_finish: needs a four-step (tiled) float plan");
    return RDL_ERR_UNSUPPORTED;
  }
  // algorithmic (see rdl_conv_forward_half): the scale's result write
  rdl::ScopedTiming t(c->s, "conv_cols", SpectrumBytes(c));
  return rdl::FastStepAInvLaunch(c->s, c->steps, d_in, d_out, c->ptw_a, c->width / 2 + 1);
}

}  // extern "C"
