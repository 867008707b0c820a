// Compile-time-planned FFT kernels for the hot transform sizes of the
// multiscale path: the float64 padded residual correction
// (SubMinorLoop::CorrectResidualDirty, cpp/algorithms/subminor_loop.cc:
// 195-218, sizes utils::GetConvolutionSize(scale, W, 1.1)) and the float32
// scale convolutions (MultiScaleTransforms::Transform,
// cpp/algorithms/multiscale/multiscale_transforms.cc:9-21, size W x H).
// Same data layouts and results (to rounding) as lds_fft.hip's runtime-plan
// kernels, which remain the path for every other size.
//
// Why a second engine: the runtime-plan kernels park their waves ~65 % of
// the time (rocprofv3 SQ_WAIT_ANY on MI355X): one 145 KiB double column or
// row pair per CU, the global loads staged through LDS behind a full
// __syncthreads(), generic index arithmetic and out-of-line passes. Here
//   * every pass is specialised at compile time (radix, span, butterflies per
//     thread), fully inlined, twiddles issued before the LDS reads,
//   * workgroups are persistent (one per CU slot) and keep their global
//     traffic in flight across LDS-only barriers: the kernel spectrum column
//     is loaded into registers while the forward column transform runs, the
//     next row pair's spectrum while the current one is transformed,
//   * rows outside the output window are never transformed, sparse inputs
//     (the sub-minor model's occupied rows) are read from a compacted list.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <vector>

#include "fft_dft.h"
#include "fft_fast.h"
#include "rdl_internal.h"

namespace rdl {
namespace ff {

// Orders LDS only: __syncthreads() would also drain the prefetch loads.
__device__ __forceinline__ void LdsSync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS slot of logical element i of a transform (see kFastPadShift)
template <typename T>
__device__ __forceinline__ uint32_t Lx(uint32_t i) {
  if constexpr (sizeof(T) == 4)
    return i + (i >> kFastPadShift);
  else
    return i;
}

// One Stockham pass (radix R, span NS) over a length-N transform in LDS, in
// place (inputs read to registers before the barrier). Twiddles come from the
// plan's pass table (MakePassTable, host): pass p's W_N^{k (q+1) M} at
// ptw[OFF + q NS + k], so a wave's load for one q is one contiguous run.
// Float reads every power; double reads w and builds w^r by recurrence (error
// ~1e-15, far below the float rounding of the result).
template <typename T, uint32_t TH, uint32_t N, uint32_t R, uint32_t NS, uint32_t OFF>
__device__ __forceinline__ void Pass(Cx<T>* buf, const Cx<T>* __restrict__ ptw,
                                     uint32_t tid) {
  constexpr uint32_t NB = N / R;
  constexpr uint32_t BPT = (NB + TH - 1) / TH;
  constexpr bool kTable = sizeof(T) == 4;
  constexpr uint32_t NW = NS > 1 ? (kTable ? R - 1 : 1) : 1;
  Cx<T> v[BPT][R];
  Cx<T> w[BPT][NW];
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
      if constexpr (NS > 1) {
        const uint32_t k = j % NS;
#pragma unroll
        for (uint32_t q = 0; q < NW; ++q) w[i][q] = ptw[OFF + q * NS + k];
      }
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) v[i][r] = buf[Lx<T>(j + r * NB)];
    }
  }
  LdsSync();
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
      const uint32_t k = j % NS;
      if constexpr (NS > 1) {
        if constexpr (kTable) {
#pragma unroll
          for (uint32_t r = 1; r < R; ++r) v[i][r] = Mul(v[i][r], w[i][r - 1]);
        } else {
          Cx<T> wr = w[i][0];
          v[i][1] = Mul(v[i][1], wr);
#pragma unroll
          for (uint32_t r = 2; r < R; ++r) {
            wr = Mul(wr, w[i][0]);
            v[i][r] = Mul(v[i][r], wr);
          }
        }
      }
      Dft<T, int(R)>::Run(v[i]);
      const uint32_t d = (j / NS) * NS * R + k;
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) buf[Lx<T>(d + r * NS)] = v[i][r];
    }
  }
  LdsSync();
}

// entries of pass (radix R, span NS) in the pass table
constexpr uint32_t PassTableSize(uint32_t R, uint32_t NS) { return NS > 1 ? NS * (R - 1) : 0; }

template <typename T, uint32_t TH, uint32_t N, uint32_t OFF, uint32_t NS, uint32_t R,
          uint32_t... Rest>
__device__ __forceinline__ void Fft(Cx<T>* buf, const Cx<T>* __restrict__ ptw,
                                    uint32_t tid) {
  Pass<T, TH, N, R, NS, OFF>(buf, ptw, tid);
  if constexpr (sizeof...(Rest) > 0)
    Fft<T, TH, N, OFF + PassTableSize(R, NS), NS * R, Rest...>(buf, ptw, tid);
}

template <uint32_t... Rs>
constexpr uint32_t Product() {
  return (Rs * ... * 1u);
}

// Float transforms with their twiddles computed from two small double tables
// in LDS instead of loaded per butterfly from the global pass tables (which
// made three quarters of the row kernels' load instructions, PMC
// SQ_INSTS_VMEM_RD): W_L^e = D1[e >> 6] x D2[e & 63] in double (exact table
// entries), powers by recurrence in double, each rounded to float once —
// the float pass table's values (long double, rounded) but for the rare
// rounding tie. L = SC x N (the base length, rows: 2H).
constexpr uint32_t kTwdLo = 64;
struct TwdLds {
  const Cx<double>* d1;  // W_L^{64 i}
  const Cx<double>* d2;  // W_L^i, i < 64
};
__device__ __forceinline__ Cx<double> TwD(const TwdLds& t, uint32_t e) {
  return Mul(t.d1[e / kTwdLo], t.d2[e % kTwdLo]);
}
__device__ __forceinline__ Cx<float> ToF(Cx<double> v) { return {float(v.x), float(v.y)}; }

template <uint32_t TH, uint32_t N, uint32_t R, uint32_t NS, uint32_t SC>
__device__ __forceinline__ void PassL(Cx<float>* buf, const TwdLds& td, uint32_t tid) {
  constexpr uint32_t NB = N / R;
  constexpr uint32_t BPT = (NB + TH - 1) / TH;
  Cx<float> v[BPT][R];
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) v[i][r] = buf[Lx<float>(j + r * NB)];
    }
  }
  LdsSync();
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
      const uint32_t k = j % NS;
      if constexpr (NS > 1) {
        const Cx<double> w = TwD(td, k * (N / (NS * R)) * SC);
        Cx<double> wr = w;
        v[i][1] = Mul(v[i][1], ToF(wr));
#pragma unroll
        for (uint32_t r = 2; r < R; ++r) {
          wr = Mul(wr, w);
          v[i][r] = Mul(v[i][r], ToF(wr));
        }
      }
      Dft<float, int(R)>::Run(v[i]);
      const uint32_t d = (j / NS) * NS * R + k;
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) buf[Lx<float>(d + r * NS)] = v[i][r];
    }
  }
  LdsSync();
}

template <uint32_t TH, uint32_t N, uint32_t SC, uint32_t NS, uint32_t R, uint32_t... Rest>
__device__ __forceinline__ void FftL(Cx<float>* buf, const TwdLds& td, uint32_t tid) {
  PassL<TH, N, R, NS, SC>(buf, td, tid);
  if constexpr (sizeof...(Rest) > 0) FftL<TH, N, SC, NS * R, Rest...>(buf, td, tid);
}

// The same transform with its pass twiddles computed ONCE per workgroup (the
// persistent row kernels transform many rows, and a thread's butterflies
// are the same in every row): PassL's float values (double recurrence, each
// power rounded once), kept in registers for a last pass with one butterfly
// per thread and in a small LDS table [q NS + k] for every other pass with
// twiddles. Same values, same arithmetic: bit-identical to FftL, without
// its per-row double math (the row kernels' largest VALU cost).
template <uint32_t NS, uint32_t R, uint32_t... Rest>
constexpr uint32_t CachedTableSize(uint32_t th, uint32_t n) {
  // entries of the LDS tables: every pass with NS > 1 except a last pass
  // with one butterfly per thread (registers)
  const bool last = sizeof...(Rest) == 0;
  const bool regs = last && (n / R + th - 1) / th == 1;
  const uint32_t here = (NS > 1 && !regs) ? NS * (R - 1) : 0;
  if constexpr (sizeof...(Rest) > 0)
    return here + CachedTableSize<NS * R, Rest...>(th, n);
  else
    return here;
}

template <uint32_t... Rs>
constexpr uint32_t LastRadix() {
  constexpr uint32_t r[] = {Rs...};
  return r[sizeof...(Rs) - 1];
}

template <uint32_t TH, uint32_t N, uint32_t SC, uint32_t NS, uint32_t R, uint32_t... Rest>
__device__ __forceinline__ void InitTwiddles(const TwdLds& td, Cx<float>* table, uint32_t off,
                                             Cx<float>* last, uint32_t tid) {
  constexpr uint32_t NB = N / R;
  constexpr bool kLast = sizeof...(Rest) == 0;
  constexpr bool kRegs = kLast && (NB + TH - 1) / TH == 1;
  if constexpr (NS > 1) {
    if constexpr (kRegs) {
      const uint32_t k = tid % NS;
      const Cx<double> w = TwD(td, k * (N / (NS * R)) * SC);
      Cx<double> wr = w;
      last[0] = ToF(wr);
#pragma unroll
      for (uint32_t r = 2; r < R; ++r) {
        wr = Mul(wr, w);
        last[r - 1] = ToF(wr);
      }
    } else {
      for (uint32_t k = tid; k < NS; k += TH) {
        const Cx<double> w = TwD(td, k * (N / (NS * R)) * SC);
        Cx<double> wr = w;
        table[off + k] = ToF(wr);
        for (uint32_t r = 2; r < R; ++r) {
          wr = Mul(wr, w);
          table[off + (r - 1) * NS + k] = ToF(wr);
        }
      }
    }
  }
  if constexpr (!kLast)
    InitTwiddles<TH, N, SC, NS * R, Rest...>(td, table,
                                             off + ((NS > 1 && !kRegs) ? NS * (R - 1) : 0), last,
                                             tid);
}

template <uint32_t TH, uint32_t N, uint32_t R, uint32_t NS, bool kLast>
__device__ __forceinline__ void PassC(Cx<float>* buf, const Cx<float>* table, uint32_t off,
                                      const Cx<float>* last, uint32_t tid) {
  constexpr uint32_t NB = N / R;
  constexpr uint32_t BPT = (NB + TH - 1) / TH;
  constexpr bool kRegs = kLast && BPT == 1;
  Cx<float> v[BPT][R];
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) v[i][r] = buf[Lx<float>(j + r * NB)];
    }
  }
  LdsSync();
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
      const uint32_t k = j % NS;
      if constexpr (NS > 1) {
#pragma unroll
        for (uint32_t r = 1; r < R; ++r)
          v[i][r] = Mul(v[i][r], kRegs ? last[r - 1] : table[off + (r - 1) * NS + k]);
      }
      Dft<float, int(R)>::Run(v[i]);
      const uint32_t d = (j / NS) * NS * R + k;
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) buf[Lx<float>(d + r * NS)] = v[i][r];
    }
  }
  LdsSync();
}

template <uint32_t TH, uint32_t N, uint32_t NS, uint32_t R, uint32_t... Rest>
__device__ __forceinline__ void FftC(Cx<float>* buf, const Cx<float>* table, uint32_t off,
                                     const Cx<float>* last, uint32_t tid) {
  constexpr bool kLast = sizeof...(Rest) == 0;
  constexpr bool kRegs = kLast && (N / R + TH - 1) / TH == 1;
  PassC<TH, N, R, NS, kLast>(buf, table, off, last, tid);
  if constexpr (!kLast)
    FftC<TH, N, NS * R, Rest...>(buf, table, off + ((NS > 1 && !kRegs) ? NS * (R - 1) : 0),
                                 last, tid);
}

// ------------------------------------------------------------- columns
// One spectrum column of length N per workgroup round (persistent grid).
struct ColArgs {
  uint32_t n_cols;    // spectrum columns = width / 2 + 1
  uint32_t ld;        // row stride of row-major buffers (= n_cols)
  uint32_t mode;      // 0 forward; 1 forward, x K x s, inverse; 2 x K x s, inverse
  uint32_t in_cm, out_cm, kern_cm;  // column-major layouts (column c at c * N)
  const uint32_t* rows;    // modes 0/1: the input's non-zero rows, or NULL:
  const uint32_t* n_rows;  //   rows [row0, row0 + row_n) (their count: device)
  uint32_t row0, row_n;
  uint32_t per_xcd;   // columns each XCD takes per round (grid / 8)
  double scale;
  // ColumnsConvD: output rows outside [out_row0, out_row0 + out_row_n) are
  // not written (the inverse row pass reads the output window's rows only)
  uint32_t out_row0, out_row_n;
  // ColumnsConvD: input and output in the tiled layout (TileIndex, column
  // length N) instead of row-major
  uint32_t tiled;
};

// PF: the kernel column is loaded into registers before the forward
// transform (in flight meanwhile); otherwise after it.
template <typename T, uint32_t TH, bool PF, uint32_t... Rs>
__global__ __launch_bounds__(TH) void Columns(ColArgs a, const Cx<T>* __restrict__ in,
                                              Cx<T>* out,
                                              const Cx<T>* __restrict__ kern,
                                              const Cx<T>* __restrict__ ptw) {
  constexpr uint32_t N = Product<Rs...>();
  constexpr uint32_t E = (N + TH - 1) / TH;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  const uint32_t tid = threadIdx.x;
  const uint32_t b = blockIdx.x, G = gridDim.x;
  const T s = T(a.scale);
  // sparse: only some rows are non-zero (a list, or a range short of N);
  // LDS then holds zeros everywhere else between columns
  const bool listed = a.rows != nullptr && a.mode != 2;
  const bool sparse = a.mode != 2 && (listed || a.row_n < N);
  const uint32_t n_rows = listed ? *a.n_rows : a.row_n;
  if (sparse) {
#pragma unroll
    for (uint32_t i = 0; i < E; ++i) {
      const uint32_t y = tid + i * TH;
      if (N % TH == 0 || y < N) buf[Lx<T>(y)] = Cx<T>{T(0), T(0)};
    }
    LdsSync();
  }
  for (uint32_t round = 0; round * G < a.n_cols; ++round) {
    // opaque per round: keeps the (loop-invariant) per-element addresses of
    // every pass from being hoisted out of the loop into spilled registers
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    // XCD-aware: the columns of one round on one XCD are contiguous, so the
    // row-major lines they share meet in one L2
    const uint32_t c = round * G + (b & 7u) * a.per_xcd + (b >> 3);
    const bool active = c < a.n_cols;
    // uniform column bases (scalar registers) + 32-bit element offsets
    const uint32_t in_stride = (a.mode == 2 && a.in_cm) ? 1u : a.ld;
    const Cx<T>* in_c = (a.mode == 2 && a.in_cm) ? in + size_t(c) * N : in + c;
    const uint32_t k_stride = a.kern_cm ? 1u : a.ld;
    const Cx<T>* kern_c = a.kern_cm ? kern + size_t(c) * N : kern + c;
    Cx<T> K[E];
    auto load_kernel = [&]() {
#pragma unroll
      for (uint32_t i = 0; i < E; ++i) {
        const uint32_t y = tid + i * TH;
        if (N % TH == 0 || y < N) K[i] = kern_c[y * k_stride];
      }
    };
    if (active) {
      if (sparse) {
        for (uint32_t q = tid; q < n_rows; q += TH) {
          const uint32_t y = listed ? a.rows[q] : a.row0 + q;
          buf[Lx<T>(y)] = in_c[y * in_stride];
        }
      } else {
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) {
          const uint32_t y = tid + i * TH;
          if (N % TH == 0 || y < N) buf[Lx<T>(y)] = in_c[y * in_stride];
        }
      }
      if (PF && a.mode != 0) load_kernel();
    }
    LdsSync();
    if (a.mode != 2) Fft<T, TH, N, 0, 1, Rs...>(buf, ptw, tid);
    if (a.mode != 0) {
      if (!PF && active) load_kernel();
      // inverse = conj(forward(conj(X K s)))
#pragma unroll
      for (uint32_t i = 0; i < E; ++i) {
        const uint32_t y = tid + i * TH;
        if (N % TH == 0 || y < N) buf[Lx<T>(y)] = Conj(Scale(Mul(buf[Lx<T>(y)], K[i]), s));
      }
      LdsSync();
      Fft<T, TH, N, 0, 1, Rs...>(buf, ptw, tid);
    }
    if (active) {
      const uint32_t o_stride = a.out_cm ? 1u : a.ld;
      Cx<T>* out_c = a.out_cm ? out + size_t(c) * N : out + c;
#pragma unroll
      for (uint32_t i = 0; i < E; ++i) {
        const uint32_t y = tid + i * TH;
        if (N % TH == 0 || y < N) {
          Cx<T> v = buf[Lx<T>(y)];
          if (a.mode != 0) v = Conj(v);
          out_c[y * o_stride] = v;
          if (sparse) buf[Lx<T>(y)] = Cx<T>{T(0), T(0)};
        }
      }
    } else if (sparse) {
#pragma unroll
      for (uint32_t i = 0; i < E; ++i) {
        const uint32_t y = tid + i * TH;
        if (N % TH == 0 || y < N) buf[Lx<T>(y)] = Cx<T>{T(0), T(0)};
      }
    }
    LdsSync();
  }
}

// Tiled spectrum layout of the four-step column passes: 16 adjacent columns
// (128 B of float complex, 256 B of double complex) of every row side by side, tile after tile, so
// both the row passes and the column passes move whole cache lines.
constexpr uint32_t kTile = 16;
__device__ __forceinline__ size_t TileIndex(uint32_t y, uint32_t k, uint32_t height) {
  return (size_t(k / kTile) * height + y) * kTile + (k % kTile);
}

// ----------------------------------- float64 correction columns (mode 1)
// ColumnsConvD: the column pass of CorrectResidualDirty's padded convolution
// (forward, x K x s, inverse; sparse input rows; input and output row-major
// or, ColArgs::tiled, in the tiled layout), with the
// per-round latency chain of Columns cut down:
//   * pass twiddles from two small LDS tables (W^e = T1[e >> 7] T2[e & 127],
//     both exact entries of the plan's length-N table) instead of a global
//     load per butterfly and pass,
//   * the first forward pass reads the input straight from global memory
//     through a row bitmap in LDS (no staging, no zeroing sweep per column),
//   * the last forward pass multiplies by K x s (prefetched into registers in
//     that pass's output order) and conjugates before its LDS store (no
//     separate multiply sweep),
//   * the last inverse pass stores to global memory from its registers.
// Same arithmetic as Columns up to the twiddle products' last bit (results
// are rounded to float by the row pass; tests/test_fft_fast.py).
constexpr uint32_t kTwShift = 7;
constexpr uint32_t kTwLo = 1u << kTwShift;

template <uint32_t TH, uint32_t N, uint32_t R, uint32_t NS, int SRC, int DST, typename Load,
          typename Store>
__device__ __forceinline__ void CPass(Cx<double>* buf, const Cx<double>* t1,
                                      const Cx<double>* t2, uint32_t tid, Load load,
                                      Store store) {
  constexpr uint32_t NB = N / R;
  constexpr uint32_t BPT = (NB + TH - 1) / TH;
  Cx<double> v[BPT][R];
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
#pragma unroll
      for (uint32_t r = 0; r < R; ++r)
        v[i][r] = SRC == 0 ? buf[j + r * NB] : load(j + r * NB);
    }
  }
  if constexpr (SRC == 0) LdsSync();  // every read done before any write
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t j = tid + i * TH;
    if (NB % TH == 0 || j < NB) {
      const uint32_t k = j % NS;
      if constexpr (NS > 1) {
        const uint32_t e = k * (N / (NS * R));
        const Cx<double> w = Mul(t1[e >> kTwShift], t2[e & (kTwLo - 1u)]);
        Cx<double> wr = w;
        v[i][1] = Mul(v[i][1], wr);
#pragma unroll
        for (uint32_t r = 2; r < R; ++r) {
          wr = Mul(wr, w);
          v[i][r] = Mul(v[i][r], wr);
        }
      }
      Dft<double, int(R)>::Run(v[i]);
      const uint32_t d = (j / NS) * NS * R + k;
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) store(i, r, d + r * NS, v[i][r]);
    }
  }
  if constexpr (DST == 0) LdsSync();
}

// passes 2 .. of the forward transform (LDS to LDS); the last one goes
// through `last` (the K multiply)
template <uint32_t TH, uint32_t N, uint32_t NS, typename Last, uint32_t R, uint32_t... Rest>
__device__ __forceinline__ void CFwdTail(Cx<double>* buf, const Cx<double>* t1,
                                         const Cx<double>* t2, uint32_t tid, Last last) {
  auto nop = [](uint32_t) { return Cx<double>{0.0, 0.0}; };
  if constexpr (sizeof...(Rest) == 0) {
    CPass<TH, N, R, NS, 0, 0>(buf, t1, t2, tid, nop, last);
  } else {
    CPass<TH, N, R, NS, 0, 0>(buf, t1, t2, tid, nop,
                              [&](uint32_t, uint32_t, uint32_t y, Cx<double> v) { buf[y] = v; });
    CFwdTail<TH, N, NS * R, Last, Rest...>(buf, t1, t2, tid, last);
  }
}

// the inverse transform's passes (LDS to LDS, the last one to `last`)
template <uint32_t TH, uint32_t N, uint32_t NS, typename Last, uint32_t R, uint32_t... Rest>
__device__ __forceinline__ void CInv(Cx<double>* buf, const Cx<double>* t1, const Cx<double>* t2,
                                     uint32_t tid, Last last) {
  auto nop = [](uint32_t) { return Cx<double>{0.0, 0.0}; };
  if constexpr (sizeof...(Rest) == 0) {
    CPass<TH, N, R, NS, 0, 1>(buf, t1, t2, tid, nop, last);
  } else {
    CPass<TH, N, R, NS, 0, 0>(buf, t1, t2, tid, nop,
                              [&](uint32_t, uint32_t, uint32_t y, Cx<double> v) { buf[y] = v; });
    CInv<TH, N, NS * R, Last, Rest...>(buf, t1, t2, tid, last);
  }
}

template <uint32_t... Rs>
constexpr uint32_t LastOf() {
  constexpr uint32_t r[] = {Rs...};
  return r[sizeof...(Rs) - 1];
}

// KF: the kernel spectrum stored as float complex (half the bytes of the
// pass's largest read), widened to double where it is multiplied
template <uint32_t TH, bool KF, uint32_t R1, uint32_t... Rs>
__global__ __launch_bounds__(TH) void ColumnsConvD(ColArgs a, const Cx<double>* __restrict__ in,
                                                   Cx<double>* out, const void* __restrict__ kern_v,
                                                   const Cx<double>* __restrict__ tw) {
  using KT = std::conditional_t<KF, Cx<float>, Cx<double>>;
  const KT* __restrict__ kern = static_cast<const KT*>(kern_v);
  constexpr uint32_t N = R1 * Product<Rs...>();
  constexpr uint32_t RL = LastOf<R1, Rs...>();
  constexpr uint32_t NBL = N / RL;  // last pass: butterflies, = its span
  constexpr uint32_t BL = (NBL + TH - 1) / TH;
  constexpr uint32_t NT1 = (N + kTwLo - 1) / kTwLo;
  constexpr uint32_t NWORDS = (N + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<double>* buf = reinterpret_cast<Cx<double>*>(lds_raw);
  Cx<double>* t1 = buf + N;
  Cx<double>* t2 = t1 + NT1;
  uint32_t* bits = reinterpret_cast<uint32_t*>(t2 + kTwLo);
  const uint32_t b = blockIdx.x, G = gridDim.x;
  const double s = a.scale;
  {
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < NT1; i += TH) t1[i] = tw[i * kTwLo];
    for (uint32_t i = tid; i < kTwLo; i += TH) t2[i] = tw[i];
    for (uint32_t i = tid; i < NWORDS; i += TH) bits[i] = 0u;
    __syncthreads();
    // the input's non-zero rows (a list, or a range)
    const bool listed = a.rows != nullptr;
    const uint32_t n_rows = listed ? *a.n_rows : a.row_n;
    for (uint32_t q = tid; q < n_rows; q += TH) {
      const uint32_t y = listed ? a.rows[q] : a.row0 + q;
      if (y < N) atomicOr(&bits[y >> 5], 1u << (y & 31u));
    }
    __syncthreads();
  }
  for (uint32_t round = 0; round * G < a.n_cols; ++round) {
    uint32_t tid = threadIdx.x;  // opaque per round (see Columns)
    asm volatile("" : "+v"(tid));
    const uint32_t c = round * G + (b & 7u) * a.per_xcd + (b >> 3);
    const bool active = c < a.n_cols;
    const uint32_t cc = active ? c : 0u;
    // column c: row-major (stride ld) or tiled (stride kTile in its tile)
    const size_t in_stride = a.tiled ? kTile : a.ld;
    const Cx<double>* in_c =
        in + (a.tiled ? size_t(cc / kTile) * N * kTile + cc % kTile : size_t(cc));
    const uint32_t k_stride = a.kern_cm ? 1u : a.ld;
    const KT* kern_c = a.kern_cm ? kern + size_t(cc) * N : kern + cc;
    auto kload = [&](uint32_t y) {
      const KT k = kern_c[y * k_stride];
      return Cx<double>{double(k.x), double(k.y)};
    };
    // K x s in the last forward pass's output order: rows j + r NBL; held in
    // registers from the round's start (512 threads), or read where it is
    // multiplied (1024 threads: the registers go to the second set of waves)
    // (register K before the forward transform costs more than it hides:
    // the first pass's input loads then wait for it in order, vmcnt; with a
    // float K at 1 024 threads: 623 -> 668 us per 9072^2 pass; the first two
    // rounds' K issued after the first pass instead: 630 -> 758 us, r05)
    constexpr bool KREG = TH <= 512;
    KT K[KREG ? BL : 1][KREG ? RL : 1];
    if constexpr (KREG) {
#pragma unroll
      for (uint32_t i = 0; i < BL; ++i) {
        const uint32_t j = tid + i * TH;
        if (NBL % TH == 0 || j < NBL)
#pragma unroll
          for (uint32_t r = 0; r < RL; ++r) K[i][r] = kern_c[(j + r * NBL) * k_stride];
      }
    }
    // forward pass 1: straight from global memory through the row bitmap
    auto load = [&](uint32_t y) {
      return ((bits[y >> 5] >> (y & 31u)) & 1u) && active ? in_c[size_t(y) * in_stride]
                                                           : Cx<double>{0.0, 0.0};
    };
    CPass<TH, N, R1, 1, 1, 0>(buf, t1, t2, tid, load,
                              [&](uint32_t, uint32_t, uint32_t y, Cx<double> v) { buf[y] = v; });
    auto mulk = [&](uint32_t i, uint32_t r, uint32_t y, Cx<double> v) {
      Cx<double> k;
      if constexpr (KREG)
        k = Cx<double>{double(K[i][r].x), double(K[i][r].y)};
      else
        k = kload(tid + i * TH + r * NBL);
      buf[y] = Conj(Scale(Mul(v, k), s));
    };
    CFwdTail<TH, N, R1, decltype(mulk), Rs...>(buf, t1, t2, tid, mulk);
    // inverse = conj(forward(conj(X K s))); the last pass stores the window rows
    auto store = [&](uint32_t, uint32_t, uint32_t y, Cx<double> v) {
      if (active && y - a.out_row0 < a.out_row_n)
        out[a.tiled ? TileIndex(y, c, N) : a.out_cm ? size_t(c) * N + y : size_t(y) * a.ld + c] =
            Conj(v);
    };
    // (its LDS reads end in a barrier, before the next round's first stores)
    CInv<TH, N, 1, decltype(store), R1, Rs...>(buf, t1, t2, tid, store);
  }
}

// ----------------------------------------------------------------- rows
// One real row of length 2H per workgroup, as a half-length complex FFT
// (z[n] = x[2n] + i x[2n+1]) with the even/odd split folded in: H complex in
// LDS (72 KiB for H = 4536 double), so two workgroups share a CU and one's
// loads overlap the other's transform. Twiddles: the length-2H table.
struct RowArgs {
  uint32_t height;      // plane rows
  uint32_t ld;          // spectrum row stride (H + 1)
  uint32_t img_w, img_h, ox, oy;  // image window inside the plane
  const uint32_t* rows;    // forward: the non-zero plane rows (NULL: the window rows)
  const uint32_t* n_rows;  // their count (device)
  int subtract;         // inverse: 0 write, 1 subtract from out
  int tiled;            // spectrum in column tiles (see TileIndex), else row-major
  int all_rows;         // forward: every plane row (zero outside the window)
  RowPeak peak;         // inverse: fused peak search when peak.partials
  int prefetch;         // inverse, subtract: load the residual row before the transform
};


// spectrum rows (X[0..H]) -> real rows written into / subtracted from the
// window. Z[k] = (X[k] + conj X[H-k]) + i W^-k (X[k] - conj X[H-k]) gives
// z = IFFT_H(Z) = N (x_even + i x_odd) (unnormalised, as C2R); the inverse
// runs as conj(FFT(conj Z)). The imaginary parts of X[0] and X[H] are
// ignored, as by C2R.
// LT (float only): twiddles from the LDS double tables (TwdLds, `twd` = the
// base table of length 2H: 2H / 64 entries W^{64 i}, then 64 entries W^i)
// and persistent workgroups (rows blockIdx, blockIdx + grid, ...: the table
// is loaded once per workgroup).
template <typename T, uint32_t TH, bool LT, uint32_t... Rs>
__global__ __launch_bounds__(TH) void RowsInverse(RowArgs a, const Cx<T>* __restrict__ spec,
                                                  float* __restrict__ out,
                                                  const Cx<T>* __restrict__ tw,
                                                  const Cx<T>* __restrict__ ptw,
                                                  const Cx<double>* __restrict__ twd) {
  constexpr uint32_t H = Product<Rs...>();
  constexpr uint32_t EH = (H + TH - 1) / TH;
  constexpr uint32_t ND1 = LT ? 2 * H / kTwdLo : 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  __shared__ uint64_t red[TH / 64];  // fused peak search
  __shared__ Cx<double> tws[LT ? ND1 + kTwdLo : 1];
  TwdLds td{tws, tws + ND1};
  // LT: the pass twiddles, made once per workgroup (FftC)
  constexpr uint32_t NCT = LT ? CachedTableSize<1, Rs...>(TH, H) : 0;
  __shared__ Cx<float> ctab[NCT > 0 ? NCT : 1];
  Cx<float> clast[LT ? LastRadix<Rs...>() - 1 : 1];
  if constexpr (LT) {
    for (uint32_t i = threadIdx.x; i < ND1 + kTwdLo; i += TH) tws[i] = twd[i];
    __syncthreads();
    InitTwiddles<TH, H, 2, 1, Rs...>(td, ctab, 0, clast, threadIdx.x);
    __syncthreads();
  }
  // bins in pairs (k, H - k): every spectrum element is read once
  constexpr uint32_t NP = H / 2 + 1;
  constexpr uint32_t EP = (NP + TH - 1) / TH;
  auto row_ptr = [&](uint32_t iy) { return spec + size_t(iy + a.oy) * a.ld; };
  auto load_at = [&](uint32_t iy, uint32_t k) {
    return *(a.tiled ? spec + TileIndex(iy + a.oy, k, a.height) : row_ptr(iy) + k);
  };
  // PF (off: measured 186.6 -> 205.8 us per 8192^2 pass on MI355X, the
  // registers cost a wave per SIMD): the next row's bins loaded into
  // registers before this row's transform and stores
  constexpr bool PF = false;
  Cx<T> pk[PF ? EP : 1], pm[PF ? EP : 1];
  auto prefetch = [&](uint32_t iy, uint32_t tid) {
#pragma unroll
    for (uint32_t i = 0; i < EP; ++i) {
      const uint32_t k = tid + i * TH;
      if (NP % TH != 0 && k >= NP) continue;
      pk[i] = load_at(iy, k);
      pm[i] = load_at(iy, H - k);
    }
  };
  if constexpr (LT && PF)
    if (blockIdx.x < a.img_h) prefetch(blockIdx.x, threadIdx.x);
  for (uint32_t iy = blockIdx.x; iy < a.img_h; iy += LT ? gridDim.x : a.img_h) {
  uint32_t tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // opaque per row (see Columns)
  // conj(Z) for bin k from X[k] = xk and X[H-k] = xm
  auto zc = [&](Cx<T> xk, Cx<T> xm, uint32_t k) {
    const Cx<T> sum = {xk.x + xm.x, xk.y - xm.y};  // X[k] + conj X[H-k]
    const Cx<T> dif = {xk.x - xm.x, xk.y + xm.y};  // X[k] - conj X[H-k]
    Cx<T> wk;
    if constexpr (LT)
      wk = ToF(TwD(td, k));
    else
      wk = tw[k];
    const Cx<T> t = Mul(Conj(wk), dif);           // W_N^-k (...)
    return Cx<T>{sum.x - t.y, -(sum.y + t.x)};      // Z = sum + i t, conjugated
  };
#pragma unroll
  for (uint32_t i = 0; i < EP; ++i) {
    const uint32_t k = tid + i * TH;
    if (NP % TH != 0 && k >= NP) continue;
    const uint32_t m = H - k;
    Cx<T> xk, xm;
    if constexpr (LT && PF) {
      xk = pk[i];
      xm = pm[i];
    } else {
      xk = load_at(iy, k);
      xm = load_at(iy, m);
    }
    if (k == 0) {  // C2R ignores the imaginary parts of X[0] and X[H]
      xk.y = T(0);
      xm.y = T(0);
    }
    buf[Lx<T>(k)] = zc(xk, xm, k);
    if (k != 0 && m != k) buf[Lx<T>(m)] = zc(xm, xk, m);
  }
  if constexpr (LT && PF)
    if (iy + gridDim.x < a.img_h) prefetch(iy + gridDim.x, tid);
  float* o = out + size_t(iy) * a.img_w;
  // subtract (the residual correction): the row's residual values loaded
  // now, issued after the spectrum loads, so they arrive during the
  // transform instead of after it (LdsSync waits for LDS only)
  const bool even_win = ((a.ox | a.img_w) & 1u) == 0;
  // only the 512-thread float64 plans (the 8192^2 / 4096^2 corrections'):
  // the registers cost the smaller plans a wave per SIMD (the gridded runs'
  // subimage corrections: 7 -> 5 waves at 128 threads, measured slower)
  constexpr bool kRpre = std::is_same_v<T, double> && TH >= 512;
  float2 rpre[kRpre ? EH : 1];
  if (kRpre && a.subtract && a.prefetch && even_win) {
#pragma unroll
    for (uint32_t i = 0; i < EH; ++i) {
      const uint32_t n = tid + i * TH;
      if (H % TH != 0 && n >= H) continue;
      const uint32_t x0 = 2 * n;
      if (x0 < a.ox || x0 >= a.ox + a.img_w) continue;
      rpre[i] = *reinterpret_cast<const float2*>(o + (x0 - a.ox));
    }
  }
  LdsSync();
  if constexpr (LT)
    FftC<TH, H, 1, Rs...>(buf, ctab, 0, clast, tid);
  else
    Fft<T, TH, H, 0, 1, Rs...>(buf, ptw, tid);
  // fused peak search over the values as written (window coordinates): per
  // thread the largest PeakKey value word (0: none qualifies) and its first
  // x, in 32-bit compares (a thread visits its x in ascending order, so the
  // strict > keeps the first of equal values, as PeakKey's index word does);
  // one 64-bit key per thread at the end of the row
  const bool peak = a.peak.partials != nullptr;
  const bool peak_row = peak && iy >= a.peak.ys && iy < a.peak.ye;
  const uint32_t pxs = a.peak.xs, pxn = a.peak.xe - a.peak.xs;
  const uint8_t* mrow = a.peak.mask ? a.peak.mask + size_t(iy) * a.img_w : nullptr;
  const uint32_t sign_mask = a.peak.allow_negative != 0 ? 0x7fffffffu : 0xffffffffu;
  uint32_t best_u = 0u, best_x = 0u;
  auto consider = [&](uint32_t x, float v) {
    if (!peak_row) return;
    const uint32_t u = __float_as_uint(v) & sign_mask;
    const bool q = u > 0x00800000u && u <= 0x7f800000u && x - pxs < pxn &&
                   (!mrow || mrow[x]);
    const uint32_t uq = q ? u : 0u;
    const bool better = uq > best_u;
    best_u = better ? uq : best_u;
    best_x = better ? x : best_x;
  };
  auto finish_peak = [&]() {
    if (!peak) return;
    uint64_t best = best_u ? ((uint64_t(best_u) << 32) |
                              uint64_t(0xffffffffu - (iy * a.img_w + best_x)))
                           : 0ull;
    best = BlockMaxU64(best, red);
    if (tid == 0) a.peak.partials[iy] = best;
  };
  if (even_win) {
    // even window: (x[2n], x[2n+1]) both in or both out, one 8-B access
#pragma unroll
    for (uint32_t i = 0; i < EH; ++i) {
      const uint32_t n = tid + i * TH;
      if (H % TH != 0 && n >= H) continue;
      const uint32_t x0 = 2 * n;
      if (x0 < a.ox || x0 >= a.ox + a.img_w) continue;
      const Cx<T> z = buf[Lx<T>(n)];  // conj(result): x[2n] = z.x, x[2n+1] = -z.y
      float2* p = reinterpret_cast<float2*>(o + (x0 - a.ox));
      float2 v = {float(z.x), float(-z.y)};
      if (a.subtract) {
        const float2 r = (kRpre && a.prefetch) ? rpre[kRpre ? i : 0] : *p;
        v = {r.x - v.x, r.y - v.y};
      }
      *p = v;
      consider(x0 - a.ox, v.x);
      consider(x0 - a.ox + 1, v.y);
    }
    finish_peak();
    if constexpr (LT) LdsSync();  // the row's LDS reads before the next row's stores
    continue;
  }
#pragma unroll
  for (uint32_t i = 0; i < EH; ++i) {
    const uint32_t n = tid + i * TH;
    if (H % TH != 0 && n >= H) continue;
    const Cx<T> z = buf[Lx<T>(n)];
    const uint32_t x0 = 2 * n, x1 = x0 + 1;
    if (x0 >= a.ox && x0 < a.ox + a.img_w) {
      float* p = o + (x0 - a.ox);
      const float v = a.subtract ? *p - float(z.x) : float(z.x);
      *p = v;
      consider(x0 - a.ox, v);
    }
    if (x1 >= a.ox && x1 < a.ox + a.img_w) {
      float* p = o + (x1 - a.ox);
      const float v = a.subtract ? *p - float(-z.y) : float(-z.y);
      *p = v;
      consider(x1 - a.ox, v);
    }
  }
  finish_peak();
  if constexpr (LT) LdsSync();
  }
}

// One 16-byte-per-lane LDS-DMA load (global_load_lds_dwordx4): lane i's 16 B
// land at LDS byte `lds` + 16 i (lds wave-uniform, through m0). In inline asm
// so the compiler does not treat it as an LDS write of unknown extent (see
// RowsInverseDma); the caller retires it with its own s_waitcnt vmcnt and a
// barrier before any wave reads those bytes.
__device__ __forceinline__ void DmaLoad16(const void* g, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}

// RowsInverse (float, tiled spectrum, write mode, even window) with the next
// row's spectrum fetched by LDS-DMA while this row is transformed and
// stored. The persistent row kernel above keeps one row per workgroup in
// flight only while that workgroup loads it (a third of its time at three
// workgroups per CU: ~3 TB/s); here every workgroup always has its next row
// in flight (global_load_lds_dwordx4: a wave instruction moves 8 tiles x
// 128 B, lane-linear into `raw`, no VGPRs), and the FFT runs in its own LDS
// buffer. The DMA is retired by a counted vmcnt (the 16 output stores per
// wave issued after it may stay in flight) and a barrier; every other
// synchronisation is LDS-only, so nothing drains it early. Same arithmetic
// as RowsInverse<float, TH, true> (FftC, zc, the fused peak search).
template <uint32_t TH, uint32_t... Rs>
__global__ __launch_bounds__(TH) void RowsInverseDma(RowArgs a, const Cx<float>* __restrict__ spec,
                                                     float* __restrict__ out,
                                                     const Cx<double>* __restrict__ twd) {
  constexpr uint32_t H = Product<Rs...>();
  constexpr uint32_t EH = H / TH;
  static_assert(H % TH == 0 && (EH == 16 || EH == 8), "vmcnt counts of 8 or 16 stores");
  constexpr uint32_t WAVES = TH / 64;
  constexpr uint32_t ND1 = 2 * H / kTwdLo;
  constexpr uint32_t NT = (H + 1 + kTile - 1) / kTile;  // spectrum tiles per row
  constexpr uint32_t NI = (NT + 7) / 8;                 // DMA wave instructions per row
  typedef __attribute__((address_space(3))) void* LdsPtr;
  // The DMA target is its own __shared__ object; the transform, tables and
  // reduction live in the dynamic array (RowsDmaLdsBytes). The DMA is issued
  // by inline asm (DmaLoad16): hipcc cannot tell which LDS bytes a
  // global_load_lds writes and, for its builtin, waits vmcnt(0) before the
  // next LDS read whatever the arrays, which drained the prefetch at once.
  __shared__ __attribute__((aligned(16))) Cx<float> raw[NI * 8 * kTile];
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  constexpr uint32_t NCT = CachedTableSize<1, Rs...>(TH, H);
  Cx<float>* buf = reinterpret_cast<Cx<float>*>(lds_raw);             // the transform
  Cx<double>* tws = reinterpret_cast<Cx<double>*>(buf + (H + (H >> kFastPadShift)));
  Cx<float>* ctab = reinterpret_cast<Cx<float>*>(tws + ND1 + kTwdLo);
  uint64_t* red = reinterpret_cast<uint64_t*>(ctab + (NCT > 0 ? (NCT + 1) / 2 * 2 : 2));
  TwdLds td{tws, tws + ND1};
  Cx<float> clast[LastRadix<Rs...>() - 1];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  auto issue = [&](uint32_t iy) {
    const size_t y = size_t(iy) + a.oy;
    for (uint32_t j = wave; j < NI; j += WAVES) {
      const uint32_t t = j * 8 + lane / 8;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          uint32_t(uintptr_t((LdsPtr)(raw + j * 8 * kTile))));
      if (t < NT) DmaLoad16(spec + (size_t(t) * a.height + y) * kTile + (lane % 8) * 2, dst);
    }
  };
  if (blockIdx.x < a.img_h) issue(blockIdx.x);
  for (uint32_t i = threadIdx.x; i < ND1 + kTwdLo; i += TH) tws[i] = twd[i];
  LdsSync();
  InitTwiddles<TH, H, 2, 1, Rs...>(td, ctab, 0, clast, threadIdx.x);
  constexpr uint32_t NP = H / 2 + 1;
  constexpr uint32_t EP = (NP + TH - 1) / TH;
  // the split's twiddles W^-k, W^-(H-k): a thread takes the same bins k in
  // every row, so they are made once (the per-row double products were a
  // tenth of the kernel's VALU)
  Cx<float> wk[EP], wm[EP];
#pragma unroll
  for (uint32_t i = 0; i < EP; ++i) {
    const uint32_t k = threadIdx.x + i * TH;
    if (NP % TH != 0 && k >= NP) continue;
    wk[i] = ToF(TwD(td, k));
    wm[i] = ToF(TwD(td, H - k));
  }
  // fused peak search: this thread's best key over all its rows (value
  // word, then the lowest index), one block reduction at the end: the
  // partials are per workgroup (FastRowsInverseLaunch's n_partials)
  const bool peak = a.peak.partials != nullptr;
  const uint32_t pxs = a.peak.xs, pxn = a.peak.xe - a.peak.xs;
  const uint32_t sign_mask = a.peak.allow_negative != 0 ? 0x7fffffffu : 0xffffffffu;
  uint64_t run_best = 0ull;
  bool first = true;
  for (uint32_t iy = blockIdx.x; iy < a.img_h; iy += gridDim.x) {
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // opaque per row (see Columns)
    // this row's DMA (issued a row ago) landed; the previous row's EH stores
    // per wave, issued after it, may still be in flight
    if (first)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (EH == 16)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    first = false;
    LdsSync();
    auto zc = [&](Cx<float> xk, Cx<float> xm, Cx<float> w) {
      const Cx<float> sum = {xk.x + xm.x, xk.y - xm.y};
      const Cx<float> dif = {xk.x - xm.x, xk.y + xm.y};
      const Cx<float> t = Mul(Conj(w), dif);
      return Cx<float>{sum.x - t.y, -(sum.y + t.x)};
    };
#pragma unroll
    for (uint32_t i = 0; i < EP; ++i) {
      const uint32_t k = tid + i * TH;
      if (NP % TH != 0 && k >= NP) continue;
      const uint32_t m = H - k;
      Cx<float> xk = raw[k], xm = raw[m];
      if (k == 0) {  // C2R ignores the imaginary parts of X[0] and X[H]
        xk.y = 0.0f;
        xm.y = 0.0f;
      }
      buf[Lx<float>(k)] = zc(xk, xm, wk[i]);
      if (k != 0 && m != k) buf[Lx<float>(m)] = zc(xm, xk, wm[i]);
    }
    LdsSync();  // raw is read: the next row's DMA may overwrite it
    if (iy + gridDim.x < a.img_h) issue(iy + gridDim.x);
    FftC<TH, H, 1, Rs...>(buf, ctab, 0, clast, tid);
    float* o = out + size_t(iy) * a.img_w;
    const bool peak_row = peak && iy >= a.peak.ys && iy < a.peak.ye;
    const uint8_t* mrow = a.peak.mask ? a.peak.mask + size_t(iy) * a.img_w : nullptr;
    // per value the PeakKey value word (|v| or v as bits; 0 when it cannot
    // be a peak: NaN, a negative value without allow_negative, outside the
    // box or the mask); values <= FLT_MIN are excluded by the row's maximum
    uint32_t uq[EH][2];
    uint32_t tb = 0u;
    // the whole plane row is the window (the launcher's condition): every
    // thread stores EH float2, in ascending x
#pragma unroll
    for (uint32_t i = 0; i < EH; ++i) {
      const uint32_t n = tid + i * TH;
      const Cx<float> z = buf[Lx<float>(n)];
      const float2 v = {z.x, -z.y};
      reinterpret_cast<float2*>(o)[n] = v;
      if (peak_row) {
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
          const uint32_t x = 2 * n + h;
          const uint32_t u = __float_as_uint(h ? v.y : v.x) & sign_mask;
          const bool q = u <= 0x7f800000u && x - pxs < pxn && (!mrow || mrow[x]);
          uq[i][h] = q ? u : 0u;
          tb = uq[i][h] > tb ? uq[i][h] : tb;
        }
      }
    }
    if (peak_row && tb > 0x00800000u) {
      // the first x holding the row's maximum (x ascends with i, h)
      uint32_t bx = 0u;
#pragma unroll
      for (int i = int(EH) - 1; i >= 0; --i)
#pragma unroll
        for (int h = 1; h >= 0; --h)
          bx = uq[i][h] == tb ? 2 * (tid + uint32_t(i) * TH) + uint32_t(h) : bx;
      const uint64_t key =
          (uint64_t(tb) << 32) | uint64_t(0xffffffffu - (iy * a.img_w + bx));
      run_best = key > run_best ? key : run_best;
    }
    LdsSync();  // the row's LDS reads (buf) before the next row's writes
  }
  if (peak) {
    const uint64_t best = WaveMaxU64(run_best);
    if (lane == 0) red[wave] = best;
    LdsSync();
    if (threadIdx.x < 64) {
      uint64_t w = lane < WAVES ? red[lane] : 0ull;
      w = WaveMaxU64(w);
      if (threadIdx.x == 0) a.peak.partials[blockIdx.x] = w;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// real plane rows (the window's image rows, zero outside) -> spectrum rows
// X[0..H]: X[k] = E[k] + W^k O[k], E = (Z[k] + conj Z[H-k]) / 2,
// O = (Z[k] - conj Z[H-k]) / 2i. Rows not listed are not touched (the
// column pass reads only listed rows).
template <typename T, uint32_t TH, bool LT, uint32_t... Rs>
__global__ __launch_bounds__(TH) void RowsForward(RowArgs a, const float* __restrict__ in,
                                                  Cx<T>* __restrict__ spec,
                                                  const Cx<T>* __restrict__ tw,
                                                  const Cx<T>* __restrict__ ptw,
                                                  const Cx<double>* __restrict__ twd) {
  constexpr uint32_t H = Product<Rs...>();
  constexpr uint32_t EH = (H + TH - 1) / TH;
  constexpr uint32_t ND1 = LT ? 2 * H / kTwdLo : 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(lds_raw);
  __shared__ Cx<double> tws[LT ? ND1 + kTwdLo : 1];
  TwdLds td{tws, tws + ND1};
  // (the per-row twiddle math stays: with the next row's input prefetched in
  // registers, FftC's cached last-pass twiddles would cost a wave per SIMD)
  if constexpr (LT) {
    for (uint32_t i = threadIdx.x; i < ND1 + kTwdLo; i += TH) tws[i] = twd[i];
    __syncthreads();
  }
  const uint32_t n_rows = a.rows ? *a.n_rows : (a.all_rows ? a.height : a.img_h);
  const bool even = ((a.ox | a.img_w) & 1u) == 0;
  auto row_of = [&](uint32_t r) { return a.rows ? a.rows[r] : (a.all_rows ? r : r + a.oy); };
  // (e, o) = (x[2n], x[2n+1]) of plane row y, zero outside the window
  auto pair_at = [&](uint32_t y, uint32_t n) {
    const int64_t iy = int64_t(y) - a.oy;
    const bool in_y = iy >= 0 && iy < a.img_h;
    const float* row = in + (in_y ? size_t(iy) * a.img_w : 0);
    const uint32_t x0 = 2 * n, x1 = x0 + 1;
    float2 v = {0.0f, 0.0f};
    if (even) {  // (x[2n], x[2n+1]) both in or both out: one 8-B load
      if (in_y && x0 >= a.ox && x0 < a.ox + a.img_w)
        v = *reinterpret_cast<const float2*>(row + (x0 - a.ox));
    } else {
      v.x = in_y && x0 >= a.ox && x0 < a.ox + a.img_w ? row[x0 - a.ox] : 0.0f;
      v.y = in_y && x1 >= a.ox && x1 < a.ox + a.img_w ? row[x1 - a.ox] : 0.0f;
    }
    return v;
  };
  // LT: the next row's input is loaded into registers before this row's
  // transform and stores (see RowsInverse)
  float2 pre[EH];
  auto prefetch = [&](uint32_t r, uint32_t tid) {
    const uint32_t y = row_of(r);
#pragma unroll
    for (uint32_t i = 0; i < EH; ++i) {
      const uint32_t n = tid + i * TH;
      if (H % TH != 0 && n >= H) continue;
      pre[i] = pair_at(y, n);
    }
  };
  if constexpr (LT)
    if (blockIdx.x < n_rows) prefetch(blockIdx.x, threadIdx.x);
  for (uint32_t r = blockIdx.x; r < n_rows; r += gridDim.x) {
    uint32_t tid = threadIdx.x;  // opaque per row (see Columns)
    asm volatile("" : "+v"(tid));
    const uint32_t y = row_of(r);
#pragma unroll
    for (uint32_t i = 0; i < EH; ++i) {
      const uint32_t n = tid + i * TH;
      if (H % TH != 0 && n >= H) continue;
      float2 v;
      if constexpr (LT)
        v = pre[i];
      else
        v = pair_at(y, n);
      buf[Lx<T>(n)] = {T(v.x), T(v.y)};
    }
    if constexpr (LT)
      if (r + gridDim.x < n_rows) prefetch(r + gridDim.x, tid);
    LdsSync();
    if constexpr (LT)
      FftL<TH, H, 2, 1, Rs...>(buf, td, tid);
    else
      Fft<T, TH, H, 0, 1, Rs...>(buf, ptw, tid);
    Cx<T>* X = spec + size_t(y) * a.ld;
    const T h = T(0.5);
    // X[k] from (Z[k], conj Z[H-k]) and X[H-k] from (Z[H-k], conj Z[k]): the
    // bins in pairs, each LDS value read once (X[0] and X[H] both come from
    // Z[0]); every output is the same expression as bin by bin
    auto put = [&](uint32_t k, Cx<T> zk, Cx<T> zc) {
      const Cx<T> ev = {h * (zk.x + zc.x), h * (zk.y + zc.y)};
      const Cx<T> od = {h * (zk.y - zc.y), -h * (zk.x - zc.x)};  // (zk - zc) / 2i
      Cx<T> wk;
      if constexpr (LT)
        wk = ToF(TwD(td, k));
      else
        wk = tw[k];
      const Cx<T> v = Add(ev, Mul(wk, od));
      // one address, one 8/16-byte store (a store per layout branch was
      // split into scalar halves)
      *(a.tiled ? spec + TileIndex(y, k, a.height) : X + k) = v;
    };
    constexpr uint32_t NP = H / 2 + 1;
    constexpr uint32_t EP = (NP + TH - 1) / TH;
#pragma unroll
    for (uint32_t i = 0; i < EP; ++i) {
      const uint32_t k = tid + i * TH;
      if (NP % TH != 0 && k >= NP) continue;
      const Cx<T> zlo = buf[Lx<T>(k)];
      const Cx<T> zhi = k == 0 ? zlo : buf[Lx<T>(H - k)];
      put(k, zlo, Conj(zhi));
      if (H - k != k) put(H - k, zhi, Conj(zlo));
    }
    LdsSync();
  }
}

// RowsForward (float, whole plane rows -> tiled spectrum) with the next
// image row fetched by LDS-DMA (DmaLoad16: a wave instruction moves 256
// contiguous floats) while this row is transformed and stored, and the pass
// twiddles made once per workgroup (FftC; the register prefetch of the
// persistent kernel left no room for them). The vmcnt count: every wave
// issues at least 2 (EP - 1) >= 16 spectrum stores after the DMA. Same
// arithmetic as RowsForward<float, TH, true>.
template <uint32_t TH, uint32_t... Rs>
__global__ __launch_bounds__(TH) void RowsForwardDma(RowArgs a, const float* __restrict__ in,
                                                     Cx<float>* __restrict__ spec,
                                                     const Cx<double>* __restrict__ twd) {
  constexpr uint32_t H = Product<Rs...>();
  constexpr uint32_t EH = H / TH;
  constexpr uint32_t NP = H / 2 + 1;
  constexpr uint32_t EP = (NP + TH - 1) / TH;
  static_assert(H % TH == 0 && (EH == 16 || EH == 8) && 2 * (EP - 1) >= EH,
                "vmcnt counts of 8 or 16 stores");
  constexpr uint32_t WAVES = TH / 64;
  constexpr uint32_t ND1 = 2 * H / kTwdLo;
  constexpr uint32_t NI = 2 * H / 256;  // DMA wave instructions per row (256 floats each)
  typedef __attribute__((address_space(3))) void* LdsPtr;
  __shared__ __attribute__((aligned(16))) float raw[2 * H];  // the DMA target (see RowsInverseDma)
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  constexpr uint32_t NCT = CachedTableSize<1, Rs...>(TH, H);
  Cx<float>* buf = reinterpret_cast<Cx<float>*>(lds_raw);
  Cx<double>* tws = reinterpret_cast<Cx<double>*>(buf + (H + (H >> kFastPadShift)));
  Cx<float>* ctab = reinterpret_cast<Cx<float>*>(tws + ND1 + kTwdLo);
  TwdLds td{tws, tws + ND1};
  Cx<float> clast[LastRadix<Rs...>() - 1];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  auto issue = [&](uint32_t y) {
    const float* row = in + size_t(y) * a.img_w;
    for (uint32_t j = wave; j < NI; j += WAVES) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          uint32_t(uintptr_t((LdsPtr)(raw + j * 256))));
      DmaLoad16(row + j * 256 + lane * 4, dst);
    }
  };
  for (uint32_t i = threadIdx.x; i < ND1 + kTwdLo; i += TH) tws[i] = twd[i];
  if (blockIdx.x < a.height) issue(blockIdx.x);
  LdsSync();
  InitTwiddles<TH, H, 2, 1, Rs...>(td, ctab, 0, clast, threadIdx.x);
  // the split's twiddles W^k, W^(H-k): the same bins in every row of this
  // thread, made once (as RowsInverseDma)
  Cx<float> wk[EP], wm[EP];
#pragma unroll
  for (uint32_t i = 0; i < EP; ++i) {
    const uint32_t k = threadIdx.x + i * TH;
    if (NP % TH != 0 && k >= NP) continue;
    wk[i] = ToF(TwD(td, k));
    wm[i] = ToF(TwD(td, H - k));
  }
  bool first = true;
  for (uint32_t y = blockIdx.x; y < a.height; y += gridDim.x) {
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // opaque per row (see Columns)
    if (first)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (EH == 16)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    first = false;
    LdsSync();
#pragma unroll
    for (uint32_t i = 0; i < EH; ++i) {
      const uint32_t n = tid + i * TH;
      const float2 v = reinterpret_cast<const float2*>(raw)[n];
      buf[Lx<float>(n)] = {v.x, v.y};
    }
    LdsSync();  // raw is read: the next row's DMA may overwrite it
    if (y + gridDim.x < a.height) issue(y + gridDim.x);
    FftC<TH, H, 1, Rs...>(buf, ctab, 0, clast, tid);
    const float h = 0.5f;
    auto put = [&](uint32_t k, Cx<float> zk, Cx<float> zc, Cx<float> w) {
      const Cx<float> ev = {h * (zk.x + zc.x), h * (zk.y + zc.y)};
      const Cx<float> od = {h * (zk.y - zc.y), -h * (zk.x - zc.x)};  // (zk - zc) / 2i
      spec[TileIndex(y, k, a.height)] = Add(ev, Mul(w, od));
    };
#pragma unroll
    for (uint32_t i = 0; i < EP; ++i) {
      const uint32_t k = tid + i * TH;
      if (NP % TH != 0 && k >= NP) continue;
      const Cx<float> zlo = buf[Lx<float>(k)];
      const Cx<float> zhi = k == 0 ? zlo : buf[Lx<float>(H - k)];
      put(k, zlo, Conj(zhi), wk[i]);
      if (H - k != k) put(H - k, zhi, Conj(zlo), wm[i]);
    }
    LdsSync();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------- four-step column passes
// A column transform of length N = N1 * N2 (float, tiled layout) as two
// passes that each move whole 128-B lines (the one-pass column kernel reads
// one 8-B element per row, which makes it L2-request bound):
//   A: for each n2, the N1 rows n2 + N2 n1 of a tile: length-N1 DFTs,
//      x W_N^(n2 k1), to rows k1 N2 + n2 of the scratch;
//   B: for each k1, the N2 consecutive scratch rows k1 N2 .. k1 N2 + N2 - 1:
//      length-N2 DFTs -> X[k1 + N1 k2] at row k1 + N1 k2 (natural order).
// The inverse convolution runs the same two passes on conj(X K s) (A's load)
// and conjugates B's store.

// LDS slot of element e of a four-step transform: one spare slot after every
// 16, so the first passes' radix-8/16 stores (lanes R elements apart) fall
// on distinct banks (PMC: 49-57 % of these kernels' LDS cycles were bank
// conflicts with the plain stride)
// Only the 4096- and 8192-point plans (the headline's and C2's columns,
// where it was measured); the smaller plans of the gridded runs' subimages
// keep the plain stride: the padded indexing raised ColStepBScales' registers
// (1792-3584 plans: occupancy 4 -> 3 waves per SIMD).
constexpr bool PadOn(uint32_t n) { return n >= 4096; }
template <bool PAD>
__device__ __forceinline__ constexpr uint32_t PdIf(uint32_t e) {
  return PAD ? e + (e >> 4) : e;
}
// column stride of a (padded) length-n transform (odd: adjacent columns on
// other banks)
template <bool PAD>
constexpr uint32_t StrideIf(uint32_t n) { return PAD ? n + (n >> 4) + 1 : n + 1; }

// `COUNT` transforms of length N at stride S in LDS (batched Pass); the
// pass tables as for Pass, read once per workgroup into LDS (`wt`, shared by
// all COUNT transforms).
template <typename T, uint32_t TH, uint32_t N, uint32_t R, uint32_t NS, uint32_t OFF,
          uint32_t COUNT, uint32_t S>
__device__ __forceinline__ void BPass(Cx<T>* buf, const Cx<T>* wt, uint32_t tid) {
  constexpr bool PAD = S != N + 1;  // the padded layout (StrideIf<true>)
  constexpr uint32_t NB = N / R;
  constexpr uint32_t TOT = COUNT * NB;
  constexpr uint32_t BPT = (TOT + TH - 1) / TH;
  Cx<T> v[BPT][R];
  Cx<T> w[BPT][NS > 1 ? R - 1 : 1];
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t b = tid + i * TH;
    if (TOT % TH == 0 || b < TOT) {
      const uint32_t t = b / NB, j = b % NB;
      if constexpr (NS > 1) {
        const uint32_t k = j % NS;
#pragma unroll
        for (uint32_t q = 0; q + 1 < R; ++q) w[i][q] = wt[OFF + q * NS + k];
      }
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) v[i][r] = buf[t * S + PdIf<PAD>(j + r * NB)];
    }
  }
  LdsSync();
#pragma unroll
  for (uint32_t i = 0; i < BPT; ++i) {
    const uint32_t b = tid + i * TH;
    if (TOT % TH == 0 || b < TOT) {
      const uint32_t t = b / NB, j = b % NB;
      const uint32_t k = j % NS;
      if constexpr (NS > 1) {
#pragma unroll
        for (uint32_t r = 1; r < R; ++r) v[i][r] = Mul(v[i][r], w[i][r - 1]);
      }
      Dft<T, int(R)>::Run(v[i]);
      const uint32_t d = (j / NS) * NS * R + k;
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) buf[t * S + PdIf<PAD>(d + r * NS)] = v[i][r];
    }
  }
  LdsSync();
}

template <typename T, uint32_t TH, uint32_t N, uint32_t COUNT, uint32_t S, uint32_t OFF,
          uint32_t NS, uint32_t R, uint32_t... Rest>
__device__ __forceinline__ void BFft(Cx<T>* buf, const Cx<T>* wt, uint32_t tid) {
  BPass<T, TH, N, R, NS, OFF, COUNT, S>(buf, wt, tid);
  if constexpr (sizeof...(Rest) > 0)
    BFft<T, TH, N, COUNT, S, OFF + PassTableSize(R, NS), NS * R, Rest...>(buf, wt, tid);
}

template <uint32_t NS, uint32_t R, uint32_t... Rest>
constexpr uint32_t TableSize() {
  if constexpr (sizeof...(Rest) > 0)
    return PassTableSize(R, NS) + TableSize<NS * R, Rest...>();
  else
    return PassTableSize(R, NS);
}

template <uint32_t... Rs>
struct Radices {};

struct StepArgs {
  uint32_t n_tiles;  // column tiles
  int inverse;       // A: load conj(X K s); B: store conj
  float scale;
};

// Pass A: workgroup = (tile, GA consecutive n2). tw: the length-N table;
// ptw: the length-N1 pass table.
template <uint32_t TH, uint32_t N1, uint32_t N2, uint32_t GA, uint32_t... R1>
__global__ __launch_bounds__(TH) void ColStepA(StepArgs a, const Cx<float>* __restrict__ in,
                                               Cx<float>* __restrict__ out,
                                               const Cx<float>* __restrict__ kern,
                                               const Cx<float>* __restrict__ tw,
                                               const Cx<float>* __restrict__ ptw) {
  constexpr uint32_t N = N1 * N2;
  constexpr bool PAD = PadOn(N1 * N2);
  constexpr uint32_t S = StrideIf<PAD>(N1);  // columns of one row on distinct banks
  constexpr uint32_t COUNT = kTile * GA;
  constexpr uint32_t EL = COUNT * N1;
  constexpr uint32_t E = (EL + TH - 1) / TH;
  constexpr uint32_t NT = TableSize<1, R1...>();
  __shared__ Cx<float> buf[COUNT * S];
  __shared__ Cx<float> wt[NT > 0 ? NT : 1];
  __shared__ Cx<float> wa[GA * N1];  // W_N^{n2 k1} of this workgroup's n2
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = blockIdx.x / (N2 / GA);
  const uint32_t n2_0 = (blockIdx.x % (N2 / GA)) * GA;
  const size_t base = size_t(tile) * N * kTile;
  for (uint32_t i = tid; i < NT; i += TH) wt[i] = ptw[i];
  for (uint32_t i = tid; i < GA * N1; i += TH) {
    const uint32_t g = i / N1, k1 = i % N1;
    wa[i] = tw[((n2_0 + g) * k1) % N];
  }
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t g = q % GA, n1 = q / GA;  // GA adjacent rows: one contiguous run
    const size_t off = base + size_t(n2_0 + g + N2 * n1) * kTile + col;
    Cx<float> v = in[off];
    if (a.inverse) v = Conj(Scale(Mul(v, kern[off]), a.scale));
    buf[(g * kTile + col) * S + PdIf<PAD>(n1)] = v;
  }
  LdsSync();
  BFft<float, TH, N1, COUNT, S, 0, 1, R1...>(buf, wt, tid);
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t g = q % GA, k1 = q / GA;
    const uint32_t n2 = n2_0 + g;
    const Cx<float> v = Mul(buf[(g * kTile + col) * S + PdIf<PAD>(k1)], wa[g * N1 + k1]);
    out[base + size_t(k1 * N2 + n2) * kTile + col] = v;
  }
}

// Pass B: workgroup = (tile, GB consecutive k1); ptw: the length-N2 pass table.
template <uint32_t TH, uint32_t N1, uint32_t N2, uint32_t GB, uint32_t... R2>
__global__ __launch_bounds__(TH) void ColStepB(StepArgs a, const Cx<float>* __restrict__ in,
                                               Cx<float>* __restrict__ out,
                                               const Cx<float>* __restrict__ ptw) {
  constexpr bool PAD = PadOn(N1 * N2);
  constexpr uint32_t S = StrideIf<PAD>(N2);
  constexpr uint32_t N = N1 * N2;
  constexpr uint32_t COUNT = kTile * GB;
  constexpr uint32_t EL = COUNT * N2;
  constexpr uint32_t E = (EL + TH - 1) / TH;
  constexpr uint32_t NT = TableSize<1, R2...>();
  __shared__ Cx<float> buf[COUNT * S];
  __shared__ Cx<float> wt[NT > 0 ? NT : 1];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = blockIdx.x / (N1 / GB);
  const uint32_t k1_0 = (blockIdx.x % (N1 / GB)) * GB;
  const size_t base = size_t(tile) * N * kTile;
  for (uint32_t i = tid; i < NT; i += TH) wt[i] = ptw[i];
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t n2 = q % N2, g = q / N2;  // rows k1 N2 .. k1 N2 + N2 - 1: contiguous
    buf[(g * kTile + col) * S + PdIf<PAD>(n2)] = in[base + size_t((k1_0 + g) * N2 + n2) * kTile + col];
  }
  LdsSync();
  BFft<float, TH, N2, COUNT, S, 0, 1, R2...>(buf, wt, tid);
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t g = q % GB, k2 = q / GB;  // rows k1 + N1 k2: GB adjacent rows per k2
    Cx<float> v = buf[(g * kTile + col) * S + PdIf<PAD>(k2)];
    if (a.inverse) v = Conj(v);
    out[base + size_t(k1_0 + g + N1 * k2) * kTile + col] = v;
  }
}

// ------------------------------- several scales from one forward half
// The scale convolutions of one image (FindMultiScalePeak: every active
// scale's kernel times the same forward spectrum) without the forward
// spectrum ever reaching HBM. After A (forward), T[k1 N2 + n2] holds, per k1,
// the inputs of the length-N2 DFTs whose outputs are X[k1 + N1 k2]. The
// inverse of Y = X K s is conj(z), z = DFT(conj Y); with k = k1 + N1 k2 and
// m = m2 + N2 m1:
//   z[m2 + N2 m1] = sum_k1 W_N1^(m1 k1) W_N^(m2 k1) sum_k2 conj Y[k1 + N1 k2] W_N2^(m2 k2),
// so a workgroup holding one k1 group runs the forward B DFT, multiplies by
// each scale's (real, even) kernel, runs the inner inverse DFT over k2 and
// the twiddle W_N^(m2 k1) in LDS, and writes U_s[k1 N2 + m2] (B*, below);
// ColStepAInv then runs the outer DFT over k1 per m2 and stores conj(z) in
// natural order. Per scale that is one write + one read + one write of the
// spectrum (against read X + K, write, read, write for A(x K) + B), and the
// forward B pass is gone.
constexpr uint32_t kMaxScaleOuts = 8;
struct ScalesArgs {
  uint32_t n_tiles;
  uint32_t n_scales;
  float scale;                          // 1 / (W H)
  const float* kern[kMaxScaleOuts];     // real kernel spectra, float tiles (16 per row)
  Cx<float>* out[kMaxScaleOuts];        // U_s, the tiled spectrum layout
};

// B*: workgroup = (tile, GB consecutive k1). ptw: the length-N2 pass table;
// tw: the length-N table W_N^e.
template <uint32_t TH, uint32_t N1, uint32_t N2, uint32_t GB, uint32_t... R2>
__global__ __launch_bounds__(TH) void ColStepBScales(ScalesArgs a,
                                                     const Cx<float>* __restrict__ in,
                                                     const Cx<float>* __restrict__ tw,
                                                     const Cx<float>* __restrict__ ptw) {
  constexpr bool PAD = PadOn(N1 * N2);
  constexpr uint32_t S = StrideIf<PAD>(N2);
  constexpr uint32_t N = N1 * N2;
  constexpr uint32_t COUNT = kTile * GB;
  constexpr uint32_t EL = COUNT * N2;
  constexpr uint32_t E = (EL + TH - 1) / TH;
  constexpr uint32_t NT = TableSize<1, R2...>();
  __shared__ Cx<float> buf[COUNT * S];
  __shared__ Cx<float> wt[NT > 0 ? NT : 1];
  __shared__ Cx<float> wb[GB * N2];  // W_N^{m2 k1} of this workgroup's k1
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = blockIdx.x / (N1 / GB);
  const uint32_t k1_0 = (blockIdx.x % (N1 / GB)) * GB;
  const size_t base = size_t(tile) * N * kTile;
  for (uint32_t i = tid; i < NT; i += TH) wt[i] = ptw[i];
  for (uint32_t i = tid; i < GB * N2; i += TH) {
    const uint32_t g = i / N2, m2 = i % N2;
    wb[i] = tw[(m2 * (k1_0 + g)) % N];
  }
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t n2 = q % N2, g = q / N2;  // rows k1 N2 .. k1 N2 + N2 - 1: contiguous
    buf[(g * kTile + col) * S + PdIf<PAD>(n2)] = in[base + size_t((k1_0 + g) * N2 + n2) * kTile + col];
  }
  LdsSync();
  BFft<float, TH, N2, COUNT, S, 0, 1, R2...>(buf, wt, tid);
  // X[k1 + N1 k2] into registers: (col, g, k2), GB adjacent rows per k2
  Cx<float> X[E];
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t g = q % GB, k2 = q / GB;
    X[i] = buf[(g * kTile + col) * S + PdIf<PAD>(k2)];
  }
  for (uint32_t sc = 0; sc < a.n_scales; ++sc) {
    // opaque per scale (see Columns): the per-element addresses are
    // recomputed, not hoisted out of the loop into registers
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const float* __restrict__ kern = a.kern[sc];
    LdsSync();  // every read of buf (X, or the previous scale's stores) done
#pragma unroll
    for (uint32_t i = 0; i < E; ++i) {
      const uint32_t idx = tid + i * TH;
      if (EL % TH != 0 && idx >= EL) continue;
      const uint32_t col = idx % kTile, q = idx / kTile;
      const uint32_t g = q % GB, k2 = q / GB;
      const float k = kern[(size_t(tile) * N + k1_0 + g + N1 * k2) * kTile + col];
      // conj(X K s), K real: the complex product's terms with Im K = 0
      const Cx<float> v = {(X[i].x * k) * a.scale, -((X[i].y * k) * a.scale)};
      buf[(g * kTile + col) * S + PdIf<PAD>(k2)] = v;
    }
    LdsSync();
    BFft<float, TH, N2, COUNT, S, 0, 1, R2...>(buf, wt, tid);
    Cx<float>* __restrict__ out = a.out[sc];
#pragma unroll
    for (uint32_t i = 0; i < E; ++i) {
      const uint32_t idx = tid + i * TH;
      if (EL % TH != 0 && idx >= EL) continue;
      const uint32_t col = idx % kTile, q = idx / kTile;
      const uint32_t m2 = q % N2, g = q / N2;  // rows k1 N2 + m2: contiguous
      out[base + size_t((k1_0 + g) * N2 + m2) * kTile + col] =
          Mul(buf[(g * kTile + col) * S + PdIf<PAD>(m2)], wb[g * N2 + m2]);
    }
  }
}

// The outer inverse step: workgroup = (tile, GA consecutive m2): the length-N1
// DFTs over k1 of U[k1 N2 + m2], conj(z) to row m2 + N2 m1 (natural order).
template <uint32_t TH, uint32_t N1, uint32_t N2, uint32_t GA, uint32_t... R1>
__global__ __launch_bounds__(TH) void ColStepAInv(StepArgs a, const Cx<float>* __restrict__ in,
                                                  Cx<float>* __restrict__ out,
                                                  const Cx<float>* __restrict__ ptw) {
  constexpr uint32_t N = N1 * N2;
  constexpr bool PAD = PadOn(N1 * N2);
  constexpr uint32_t S = StrideIf<PAD>(N1);
  constexpr uint32_t COUNT = kTile * GA;
  constexpr uint32_t EL = COUNT * N1;
  constexpr uint32_t E = (EL + TH - 1) / TH;
  constexpr uint32_t NT = TableSize<1, R1...>();
  __shared__ Cx<float> buf[COUNT * S];
  __shared__ Cx<float> wt[NT > 0 ? NT : 1];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = blockIdx.x / (N2 / GA);
  const uint32_t m2_0 = (blockIdx.x % (N2 / GA)) * GA;
  const size_t base = size_t(tile) * N * kTile;
  for (uint32_t i = tid; i < NT; i += TH) wt[i] = ptw[i];
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t g = q % GA, k1 = q / GA;  // rows k1 N2 + m2_0 ..: GA contiguous
    buf[(g * kTile + col) * S + PdIf<PAD>(k1)] = in[base + size_t(k1 * N2 + m2_0 + g) * kTile + col];
  }
  LdsSync();
  BFft<float, TH, N1, COUNT, S, 0, 1, R1...>(buf, wt, tid);
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t idx = tid + i * TH;
    if (EL % TH != 0 && idx >= EL) continue;
    const uint32_t col = idx % kTile, q = idx / kTile;
    const uint32_t g = q % GA, m1 = q / GA;  // rows m2 + N2 m1: GA adjacent per m1
    out[base + size_t(m2_0 + g + N2 * m1) * kTile + col] =
        Conj(buf[(g * kTile + col) * S + PdIf<PAD>(m1)]);
  }
  (void)a;
}

// The real, even spectrum of a symmetric small kernel placed as
// PrepareSmallConvolutionKernel (centre at (0, 0), wrapped): with k even in
// x and y, K(u, v) = sum_y cos(2 pi v y / H) sum_x k(x, y) cos(2 pi u x / W),
// evaluated in double from cosine tables (cos_w[j] = cos(2 pi j / W), long
// double on the host, angles reduced exactly: (u x) mod W), rounded to float
// once. Stage 1: A[y][u] = k(0, y) + 2 sum_{x=1..r} k(x, y) cos(2 pi u x / W)
// for the kernel rows y = 0..r.
__global__ __launch_bounds__(256) void RealKernelRows(const float* __restrict__ shape,
                                                      uint32_t n, uint32_t w, uint32_t nu,
                                                      const double* __restrict__ cos_w,
                                                      double* __restrict__ a_out) {
  const uint32_t u = blockIdx.x * 256 + threadIdx.x;
  const uint32_t y = blockIdx.y;  // 0 .. r
  const uint32_t r = n / 2;
  if (u >= nu) return;
  const float* row = shape + size_t(r + y) * n + r;  // k(x, y) = row[x], x >= 0
  double acc = 0.0;
  uint32_t e = 0;  // (u x) mod w
  for (uint32_t x = 1; x <= r; ++x) {
    e += u;
    if (e >= w) e -= w;
    acc += double(row[x]) * cos_w[e];
  }
  a_out[size_t(y) * nu + u] = double(row[0]) + 2.0 * acc;
}

// Stage 2: K(u, v) = A[0][u] + 2 sum_{y=1..r} A[y][u] cos(2 pi v y / H), float,
// tiled (16 columns per row, tile after tile; columns >= nu zero).
__global__ __launch_bounds__(256) void RealKernelCols(const double* __restrict__ a_in,
                                                      uint32_t r, uint32_t h, uint32_t nu,
                                                      uint32_t n_tiles,
                                                      const double* __restrict__ cos_h,
                                                      float* __restrict__ out) {
  const size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  const size_t total = size_t(n_tiles) * h * kTile;
  if (i >= total) return;
  const uint32_t col = uint32_t(i % kTile);
  const uint32_t v = uint32_t((i / kTile) % h);
  const uint32_t tile = uint32_t(i / (size_t(kTile) * h));
  const uint32_t u = tile * kTile + col;
  if (u >= nu) {
    out[i] = 0.0f;
    return;
  }
  double acc = 0.0;
  uint32_t e = 0;  // (v y) mod h
  for (uint32_t y = 1; y <= r; ++y) {
    e += v;
    if (e >= h) e -= h;
    acc += a_in[size_t(y) * nu + u] * cos_h[e];
  }
  out[i] = float(a_in[u] + 2.0 * acc);
}

// row mask (one byte per plane row) -> ascending list of the non-zero rows
__global__ __launch_bounds__(1024) void CompactRows(const uint8_t* __restrict__ mask,
                                                    uint32_t n, uint32_t* __restrict__ rows,
                                                    uint32_t* __restrict__ count) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t base;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  if (tid == 0) base = 0;
  __syncthreads();
  for (uint32_t off = 0; off < n; off += 1024) {
    const uint32_t y = off + tid;
    const bool f = y < n && mask[y] != 0;
    const uint64_t bal = __ballot(f);
    const uint32_t before = __popcll(bal & ((uint64_t(1) << lane) - 1));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    uint32_t wbase = base;
    for (uint32_t w = 0; w < wave; ++w) wbase += wsum[w];
    if (f) rows[wbase + before] = y;
    __syncthreads();
    if (tid == 0)
      for (uint32_t w = 0; w < 16; ++w) base += wsum[w];
    __syncthreads();
  }
  if (tid == 0) *count = base;
}

}  // namespace ff

// ---------------------------------------------------------------- plans
// Supported transform lengths: columns (full length N) and rows (half length
// H = N / 2). Radices in pass order; double stays at radix <= 9 and keeps
// each pass's butterflies-per-thread x radix small (1024 threads leave 128
// VGPRs; checked spill-free with -Rpass-analysis=kernel-resource-usage).
#define RDL_FAST_COLS(T, TH, PF, ...)                                          \
  FastColumns {                                                                \
    ff::Product<__VA_ARGS__>(), sizeof(T) == 8, TH,                            \
        reinterpret_cast<const void*>(&ff::Columns<T, TH, PF, __VA_ARGS__>),   \
        MakeRadixList<__VA_ARGS__>()                                           \
  }
#define RDL_FAST_ROWS(T, TH, ...)                                                      \
  FastRows {                                                                           \
    2 * ff::Product<__VA_ARGS__>(), sizeof(T) == 8, TH,                                \
        reinterpret_cast<const void*>(&ff::RowsInverse<T, TH, false, __VA_ARGS__>),    \
        reinterpret_cast<const void*>(&ff::RowsForward<T, TH, false, __VA_ARGS__>),    \
        MakeRadixList<__VA_ARGS__>(), RowsLt<T, TH, __VA_ARGS__>(true),                \
        RowsLt<T, TH, __VA_ARGS__>(false), RowsDma<T, TH, __VA_ARGS__>(),             \
        RowsDmaLds<T, TH, __VA_ARGS__>(), RowsFwdDma<T, TH, __VA_ARGS__>(),             \
        RowsFwdDmaLds<T, TH, __VA_ARGS__>()                                            \
  }

// the LDS-DMA inverse rows (float, 8 or 16 output pairs per thread) and
// their one dynamic LDS array (RowsInverseDma's layout)
template <uint32_t TH, uint32_t... Rs>
constexpr size_t RowsDmaLdsBytes() {
  constexpr uint32_t H = ff::Product<Rs...>();
  constexpr uint32_t NT = (H + 1 + ff::kTile - 1) / ff::kTile;
  constexpr uint32_t NI = (NT + 7) / 8;
  constexpr uint32_t NCT = ff::CachedTableSize<1, Rs...>(TH, H);
  (void)NI;  // (the DMA target is a static array of the kernel)
  return size_t(H + (H >> kFastPadShift)) * 8 +
         size_t(2 * H / ff::kTwdLo + ff::kTwdLo) * 16 + size_t(NCT > 0 ? (NCT + 1) / 2 * 2 : 2) * 8 +
         size_t(TH / 64) * 8;
}
template <typename T, uint32_t TH, uint32_t... Rs>
size_t RowsDmaLds() {
  if constexpr (sizeof(T) == 4)
    return RowsDmaLdsBytes<TH, Rs...>();
  else
    return 0;
}
template <uint32_t TH, uint32_t... Rs>
constexpr size_t RowsFwdDmaLdsBytes() {
  constexpr uint32_t H = ff::Product<Rs...>();
  constexpr uint32_t NCT = ff::CachedTableSize<1, Rs...>(TH, H);
  return size_t(H + (H >> kFastPadShift)) * 8 + size_t(2 * H / ff::kTwdLo + ff::kTwdLo) * 16 +
         size_t(NCT > 0 ? NCT : 1) * 8;
}
template <typename T, uint32_t TH, uint32_t... Rs>
const void* RowsFwdDma() {
  constexpr uint32_t H = ff::Product<Rs...>();
  constexpr uint32_t NP = H / 2 + 1;
  constexpr uint32_t EP = (NP + TH - 1) / TH;
  if constexpr (sizeof(T) == 4 && H % TH == 0 && (H / TH == 16 || H / TH == 8) &&
                2 * (EP - 1) >= H / TH)
    return reinterpret_cast<const void*>(&ff::RowsForwardDma<TH, Rs...>);
  else
    return nullptr;
}
template <typename T, uint32_t TH, uint32_t... Rs>
size_t RowsFwdDmaLds() {
  if constexpr (sizeof(T) == 4)
    return RowsFwdDmaLdsBytes<TH, Rs...>();
  else
    return 0;
}
template <typename T, uint32_t TH, uint32_t... Rs>
const void* RowsDma() {
  constexpr uint32_t H = ff::Product<Rs...>();
  if constexpr (sizeof(T) == 4 && H % TH == 0 && (H / TH == 16 || H / TH == 8))
    return reinterpret_cast<const void*>(&ff::RowsInverseDma<TH, Rs...>);
  else
    return nullptr;
}

// the float row kernels with LDS double twiddles (none for double)
template <typename T, uint32_t TH, uint32_t... Rs>
const void* RowsLt(bool inverse) {
  if constexpr (sizeof(T) == 4)
    return inverse ? reinterpret_cast<const void*>(&ff::RowsInverse<T, TH, true, Rs...>)
                   : reinterpret_cast<const void*>(&ff::RowsForward<T, TH, true, Rs...>);
  else
    return nullptr;
}

const FastColumns* FindFastColumns(uint32_t n, bool f64) {
  static const FastColumns kPlans[] = {
      // float64 padded correction sizes of 8192^2 (scales 0..256) and 4096^2
      RDL_FAST_COLS(double, 1024, true, 7, 9, 9, 4, 4),        // 9072
      RDL_FAST_COLS(double, 1024, true, 9, 4, 4, 4, 4, 4),     // 9216
      RDL_FAST_COLS(double, 1024, true, 7, 3, 7, 4, 4, 4),     // 9408
      RDL_FAST_COLS(double, 1024, true, 7, 5, 3, 5, 3, 3, 2),  // 9450
      RDL_FAST_COLS(double, 1024, true, 7, 9, 9, 8),           // 4536
      RDL_FAST_COLS(double, 1024, true, 9, 8, 8, 8),           // 4608
      RDL_FAST_COLS(double, 1024, true, 7, 3, 7, 8, 4),        // 4704
      RDL_FAST_COLS(double, 1024, true, 5, 3, 5, 8, 8),        // 4800
      RDL_FAST_COLS(double, 1024, true, 5, 5, 5, 5, 8),        // 5000
      // float64 padded corrections of gridded runs' subimages
      // (GetConvolutionSize of ~1000-1700 pixel subimages; 1 KiB-36 KiB per
      // column, several workgroups per CU)
      RDL_FAST_COLS(double, 256, true, 7, 5, 5, 3, 2),                 // 1050
      RDL_FAST_COLS(double, 256, true, 5, 9, 3, 8),                    // 1080
      RDL_FAST_COLS(double, 256, true, 7, 5, 8, 4),                    // 1120
      RDL_FAST_COLS(double, 256, true, 7, 9, 9, 2),                    // 1134
      RDL_FAST_COLS(double, 256, true, 9, 8, 4, 4),                    // 1152
      RDL_FAST_COLS(double, 256, true, 7, 7, 3, 8),                    // 1176
      RDL_FAST_COLS(double, 256, true, 5, 5, 3, 4, 4),                 // 1200
      RDL_FAST_COLS(double, 256, true, 5, 5, 5, 5, 2),                 // 1250
      RDL_FAST_COLS(double, 256, true, 7, 5, 9, 4),                    // 1260
      RDL_FAST_COLS(double, 256, true, 5, 8, 8, 4),                    // 1280
      RDL_FAST_COLS(double, 256, true, 9, 9, 4, 4),                    // 1296
      RDL_FAST_COLS(double, 256, true, 7, 3, 8, 8),                    // 1344
      RDL_FAST_COLS(double, 256, true, 7, 7, 7, 4),                    // 1372
      RDL_FAST_COLS(double, 256, true, 7, 5, 5, 8),                    // 1400
      RDL_FAST_COLS(double, 256, true, 5, 9, 8, 4),                    // 1440
      RDL_FAST_COLS(double, 256, true, 9, 9, 9, 2),                    // 1458
      RDL_FAST_COLS(double, 256, true, 7, 7, 5, 3, 2),                 // 1470
      RDL_FAST_COLS(double, 256, true, 5, 5, 5, 3, 4),                 // 1500
      RDL_FAST_COLS(double, 256, true, 7, 9, 3, 8),                    // 1512
      RDL_FAST_COLS(double, 256, true, 3, 8, 8, 8),                    // 1536
      RDL_FAST_COLS(double, 256, true, 7, 7, 8, 4),                    // 1568
      RDL_FAST_COLS(double, 256, true, 5, 9, 9, 4),                    // 1620
      RDL_FAST_COLS(double, 256, true, 7, 5, 3, 4, 4),                 // 1680
      RDL_FAST_COLS(double, 256, true, 7, 5, 9, 3, 2),                 // 1890
      RDL_FAST_COLS(double, 256, true, 5, 3, 8, 8, 2),              // 1920
      RDL_FAST_COLS(double, 256, true, 9, 9, 3, 8),                 // 1944
      RDL_FAST_COLS(double, 256, true, 7, 7, 5, 8),                 // 1960
      RDL_FAST_COLS(double, 256, true, 5, 5, 5, 8, 2),              // 2000
      RDL_FAST_COLS(double, 256, true, 7, 9, 8, 4),                 // 2016
      RDL_FAST_COLS(double, 256, true, 8, 8, 8, 4),                 // 2048
      RDL_FAST_COLS(double, 256, true, 7, 5, 5, 3, 4),              // 2100
      RDL_FAST_COLS(double, 256, true, 5, 9, 3, 8, 2),              // 2160
      RDL_FAST_COLS(double, 256, true, 7, 5, 8, 8),                 // 2240
      RDL_FAST_COLS(double, 256, true, 5, 5, 5, 9, 2),              // 2250
      RDL_FAST_COLS(double, 256, true, 7, 9, 9, 4),                 // 2268
      RDL_FAST_COLS(double, 256, true, 9, 8, 8, 4),                 // 2304
      RDL_FAST_COLS(double, 256, true, 7, 7, 3, 8, 2),              // 2352
      RDL_FAST_COLS(double, 256, true, 5, 5, 3, 8, 4),              // 2400
      RDL_FAST_COLS(double, 256, true, 5, 9, 9, 3, 2),              // 2430
      RDL_FAST_COLS(double, 256, true, 7, 7, 5, 5, 2),              // 2450
      RDL_FAST_COLS(double, 256, true, 5, 5, 5, 5, 4),              // 2500
      RDL_FAST_COLS(double, 256, true, 7, 5, 9, 8),                 // 2520
      RDL_FAST_COLS(double, 256, true, 5, 8, 8, 8),                 // 2560
      RDL_FAST_COLS(double, 256, true, 9, 9, 8, 4),                 // 2592
      RDL_FAST_COLS(double, 256, true, 7, 7, 9, 3, 2),              // 2646
      RDL_FAST_COLS(double, 256, true, 7, 3, 8, 8, 2),              // 2688
      RDL_FAST_COLS(double, 256, true, 7, 7, 7, 8),                 // 2744
      RDL_FAST_COLS(double, 256, true, 7, 5, 5, 8, 2),              // 2800
      RDL_FAST_COLS(double, 256, true, 5, 9, 8, 8),                 // 2880
      RDL_FAST_COLS(double, 256, true, 9, 9, 9, 4),                 // 2916
      RDL_FAST_COLS(double, 256, true, 7, 7, 5, 3, 4),              // 2940
      RDL_FAST_COLS(double, 256, true, 5, 5, 5, 3, 8),              // 3000
      RDL_FAST_COLS(double, 256, true, 7, 9, 3, 8, 2),              // 3024
      RDL_FAST_COLS(double, 256, true, 3, 8, 8, 8, 2),              // 3072
      RDL_FAST_COLS(double, 256, true, 7, 7, 8, 8),                 // 3136
      RDL_FAST_COLS(double, 256, true, 7, 5, 5, 9, 2),              // 3150
      RDL_FAST_COLS(double, 256, true, 5, 5, 8, 8, 2),              // 3200
      RDL_FAST_COLS(double, 256, true, 5, 9, 9, 8),                 // 3240
      RDL_FAST_COLS(double, 256, true, 7, 5, 3, 8, 4),              // 3360
      RDL_FAST_COLS(double, 256, true, 7, 9, 9, 3, 2),              // 3402
      RDL_FAST_COLS(double, 256, true, 7, 7, 7, 5, 2),              // 3430
      RDL_FAST_COLS(double, 256, true, 7, 5, 5, 5, 4),              // 3500
      // float32 scale convolutions (two workgroups per CU)
      RDL_FAST_COLS(float, 512, true, 8, 8, 8, 16),            // 8192
      RDL_FAST_COLS(float, 512, true, 8, 8, 8, 8),             // 4096
      // the periodically extended subimage planes of a tiled run
      // (MultiScaleTransforms' CanonicalFftSize ladder)
      RDL_FAST_COLS(float, 512, true, 8, 8, 8, 7),             // 3584
      RDL_FAST_COLS(float, 512, true, 8, 8, 16, 3),            // 3072
      RDL_FAST_COLS(float, 512, true, 8, 8, 8, 5),             // 2560
      RDL_FAST_COLS(float, 512, true, 8, 8, 8, 4),             // 2048
      RDL_FAST_COLS(float, 512, true, 8, 8, 4, 7),             // 1792
      RDL_FAST_COLS(float, 512, true, 8, 8, 8, 3),             // 1536
      RDL_FAST_COLS(float, 512, true, 8, 8, 4, 5),             // 1280
  };
  for (const FastColumns& p : kPlans)
    if (p.n == n && p.f64 == f64) return &p;
  return nullptr;
}

const FastRows* FindFastRows(uint32_t n, bool f64) {
  static const FastRows kPlans[] = {
      RDL_FAST_ROWS(double, 512, 7, 9, 9, 8),      // 9072
      RDL_FAST_ROWS(double, 512, 9, 8, 8, 8),      // 9216
      RDL_FAST_ROWS(double, 512, 7, 3, 7, 8, 4),   // 9408
      RDL_FAST_ROWS(double, 512, 7, 5, 3, 5, 9),   // 9450
      RDL_FAST_ROWS(double, 256, 7, 9, 9, 4),      // 4536
      RDL_FAST_ROWS(double, 256, 9, 4, 4, 4, 4),   // 4608
      RDL_FAST_ROWS(double, 256, 7, 3, 7, 4, 4),   // 4704
      RDL_FAST_ROWS(double, 256, 5, 3, 5, 8, 4),   // 4800
      RDL_FAST_ROWS(double, 256, 5, 5, 5, 5, 4),   // 5000
      RDL_FAST_ROWS(double, 128, 7, 5, 5, 3),            // 1050
      RDL_FAST_ROWS(double, 128, 5, 9, 3, 4),            // 1080
      RDL_FAST_ROWS(double, 128, 7, 5, 4, 4),            // 1120
      RDL_FAST_ROWS(double, 128, 7, 9, 9),               // 1134
      RDL_FAST_ROWS(double, 128, 9, 8, 8),               // 1152
      RDL_FAST_ROWS(double, 128, 7, 7, 3, 4),            // 1176
      RDL_FAST_ROWS(double, 128, 5, 5, 3, 8),            // 1200
      RDL_FAST_ROWS(double, 128, 5, 5, 5, 5),            // 1250
      RDL_FAST_ROWS(double, 128, 7, 5, 9, 2),            // 1260
      RDL_FAST_ROWS(double, 128, 5, 8, 4, 4),            // 1280
      RDL_FAST_ROWS(double, 128, 9, 9, 8),               // 1296
      RDL_FAST_ROWS(double, 128, 7, 3, 8, 4),            // 1344
      RDL_FAST_ROWS(double, 128, 7, 7, 7, 2),            // 1372
      RDL_FAST_ROWS(double, 128, 7, 5, 5, 4),            // 1400
      RDL_FAST_ROWS(double, 128, 5, 9, 4, 4),            // 1440
      RDL_FAST_ROWS(double, 128, 9, 9, 9),               // 1458
      RDL_FAST_ROWS(double, 128, 7, 7, 5, 3),            // 1470
      RDL_FAST_ROWS(double, 128, 5, 5, 5, 3, 2),         // 1500
      RDL_FAST_ROWS(double, 128, 7, 9, 3, 4),            // 1512
      RDL_FAST_ROWS(double, 128, 3, 8, 8, 4),            // 1536
      RDL_FAST_ROWS(double, 128, 7, 7, 4, 4),            // 1568
      RDL_FAST_ROWS(double, 128, 5, 9, 9, 2),            // 1620
      RDL_FAST_ROWS(double, 128, 7, 5, 3, 8),            // 1680
      RDL_FAST_ROWS(double, 128, 7, 5, 9, 3),            // 1890
      RDL_FAST_ROWS(double, 256, 5, 3, 8, 8),         // 1920
      RDL_FAST_ROWS(double, 256, 9, 9, 3, 4),         // 1944
      RDL_FAST_ROWS(double, 256, 7, 7, 5, 4),         // 1960
      RDL_FAST_ROWS(double, 256, 5, 5, 5, 8),         // 2000
      RDL_FAST_ROWS(double, 256, 7, 9, 8, 2),         // 2016
      RDL_FAST_ROWS(double, 256, 8, 8, 8, 2),         // 2048
      RDL_FAST_ROWS(double, 256, 7, 5, 5, 3, 2),      // 2100
      RDL_FAST_ROWS(double, 256, 5, 9, 3, 8),         // 2160
      RDL_FAST_ROWS(double, 256, 7, 5, 8, 4),         // 2240
      RDL_FAST_ROWS(double, 256, 5, 5, 5, 9),         // 2250
      RDL_FAST_ROWS(double, 256, 7, 9, 9, 2),         // 2268
      RDL_FAST_ROWS(double, 256, 9, 8, 8, 2),         // 2304
      RDL_FAST_ROWS(double, 256, 7, 7, 3, 8),         // 2352
      RDL_FAST_ROWS(double, 256, 5, 5, 3, 8, 2),      // 2400
      RDL_FAST_ROWS(double, 256, 5, 9, 9, 3),         // 2430
      RDL_FAST_ROWS(double, 256, 7, 7, 5, 5),         // 2450
      RDL_FAST_ROWS(double, 256, 5, 5, 5, 5, 2),      // 2500
      RDL_FAST_ROWS(double, 256, 7, 5, 9, 4),         // 2520
      RDL_FAST_ROWS(double, 256, 5, 8, 8, 4),         // 2560
      RDL_FAST_ROWS(double, 256, 9, 9, 8, 2),         // 2592
      RDL_FAST_ROWS(double, 256, 7, 7, 9, 3),         // 2646
      RDL_FAST_ROWS(double, 256, 7, 3, 8, 8),         // 2688
      RDL_FAST_ROWS(double, 256, 7, 7, 7, 4),         // 2744
      RDL_FAST_ROWS(double, 256, 7, 5, 5, 8),         // 2800
      RDL_FAST_ROWS(double, 256, 5, 9, 8, 4),         // 2880
      RDL_FAST_ROWS(double, 256, 9, 9, 9, 2),         // 2916
      RDL_FAST_ROWS(double, 256, 7, 7, 5, 3, 2),      // 2940
      RDL_FAST_ROWS(double, 256, 5, 5, 5, 3, 4),      // 3000
      RDL_FAST_ROWS(double, 256, 7, 9, 3, 8),         // 3024
      RDL_FAST_ROWS(double, 256, 3, 8, 8, 8),         // 3072
      RDL_FAST_ROWS(double, 256, 7, 7, 8, 4),         // 3136
      RDL_FAST_ROWS(double, 256, 7, 5, 5, 9),         // 3150
      RDL_FAST_ROWS(double, 256, 5, 5, 8, 8),         // 3200
      RDL_FAST_ROWS(double, 256, 5, 9, 9, 4),         // 3240
      RDL_FAST_ROWS(double, 256, 7, 5, 3, 8, 2),      // 3360
      RDL_FAST_ROWS(double, 256, 7, 9, 9, 3),         // 3402
      RDL_FAST_ROWS(double, 256, 7, 7, 7, 5),         // 3430
      RDL_FAST_ROWS(double, 256, 7, 5, 5, 5, 2),      // 3500
      RDL_FAST_ROWS(float, 256, 16, 16, 16),       // 8192
      RDL_FAST_ROWS(float, 256, 16, 16, 8),        // 4096
      RDL_FAST_ROWS(float, 256, 16, 16, 7),        // 3584
      RDL_FAST_ROWS(float, 256, 16, 16, 2, 3),     // 3072
      RDL_FAST_ROWS(float, 256, 16, 16, 5),        // 2560
      RDL_FAST_ROWS(float, 256, 16, 16, 4),        // 2048
      RDL_FAST_ROWS(float, 256, 16, 8, 7),         // 1792
      RDL_FAST_ROWS(float, 256, 16, 16, 3),        // 1536
      RDL_FAST_ROWS(float, 256, 16, 8, 5),         // 1280
  };
  for (const FastRows& p : kPlans)
    if (p.n == n && p.f64 == f64) return &p;
  return nullptr;
}

#undef RDL_FAST_COLS
#undef RDL_FAST_ROWS

#define RDL_CONV_D(TH, ...)                                                    \
  FastColumns {                                                                \
    ff::Product<__VA_ARGS__>(), true, TH,                                      \
        reinterpret_cast<const void*>(&ff::ColumnsConvD<TH, false, __VA_ARGS__>), \
        MakeRadixList<__VA_ARGS__>(),                                          \
        reinterpret_cast<const void*>(&ff::ColumnsConvD<TH, true, __VA_ARGS__>)  \
  }
const FastColumns* FindConvColumnsD(uint32_t n) {
  static const FastColumns kPlans[] = {
      RDL_CONV_D(512, 7, 9, 9, 4, 4),        // 9072
      RDL_CONV_D(512, 9, 4, 4, 4, 4, 4),     // 9216
      RDL_CONV_D(512, 7, 3, 7, 4, 4, 4),     // 9408
      RDL_CONV_D(512, 7, 5, 3, 5, 3, 3, 2),  // 9450
      RDL_CONV_D(512, 7, 9, 9, 8),           // 4536
      RDL_CONV_D(512, 9, 8, 8, 8),           // 4608
      RDL_CONV_D(512, 7, 3, 7, 8, 4),        // 4704
      RDL_CONV_D(512, 5, 3, 5, 8, 8),        // 4800
      RDL_CONV_D(512, 5, 5, 5, 5, 8),        // 5000
  };
  // 1024-thread plans of the large sizes (one column's 145 KiB of LDS per
  // CU: twice the waves cover the passes' LDS and memory waits; 9072:
  // 779 -> 661 us, tools/bench_fftk.py f64); RDL_FFT_CONVD=512 keeps the
  // 512-thread plans, =0 disables the engine
  static const FastColumns kPlans1024[] = {
      RDL_CONV_D(1024, 7, 9, 9, 4, 4),        // 9072
      RDL_CONV_D(1024, 9, 4, 4, 4, 4, 4),     // 9216
      RDL_CONV_D(1024, 7, 3, 7, 4, 4, 4),     // 9408
      RDL_CONV_D(1024, 7, 5, 3, 5, 3, 3, 2),  // 9450
  };
  static const int mode = [] {
    const char* e = std::getenv("RDL_FFT_CONVD");
    return !e ? 2 : e[0] == '0' ? 0 : std::atoi(e) == 512 ? 1 : 2;
  }();
  if (mode == 0) return nullptr;
  if (mode == 2)
    for (const FastColumns& p : kPlans1024)
      if (p.n == n) return &p;
  for (const FastColumns& p : kPlans)
    if (p.n == n) return &p;
  return nullptr;
}
#undef RDL_CONV_D

size_t ConvColumnsDLdsBytes(uint32_t n) {
  return size_t(n) * 16 + size_t((n + ff::kTwLo - 1) / ff::kTwLo + ff::kTwLo) * 16 +
         size_t((n + 31) / 32) * 4;
}

#define RDL_FAST_STEPS(N1, N2, GA, GB, RA, RB)                                     \
  FastSteps {                                                                      \
    N1 * N2, N1, N2, GA, GB, 256,                                                  \
        reinterpret_cast<const void*>(&ff::ColStepA<256, N1, N2, GA, RA>),         \
        reinterpret_cast<const void*>(&ff::ColStepB<256, N1, N2, GB, RB>),         \
        MakeRadixList<RA>(), MakeRadixList<RB>(),                                  \
        reinterpret_cast<const void*>(&ff::ColStepBScales<256, N1, N2, GB, RB>),   \
        reinterpret_cast<const void*>(&ff::ColStepAInv<256, N1, N2, GA, RA>)       \
  }
#define RDL_R(...) __VA_ARGS__

const FastSteps* FindFastSteps(uint32_t n) {
  static const FastSteps kPlans[] = {
      RDL_FAST_STEPS(64, 128, 4, 2, RDL_R(8, 8), RDL_R(16, 8)),  // 8192
      RDL_FAST_STEPS(64, 64, 4, 4, RDL_R(8, 8), RDL_R(8, 8)),    // 4096
      RDL_FAST_STEPS(64, 56, 4, 4, RDL_R(8, 8), RDL_R(8, 7)),    // 3584
      RDL_FAST_STEPS(64, 48, 4, 4, RDL_R(8, 8), RDL_R(16, 3)),   // 3072
      RDL_FAST_STEPS(64, 40, 4, 4, RDL_R(8, 8), RDL_R(8, 5)),    // 2560
      RDL_FAST_STEPS(32, 64, 4, 4, RDL_R(8, 4), RDL_R(8, 8)),    // 2048
      RDL_FAST_STEPS(32, 56, 4, 4, RDL_R(8, 4), RDL_R(8, 7)),    // 1792
      RDL_FAST_STEPS(32, 48, 4, 4, RDL_R(8, 4), RDL_R(16, 3)),   // 1536
      RDL_FAST_STEPS(32, 40, 4, 4, RDL_R(8, 4), RDL_R(8, 5)),    // 1280
  };
  for (const FastSteps& p : kPlans)
    if (p.n == n) return &p;
  return nullptr;
}

#undef RDL_FAST_STEPS
#undef RDL_R

namespace {
// workgroups per CU for a kernel at its LDS size (cached), after raising its
// dynamic LDS limit once per device
int SlotsPerCu(rdl_session* s, const void* fn, uint32_t threads, size_t lds) {
  static std::mutex mutex;
  static std::map<std::tuple<const void*, int, size_t>, int> cache;
  std::lock_guard<std::mutex> lock(mutex);
  const auto key = std::make_tuple(fn, s->device, lds);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  // (below the CU's LDS by the kernel's static arrays: the row kernels'
  // reduction array for the fused peak search and the float rows' twiddle
  // tables)
  hipFuncAttributes attr{};
  if (hipFuncGetAttributes(&attr, fn) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if (attr.sharedSizeBytes >= kFftLdsBytesFast ||
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                          int(kFftLdsBytesFast - attr.sharedSizeBytes)) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, int(threads), lds) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  cache[key] = std::max(n, 1);
  return cache[key];
}
}  // namespace

int FastColumnsLaunch(rdl_session* s, const FastColumns* p, const void* in, void* out,
                      const void* kern, const void* ptw, uint32_t n_cols, uint32_t mode,
                      int in_cm, int out_cm, int kern_cm, const uint32_t* rows,
                      const uint32_t* n_rows, uint32_t row0, uint32_t row_n,
                      double scale) {
  const size_t lds = FastLdsBytes(p->n, p->f64);
  const int slots = SlotsPerCu(s, p->kernel, p->threads, lds);
  if (slots < 0) {
    SetError("fast FFT columns: occupancy query failed");
    return RDL_ERR_HIP;
  }
  ff::ColArgs a{};
  a.n_cols = n_cols;
  a.ld = n_cols;
  a.mode = mode;
  a.in_cm = in_cm ? 1u : 0u;
  a.out_cm = out_cm ? 1u : 0u;
  a.kern_cm = kern_cm ? 1u : 0u;
  a.rows = rows;
  a.n_rows = n_rows;
  a.row0 = rows ? 0u : row0;
  a.row_n = rows ? p->n : row_n;
  a.scale = scale;
  const uint32_t want = std::min<uint32_t>(n_cols, uint32_t(s->n_cus) * uint32_t(slots));
  a.per_xcd = std::max<uint32_t>(1, (want + 7) / 8);
  const uint32_t grid = 8 * a.per_xcd;
  void* args[] = {&a, (void*)&in, (void*)&out, (void*)&kern, (void*)&ptw};
  RDL_HIP_CHECK(hipLaunchKernel(p->kernel, dim3(grid), dim3(p->threads), args, lds,
                                s->stream));
  return RDL_OK;
}

int ConvColumnsDLaunch(rdl_session* s, const FastColumns* p, const void* in, void* out,
                       const void* kern, const void* tw, uint32_t n_cols, int kern_cm,
                       int out_cm, const uint32_t* rows, const uint32_t* n_rows, uint32_t row0,
                       uint32_t row_n, double scale, uint32_t out_row0, uint32_t out_row_n,
                       bool kernel_f32, bool tiled) {
  const size_t lds = ConvColumnsDLdsBytes(p->n);
  const void* fn = kernel_f32 ? p->kernel_kf : p->kernel;
  if (!fn) {
    SetError("float64 correction columns: no float-kernel plan");
    return RDL_ERR_UNSUPPORTED;
  }
  const int slots = SlotsPerCu(s, fn, p->threads, lds);
  if (slots < 0) {
    SetError("float64 correction columns: occupancy query failed");
    return RDL_ERR_HIP;
  }
  ff::ColArgs a{};
  a.n_cols = n_cols;
  a.ld = n_cols;
  a.mode = 1;
  a.kern_cm = kern_cm ? 1u : 0u;
  a.out_cm = out_cm ? 1u : 0u;
  a.rows = rows;
  a.n_rows = n_rows;
  a.row0 = rows ? 0u : row0;
  a.row_n = rows ? p->n : row_n;
  a.scale = scale;
  a.out_row0 = out_row0;
  a.out_row_n = out_row_n;
  a.tiled = tiled ? 1u : 0u;

  const uint32_t want = std::min<uint32_t>(n_cols, uint32_t(s->n_cus) * uint32_t(slots));
  a.per_xcd = std::max<uint32_t>(1, (want + 7) / 8);
  const uint32_t grid = 8 * a.per_xcd;
  void* args[] = {&a, (void*)&in, (void*)&out, (void*)&kern, (void*)&tw};
  RDL_HIP_CHECK(hipLaunchKernel(fn, dim3(grid), dim3(p->threads), args, lds, s->stream));
  return RDL_OK;
}

namespace {
// RDL_FFT_ROWTW=0: the float row kernels with global pass tables (comparison)
bool RowTwiddlesInLds() {
  static const bool on = [] {
    const char* e = std::getenv("RDL_FFT_ROWTW");
    return !(e && e[0] == '0');
  }();
  return on;
}
}  // namespace

int FastRowsInverseLaunch(rdl_session* s, const FastRows* p, const void* spec, float* out,
                          const void* tw, const void* ptw, uint32_t height, uint32_t img_w, uint32_t img_h,
                          uint32_t ox, uint32_t oy, int subtract, int tiled, const RowPeak* peak,
                          const void* twd, uint32_t* n_partials) {
  // the LDS-DMA kernel: a tiled float spectrum written whole into the
  // window (RDL_ROWS_DMA=0: the persistent row kernel)
  if (n_partials) *n_partials = img_h;  // per-row partials (the persistent row kernel)
  static const bool dma_on = [] {
    const char* e = std::getenv("RDL_ROWS_DMA");
    return !(e && e[0] == '0');
  }();
  const uint32_t half = p->n / 2;
  if (dma_on && p->inverse_dma && twd && RowTwiddlesInLds() && tiled && !subtract && ox == 0 && img_w == p->n &&
      img_h > 0) {
    const size_t lds = p->inverse_dma_lds;
    const int slots = SlotsPerCu(s, p->inverse_dma, p->threads, lds);
    if (slots < 0) {
      SetError("fast FFT rows (DMA): occupancy query failed");
      return RDL_ERR_HIP;
    }
    ff::RowArgs a{};
    a.height = height;
    a.ld = half + 1;
    a.img_w = img_w;
    a.img_h = img_h;
    a.ox = ox;
    a.oy = oy;
    a.tiled = 1;
    if (peak) a.peak = *peak;
    const uint32_t grid = std::min<uint32_t>(img_h, uint32_t(s->n_cus) * uint32_t(slots));
    void* args[] = {&a, (void*)&spec, (void*)&out, (void*)&twd};
    RDL_HIP_CHECK(hipLaunchKernel(p->inverse_dma, dim3(grid), dim3(p->threads), args, lds,
                                  s->stream));
    if (n_partials) *n_partials = grid;  // one partial per workgroup
    return RDL_OK;
  }
  const size_t lds = FastLdsBytes(p->n / 2, p->f64);
  const bool lt = p->inverse_lt && twd && RowTwiddlesInLds();
  const void* fn = lt ? p->inverse_lt : p->inverse;
  const int slots = SlotsPerCu(s, fn, p->threads, lds);
  if (slots < 0) {
    SetError("fast FFT rows: occupancy query failed");
    return RDL_ERR_HIP;
  }
  if (img_h == 0) return RDL_OK;
  ff::RowArgs a{};
  a.height = height;
  a.ld = p->n / 2 + 1;
  a.img_w = img_w;
  a.img_h = img_h;
  a.ox = ox;
  a.oy = oy;
  a.subtract = subtract;
  a.tiled = tiled;
  if (peak) a.peak = *peak;
  // RDL_ROWS_RPRE=0: the residual read where it is subtracted (comparison)
  static const int rpre = [] {
    const char* e = std::getenv("RDL_ROWS_RPRE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  a.prefetch = rpre;
  // LT kernels are persistent (rows grid-strided): one table load per workgroup.
  // A session with a second lane keeps one slot per CU free for the other
  // lane's column passes (8192^2 bench: 762.8 -> 757.3 ms per step; 770.9
  // with one lane), RDL_ROWS_PER_CU sets the cap
  static const int cap_env = [] {
    const char* e = std::getenv("RDL_ROWS_PER_CU");
    return e ? std::atoi(e) : 0;
  }();
  const int cap = cap_env > 0 ? cap_env : (s->aux && slots >= 4 ? slots - 1 : slots);
  const uint32_t per_cu = uint32_t(cap < slots ? cap : slots);
  const uint32_t grid =
      lt ? std::min<uint32_t>(img_h, uint32_t(s->n_cus) * per_cu) : img_h;
  void* args[] = {&a, (void*)&spec, (void*)&out, (void*)&tw, (void*)&ptw, (void*)&twd};
  RDL_HIP_CHECK(hipLaunchKernel(fn, dim3(grid), dim3(p->threads), args, lds, s->stream));
  return RDL_OK;
}

int FastRowsForwardLaunch(rdl_session* s, const FastRows* p, const float* in, void* spec,
                          const void* tw, const void* ptw, uint32_t height, uint32_t img_w, uint32_t img_h,
                          uint32_t ox, uint32_t oy, const uint32_t* rows,
                          const uint32_t* n_rows, int tiled, const void* twd, int all_rows) {
  // the LDS-DMA kernel: a whole float plane into a tiled spectrum
  // (RDL_ROWS_DMA=0: the persistent row kernel)
  static const bool dma_on = [] {
    const char* e = std::getenv("RDL_ROWS_DMA");
    return !(e && e[0] == '0');
  }();
  if (dma_on && p->forward_dma && twd && RowTwiddlesInLds() && tiled && !rows && ox == 0 &&
      oy == 0 && img_w == p->n && img_h == height && height > 0) {
    const size_t lds = p->forward_dma_lds;
    const int slots = SlotsPerCu(s, p->forward_dma, p->threads, lds);
    if (slots < 0) {
      SetError("fast FFT rows (DMA): occupancy query failed");
      return RDL_ERR_HIP;
    }
    ff::RowArgs a{};
    a.height = height;
    a.ld = p->n / 2 + 1;
    a.img_w = img_w;
    a.img_h = img_h;
    a.tiled = 1;
    a.all_rows = 1;
    const uint32_t grid = std::min<uint32_t>(height, uint32_t(s->n_cus) * uint32_t(slots));
    void* args[] = {&a, (void*)&in, (void*)&spec, (void*)&twd};
    RDL_HIP_CHECK(hipLaunchKernel(p->forward_dma, dim3(grid), dim3(p->threads), args, lds,
                                  s->stream));
    return RDL_OK;
  }
  const size_t lds = FastLdsBytes(p->n / 2, p->f64);
  const bool lt = p->forward_lt && twd && RowTwiddlesInLds();
  const void* fn = lt ? p->forward_lt : p->forward;
  const int slots = SlotsPerCu(s, fn, p->threads, lds);
  if (slots < 0) {
    SetError("fast FFT rows: occupancy query failed");
    return RDL_ERR_HIP;
  }
  ff::RowArgs a{};
  a.height = height;
  a.ld = p->n / 2 + 1;
  a.img_w = img_w;
  a.img_h = img_h;
  a.ox = ox;
  a.oy = oy;
  a.rows = rows;
  a.n_rows = n_rows;
  a.tiled = tiled;
  // (all_rows < 0: every plane row for a tiled spectrum, the window rows otherwise)
  a.all_rows = all_rows < 0 ? tiled : all_rows;
  const uint32_t max_rows = (rows || a.all_rows) ? height : img_h;
  if (max_rows == 0) return RDL_OK;
  const uint32_t grid =
      std::min<uint32_t>(max_rows, uint32_t(s->n_cus) * uint32_t(slots) * 2);
  void* args[] = {&a, (void*)&in, (void*)&spec, (void*)&tw, (void*)&ptw, (void*)&twd};
  RDL_HIP_CHECK(hipLaunchKernel(fn, dim3(grid), dim3(p->threads), args, lds, s->stream));
  return RDL_OK;
}

int MakeTwiddleBase(uint32_t base, void** out, hipStream_t stream) {
  // W_base^{64 i} for i < base / 64, then W_base^i for i < 64, in double
  std::vector<double> host;
  auto put = [&](uint64_t e) {
    const long double ang = -2.0L * 3.14159265358979323846264338327950288L *
                            (long double)(e % base) / base;
    host.push_back(double(std::cos(ang)));
    host.push_back(double(std::sin(ang)));
  };
  for (uint32_t i = 0; i < base / ff::kTwdLo; ++i) put(uint64_t(i) * ff::kTwdLo);
  for (uint32_t i = 0; i < ff::kTwdLo; ++i) put(i);
  RDL_HIP_CHECK(rdl::DevMalloc(out, host.size() * sizeof(double)));
  RDL_HIP_CHECK(UploadSync(*out, host.data(), host.size() * sizeof(double), stream));
  return RDL_OK;
}

int FastStepLaunch(rdl_session* s, const FastSteps* p, bool pass_b, const void* in,
                   void* out, const void* kern, const void* tw, const void* ptw,
                   uint32_t n_cols, int inverse, float scale) {
  ff::StepArgs a{};
  a.n_tiles = (n_cols + ff::kTile - 1) / ff::kTile;
  a.inverse = inverse;
  a.scale = scale;
  if (pass_b) {
    const uint32_t grid = a.n_tiles * (p->n1 / p->gb);
    void* args[] = {&a, (void*)&in, (void*)&out, (void*)&ptw};
    RDL_HIP_CHECK(hipLaunchKernel(p->step_b, dim3(grid), dim3(p->threads), args, 0,
                                  s->stream));
  } else {
    const uint32_t grid = a.n_tiles * (p->n2 / p->ga);
    void* args[] = {&a, (void*)&in, (void*)&out, (void*)&kern, (void*)&tw, (void*)&ptw};
    RDL_HIP_CHECK(hipLaunchKernel(p->step_a, dim3(grid), dim3(p->threads), args, 0,
                                  s->stream));
  }
  return RDL_OK;
}

int FastScalesLaunch(rdl_session* s, const FastSteps* p, const void* in, const void* tw,
                     const void* ptw_b, uint32_t n_cols, uint32_t n_scales,
                     const float* const* kerns, void* const* outs, float scale) {
  if (n_scales == 0) return RDL_OK;
  if (n_scales > ff::kMaxScaleOuts) {
    SetError("scale convolutions: at most 8 scales per launch");
    return RDL_ERR_ARG;
  }
  ff::ScalesArgs a{};
  a.n_tiles = (n_cols + ff::kTile - 1) / ff::kTile;
  a.n_scales = n_scales;
  a.scale = scale;
  for (uint32_t i = 0; i < n_scales; ++i) {
    a.kern[i] = kerns[i];
    a.out[i] = static_cast<Cx<float>*>(outs[i]);
  }
  const uint32_t grid = a.n_tiles * (p->n1 / p->gb);
  void* args[] = {&a, (void*)&in, (void*)&tw, (void*)&ptw_b};
  RDL_HIP_CHECK(hipLaunchKernel(p->step_b_scales, dim3(grid), dim3(p->threads), args, 0,
                                s->stream));
  return RDL_OK;
}

int FastStepAInvLaunch(rdl_session* s, const FastSteps* p, const void* in, void* out,
                       const void* ptw_a, uint32_t n_cols) {
  ff::StepArgs a{};
  a.n_tiles = (n_cols + ff::kTile - 1) / ff::kTile;
  const uint32_t grid = a.n_tiles * (p->n2 / p->ga);
  void* args[] = {&a, (void*)&in, (void*)&out, (void*)&ptw_a};
  RDL_HIP_CHECK(hipLaunchKernel(p->step_a_inv, dim3(grid), dim3(p->threads), args, 0,
                                s->stream));
  return RDL_OK;
}

int MakeCosTable(uint32_t n, void** out, hipStream_t stream) {
  std::vector<double> host(n);
  for (uint32_t j = 0; j < n; ++j)
    host[j] = double(std::cos(2.0L * 3.14159265358979323846264338327950288L *
                              (long double)j / n));
  RDL_HIP_CHECK(rdl::DevMalloc(out, host.size() * sizeof(double)));
  RDL_HIP_CHECK(UploadSync(*out, host.data(), host.size() * sizeof(double), stream));
  return RDL_OK;
}

int RealKernelLaunch(rdl_session* s, const float* shape, uint32_t n, uint32_t w, uint32_t h,
                     const void* cos_w, const void* cos_h, void* a_scratch, float* out) {
  const uint32_t nu = w / 2 + 1;
  const uint32_t r = n / 2;
  const uint32_t n_tiles = (nu + ff::kTile - 1) / ff::kTile;
  ff::RealKernelRows<<<dim3((nu + 255) / 256, r + 1), 256, 0, s->stream>>>(
      shape, n, w, nu, static_cast<const double*>(cos_w), static_cast<double*>(a_scratch));
  RDL_HIP_CHECK(hipGetLastError());
  const size_t total = size_t(n_tiles) * h * ff::kTile;
  ff::RealKernelCols<<<dim3(uint32_t((total + 255) / 256)), 256, 0, s->stream>>>(
      static_cast<const double*>(a_scratch), r, h, nu, n_tiles,
      static_cast<const double*>(cos_h), out);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int MakePassTable(uint32_t n, const RadixList& radix, bool f64, void** out,
                  hipStream_t stream) {
  std::vector<double> re, im;
  uint32_t ns = 1;
  for (uint32_t p = 0; p < radix.n; ++p) {
    const uint32_t r = radix.r[p];
    const uint32_t m = n / (ns * r);
    if (ns > 1)
      for (uint32_t q = 0; q + 1 < r; ++q)
        for (uint32_t k = 0; k < ns; ++k) {
          const uint64_t e = (uint64_t(k) * (q + 1) * m) % n;
          const long double ang =
              -2.0L * 3.14159265358979323846264338327950288L * (long double)e / n;
          re.push_back(double(std::cos(ang)));
          im.push_back(double(std::sin(ang)));
        }
    ns *= r;
  }
  const size_t count = std::max<size_t>(re.size(), 1);
  std::vector<unsigned char> host(count * (f64 ? 16 : 8), 0);
  for (size_t i = 0; i < re.size(); ++i) {
    if (f64) {
      const double v[2] = {re[i], im[i]};
      std::memcpy(&host[i * 16], v, 16);
    } else {
      const float v[2] = {float(re[i]), float(im[i])};
      std::memcpy(&host[i * 8], v, 8);
    }
  }
  RDL_HIP_CHECK(rdl::DevMalloc(out, host.size()));
  RDL_HIP_CHECK(UploadSync(*out, host.data(), host.size(), stream));
  return RDL_OK;
}

int FastCompactRows(rdl_session* s, const uint8_t* mask, uint32_t n, uint32_t* rows,
                    uint32_t* count) {
  ff::CompactRows<<<1, 1024, 0, s->stream>>>(mask, n, rows, count);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // namespace rdl
