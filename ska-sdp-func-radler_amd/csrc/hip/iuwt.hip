// IUWT à-trous B3-spline decomposition and recomposition (IuwtDecomposition,
// cpp/algorithms/iuwt/iuwt_decomposition.cc:9-237, .h:94-146, 243-261).
//
// Separable 5-tap filter h = (1, 4, 6, 4, 1)/16 with spacing d = 2^(s+1)-1 and
// zero boundaries. Each output pixel is computed by one thread with the
// reference's tap order per boundary region and its FMA contraction
// (t0 + t1 + ... -> fma(x_k, h_k, ... fma(x_0, h_0, x_1*h_1)); see
// oracle/iuwt.cc), so results are bit-identical to the reference build.
// Decompose(x, x, ..) — input used as its own scratch, as the reference's IUWT
// deconvolution does — makes the first horizontal pass a recursive in-place row
// filter; that case runs one thread per row, left to right.
#include "rdl_internal.h"

namespace rdl {

__device__ __forceinline__ float IuwtTap(int k) {
  return k == 2 ? 6.0f / 16.0f : (k == 1 || k == 3) ? 4.0f / 16.0f : 1.0f / 16.0f;
}

// taps in `order` (first two: x[o0]*h + x[o1]*h contracted as fma(x0, h0, x1*h1))
template <int N>
__device__ __forceinline__ float TapSum(const float* t, const int (&order)[N]) {
  float acc = t[order[1]] * IuwtTap(order[1]);
  acc = __builtin_fmaf(t[order[0]], IuwtTap(order[0]), acc);
#pragma unroll
  for (int i = 2; i < N; ++i) acc = __builtin_fmaf(t[order[i]], IuwtTap(order[i]), acc);
  return acc;
}

// convolveHorizontalFast regions (iuwt_decomposition.cc:84-131)
__device__ __forceinline__ float HorizontalValue(const float* t, int64_t x,
                                                 int64_t w, int d) {
  if (x < d) return TapSum<3>(t, {2, 3, 4});
  if (x < 2 * d) return TapSum<4>(t, {2, 1, 3, 4});
  if (x < w - 2 * d) return TapSum<5>(t, {2, 1, 0, 3, 4});
  if (x < w - d) return TapSum<4>(t, {2, 1, 0, 3});
  return TapSum<3>(t, {2, 1, 0});
}

// convolveVerticalPartialFast regions (iuwt_decomposition.cc:172-235)
__device__ __forceinline__ float VerticalValue(const float* t, int64_t y,
                                               int64_t h, int d) {
  if (y < d) return TapSum<3>(t, {2, 3, 4});
  if (y < 2 * d) return TapSum<4>(t, {1, 2, 3, 4});
  if (y < h - 2 * d) return TapSum<5>(t, {0, 1, 2, 3, 4});
  if (y < h - d) return TapSum<4>(t, {0, 1, 2, 3});
  return TapSum<3>(t, {0, 1, 2});
}

// The dispatcher deals workgroups round-robin over the 8 XCDs; a workgroup's
// row comes from its XCD's contiguous band of rows, so the vertical taps
// (rows y +- d, y +- 2d) another workgroup of the same XCD read moments
// earlier are still in that XCD's L2.
__device__ __forceinline__ int64_t XcdBandRow(uint32_t block, uint32_t h) {
  const uint32_t band = (h + 7u) / 8u;
  return int64_t((block % 8u) * band + block / 8u);
}
inline unsigned XcdBandBlocks(uint32_t h) { return 8u * ((h + 7u) / 8u); }

__global__ __launch_bounds__(256) void IuwtHorizontalKernel(float* out,
                                                            const float* in,
                                                            uint32_t w, uint32_t h,
                                                            int d) {
  const size_t n = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const int64_t x = int64_t(i % w);
    const float* row = in + (i - size_t(x));
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = x + int64_t(d) * (k - 2);
      t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
    }
    out[i] = HorizontalValue(t, x, int64_t(w), d);
  }
}

// in-place (aliased) variant: one thread per row, left to right
__global__ __launch_bounds__(64) void IuwtHorizontalInPlaceKernel(float* data,
                                                                  uint32_t w,
                                                                  uint32_t h, int d) {
  const uint32_t y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= h) return;
  float* row = data + size_t(y) * w;
  for (int64_t x = 0; x < int64_t(w); ++x) {
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = x + int64_t(d) * (k - 2);
      t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
    }
    row[x] = HorizontalValue(t, x, int64_t(w), d);
  }
}

// 32-bit forms for the chain kernels: the interior region (five taps) first,
// the boundary regions as HorizontalValue orders them
__device__ __forceinline__ float HorizontalValue32(const float* t, int x, int w, int d) {
  if (x >= 2 * d && x < w - 2 * d) return TapSum<5>(t, {2, 1, 0, 3, 4});
  if (x < d) return TapSum<3>(t, {2, 3, 4});
  if (x < 2 * d) return TapSum<4>(t, {2, 1, 3, 4});
  if (x < w - d) return TapSum<4>(t, {2, 1, 0, 3});
  return TapSum<3>(t, {2, 1, 0});
}
// The in-place pass as recurrences (r06): along one row, position x reads
// the already-filtered x - d, x - 2d and the original x, x + d, x + 2d, so the
// residue classes mod d are independent recurrences. One thread per (row,
// residue) keeps the two filtered and two original taps in registers and
// loads the original x + 2d values a block of steps ahead (they are read
// before this thread overwrites them), instead of a dependent global
// round trip per pixel. Same per-pixel expression (HorizontalValue), same
// order of writes within each recurrence, so the result is identical.
__global__ __launch_bounds__(64) void IuwtHorizontalInPlaceChains(float* data, uint32_t w,
                                                                  uint32_t h, int d) {
  const uint64_t t = blockIdx.x * 64ull + threadIdx.x;
  const uint32_t dd = uint32_t(d);
  const uint64_t y = t / dd;
  const int r = int(t % dd);
  if (y >= h || uint32_t(r) >= w) return;
  float* row = data + y * w;
  const int wi = int(w);
  const int n = (wi - r + d - 1) / d;  // recurrence length
  auto orig = [&](int k) -> float { return k < n ? row[r + k * d] : 0.0f; };
  constexpr int B = 8;
  float t0 = 0.0f, t1 = 0.0f;  // filtered x - 2d, x - d
  float t2 = orig(0), t3 = orig(1);
  float cur[B], nxt[B];
#pragma unroll
  for (int i = 0; i < B; ++i) cur[i] = orig(2 + i);
  for (int k0 = 0; k0 < n; k0 += B) {
#pragma unroll
    for (int i = 0; i < B; ++i) nxt[i] = orig(k0 + B + 2 + i);
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int k = k0 + i;
      if (k < n) {
        const int x = r + k * d;
        const float tt[5] = {t0, t1, t2, t3, cur[i]};
        const float v = HorizontalValue32(tt, x, wi, d);
        row[x] = v;
        t0 = t1;
        t1 = v;
        t2 = t3;
        t3 = cur[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B; ++i) cur[i] = nxt[i];
  }
}

// out = V(in), or with lhs: out = lhs - V(in) (differenceMT fused)
__global__ __launch_bounds__(256) void IuwtVerticalKernel(float* out,
                                                          const float* in,
                                                          const float* lhs,
                                                          uint32_t w, uint32_t h,
                                                          int d) {
  // one row per workgroup, rows in XCD bands (XcdBandRow)
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  for (uint32_t x = threadIdx.x; x < w; x += blockDim.x) {
    const size_t i = size_t(y) * w + x;
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      t[k] = (yy >= 0 && yy < int64_t(h)) ? in[size_t(yy) * w + x] : 0.0f;
    }
    const float v = VerticalValue(t, y, int64_t(h), d);
    out[i] = lhs ? lhs[i] - v : v;
  }
}

// IuwtDecomposition::convolve (.h:243-261) per pixel: accumulators start at 0
// and take the taps h0..h4 in order where in range, each as fma(x, h, acc)
__global__ __launch_bounds__(256) void IuwtAccumulateH(float* out, const float* in,
                                                       uint32_t w, uint32_t h,
                                                       int d) {
  const size_t n = size_t(w) * h;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const int64_t x = int64_t(i % w);
    const float* row = in + (i - size_t(x));
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = x + int64_t(d) * (k - 2);
      if (xx >= 0 && xx < int64_t(w)) acc = __builtin_fmaf(row[xx], IuwtTap(k), acc);
    }
    out[i] = acc;
  }
}

// vertical accumulate, then + coefficients (Recompose, .h:138-142)
__global__ __launch_bounds__(256) void IuwtAccumulateVAdd(float* out,
                                                          const float* in,
                                                          const float* add,
                                                          uint32_t w, uint32_t h,
                                                          int d) {
  // one row per workgroup, rows in XCD bands (XcdBandRow)
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  for (uint32_t x = threadIdx.x; x < w; x += blockDim.x) {
    const size_t i = size_t(y) * w + x;
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      if (yy >= 0 && yy < int64_t(h))
        acc = __builtin_fmaf(in[size_t(yy) * w + x], IuwtTap(k), acc);
    }
    out[i] = acc + add[i];
  }
}

// ---- fused row kernels (r06). Each block owns image rows; a row of the
// intermediate lives in LDS between the vertical and horizontal filters, so
// the intermediates of the four passes per scale do not all reach HBM. Every
// value is computed by the same per-pixel operations as the kernels above
// (VerticalValue / HorizontalValue / the Recompose accumulations), so the
// outputs are bit-identical.
//
// DecomposeRows (one scale, spacing d; DecomposeMt's i1 = V(H(a)) and the
// scratch = H(i1) of iuwt_decomposition.cc:9-54): row y of i1 = V_d(s1) from
// rows y + k d of s1 = H_d(a), kept in LDS, then s2 = H_d(i1) for this
// scale's difference pass and, when d_next > 0, s1' = H_d_next(i1), the
// next scale's first pass (a_{s+1} = i1).
__global__ __launch_bounds__(256) void IuwtDecomposeRows(float* __restrict__ i1,
                                                         float* __restrict__ s2,
                                                         float* __restrict__ s1_next,
                                                         const float* __restrict__ s1,
                                                         uint32_t w, uint32_t h, int d,
                                                         int d_next) {
  extern __shared__ float row[];
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  // the vertical filter four pixels (one float4 per tap row) at a time, all
  // five tap rows' loads issued before the sums (w % 4 == 0: the launcher)
  const float4* s1v = reinterpret_cast<const float4*>(s1);
  float4* i1v = reinterpret_cast<float4*>(i1);
  const uint32_t w4 = w / 4;
  // (restrict pointers and unrolling: every tap row's load of the next
  // float4s issues before this one's sums and stores)
#pragma unroll 4
  for (uint32_t x4 = threadIdx.x; x4 < w4; x4 += blockDim.x) {
    float4 t4[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      t4[k] = (yy >= 0 && yy < int64_t(h)) ? s1v[size_t(yy) * w4 + x4]
                                            : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    float4 v;
    {
      float t[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].x;
      v.x = VerticalValue(t, y, int64_t(h), d);
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].y;
      v.y = VerticalValue(t, y, int64_t(h), d);
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].z;
      v.z = VerticalValue(t, y, int64_t(h), d);
#pragma unroll
      for (int k = 0; k < 5; ++k) t[k] = t4[k].w;
      v.w = VerticalValue(t, y, int64_t(h), d);
    }
    reinterpret_cast<float4*>(row)[x4] = v;
    i1v[size_t(y) * w4 + x4] = v;
  }
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < w; x += blockDim.x) {
    float t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t xx = int64_t(x) + int64_t(d) * (k - 2);
      t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
    }
    s2[size_t(y) * w + x] = HorizontalValue(t, x, int64_t(w), d);
    if (d_next > 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int64_t xx = int64_t(x) + int64_t(d_next) * (k - 2);
        t[k] = (xx >= 0 && xx < int64_t(w)) ? row[xx] : 0.0f;
      }
      s1_next[size_t(y) * w + x] = HorizontalValue(t, x, int64_t(w), d_next);
    }
  }
}

// out = lhs - V_d(in), four pixels per thread (w % 4 == 0): the difference
// pass of the fused decomposition, one float4 per tap row in flight
__global__ __launch_bounds__(256) void IuwtVerticalDiff4(float* __restrict__ out,
                                                         const float* __restrict__ in,
                                                         const float* __restrict__ lhs,
                                                         uint32_t w, uint32_t h, int d) {
  // one row per workgroup, rows in XCD bands (XcdBandRow)
  const uint32_t w4 = w / 4;
  const int64_t y = XcdBandRow(blockIdx.x, h);
  if (y >= int64_t(h)) return;
  const float4* inv = reinterpret_cast<const float4*>(in);
#pragma unroll 4
  for (uint32_t x4 = threadIdx.x; x4 < w4; x4 += blockDim.x) {
    const size_t i = size_t(y) * w4 + x4;
    float4 t4[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int64_t yy = y + int64_t(d) * (k - 2);
      t4[k] = (yy >= 0 && yy < int64_t(h)) ? inv[size_t(yy) * w4 + x4]
                                            : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    const float4 l = reinterpret_cast<const float4*>(lhs)[i];
    float t[5];
    float4 o;
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].x;
    o.x = l.x - VerticalValue(t, y, int64_t(h), d);
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].y;
    o.y = l.y - VerticalValue(t, y, int64_t(h), d);
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].z;
    o.z = l.z - VerticalValue(t, y, int64_t(h), d);
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = t4[k].w;
    o.w = l.w - VerticalValue(t, y, int64_t(h), d);
    reinterpret_cast<float4*>(out)[i] = o;
  }
}

// VerticalValue's region of row y (uniform over a chain step), then its sum
__device__ __forceinline__ int VerticalRegion(int64_t y, int64_t h, int64_t d) {
  return y < d ? 0 : y < 2 * d ? 1 : y < h - 2 * d ? 2 : y < h - d ? 3 : 4;
}
__device__ __forceinline__ float VerticalByRegion(const float* t, int region) {
  switch (region) {
    case 0: return TapSum<3>(t, {2, 3, 4});
    case 1: return TapSum<4>(t, {1, 2, 3, 4});
    case 2: return TapSum<5>(t, {0, 1, 2, 3, 4});
    case 3: return TapSum<4>(t, {0, 1, 2, 3});
    default: return TapSum<3>(t, {0, 1, 2});
  }
}

// ---- row-chain kernels (r06): one launch per scale. Along the vertical axis
// the à-trous taps of row y are rows y + k d, so the rows r, r + d, r + 2d, ...
// (one residue class mod d, a "chain") share their taps: a workgroup walks
// one segment of a chain over one column strip, keeping the last five
// filtered rows in LDS rings, and every image row is read once per pass
// instead of five times. Decomposition per step j (chain position):
//   phase A: ring1[j] = H_d(a_j) over the strip + 2d columns each side;
//            ring2[j-3] = H_d(i1_{j-3}) over the strip (i1 row from LDS)
//   phase B: i1_{j-2} = V_d(ring1[j-4..j]) -> LDS and the i1 plane;
//            coef_{j-5} = a_{j-5} - V_d(ring2[j-7..j-3]) -> coefficient plane
// with the next a row and the coefficient's a row loaded one step ahead in
// registers. Each value is the same per-pixel expression as the kernels
// above (HorizontalValue / VerticalValue and the subtraction), so the planes
// are bit-identical; a segment of K outputs reads K + 8 rows of a (the tap
// rows of its first and last outputs), the strip 4d extra columns each side.
struct ChainArgs {
  const float* a;     // this scale's approximation (decompose) / the coarser
                      // recomposition (recompose)
  float* i1;          // next approximation (decompose) / finer recomposition
  float* coef;        // this scale's coefficients: written (decompose) or
                      // added (recompose)
  uint32_t w, h;
  int d;
  uint32_t ws;        // output columns per workgroup (multiple of 4, <= 1024)
  uint32_t n_strips;  // ceil(w / ws)
  uint32_t n_seg;     // segments per chain
  uint32_t n_res;     // chains: min(d, h) residues
  float* dummy;       // 256 floats: the stores of lanes with nothing to store
};
// block -> (residue r, segment, strip), consecutive strips of one segment on
// one XCD (their halo columns are shared through its L2)
struct ChainPlace {
  int64_t r, kb, ke, x0;
  bool ok;
};
__device__ __forceinline__ ChainPlace ChainBlock(const ChainArgs& p) {
  ChainPlace c;
  const uint32_t n_blocks = p.n_res * p.n_seg * p.n_strips;
  const uint32_t per = (n_blocks + 7u) / 8u;
  const uint32_t L = (blockIdx.x % 8u) * per + blockIdx.x / 8u;
  c.ok = L < n_blocks;
  if (!c.ok) return c;
  const uint32_t strip = L % p.n_strips;
  const uint32_t rest = L / p.n_strips;
  const int64_t seg = rest % p.n_seg;
  c.r = rest / p.n_seg;
  const int64_t h = p.h, d = p.d;
  c.x0 = int64_t(strip) * p.ws;
  const int64_t k_r = c.r < h ? (h - c.r + d - 1) / d : 0;  // chain length
  const int64_t k_max = (h + d - 1) / d;
  const int64_t kseg = (k_max + p.n_seg - 1) / p.n_seg;
  c.kb = seg * kseg;
  c.ke = c.kb + kseg < k_r ? c.kb + kseg : k_r;
  c.ok = c.kb < c.ke;
  return c;
}

__device__ __forceinline__ int64_t Floor4(int64_t v) {
  return v >= 0 ? v & ~int64_t(3) : -((-v + 3) & ~int64_t(3));
}

// Every global load and store of a step is unconditional: out-of-range lanes
// load the plane's first float4 (zeroed after) and store to a dummy area, and
// the first and last steps of a segment run the same code with their
// results discarded. So the memory operations of a step are a fixed sequence
// and the compiler's wait counts stay exact across the loop; each step
// alternates between two register sets, so a row's loads are issued two
// steps before its LDS store.
template <int NA>
struct ChainRow {
  float4 v[NA];
  bool ok[NA];
  __device__ __forceinline__ void Load(const float* a, int64_t j, int64_t r, int64_t d,
                                       int64_t w, int64_t h, int64_t ab, int64_t wa4) {
    const int64_t y = r + j * d;
    const bool row_ok = j >= 0 && y < h;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int64_t g = threadIdx.x + int64_t(i) * 256;
      const int64_t c = ab + 4 * g;
      ok[i] = row_ok && g < wa4 && c >= 0 && c < w;
      v[i] = *reinterpret_cast<const float4*>(a + (ok[i] ? y * w + c : 0));
    }
  }
  // the LDS row slot holds 256 NA float4s, so every lane stores
  __device__ __forceinline__ void Store(float* row) const {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      reinterpret_cast<float4*>(row)[threadIdx.x + i * 256] =
          ok[i] ? v[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
};
// one row of a plane at chain position j, this thread's output columns
template <int NO>
struct ChainOut {
  float v[NO];
  __device__ __forceinline__ void Load(const float* src, int64_t j, int64_t r, int64_t d,
                                       int64_t w, int64_t h, int64_t x0, int64_t ws) {
    const int64_t y = r + j * d;
    const bool row_ok = j >= 0 && y < h;
#pragma unroll
    for (int i = 0; i < NO; ++i) {
      const int64_t q = threadIdx.x + int64_t(i) * 256;
      const bool ok = row_ok && q < ws && x0 + q < w;
      v[i] = src[ok ? y * w + x0 + q : 0];
    }
  }
};
__device__ __forceinline__ int64_t Mod5(int64_t v) {
  const int32_t m = int32_t(v) % 5;  // positions fit 32 bits
  return m < 0 ? m + 5 : m;
}

template <int NA, int NO, int NI>
__global__ __launch_bounds__(256) void IuwtDecomposeChain(ChainArgs p) {
  extern __shared__ float lds[];
  const ChainPlace c = ChainBlock(p);
  if (!c.ok) return;
  const int64_t w = p.w, h = p.h, d = p.d, ws = p.ws;
  const int64_t r = c.r, kb = c.kb, ke = c.ke, x0 = c.x0;
  const int64_t xi0 = x0 - 2 * d;  // i1 / H(a) columns [xi0, xi0 + wi)
  const int64_t wi = ws + 4 * d;
  const int64_t ab = Floor4(x0 - 4 * d);  // a row columns [ab, ab + 4 wa4)
  const int64_t wa4 = (x0 + ws + 4 * d - ab + 3) / 4;
  constexpr int kSlot = 1024 * NA;  // floats per a-row slot
  float* arow = lds;                // [2][kSlot]
  float* ring1 = arow + 2 * kSlot;  // [5][wi]: H(a)
  float* i1row = ring1 + 5 * wi;    // [2][wi]
  float* ring2 = i1row + 2 * wi;    // [5][ws]: H(i1)
  float* aring = ring2 + 5 * ws;    // [6][ws]: a over the strip, the
                                    // coefficient rows' left-hand side
  float* dummy = p.dummy + threadIdx.x;
  const int64_t j0 = kb - 4;  // first a position
  // steps j0 .. j0 + n_steps - 1 (>= ke + 4), an even count
  const int64_t n_steps = (ke + 5 - j0 + 1) & ~int64_t(1);
  const int64_t xe = x0 + ws < w ? x0 + ws : w;

  // 32-bit column arithmetic inside the steps (w, h < 2^31; positions of
  // one chain fit 32 bits): the taps' offsets d (k - 2) are uniform
  const int wi32 = int(wi), ws32 = int(ws), w32 = int(w), d32 = int(d);
  const int xi32 = int(xi0), x032 = int(x0), xe32 = int(xe), ab32 = int(ab);
  const int tid = int(threadIdx.x);
  auto step = [&](int64_t j, ChainRow<NA>& pa) {
    // phase A: ring1[j] = H(a_j); ring2[j-3] = H(i1_{j-3}); aring[j] = a_j
    {
      const float* ar = arow + ((j - j0) & 1) * kSlot - ab32;
      {
        float* as = aring + int64_t(uint32_t(j - j0) % 6u) * ws32 - x032;
#pragma unroll
        for (int i = 0; i < NO; ++i) {
          const int x = x032 + tid + i * 256;
          if (x < x032 + ws32) as[x] = ar[x];
        }
      }
      float* out = ring1 + Mod5(j - j0) * wi32 - xi32;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int x = xi32 + tid + i * 256;
        if (x < xi32 + wi32) {
          float t[5];
#pragma unroll
          for (int k = 0; k < 5; ++k) t[k] = ar[x + d32 * (k - 2)];
          out[x] = HorizontalValue32(t, x, w32, d32);
        }
      }
      const int64_t m = j - 3;
      const float* ir = i1row + ((m - j0) & 1) * wi32 - xi32;
      float* out2 = ring2 + Mod5(m - j0) * ws32 - x032;
#pragma unroll
      for (int i = 0; i < NO; ++i) {
        const int x = x032 + tid + i * 256;
        if (x < x032 + ws32) {
          float t[5];
#pragma unroll
          for (int k = 0; k < 5; ++k) t[k] = ir[x + d32 * (k - 2)];
          out2[x] = HorizontalValue32(t, x, w32, d32);
        }
      }
    }
    __syncthreads();
    // phase B: i1_{j-2} = V(ring1[j-4..j]); coef_{j-5} = a - V(ring2[j-7..j-3])
    {
      const int64_t pi = j - 2;
      const int64_t y = r + pi * d;
      const bool row_in = pi >= 0 && y < h;
      const bool store = pi >= kb && pi < ke;
      const int vreg = VerticalRegion(y, h, d);  // uniform over the step
      const float* rows[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) rows[k] = ring1 + Mod5(pi - 2 + k - j0) * wi32 - xi32;
      float* keep = i1row + ((pi - j0) & 1) * wi32 - xi32;
      float* i1_row = p.i1 + y * w;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int x = xi32 + tid + i * 256;
        const bool in = x < xi32 + wi32;
        const int xc = in ? x : xi32;
        float t[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) t[k] = rows[k][xc];
        // rows and columns outside the image are the zero padding of the
        // next horizontal pass, as the four-pass kernels read them
        const float v = (row_in && x >= 0 && x < w32) ? VerticalByRegion(t, vreg) : 0.0f;
        if (in) keep[x] = v;
        const bool st = store && in && x >= x032 && x < xe32;
        *(st ? i1_row + x : dummy) = v;
      }
      const int64_t q = j - 5;
      const int64_t yq = r + q * d;
      const bool qok = q >= kb && q < ke;
      const int vreg2 = VerticalRegion(yq, h, d);
      const float* rows2[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) rows2[k] = ring2 + Mod5(q - 2 + k - j0) * ws32;
      const float* lhs = aring + int64_t(uint32_t(q - j0 + 6) % 6u) * ws32;
      float* coef_row = p.coef + yq * w + x0;
#pragma unroll
      for (int i = 0; i < NO; ++i) {
        const int o = tid + i * 256;
        const bool in = o < ws32;
        const int oc = in ? o : 0;
        float t[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) t[k] = rows2[k][oc];
        const float v = lhs[oc] - VerticalByRegion(t, vreg2);
        const bool st = qok && in && x032 + o < w32;
        *(st ? coef_row + o : dummy) = v;
      }
    }
    // row j + 1 (loaded two steps ago) into LDS, row j + 3 into this step's
    // register set
    pa.Store(arow + ((j + 1 - j0) & 1) * kSlot);
    pa.Load(p.a, j + 3, r, d, w, h, ab, wa4);
    __syncthreads();
  };

  ChainRow<NA> pa0, pa1;
  pa0.Load(p.a, j0, r, d, w, h, ab, wa4);
  pa0.Store(arow + 0 * kSlot);
  pa0.Load(p.a, j0 + 1, r, d, w, h, ab, wa4);
  pa1.Load(p.a, j0 + 2, r, d, w, h, ab, wa4);
  __syncthreads();
  for (int64_t t = 0; t < n_steps; t += 2) {
    step(j0 + t, pa0);
    step(j0 + t + 1, pa1);
  }
}

// Recompose per scale (IuwtDecomposition::Recompose, .h:121-146): out =
// V_acc(H_acc(prev)) + coef, the accumulations of IuwtAccumulateH /
// IuwtAccumulateVAdd (taps in order, out-of-range taps skipped: a select,
// so the five LDS reads issue together), along chains as above:
// ring1[j] = H_acc(prev_j) over the strip, out_{j-2} from ring1[j-4..j].
template <int NA, int NO>
__global__ __launch_bounds__(256) void IuwtRecomposeChain(ChainArgs p) {
  extern __shared__ float lds[];
  const ChainPlace c = ChainBlock(p);
  if (!c.ok) return;
  const int64_t w = p.w, h = p.h, d = p.d, ws = p.ws;
  const int64_t r = c.r, kb = c.kb, ke = c.ke, x0 = c.x0;
  const int64_t ab = Floor4(x0 - 2 * d);
  const int64_t wa4 = (x0 + ws + 2 * d - ab + 3) / 4;
  constexpr int kSlot = 1024 * NA;
  float* arow = lds;                // [2][kSlot]
  float* ring1 = arow + 2 * kSlot;  // [5][ws]
  float* dummy = p.dummy + threadIdx.x;
  const int64_t j0 = kb - 2;
  const int64_t n_steps = (ke + 2 - j0 + 1) & ~int64_t(1);

  const int ws32 = int(ws), w32 = int(w), d32 = int(d), x032 = int(x0), ab32 = int(ab);
  const int tid = int(threadIdx.x);
  auto step = [&](int64_t j, ChainRow<NA>& pa, ChainOut<NO>& pl) {
    {
      const float* ar = arow + ((j - j0) & 1) * kSlot - ab32;
      float* out = ring1 + Mod5(j - j0) * ws32 - x032;
#pragma unroll
      for (int i = 0; i < NO; ++i) {
        const int x = x032 + tid + i * 256;
        if (x < x032 + ws32) {
          float t[5];
#pragma unroll
          for (int k = 0; k < 5; ++k) t[k] = ar[x + d32 * (k - 2)];
          float acc = 0.0f;
#pragma unroll
          for (int k = 0; k < 5; ++k) {
            const int xx = x + d32 * (k - 2);
            const float f = __builtin_fmaf(t[k], IuwtTap(k), acc);
            acc = (xx >= 0 && xx < w32) ? f : acc;
          }
          out[x] = acc;
        }
      }
    }
    __syncthreads();
    {
      const int64_t pi = j - 2;
      const int64_t y = r + pi * d;
      const bool pok = pi >= kb && pi < ke;
      bool yin[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int64_t yy = y + d * (k - 2);
        yin[k] = yy >= 0 && yy < h;  // uniform
      }
      const float* rows[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) rows[k] = ring1 + Mod5(pi - 2 + k - j0) * ws32;
      float* out_row = p.i1 + y * w + x0;
#pragma unroll
      for (int i = 0; i < NO; ++i) {
        const int o = tid + i * 256;
        const bool in = o < ws32;
        const int oc = in ? o : 0;
        float t[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) t[k] = rows[k][oc];
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const float f = __builtin_fmaf(t[k], IuwtTap(k), acc);
          acc = yin[k] ? f : acc;
        }
        const bool st = pok && in && x032 + o < w32;
        *(st ? out_row + o : dummy) = acc + pl.v[i];
      }
    }
    pa.Store(arow + ((j + 1 - j0) & 1) * kSlot);
    pl.Load(p.coef, j, r, d, w, h, x0, ws);
    pa.Load(p.a, j + 3, r, d, w, h, ab, wa4);
    __syncthreads();
  };

  ChainRow<NA> pa0, pa1;
  ChainOut<NO> pl0, pl1;
  pa0.Load(p.a, j0, r, d, w, h, ab, wa4);
  pa0.Store(arow + 0 * kSlot);
  pa0.Load(p.a, j0 + 1, r, d, w, h, ab, wa4);
  pa1.Load(p.a, j0 + 2, r, d, w, h, ab, wa4);
  pl0.Load(p.coef, j0 - 2, r, d, w, h, x0, ws);
  pl1.Load(p.coef, j0 - 1, r, d, w, h, x0, ws);
  __syncthreads();
  for (int64_t t = 0; t < n_steps; t += 2) {
    step(j0 + t, pa0, pl0);
    step(j0 + t + 1, pa1, pl1);
  }
}

// RDL_IUWT_FUSED selects the IUWT kernels (comparison): 0 the four-pass
// kernels and the one-thread-per-row in-place pass; 1 the fused row
// decomposition, four-pass recomposition; unset (2) the fused row
// decomposition and the row-chain recomposition; 3 the row chains for both
// (the chain decomposition measured slower than the fused rows: 0.93-1.23 ms
// against 0.88 ms at 4096^2, 6 scales). Modes 1-3 run the in-place pass as
// recurrences (IuwtHorizontalInPlaceChains).
inline int IuwtMode() {
  const char* e = std::getenv("RDL_IUWT_FUSED");
  if (!e || !e[0]) return 2;
  return e[0] == '0' ? 0 : e[0] == '1' ? 1 : e[0] == '3' ? 3 : 2;
}
inline bool IuwtFusedOn() { return IuwtMode() != 0; }

// the chain launch's geometry for spacing d, or false when the rows do not
// fit its register/LDS budget (the row kernels then run)
struct ChainPlan {
  ChainArgs a;
  unsigned blocks;
  size_t lds;
  int na, no, ni;  // float4 loads per thread per row; output and halo-strip
                   // columns per thread (multiples of 256)
};
inline bool PlanChain(uint32_t w, uint32_t h, int d, bool decompose, ChainPlan* pl) {
  // 512 columns per workgroup at every spacing: 1024 (fewer halo columns at
  // d >= 31) lowers the occupancy more than it saves (r06 measurement)
  uint32_t ws = 512u;
  if (const char* e = std::getenv("RDL_IUWT_CHAIN_WS")) {  // (measurement)
    const unsigned v = unsigned(std::atoi(e));
    if (v >= 256 && v <= 1024 && v % 256 == 0) ws = v;
  }
  if (ws > (w + 3u) / 4u * 4u) ws = (w + 3u) / 4u * 4u;
  const int64_t halo = decompose ? 4 * int64_t(d) : 2 * int64_t(d);
  const int64_t wa4 = (int64_t(ws) + 2 * halo + 6) / 4;
  if (wa4 > 512) return false;
  pl->na = wa4 <= 256 ? 1 : 2;
  pl->no = int(DivUp(ws, 256));
  if (pl->no == 3) pl->no = 4;
  const int64_t wi = int64_t(ws) + 4 * int64_t(d);
  pl->ni = std::max(pl->no, int((wi + 255) / 256));
  if (pl->ni > pl->no + 2) return false;
  const uint32_t n_strips = (w + ws - 1) / ws;
  const uint32_t n_res = uint32_t(d) < h ? uint32_t(d) : h;  // chains with rows
  const uint32_t k_max = (h + uint32_t(d) - 1) / uint32_t(d);
  uint32_t n_seg = std::min(DivUp(k_max, 24), DivUp(1536, size_t(n_res) * n_strips));
  n_seg = std::max(1u, std::min(n_seg, k_max));
  const uint64_t n_blocks = uint64_t(n_res) * n_seg * n_strips;
  if (n_blocks > (uint64_t(1) << 30)) return false;
  ChainArgs& a = pl->a;
  a.w = w;
  a.h = h;
  a.d = d;
  a.ws = ws;
  a.n_strips = n_strips;
  a.n_seg = n_seg;
  a.n_res = n_res;
  pl->blocks = unsigned(8 * ((n_blocks + 7) / 8));
  const int64_t slots = 2 * 1024 * int64_t(pl->na);
  pl->lds = decompose ? size_t(slots + 7 * wi + 11 * int64_t(ws)) * sizeof(float)
                      : size_t(slots + 5 * int64_t(ws)) * sizeof(float);
  return pl->lds <= 160 * 1024;
}
template <typename Fn>
int LaunchChainKernel(rdl_session* s, const ChainPlan& pl, Fn* fn,
                      std::atomic<uint64_t>& lds_set) {
  if (pl.lds > 64 * 1024)
    RDL_TRY(SetMaxLdsOnce(reinterpret_cast<const void*>(fn), 160 * 1024, s->device,
                          lds_set));
  fn<<<pl.blocks, 256, pl.lds, s->stream>>>(pl.a);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}
template <int NA, int NO>
int LaunchChainT(rdl_session* s, const ChainPlan& pl, bool decompose) {
  static std::atomic<uint64_t> lds_set[4] = {{0}, {0}, {0}, {0}};
  if (!decompose) return LaunchChainKernel(s, pl, IuwtRecomposeChain<NA, NO>, lds_set[3]);
  switch (pl.ni - NO) {
    case 0: return LaunchChainKernel(s, pl, IuwtDecomposeChain<NA, NO, NO>, lds_set[0]);
    case 1: return LaunchChainKernel(s, pl, IuwtDecomposeChain<NA, NO, NO + 1>, lds_set[1]);
    default: return LaunchChainKernel(s, pl, IuwtDecomposeChain<NA, NO, NO + 2>, lds_set[2]);
  }
}
template <int NA>
int LaunchChainO(rdl_session* s, const ChainPlan& pl, bool decompose) {
  switch (pl.no) {
    case 1: return LaunchChainT<NA, 1>(s, pl, decompose);
    case 2: return LaunchChainT<NA, 2>(s, pl, decompose);
    default: return LaunchChainT<NA, 4>(s, pl, decompose);
  }
}
inline int LaunchChain(rdl_session* s, const ChainPlan& pl, bool decompose) {
  return pl.na == 1 ? LaunchChainO<1>(s, pl, decompose) : LaunchChainO<2>(s, pl, decompose);
}

// rows of at most this many floats go through LDS (one row per block: 64 KiB
// at most)
constexpr uint32_t kIuwtFusedMaxWidth = 16384;

inline unsigned IuwtGrid(size_t n) {
  return unsigned(std::min<size_t>(16384, std::max<size_t>(1, (n + 255) / 256)));
}

int Horizontal(rdl_session* s, float* out, const float* in, uint32_t w, uint32_t h,
               int d) {
  ScopedTiming t(s, "iuwt", double(w) * h * 8.0);
  if (out == in) {
    // RDL_IUWT_FUSED=0: the one-thread-per-row kernel (comparison)
    if (IuwtMode() == 0)
      IuwtHorizontalInPlaceKernel<<<DivUp(h, 64), 64, 0, s->stream>>>(out, w, h, d);
    else
      IuwtHorizontalInPlaceChains<<<DivUp(uint64_t(h) * uint32_t(d), 64), 64, 0,
                                    s->stream>>>(out, w, h, d);
  } else {
    IuwtHorizontalKernel<<<IuwtGrid(size_t(w) * h), 256, 0, s->stream>>>(out, in, w,
                                                                          h, d);
  }
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int Vertical(rdl_session* s, float* out, const float* in, const float* lhs,
             uint32_t w, uint32_t h, int d) {
  ScopedTiming t(s, "iuwt", double(w) * h * (lhs ? 12.0 : 8.0));
  IuwtVerticalKernel<<<XcdBandBlocks(h), 256, 0, s->stream>>>(out, in, lhs, w, h, d);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // namespace rdl

extern "C" {

int rdl_iuwt_decompose(rdl_session* s, float* d_input, float* d_scratch,
                       uint32_t width, uint32_t height, uint32_t n_scales,
                       float* d_coeffs, int include_largest) {
  RDL_ARG_CHECK(s && d_input && d_scratch && d_coeffs, "NULL argument");
  RDL_ARG_CHECK(n_scales >= 1 && n_scales <= 24, "n_scales out of range");
  RDL_ARG_CHECK(width >= 1 && height >= 1, "bad size");
  // DecomposeMt (iuwt_decomposition.cc:9-54)
  const size_t n = size_t(width) * height;
  const bool vec_ok =
      d_input != d_scratch && width % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(d_input) | reinterpret_cast<uintptr_t>(d_coeffs)) % 16 == 0;
  if (vec_ok && rdl::IuwtMode() == 3) {
    // row chains: one launch per scale (IuwtDecomposeChain). The approximation
    // planes alternate between the largest-scale plane and one scratch plane,
    // the last landing in the largest-scale plane.
    std::vector<rdl::ChainPlan> plans(n_scales);
    bool all = true;
    for (uint32_t sc = 0; sc < n_scales && all; ++sc)
      all = rdl::PlanChain(width, height, (1 << (sc + 1)) - 1, true, &plans[sc]);
    if (all) {
      RDL_TRY(s->EnsureScratch(s->iuwt, (n + 256) * sizeof(float)));
      float* big = d_coeffs + size_t(n_scales) * n;
      float* spare = static_cast<float*>(s->iuwt.ptr);
      for (auto& pl : plans) pl.a.dummy = spare + n;
      const float* a = d_input;
      for (uint32_t sc = 0; sc < n_scales; ++sc) {
        rdl::ChainPlan& pl = plans[sc];
        float* i1 = ((n_scales - 1 - sc) % 2 == 0) ? big : spare;
        pl.a.a = a;
        pl.a.i1 = i1;
        pl.a.coef = d_coeffs + size_t(sc) * n;
        rdl::ScopedTiming t(s, "iuwt", double(n) * 12.0);
        RDL_TRY(rdl::LaunchChain(s, pl, true));
        a = i1;
      }
      if (!include_largest)
        RDL_HIP_CHECK(hipMemsetAsync(big, 0, n * sizeof(float), s->stream));
      return RDL_OK;
    }
  }
  if (vec_ok && width <= rdl::kIuwtFusedMaxWidth && rdl::IuwtFusedOn()) {
    // fused: per scale one row kernel (i1, s2 = H(i1), next scale's H(i1))
    // and the difference pass; the approximation planes alternate between
    // the largest-scale plane and a scratch plane (no copy), arranged so the
    // last one lands in the largest-scale plane as the four-pass form leaves
    // it. The caller's scratch is not written (not aliased: nothing reads it).
    RDL_TRY(s->EnsureScratch(s->iuwt, 4 * n * sizeof(float)));
    float* big = d_coeffs + size_t(n_scales) * n;
    float* spare = static_cast<float*>(s->iuwt.ptr);
    float* s1[2] = {spare + n, spare + 2 * n};
    float* s2 = spare + 3 * n;
    RDL_TRY(rdl::Horizontal(s, s1[0], d_input, width, height, 1));
    const float* a = d_input;
    for (uint32_t sc = 0; sc < n_scales; ++sc) {
      const int d = (1 << (sc + 1)) - 1;
      const int d_next = sc + 1 < n_scales ? (1 << (sc + 2)) - 1 : 0;
      float* i1 = ((n_scales - 1 - sc) % 2 == 0) ? big : spare;
      {
        rdl::ScopedTiming t(s, "iuwt", double(n) * (d_next ? 16.0 : 12.0));
        rdl::IuwtDecomposeRows<<<rdl::XcdBandBlocks(height), 256, width * sizeof(float),
                                 s->stream>>>(
            i1, s2, s1[(sc + 1) & 1u], s1[sc & 1u], width, height, d, d_next);
        RDL_HIP_CHECK(hipGetLastError());
      }
      {
        rdl::ScopedTiming t(s, "iuwt", double(n) * 12.0);
        rdl::IuwtVerticalDiff4<<<rdl::XcdBandBlocks(height), 256, 0, s->stream>>>(
            d_coeffs + size_t(sc) * n, s2, a, width, height, d);
        RDL_HIP_CHECK(hipGetLastError());
      }
      a = i1;
    }
    if (!include_largest)
      RDL_HIP_CHECK(hipMemsetAsync(big, 0, n * sizeof(float), s->stream));
    return RDL_OK;
  }
  RDL_TRY(s->EnsureScratch(s->iuwt, n * sizeof(float)));
  float* i0 = static_cast<float*>(s->iuwt.ptr);
  float* i1 = d_coeffs + size_t(n_scales) * n;  // the largest scale aliases i1
  RDL_TRY(rdl::Horizontal(s, d_scratch, d_input, width, height, 1));
  RDL_TRY(rdl::Vertical(s, i1, d_scratch, nullptr, width, height, 1));
  RDL_TRY(rdl::Horizontal(s, d_scratch, i1, width, height, 1));
  // coefficients0 = input - V(...); `input` has become the scratch when aliased
  RDL_TRY(rdl::Vertical(s, d_coeffs, d_scratch, d_input, width, height, 1));
  RDL_HIP_CHECK(hipMemcpyAsync(i0, i1, n * sizeof(float), hipMemcpyDeviceToDevice,
                               s->stream));
  for (uint32_t sc = 1; sc < n_scales; ++sc) {
    const int d = (1 << (sc + 1)) - 1;
    float* coef = d_coeffs + size_t(sc) * n;
    RDL_TRY(rdl::Horizontal(s, d_scratch, i0, width, height, d));
    RDL_TRY(rdl::Vertical(s, i1, d_scratch, nullptr, width, height, d));
    RDL_TRY(rdl::Horizontal(s, d_scratch, i1, width, height, d));
    RDL_TRY(rdl::Vertical(s, coef, d_scratch, i0, width, height, d));
    if (sc + 1 != n_scales)
      RDL_HIP_CHECK(hipMemcpyAsync(i0, i1, n * sizeof(float),
                                   hipMemcpyDeviceToDevice, s->stream));
  }
  if (!include_largest)
    RDL_HIP_CHECK(hipMemsetAsync(i1, 0, n * sizeof(float), s->stream));
  return RDL_OK;
}

int rdl_iuwt_recompose(rdl_session* s, const float* d_coeffs, uint32_t width,
                       uint32_t height, uint32_t n_scales, int include_largest,
                       float* d_out) {
  RDL_ARG_CHECK(s && d_coeffs && d_out, "NULL argument");
  RDL_ARG_CHECK(n_scales >= 1 && n_scales <= 24, "n_scales out of range");
  // Recompose (iuwt_decomposition.h:121-146)
  const size_t n = size_t(width) * height;
  RDL_TRY(s->EnsureScratch(s->iuwt, (n + 256) * sizeof(float)));
  float* tmp = static_cast<float*>(s->iuwt.ptr);
  if (rdl::IuwtMode() >= 2 && width % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(d_coeffs) | reinterpret_cast<uintptr_t>(d_out)) % 16 == 0) {
    // row chains (IuwtRecomposeChain): each scale reads the coarser
    // recomposition (first: the approximation or the last detail plane,
    // in place in the coefficients) and writes the finer one, alternating
    // between the scratch plane and d_out so that the last lands in d_out
    const int first = include_largest ? int(n_scales) : int(n_scales) - 1;
    std::vector<rdl::ChainPlan> plans(static_cast<size_t>(first));
    bool all = true;
    for (int sc = 0; sc < first && all; ++sc)
      all = rdl::PlanChain(width, height, (1 << (sc + 1)) - 1, false, &plans[size_t(sc)]);
    if (all) {
      for (auto& pl : plans) pl.a.dummy = tmp + n;
      const float* prev = d_coeffs + size_t(first) * n;
      if (first == 0) {
        RDL_HIP_CHECK(hipMemcpyAsync(d_out, prev, n * sizeof(float),
                                     hipMemcpyDeviceToDevice, s->stream));
        return RDL_OK;
      }
      for (int sc = first - 1; sc >= 0; --sc) {
        rdl::ChainPlan& pl = plans[size_t(sc)];
        float* out = (sc % 2 == 0) ? d_out : tmp;
        pl.a.a = prev;
        pl.a.i1 = out;
        pl.a.coef = const_cast<float*>(d_coeffs + size_t(sc) * n);
        rdl::ScopedTiming t(s, "iuwt", double(n) * 12.0);
        RDL_TRY(rdl::LaunchChain(s, pl, false));
        prev = out;
      }
      return RDL_OK;
    }
  }
  int sc = int(n_scales) - 1;
  if (include_largest) {
    RDL_HIP_CHECK(hipMemcpyAsync(d_out, d_coeffs + size_t(n_scales) * n,
                                 n * sizeof(float), hipMemcpyDeviceToDevice,
                                 s->stream));
  } else {
    RDL_HIP_CHECK(hipMemcpyAsync(d_out, d_coeffs + size_t(sc) * n, n * sizeof(float),
                                 hipMemcpyDeviceToDevice, s->stream));
    --sc;
  }
  for (; sc >= 0; --sc) {
    const int d = (1 << (sc + 1)) - 1;
    {
      rdl::ScopedTiming t(s, "iuwt", double(n) * 20.0);
      rdl::IuwtAccumulateH<<<rdl::IuwtGrid(n), 256, 0, s->stream>>>(tmp, d_out, width,
                                                                  height, d);
      rdl::IuwtAccumulateVAdd<<<rdl::XcdBandBlocks(height), 256, 0, s->stream>>>(
          d_out, tmp, d_coeffs + size_t(sc) * n, width, height, d);
    }
    RDL_HIP_CHECK(hipGetLastError());
  }
  return RDL_OK;
}

}  // extern "C"
