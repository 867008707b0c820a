// The sub-minor (Clark-style) loop: replaces SubMinorLoop::Run with
// findPeakPositions / MakeSets / GetMaxComponent
// (cpp/algorithms/subminor_loop.cc:13-184).
//
// Selection: three streaming passes over the border box (count, scan,
// scatter) compact the pixels whose integrated value passes the threshold
// into a row-major list (packed y<<16|x) and gather their N_img residual
// values — the same order the reference's nested x/y loops produce.
//
// Loop: one persistent launch. The selected set is partitioned over G
// workgroups (one per CU); each keeps its pixels' positions, residual and
// model values in LDS (global scratch when the set outgrows G x 160 KiB).
// Per iteration every workgroup subtracts the current component's shifted
// twice-convolved PSF from its pixels (one FMA per pixel and image, PSF
// gathered from HBM/L2), re-integrates and reduces its argmax; with G > 1 the
// winners are exchanged through write-through (sc1) records and a monotonic
// arrival counter, so all workgroups take the same next component. The
// per-iteration argmax key orders the signed (or absolute) integrated value
// with the first index winning ties, which is GetMaxComponent's
// "start at scratch[0], strict '>'" scan.
#include <cmath>

#include <cstdio>

#include <cstdlib>

#include "rdl_internal.h"
#include "logpoly.h"

struct rdl_subminor {
  rdl_session* s = nullptr;
  void* counts = nullptr;  // per-chunk counts / offsets
  size_t counts_bytes = 0;
  void* sel = nullptr;     // positions + R + M for the selected set
  size_t sel_bytes = 0;
  void* sync = nullptr;    // records + counter + result + trace
  size_t sync_bytes = 0;
  uint64_t n_selected = 0;
  uint32_t n_images = 0;
  uint32_t width = 0, height = 0;
  uint32_t* d_pos = nullptr;
  float* d_r = nullptr;
  float* d_m = nullptr;
  int mode = 0;  // 0 auto, 1 LDS kernel, 2 register kernel, 3 single-wave kernel,
                 // 4 one 1024-thread workgroup, 5 1024-thread grid, 6 table kernel
  uint32_t target_per_block = 1024;  // pixels per workgroup (multi-workgroup)
  uint32_t single_max = 2048;         // largest selection kept on one workgroup
  uint32_t wave_max = 128;            // largest selection on the single-wave kernel
  uint32_t big_max = 3584;            // largest selection on one 1024-thread workgroup
  uint32_t big_target = 0;            // > 0: larger selections on 1024-thread grids
  uint32_t table_max = 16384;         // largest selection given a pairwise PSF table
  void* table = nullptr;              // [n_psf][n_sel][n_sel] PSF values at the
  size_t table_bytes = 0;             //   selected pixels' pairwise offsets
  void* pos_buf = nullptr;            // selected positions (sparse / single pass)
  size_t pos_bytes = 0;
  void* local_buf = nullptr;          // sparse selection: the chunks' own lists
  size_t local_bytes = 0;
  void* stamp_mark = nullptr;         // shape-model stamping: tiles a stamp reaches
  size_t stamp_mark_bytes = 0;
  int select_passes = 0;              // 0 sparse two-phase, 1 single pass, 3 count + scan + scatter
  int select_ticket = 1;              // single pass: chunk order by ticket
  int select_quad = 1;                // sparse: 16-byte loads where they apply
  uint64_t select_spin_limit = uint64_t(1) << 26;  // look-back polls before failing
  int tab = 1;                        // SubminorLoopTab where it applies (RDL_SUBMINOR_TAB=0: off)
  uint32_t tab_threads = 0;           // 0: 512 up to 2048 pixels per participant, else 1024
  uint32_t tab_target = 1024;         // pixels per participant (RDL_SUBMINOR_TAB_TARGET)
  uint32_t tab_single = 8192;         // one workgroup up to this (RDL_SUBMINOR_TAB_SINGLE)
  // a launched loop whose result has not been read (rdl_subminor_launch ->
  // rdl_subminor_collect)
  bool pending = false;
  uint64_t pending_start = 0;       // iteration_start of the launch
  double pending_bytes_per_it = 0;  // algorithmic bytes per iteration
  const uint32_t* pending_result = nullptr;
  hipEvent_t pending_ev0 = nullptr, pending_ev1 = nullptr;  // RDL_TRACE_SUBMINOR
  uint64_t pending_n_sel = 0;
  uint32_t pending_g = 0;
  int pending_kind = 0, pending_threads = 0, pending_table = 0;
};

namespace rdl {

constexpr uint32_t kChunk = 2048;  // box pixels per selection workgroup
constexpr uint32_t kSelThreads = 256;
constexpr uint32_t kLoopThreads = 512;

struct SelArgs {
  const float* residuals;
  const uint8_t* mask;
  uint32_t width, height, n;  // n = width*height
  uint32_t xs, xe, ys, ye, bw;
  uint64_t box_pixels;
  rdl_integration integ;
  float threshold;
  int32_t allow_negative;
  const float* rms;  // RMS factor image (W x H) or nullptr
};

// A thread's box position, advanced by a fixed stride without dividing (a
// 64-bit divide per pixel made the selection passes ALU-bound).
struct BoxWalker {
  uint64_t b;
  uint32_t x, y;  // inside the box
  __device__ BoxWalker(const SelArgs& a, uint64_t b0)
      : b(b0), x(uint32_t(b0 % a.bw)), y(uint32_t(b0 / a.bw)) {}
  __device__ void Advance(const SelArgs& a, uint32_t stride) {
    b += stride;
    x += stride;
    while (x >= a.bw) {
      x -= a.bw;
      ++y;
    }
  }
};

// the selection test of pixel idx whose first image's residual v0 the
// caller loaded (so a thread's loads can all be in flight at once)
__device__ __forceinline__ bool SelectedValue(const SelArgs& a, uint32_t idx, float v0) {
  if (a.mask && !a.mask[idx]) return false;
  float v = IntegratePixel(a.integ, [&](uint32_t k) {
    return k == 0 ? v0 : a.residuals[size_t(k) * a.n + idx];
  });
  if (a.rms) v *= a.rms[idx];  // integratedScratch *= rms (subminor_loop.cc:147-149)
  const float value = a.allow_negative ? fabsf(v) : v;
  return value >= a.threshold;
}

__device__ __forceinline__ bool Selected(const SelArgs& a, const BoxWalker& w,
                                         uint32_t& idx) {
  if (w.b >= a.box_pixels) return false;
  idx = (a.ys + w.y) * a.width + a.xs + w.x;
  if (a.mask && !a.mask[idx]) return false;
  float v = IntegratePixel(
      a.integ, [&](uint32_t k) { return a.residuals[size_t(k) * a.n + idx]; });
  if (a.rms) v *= a.rms[idx];  // integratedScratch *= rms (subminor_loop.cc:147-149)
  const float value = a.allow_negative ? fabsf(v) : v;
  return value >= a.threshold;
}

__global__ __launch_bounds__(kSelThreads) void SelCount(SelArgs a,
                                                        uint32_t* counts) {
  __shared__ uint32_t lds[kSelThreads / 64];
  uint32_t c = 0;
  const uint64_t base = uint64_t(blockIdx.x) * kChunk;
  BoxWalker bw(a, base + threadIdx.x);
  constexpr uint32_t kItems = kChunk / kSelThreads;
  uint32_t idx[kItems];
  float v0[kItems];
#pragma unroll
  for (uint32_t i = 0; i < kItems; ++i) {
    idx[i] = bw.b < a.box_pixels ? (a.ys + bw.y) * a.width + a.xs + bw.x : 0xffffffffu;
    bw.Advance(a, kSelThreads);
  }
#pragma unroll
  for (uint32_t i = 0; i < kItems; ++i)
    v0[i] = a.residuals[idx[i] == 0xffffffffu ? 0u : idx[i]];
#pragma unroll
  for (uint32_t i = 0; i < kItems; ++i)
    c += (idx[i] != 0xffffffffu && SelectedValue(a, idx[i], v0[i])) ? 1u : 0u;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kSelThreads / 64; ++w) t += lds[w];
    counts[blockIdx.x] = t;
  }
}

// Exclusive scan of the chunk counts in one workgroup; writes the total.
// Thread t owns the contiguous segment [t seg, (t + 1) seg): sums it, one
// block scan of the 1024 sums, then rewrites its segment as offsets.
__global__ __launch_bounds__(1024) void SelScan(uint32_t* counts, uint32_t n,
                                                uint64_t* total, uint64_t* total_host) {
  __shared__ uint64_t lds[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t seg = (n + 1023) / 1024;
  const uint32_t lo = min(n, t * seg), hi = min(n, lo + seg);
  uint64_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += counts[i];
  lds[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    const uint64_t v = t >= off ? lds[t - off] : 0;
    __syncthreads();
    lds[t] += v;
    __syncthreads();
  }
  uint64_t run = lds[t] - sum;  // exclusive
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = counts[i];
    counts[i] = uint32_t(run);
    run += c;
  }
  if (t == 1023) {
    *total = lds[1023];
    *total_host = lds[1023];  // the host's copy (mapped memory, no read-back copy)
  }
}

__global__ __launch_bounds__(kSelThreads) void SelScatter(
    SelArgs a, const uint32_t* offsets, uint32_t n_img, uint64_t n_sel,
    uint32_t* pos, float* r) {
  __shared__ uint32_t wave_tot[kSelThreads / 64];
  const uint64_t base = uint64_t(blockIdx.x) * kChunk;
  uint32_t running = offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  BoxWalker bw(a, base + threadIdx.x);
  for (uint32_t j0 = 0; j0 < kChunk; j0 += kSelThreads) {
    uint32_t idx = 0;
    const bool sel = Selected(a, bw, idx);
    bw.Advance(a, kSelThreads);
    const uint64_t ballot = __ballot(sel);
    const uint32_t before = __popcll(ballot & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wave] = __popcll(ballot);
    __syncthreads();
    uint32_t woff = 0;
    for (int w = 0; w < wave; ++w) woff += wave_tot[w];
    uint32_t step = 0;
    for (uint32_t w = 0; w < kSelThreads / 64; ++w) step += wave_tot[w];
    if (sel) {
      const uint64_t o = running + woff + before;
      const uint32_t x = idx % a.width, y = idx / a.width;
      pos[o] = (y << 16) | x;
      for (uint32_t k = 0; k < n_img; ++k)
        r[size_t(k) * n_sel + o] = a.residuals[size_t(k) * a.n + idx];
    }
    running += step;
    __syncthreads();
  }
}

// Single-pass selection (replaces SelCount + SelScan + SelScatter): each
// workgroup takes the next chunk in launch order (a ticket), flags its
// pixels once, publishes its count, and finds its output offset by
// decoupled look-back over its predecessors' published counts / prefixes
// (status words {flag, value}, single-copy-atomic 8-byte stores; flag 1 =
// the chunk's count, 2 = the inclusive prefix). Positions only; the residual
// values follow in SelGather once the host knows the count. One read of the
// box instead of two, no scan launch. Output order = ascending box order,
// as the three-kernel path.
constexpr uint32_t kSpThreads = 512;
constexpr uint32_t kSelItems = 16;
constexpr uint32_t kSpChunk = kSpThreads * kSelItems;  // box pixels per workgroup
constexpr uint64_t kStatusAggregate = uint64_t(1) << 32;
constexpr uint64_t kStatusPrefix = uint64_t(2) << 32;

__global__ __launch_bounds__(kSpThreads) void SelSinglePass(SelArgs a, uint32_t* ticket,
                                                             uint64_t* status,
                                                             uint32_t n_chunks, uint32_t* pos,
                                                             uint64_t* total,
                                                             uint32_t* failed,
                                                             uint64_t spin_limit) {
  __shared__ uint32_t chunk_s;
  __shared__ uint32_t wave_tot[kSelItems][kSpThreads / 64];
  __shared__ uint32_t excl_s;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  // ticket: chunks in the order workgroups start (NULL: blockIdx, which the
  // dispatcher hands out in order on each XCD)
  if (tid == 0) chunk_s = ticket ? atomicAdd(ticket, 1u) : blockIdx.x;
  __syncthreads();
  const uint32_t b = chunk_s;
  const uint64_t base = uint64_t(b) * kSpChunk;
  uint64_t ballots[kSelItems];
  uint32_t idx[kSelItems];
  BoxWalker bw(a, base + tid);
  float v0[kSelItems];
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i) {
    idx[i] = bw.b < a.box_pixels ? (a.ys + bw.y) * a.width + a.xs + bw.x : 0xffffffffu;
    bw.Advance(a, kSpThreads);
  }
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i)  // every load in flight at once
    v0[i] = a.residuals[idx[i] == 0xffffffffu ? 0u : idx[i]];
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i) {
    const bool sel = idx[i] != 0xffffffffu && SelectedValue(a, idx[i], v0[i]);
    ballots[i] = __ballot(sel);
    if (lane == 0) wave_tot[i][wave] = uint32_t(__popcll(ballots[i]));
  }
  __syncthreads();
  uint32_t count = 0;
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i)
#pragma unroll
    for (uint32_t w = 0; w < kSpThreads / 64; ++w) count += wave_tot[i][w];
  if (wave == 0) {
    uint64_t excl = 0;
    if (b == 0) {
      if (lane == 0)
        __hip_atomic_store(&status[0], kStatusPrefix | count, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(&status[b], kStatusAggregate | count, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      // look back 64 predecessors at a time (lane l: chunk b - 1 - l)
      int64_t p = int64_t(b) - 1 - int64_t(lane);
      uint64_t spins = 0;
      while (true) {
        uint64_t st = p >= 0 ? __hip_atomic_load(&status[p], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : kStatusPrefix;  // before chunk 0: prefix 0
        // every predecessor publishes its count before it looks back
        while (!__all((st >> 32) != 0u)) {
          __builtin_amdgcn_s_sleep(1);
          if ((st >> 32) == 0u)
            st = __hip_atomic_load(&status[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (++spins > spin_limit) break;  // never expected; ends the wave
        }
        const uint64_t pm = __ballot((st >> 32) == 2u);
        const uint32_t v = uint32_t(st);
        if (pm) {
          const uint32_t first = uint32_t(__builtin_ctzll(pm));  // nearest prefix
          uint64_t part = lane <= first ? uint64_t(v) : 0ull;
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
          excl += part;
          break;
        }
        uint64_t part = v;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
        excl += part;
        p -= 64;
        if (spins > spin_limit) break;
      }
      // a predecessor never published (never expected): the prefix is wrong,
      // so the selection is reported failed rather than silently corrupt
      if (spins > spin_limit && lane == 0) atomicOr(failed, 1u);
      if (lane == 0)
        __hip_atomic_store(&status[b], kStatusPrefix | uint32_t(excl + count),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      excl_s = uint32_t(excl);
      if (b == n_chunks - 1) *total = excl + count;
    }
  }
  __syncthreads();
  uint32_t o = excl_s;
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i) {
    uint32_t woff = 0, step = 0;
#pragma unroll
    for (uint32_t w = 0; w < kSpThreads / 64; ++w) {
      woff += w < wave ? wave_tot[i][w] : 0u;
      step += wave_tot[i][w];
    }
    if ((ballots[i] >> lane) & 1ull) {
      const uint32_t before = uint32_t(__popcll(ballots[i] & ((1ull << lane) - 1ull)));
      const uint32_t x = idx[i] % a.width, y = idx[i] / a.width;
      pos[o + woff + before] = (y << 16) | x;
    }
    o += step;
  }
}

// Sparse two-phase selection (the default): SelLocal flags each chunk's
// pixels once (the single pass's loads and tests) and stores the chunk's
// count and its selected positions, ascending, in the chunk's own slot of
// `local`; SelScan turns the counts into offsets; SelPlace moves every
// non-empty chunk's positions to its offset. No workgroup waits for another
// (the single pass's look-back chained the chunks), and a selection is a few
// thousand pixels, so the second pass touches a few hundred chunks.
__global__ __launch_bounds__(kSpThreads) void SelLocal(SelArgs a, uint32_t* __restrict__ counts,
                                                       uint32_t* __restrict__ local) {
  __shared__ uint32_t wave_tot[kSelItems][kSpThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t b = blockIdx.x;
  const uint64_t base = uint64_t(b) * kSpChunk;
  uint64_t ballots[kSelItems];
  uint32_t idx[kSelItems];
  BoxWalker bw(a, base + tid);
  float v0[kSelItems];
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i) {
    idx[i] = bw.b < a.box_pixels ? (a.ys + bw.y) * a.width + a.xs + bw.x : 0xffffffffu;
    bw.Advance(a, kSpThreads);
  }
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i)  // every load in flight at once
    v0[i] = a.residuals[idx[i] == 0xffffffffu ? 0u : idx[i]];
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i) {
    const bool sel = idx[i] != 0xffffffffu && SelectedValue(a, idx[i], v0[i]);
    ballots[i] = __ballot(sel);
    if (lane == 0) wave_tot[i][wave] = uint32_t(__popcll(ballots[i]));
  }
  __syncthreads();
  uint32_t count = 0;
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i)
#pragma unroll
    for (uint32_t w = 0; w < kSpThreads / 64; ++w) count += wave_tot[i][w];
  if (tid == 0) counts[b] = count;
  if (count == 0) return;
  uint32_t* out = local + base;
  uint32_t o = 0;
#pragma unroll
  for (uint32_t i = 0; i < kSelItems; ++i) {
    uint32_t woff = 0, step = 0;
#pragma unroll
    for (uint32_t w = 0; w < kSpThreads / 64; ++w) {
      woff += w < wave ? wave_tot[i][w] : 0u;
      step += wave_tot[i][w];
    }
    if ((ballots[i] >> lane) & 1ull) {
      const uint32_t before = uint32_t(__popcll(ballots[i] & ((1ull << lane) - 1ull)));
      const uint32_t x = idx[i] % a.width, y = idx[i] / a.width;
      out[o + woff + before] = (y << 16) | x;
    }
    o += step;
  }
}

// SelLocal with 16-byte loads (rows whose width is a multiple of 4, one
// image with the identity integration, no RMS weights): a workgroup takes
// `rpb` box rows, each as `ipr` items of 512 float4 (items of a row in
// order, rows in order: box order), so the selection costs a peak search's
// read. A lane's 4-pixel flags are ranked across the wave from three
// ballots of its count's bits.
constexpr uint32_t kQuadItems = 8;
constexpr uint32_t kQuadChunk = kSpThreads * kQuadItems * 4;  // pixel slots per chunk

__global__ __launch_bounds__(kSpThreads) void SelLocalQuad(SelArgs a, uint32_t ipr, uint32_t rpb,
                                                           uint32_t* __restrict__ counts,
                                                           uint32_t* __restrict__ local) {
  __shared__ uint32_t wave_tot[kQuadItems][kSpThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t b = blockIdx.x;
  const uint32_t y0 = a.ys + b * rpb;
  const uint32_t y1 = min(a.ye, y0 + rpb);
  const uint32_t q0 = a.xs >> 2, q1 = (a.xe + 3) >> 2;
  const uint64_t lower = (uint64_t(1) << lane) - 1ull;
  float4 v[kQuadItems];
  uint32_t mk[kQuadItems];
#pragma unroll
  for (uint32_t i = 0; i < kQuadItems; ++i) {  // every load in flight at once
    const uint32_t y = y0 + i / ipr, q = q0 + (i % ipr) * kSpThreads + tid;
    const bool in = y < y1 && q < q1;
    v[i] = in ? reinterpret_cast<const float4*>(a.residuals + size_t(y) * a.width)[q]
              : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    mk[i] = in ? 0x01010101u : 0u;
    if (in && a.mask) mk[i] = reinterpret_cast<const uint32_t*>(a.mask + size_t(y) * a.width)[q];
  }
  uint32_t m4[kQuadItems], pre[kQuadItems];
  uint32_t any_m = 0u;
#pragma unroll
  for (uint32_t i = 0; i < kQuadItems; ++i) {
    const uint32_t q = q0 + (i % ipr) * kSpThreads + tid;
    const float vv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    uint32_t m = 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t x = 4 * q + j;
      const float value = a.allow_negative ? fabsf(vv[j]) : vv[j];
      const bool sel = ((mk[i] >> (8 * j)) & 0xffu) && x >= a.xs && x < a.xe &&
                       value >= a.threshold;
      m |= sel ? (1u << j) : 0u;
    }
    m4[i] = m;
    any_m |= m;
  }
  // a selection is sparse: most waves select nothing and skip the ranking
  if (__any(any_m != 0u)) {
#pragma unroll
    for (uint32_t i = 0; i < kQuadItems; ++i) {
      const uint32_t c = uint32_t(__popc(m4[i]));
      const uint64_t b0 = __ballot(c & 1u), b1 = __ballot(c & 2u), b2 = __ballot(c & 4u);
      pre[i] = uint32_t(__popcll(b0 & lower) + 2 * __popcll(b1 & lower) + 4 * __popcll(b2 & lower));
      if (lane == 0)
        wave_tot[i][wave] = uint32_t(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kQuadItems; ++i) {
      pre[i] = 0u;
      if (lane == 0) wave_tot[i][wave] = 0u;
    }
  }
  __syncthreads();
  uint32_t count = 0;
#pragma unroll
  for (uint32_t i = 0; i < kQuadItems; ++i)
#pragma unroll
    for (uint32_t w = 0; w < kSpThreads / 64; ++w) count += wave_tot[i][w];
  if (tid == 0) counts[b] = count;
  if (count == 0) return;
  uint32_t* out = local + uint64_t(b) * kQuadChunk;
  uint32_t o = 0;
#pragma unroll
  for (uint32_t i = 0; i < kQuadItems; ++i) {
    uint32_t woff = 0, step = 0;
#pragma unroll
    for (uint32_t w = 0; w < kSpThreads / 64; ++w) {
      woff += w < wave ? wave_tot[i][w] : 0u;
      step += wave_tot[i][w];
    }
    if (m4[i]) {
      const uint32_t y = y0 + i / ipr, q = q0 + (i % ipr) * kSpThreads + tid;
      uint32_t k = o + woff + pre[i];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j)
        if ((m4[i] >> j) & 1u) out[k++] = (y << 16) | (4 * q + j);
    }
    o += step;
  }
}

// chunk b's positions (offsets[b] .. offsets[b + 1], the last to *total)
__global__ __launch_bounds__(256) void SelPlace(const uint32_t* __restrict__ offsets,
                                                uint32_t n_chunks,
                                                const uint64_t* __restrict__ total,
                                                const uint32_t* __restrict__ local,
                                                uint32_t chunk_slots,
                                                uint32_t* __restrict__ pos) {
  const uint32_t b = blockIdx.x;
  const uint32_t off = offsets[b];
  const uint32_t end = b + 1 < n_chunks ? offsets[b + 1] : uint32_t(*total);
  const uint32_t* src = local + uint64_t(b) * chunk_slots;
  for (uint32_t k = threadIdx.x; off + k < end; k += 256) pos[off + k] = src[k];
}

// the selected pixels' residual values, [image][n_sel]
__global__ __launch_bounds__(256) void SelGather(const float* residuals, uint32_t width,
                                                 uint32_t n, const uint32_t* pos,
                                                 uint64_t n_sel, uint32_t n_img, float* r) {
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < n_sel;
       j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t p = pos[j];
    const uint32_t idx = (p >> 16) * width + (p & 0xffffu);
    for (uint32_t k = 0; k < n_img; ++k) r[k * n_sel + j] = residuals[size_t(k) * n + idx];
  }
}

// ----------------------------------------------------------------- loop
struct LoopArgs {
  const uint32_t* pos;    // n_sel
  float* r;               // [n_img][n_sel] (in: gathered residuals)
  float* m;               // [n_img][n_sel] (out: model values)
  const float* psfs;      // twice-convolved PSFs, W*H planes
  const float* spectral;  // n_img x n_img spectral-fit map, or nullptr
  const float* rms;       // RMS factor image (W x H), or nullptr
  uint32_t* records;      // [2][G][rec_words] (G > 1)
  uint32_t* counter;      // arrival counter (G > 1), zeroed per launch
  uint32_t* result;       // LoopResult
  uint32_t* trace;        // 2 x u32 per component
  uint64_t trace_cap;
  uint64_t n_sel;
  uint32_t per_block;
  uint32_t n_blocks;
  uint32_t rec_words;
  uint32_t width, height, n_img, n_pol;
  rdl_integration integ;
  float threshold, gain, divergence_limit;
  uint64_t iteration_start, max_iterations;
  int32_t allow_negative, stop_on_negative;
  int32_t use_lds;
  int32_t prof;           // accumulate per-phase cycles (block 0, wave 0)
  const float* table;     // pairwise PSF table (BuildPairTable) or nullptr
  rdl_logpoly lp;         // log-polynomial fit (has_lp; SubminorLoop only)
  int32_t has_lp;
  // table loops on a grid: launched blocks per participant (the participants
  // are blocks 0, S, 2S, ...: S = 8 puts them on one XCD under round-robin
  // dispatch; a pooled session whose share of the GPU is below 8 blocks per
  // participant launches S = 1), and 1 to exchange through agent-scope
  // stores even when every participant is on one XCD (RDL_SUBMINOR_EXCHANGE=agent)
  uint32_t part_stride;
  int32_t agent_exchange;
  // SubminorLoopTab with one workgroup: the block argmax as ONE 64-bit LDS
  // atomic max per 16-lane row (RDL_SUBMINOR_ATOMIC=0: the wave slots)
  int32_t atomic_reduce;
};

struct LoopResult {
  uint64_t iteration;
  float peak;
  int32_t diverging;
  float flux;
  uint32_t error;
};

__device__ __forceinline__ uint64_t MaxKey(float integ, bool allow_negative,
                                           uint64_t p) {
  const float v = allow_negative ? fabsf(integ) : integ;
  if (v != v) return 0ull;  // NaN never wins (unless everything is NaN)
  uint32_t u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return (uint64_t(u) << 32) | uint64_t(0xffffffffu - uint32_t(p));
}

// The float MaxKey encoded (|v| when allow_negative).
__device__ __forceinline__ float KeyValue(uint64_t key) {
  uint32_t u = uint32_t(key >> 32);
  u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  return __uint_as_float(u);
}

__device__ __forceinline__ void StoreSc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t LoadSc1(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Winner record layout (u32 words): key lo, key hi, integ (f32), pos, r[n_img]
template <int NI>
__global__ __launch_bounds__(kLoopThreads) void SubminorLoop(LoopArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ uint64_t red[kLoopThreads / 64];
  __shared__ uint32_t win[4 + RDL_MAX_IMAGES];
  __shared__ uint32_t flags[2];

  const uint32_t tid = threadIdx.x;
  const uint64_t base = uint64_t(blockIdx.x) * a.per_block;
  const uint32_t cnt =
      base >= a.n_sel ? 0u : uint32_t(min<uint64_t>(a.per_block, a.n_sel - base));
  const uint32_t n_img = a.n_img;

  uint32_t* pos;
  float* R;
  float* M;
  size_t stride;  // between images
  if (a.use_lds) {
    pos = smem;
    R = reinterpret_cast<float*>(smem + a.per_block);
    M = R + size_t(n_img) * a.per_block;
    stride = a.per_block;
    for (uint32_t j = tid; j < cnt; j += kLoopThreads) {
      pos[j] = a.pos[base + j];
      for (uint32_t k = 0; k < n_img; ++k) {
        R[k * stride + j] = a.r[size_t(k) * a.n_sel + base + j];
        M[k * stride + j] = 0.0f;
      }
    }
  } else {
    pos = const_cast<uint32_t*>(a.pos) + base;
    R = a.r + base;
    M = a.m + base;
    stride = a.n_sel;
    for (uint32_t j = tid; j < cnt; j += kLoopThreads)
      for (uint32_t k = 0; k < n_img; ++k) M[k * stride + j] = 0.0f;
  }
  __syncthreads();

  const int W = int(a.width), H = int(a.height);
  const size_t plane = size_t(a.width) * a.height;
  float c[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) c[k] = 0.0f;
  int cx = 0, cy = 0;
  bool have_component = false;
  float start_abs = 0.0f;
  bool diverging = false;
  float flux = 0.0f;
  uint64_t iteration = a.iteration_start;
  uint32_t gen = 0;
  float m = 0.0f;
  uint64_t winner_p = 0;

  while (true) {
    // ---- subtract the current component, integrate, local argmax
    uint64_t best = 0;
    for (uint32_t j = tid; j < cnt; j += kLoopThreads) {
      const uint32_t pk = pos[j];
      const int px = int(pk & 0xffffu), py = int(pk >> 16);
      float v[NI];
      if (have_component) {
        const int dx = px - cx + W / 2, dy = py - cy + H / 2;
        const bool in = dx >= 0 && dx < W && dy >= 0 && dy < H;
        const size_t off = size_t(dy) * a.width + size_t(dx);
#pragma unroll
        for (int k = 0; k < NI; ++k) {
          if (k < int(n_img)) {
            float rv = R[k * stride + j];
            if (in) {
              const float pv = a.psfs[size_t(k / int(a.n_pol)) * plane + off];
              rv = __builtin_fmaf(-pv, c[k], rv);
              R[k * stride + j] = rv;
            }
            v[k] = rv;
          } else {
            v[k] = 0.0f;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < NI; ++k)
          v[k] = k < int(n_img) ? R[k * stride + j] : 0.0f;
      }
      float integ = IntegratePixel(a.integ, [&](uint32_t kk) {
        float r = v[0];
#pragma unroll
        for (int q = 1; q < NI; ++q) r = (uint32_t(q) == kk) ? v[q] : r;
        return r;
      });
      if (a.rms) integ *= a.rms[size_t(py) * a.width + px];  // GetMaxComponent
      uint64_t key = MaxKey(integ, a.allow_negative, base + j);
      if (base + j == 0 && integ != integ) key = ~0ull;  // scratch[0] is NaN
      best = key > best ? key : best;
    }
    // block reduce
    {
      uint64_t w = WaveMaxU64(best);
      if ((tid & 63) == 0) red[tid >> 6] = w;
      __syncthreads();
      if (tid < 64) {
        uint64_t x = tid < kLoopThreads / 64 ? red[tid] : 0ull;
        x = WaveMaxU64(x);
        if (tid == 0) red[0] = x;
      }
      __syncthreads();
    }
    const uint64_t block_best = red[0];
    // owner of the block winner fills the local record
    if (cnt > 0) {
      const uint64_t lp = block_best == 0 ? 0ull
                          : block_best == ~0ull ? 0ull
                          : uint64_t(0xffffffffu - uint32_t(block_best));
      const uint64_t j = lp - base;
      if (lp >= base && j < cnt && (j % kLoopThreads) == tid) {
        win[0] = uint32_t(block_best);
        win[1] = uint32_t(block_best >> 32);
        float vv[NI];
#pragma unroll
        for (int k = 0; k < NI; ++k)
          vv[k] = k < int(n_img) ? R[k * stride + j] : 0.0f;
        float integ = IntegratePixel(a.integ, [&](uint32_t kk) {
          float r = vv[0];
#pragma unroll
          for (int q = 1; q < NI; ++q) r = (uint32_t(q) == kk) ? vv[q] : r;
          return r;
        });
        if (a.rms)
          integ *= a.rms[size_t(pos[j] >> 16) * a.width + (pos[j] & 0xffffu)];
        win[2] = __float_as_uint(integ);
        win[3] = pos[j];
        for (uint32_t k = 0; k < n_img; ++k) win[4 + k] = __float_as_uint(vv[k]);
      }
    } else if (tid == 0) {
      win[0] = 0;
      win[1] = 0;
    }
    __syncthreads();

    if (a.n_blocks > 1) {
      // ---- exchange records: write-through stores, arrival counter
      uint32_t* rec_base = a.records + size_t(gen & 1) * a.n_blocks * a.rec_words;
      if (tid == 0) {
        uint32_t* rec = rec_base + size_t(blockIdx.x) * a.rec_words;
        for (uint32_t w = 0; w < 4 + n_img; ++w) StoreSc1(rec + w, win[w]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t target = (gen + 1) * a.n_blocks;
        uint64_t spins = 0;
        flags[0] = 0;
        while (LoadSc1(a.counter) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1ull << 28)) {  // ~minutes: a lost workgroup
            flags[0] = 1;
            break;
          }
        }
      }
      __syncthreads();
      if (flags[0]) {
        if (tid == 0) StoreSc1(&a.result[8], 1u);
        return;
      }
      // wave 0 reduces the G keys
      if (tid < 64) {
        uint64_t bk = 0;
        uint32_t bb = 0;
        for (uint32_t b = tid; b < a.n_blocks; b += 64) {
          uint32_t* rec = rec_base + size_t(b) * a.rec_words;
          const uint64_t k =
              uint64_t(LoadSc1(rec)) | (uint64_t(LoadSc1(rec + 1)) << 32);
          if (k > bk) {
            bk = k;
            bb = b;
          }
        }
        // wave argmax over (key, block)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const uint64_t ok = __shfl_xor(bk, off, 64);
          const uint32_t ob = __shfl_xor(bb, off, 64);
          if (ok > bk || (ok == bk && ob < bb)) {
            bk = ok;
            bb = ob;
          }
        }
        if (tid == 0) flags[1] = bb;
      }
      __syncthreads();
      if (tid < 4 + n_img) {
        uint32_t* rec = rec_base + size_t(flags[1]) * a.rec_words;
        win[tid] = LoadSc1(rec + tid);
      }
      __syncthreads();
      ++gen;
    }

    // ---- the global winner is in win[]; identical decisions everywhere
    const uint64_t gkey = uint64_t(win[0]) | (uint64_t(win[1]) << 32);
    winner_p = (gkey == 0 || gkey == ~0ull)
                   ? 0ull
                   : uint64_t(0xffffffffu - uint32_t(gkey));
    m = __uint_as_float(win[2]);
    if (!have_component) {
      start_abs = fabsf(m);  // subminor_loop.cc:59
    } else {
      if (a.divergence_limit != 0.0f)
        diverging = fabsf(m) > start_abs * a.divergence_limit;
      ++iteration;
    }
    // loop condition (subminor_loop.cc:61-63)
    const bool go = fabsf(m) > a.threshold && iteration < a.max_iterations &&
                    (!a.stop_on_negative || m >= 0.0f) && !diverging;
    if (!go) break;
    // next component (subminor_loop.cc:64-89)
    if (a.has_lp) {
      // PerformSpectralFit of the gain-scaled values (subminor_loop.cc:66-76)
      // with the log-polynomial fitter: every thread runs the same fit on
      // the same values (identical bits, no broadcast needed)
      float v[NI];
      for (int k = 0; k < NI; ++k)
        v[k] = k < int(n_img) ? __uint_as_float(win[4 + k]) * a.gain : 0.0f;
      lp::PerformSpectralFit(a.lp, a.n_pol, v);
#pragma unroll
      for (int k = 0; k < NI; ++k) c[k] = k < int(n_img) ? v[k] : 0.0f;
    } else if (a.spectral) {
      // PerformSpectralFit of the gain-scaled values (subminor_loop.cc:66-76)
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        float acc = 0.0f;
        if (k < int(n_img))
          for (uint32_t q = 0; q < n_img; ++q)
            acc = __builtin_fmaf(a.spectral[k * n_img + q],
                                 __uint_as_float(win[4 + q]) * a.gain, acc);
        c[k] = acc;
      }
    } else {
#pragma unroll
      for (int k = 0; k < NI; ++k)
        c[k] = k < int(n_img) ? __uint_as_float(win[4 + k]) * a.gain : 0.0f;
    }
    flux += m * a.gain;
    cx = int(win[3] & 0xffffu);
    cy = int(win[3] >> 16);
    {
      const uint64_t j = winner_p - base;
      if (winner_p >= base && j < cnt && (j % kLoopThreads) == tid) {
#pragma unroll
        for (int k = 0; k < NI; ++k)
          if (k < int(n_img)) M[k * stride + j] += c[k];
      }
    }
    if (blockIdx.x == 0 && tid == 0 && a.trace) {
      const uint64_t t = iteration - a.iteration_start;
      if (t < a.trace_cap) {
        a.trace[2 * t] = uint32_t(cx);
        a.trace[2 * t + 1] = uint32_t(cy);
      }
    }
    have_component = true;
    __syncthreads();
  }

  // write back model values (LDS variant)
  if (a.use_lds) {
    for (uint32_t j = tid; j < cnt; j += kLoopThreads)
      for (uint32_t k = 0; k < n_img; ++k)
        a.m[size_t(k) * a.n_sel + base + j] = M[k * stride + j];
  }
  if (blockIdx.x == 0 && tid == 0) {
    LoopResult* r = reinterpret_cast<LoopResult*>(a.result);
    r->iteration = iteration;
    r->peak = m;
    r->diverging = diverging ? 1 : 0;
    r->flux = flux;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ScatterModel(const uint32_t* pos,
                                                    const float* m,
                                                    uint64_t n_sel,
                                                    T* dest, uint32_t dw,
                                                    uint32_t ox, uint32_t oy,
                                                    int add) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n_sel;
       i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t pk = pos[i];
    const size_t d = size_t((pk >> 16) + oy) * dw + (pk & 0xffffu) + ox;
    if (add)
      dest[d] += T(m[i]);
    else
      dest[d] = T(m[i]);
  }
}

// rows of the (untrimmed) model plane that hold a non-zero component
// SubMinorLoop::UpdateAutoMask (subminor_loop.cc:220-228)
__global__ __launch_bounds__(256) void UpdateMaskKernel(const uint32_t* pos,
                                                        const float* m, uint64_t n_sel,
                                                        uint32_t n_img, uint32_t width,
                                                        uint8_t* mask) {
  const uint64_t p = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (p >= n_sel) return;
  bool any = false;
  for (uint32_t k = 0; k < n_img; ++k) any |= m[size_t(k) * n_sel + p] != 0.0f;
  if (any) mask[size_t(pos[p] >> 16) * width + (pos[p] & 0xffffu)] = 1;
}

__global__ __launch_bounds__(256) void MarkModelRows(const uint32_t* pos,
                                                     const float* m, uint64_t n_sel,
                                                     uint8_t* rows, uint32_t oy) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n_sel;
       i += uint64_t(gridDim.x) * blockDim.x)
    if (m[i] != 0.0f) rows[(pos[i] >> 16) + oy] = 1;
}

// zero the rows y of a width-wide plane whose mark rows[y + oy] is set
__global__ __launch_bounds__(256) void ZeroMarkedRows(float* __restrict__ plane, uint32_t width,
                                                      uint32_t height,
                                                      const uint8_t* __restrict__ rows,
                                                      uint32_t oy) {
  for (uint32_t y = blockIdx.x; y < height; y += gridDim.x) {
    if (!rows[y + oy]) continue;
    float* row = plane + size_t(y) * width;
    for (uint32_t x = threadIdx.x; x < width; x += 256) row[x] = 0.0f;
  }
}

// Model update of a scale > 0 outer iteration: model += the selection's
// component values convolved (circularly, as the FFT convolution of the
// reference does) with the scale's n x n shape kernel, by direct stamping.
// One workgroup per 64 x 64 output tile walks the selection in index order,
// keeps the components whose (wrapped) stamp reaches the tile, and sums
// m_c * k[y - y_c + n/2][x - x_c + n/2] per pixel in that order: a fixed
// summation order, so the result is reproducible.
constexpr uint32_t kStampTile = 64;
constexpr uint32_t kStampThreads = 256;
constexpr uint32_t kStampRows = kStampTile * kStampTile / kStampThreads;  // 16

// d in (-size, 2*size) -> d mod size
__device__ __forceinline__ uint32_t WrapDist(int32_t d, uint32_t size) {
  if (d < 0) d += int32_t(size);
  if (d >= int32_t(size)) d -= int32_t(size);
  return uint32_t(d);
}

// the tiles some component's n x n stamp reaches (circularly, as the
// stamping's hit test): a conservative byte map, so a tile no stamp reaches
// skips its walk over the selection
__device__ __forceinline__ void TileSpan(int32_t lo, int32_t hi, uint32_t size,
                                         uint32_t (&a)[2], uint32_t (&b)[2], int& k) {
  // [lo, hi] (hi - lo < size) as tile ranges, split where it wraps
  k = 0;
  if (lo < 0) {
    a[k] = uint32_t(lo + int32_t(size)) / kStampTile;
    b[k++] = (size - 1) / kStampTile;
    lo = 0;
  }
  if (hi >= int32_t(size)) {
    a[k] = 0;
    b[k++] = uint32_t(hi - int32_t(size)) / kStampTile;
    hi = int32_t(size) - 1;
  }
  a[k] = uint32_t(lo) / kStampTile;
  b[k++] = uint32_t(hi) / kStampTile;
}

// Per chunk of kStampThreads components (StampShapeModel's walk), the box
// its stamps cover, unwrapped: {x lo, x hi, y lo, y hi}; x lo > x hi when no
// component of the chunk is non-zero. One workgroup per chunk.
__global__ __launch_bounds__(256) void MarkStampTiles(const uint32_t* __restrict__ pos,
                                                      const float* __restrict__ m,
                                                      uint64_t n_sel, uint32_t n,
                                                      uint32_t width, uint32_t height,
                                                      uint32_t tiles_x,
                                                      uint8_t* __restrict__ mark,
                                                      int4* __restrict__ bounds) {
  const int32_t h = int32_t(n / 2);
  __shared__ int32_t red[4][256 / 64];
  int32_t bx0 = INT32_MAX, bx1 = INT32_MIN, by0 = INT32_MAX, by1 = INT32_MIN;
  const uint64_t c = blockIdx.x * uint64_t(256) + threadIdx.x;
  if (c < n_sel && m[c] != 0.0f) {
    const int32_t xc = int32_t(pos[c] & 0xffffu), yc = int32_t(pos[c] >> 16);
    bx0 = xc - h;
    bx1 = xc + h;
    by0 = yc - h;
    by1 = yc + h;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    bx0 = min(bx0, __shfl_xor(bx0, off, 64));
    bx1 = max(bx1, __shfl_xor(bx1, off, 64));
    by0 = min(by0, __shfl_xor(by0, off, 64));
    by1 = max(by1, __shfl_xor(by1, off, 64));
  }
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = bx0;
    red[1][wave] = bx1;
    red[2][wave] = by0;
    red[3][wave] = by1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < 256 / 64; ++w) {
      red[0][0] = min(red[0][0], red[0][w]);
      red[1][0] = max(red[1][0], red[1][w]);
      red[2][0] = min(red[2][0], red[2][w]);
      red[3][0] = max(red[3][0], red[3][w]);
    }
    bounds[blockIdx.x] = make_int4(red[0][0], red[1][0], red[2][0], red[3][0]);
  }
  {
    if (c >= n_sel || m[c] == 0.0f) return;
    const int32_t xc = int32_t(pos[c] & 0xffffu), yc = int32_t(pos[c] >> 16);
    uint32_t xa[2], xb[2], ya[2], yb[2];
    int nx, ny;
    TileSpan(xc - h, xc + h, width, xa, xb, nx);
    TileSpan(yc - h, yc + h, height, ya, yb, ny);
    for (int i = 0; i < ny; ++i)
      for (uint32_t ty = ya[i]; ty <= yb[i]; ++ty)
        for (int j = 0; j < nx; ++j)
          for (uint32_t tx = xa[j]; tx <= xb[j]; ++tx) mark[ty * tiles_x + tx] = 1;
  }
}

// a chunk's stamps miss the tile [t0, t0 + l) on one axis (a box that wraps
// around the plane never misses)
__device__ __forceinline__ bool StampMisses(int32_t lo, int32_t hi, uint32_t t0, uint32_t l,
                                            uint32_t size) {
  if (lo < 0 || hi >= int32_t(size)) return false;
  return hi < int32_t(t0) || lo >= int32_t(t0 + l);
}

__global__ __launch_bounds__(kStampThreads) void StampShapeModel(
    const uint32_t* __restrict__ pos, const float* __restrict__ m, uint64_t n_sel,
    const float* __restrict__ kern, uint32_t n, float* __restrict__ model,
    uint32_t width, uint32_t height, uint32_t tiles_x, const uint8_t* __restrict__ mark,
    const int4* __restrict__ bounds) {
  if (!mark[blockIdx.x]) return;
  __shared__ uint32_t list[kStampThreads];
  __shared__ uint32_t wave_count[kStampThreads / 64];
  __shared__ uint32_t n_list;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t tx0 = (blockIdx.x % tiles_x) * kStampTile;
  const uint32_t ty0 = (blockIdx.x / tiles_x) * kStampTile;
  const uint32_t lx = min(kStampTile, width - tx0), ly = min(kStampTile, height - ty0);
  const uint32_t h = n / 2;
  const uint32_t px = tx0 + (tid % kStampTile);
  const uint32_t py0 = ty0 + tid / kStampTile;
  float acc[kStampRows];
#pragma unroll
  for (uint32_t r = 0; r < kStampRows; ++r) acc[r] = 0.0f;
  bool any = false;
  for (uint64_t base = 0; base < n_sel; base += kStampThreads) {
    // chunks whose stamps cannot reach this tile (components come in raster
    // order, so a chunk covers a few rows): skipped whole, uniformly
    if (bounds) {
      const int4 bb = bounds[base / kStampThreads];
      if (bb.x > bb.y || StampMisses(bb.x, bb.y, tx0, lx, width) ||
          StampMisses(bb.z, bb.w, ty0, ly, height))
        continue;
    }
    const uint64_t c = base + tid;
    bool hit = false;
    if (c < n_sel && m[c] != 0.0f) {
      const uint32_t pk = pos[c];
      const uint32_t xc = pk & 0xffffu, yc = pk >> 16;
      const uint32_t dx0 = WrapDist(int32_t(tx0) - int32_t(xc) + int32_t(h), width);
      const uint32_t dy0 = WrapDist(int32_t(ty0) - int32_t(yc) + int32_t(h), height);
      hit = (dx0 < n || dx0 + lx - 1 >= width) && (dy0 < n || dy0 + ly - 1 >= height);
    }
    // order-preserving compaction of the hits (wave order, then lane order)
    const uint64_t b = __ballot(hit);
    if (lane == 0) wave_count[wave] = uint32_t(__popcll(b));
    __syncthreads();
    uint32_t off = 0, total = 0;
    for (uint32_t w = 0; w < kStampThreads / 64; ++w) {
      if (w < wave) off += wave_count[w];
      total += wave_count[w];
    }
    if (hit) list[off + uint32_t(__popcll(b & ((uint64_t(1) << lane) - 1)))] = uint32_t(c - base);
    if (tid == 0) n_list = total;
    __syncthreads();
    const uint32_t cnt = n_list;
    any |= cnt != 0;
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint64_t cc = base + list[i];
      const uint32_t pk = pos[cc];
      const float v = m[cc];
      const uint32_t xc = pk & 0xffffu, yc = pk >> 16;
      const uint32_t dx = WrapDist(int32_t(px) - int32_t(xc) + int32_t(h), width);
      if (dx >= n || px >= width) continue;
      constexpr uint32_t kStep = kStampThreads / kStampTile;
      uint32_t dy = WrapDist(int32_t(py0) - int32_t(yc) + int32_t(h), height);
#pragma unroll
      for (uint32_t r = 0; r < kStampRows; ++r) {
        if (dy < n && py0 + r * kStep < height) acc[r] += v * kern[dy * n + dx];
        dy += kStep;
        if (dy >= height) dy -= height;
      }
    }
    __syncthreads();
  }
  if (!any || px >= width) return;
#pragma unroll
  for (uint32_t r = 0; r < kStampRows; ++r) {
    const uint32_t py = py0 + r * (kStampThreads / kStampTile);
    if (py < height) model[size_t(py) * width + px] += acc[r];
  }
}

// ------------------------------------------------- pairwise PSF table
// table[q][p][j] = PSF q at the offset of selected pixel j from selected
// pixel p (the value the loop gathers for pixel j when p is the component),
// or kOutsideBits where that offset leaves the PSF plane (no subtraction,
// subminor_loop.cc:100-106). Built once per loop by the whole GPU; the loop
// then reads ONE contiguous row per component (coalesced, L2-reusable when a
// component repeats) instead of n_sel scattered gathers.
constexpr uint32_t kOutsideBits = 0x7fbadbadu;  // a NaN payload no PSF value carries

__global__ __launch_bounds__(256) void BuildPairTable(const uint32_t* __restrict__ pos,
                                                      const float* __restrict__ psfs,
                                                      uint32_t n_sel, uint32_t n_psf,
                                                      uint32_t width, uint32_t height,
                                                      float* __restrict__ table,
                                                      uint64_t* __restrict__ zero,
                                                      uint32_t zero_words) {
  // the loop's per-launch exchange area, zeroed here (no memset launch: the
  // loop runs after this kernel on the same stream)
  if (blockIdx.x == 0 && blockIdx.y == 0)
    for (uint32_t w = threadIdx.x; w < zero_words; w += 256) zero[w] = 0ull;
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  const uint32_t p = blockIdx.y;
  if (j >= n_sel) return;
  const uint32_t pp = pos[p], pj = pos[j];
  const int dx = int(pj & 0xffffu) - int(pp & 0xffffu) + int(width / 2);
  const int dy = int(pj >> 16) - int(pp >> 16) + int(height / 2);
  const bool in = dx >= 0 && dx < int(width) && dy >= 0 && dy < int(height);
  const size_t plane = size_t(width) * height;
  const size_t off = in ? size_t(dy) * width + size_t(dx) : 0;
  for (uint32_t q = 0; q < n_psf; ++q)
    table[(size_t(q) * n_sel + p) * n_sel + j] =
        in ? psfs[size_t(q) * plane + off] : __uint_as_float(kOutsideBits);
}

// ------------------------------------------------- register-resident loop
// SubminorLoopReg: the same loop with each thread's ITEMS selected pixels
// (positions, residuals, model values) held in VGPRs, so one iteration is
//   * ITEMS x N_img PSF gathers issued back to back (one memory round trip),
//   * FMAs + integration + per-thread argmax in registers,
//   * a wave argmax, the wave winner's payload into a parity slot in LDS,
//   * ONE workgroup barrier; every wave then reduces the slots itself.
// With G > 1 workgroups the block winners are exchanged through epoch-tagged
// 8-byte granules ({epoch, word}, single-copy-atomic sc1 stores/loads): wave 0
// sweeps all G records until every tag matches, so the data is the flag and
// no counter or fence round trip is needed (parity-double-buffered so a fast
// block never overwrites a record a slow one has not read).
constexpr uint32_t kRegThreads = 512;
constexpr uint32_t kRegWaves = kRegThreads / 64;

// DPP cross-lane moves (gfx9 family): a 64-lane max in 6 VALU steps instead
// of 6 ds_bpermute round trips; the result is read from lane 63 (or lane 0
// for the 8-lane form) into a scalar.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint64_t DppU64(uint64_t v) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_update_dpp(
      0, int(uint32_t(v)), CTRL, ROW_MASK, 0xf, false));
  const uint32_t hi = uint32_t(__builtin_amdgcn_update_dpp(
      0, int(uint32_t(v >> 32)), CTRL, ROW_MASK, 0xf, false));
  return (uint64_t(hi) << 32) | lo;
}
__device__ __forceinline__ uint64_t ReadLaneU64(uint64_t v, int lane) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), lane));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), lane));
  return (uint64_t(hi) << 32) | lo;
}
// Max over lanes 0..7 (others must hold 0); uniform result.
__device__ __forceinline__ uint64_t Max8U64(uint64_t v) {
  uint64_t t;
  t = DppU64<0xb1>(v);  // quad_perm [1,0,3,2]
  v = t > v ? t : v;
  t = DppU64<0x4e>(v);  // quad_perm [2,3,0,1]
  v = t > v ? t : v;
  t = DppU64<0x141>(v);  // row_half_mirror
  v = t > v ? t : v;
  return ReadLaneU64(v, 0);
}
// Max over lanes 0..15 (others must hold 0); uniform result.
__device__ __forceinline__ uint64_t Max16U64(uint64_t v) {
  uint64_t t;
  t = DppU64<0xb1>(v);
  v = t > v ? t : v;
  t = DppU64<0x4e>(v);
  v = t > v ? t : v;
  t = DppU64<0x141>(v);
  v = t > v ? t : v;
  t = DppU64<0x140>(v);  // row_mirror
  v = t > v ? t : v;
  return ReadLaneU64(v, 0);
}
// Max over the 64 lanes; uniform result.
__device__ __forceinline__ uint64_t Max64U64(uint64_t v) {
  uint64_t t;
  t = DppU64<0xb1>(v);
  v = t > v ? t : v;
  t = DppU64<0x4e>(v);
  v = t > v ? t : v;
  t = DppU64<0x141>(v);
  v = t > v ? t : v;
  t = DppU64<0x140>(v);  // row_mirror
  v = t > v ? t : v;
  t = DppU64<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v = t > v ? t : v;
  t = DppU64<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
  v = t > v ? t : v;
  return ReadLaneU64(v, 63);
}
// Workgroup barrier that orders LDS only: __syncthreads() also drains vmcnt,
// which would make every iteration wait for its own trace/granule stores.
__device__ __forceinline__ void LdsBarrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ int FirstLane(bool pred) {
  const uint64_t b = __ballot(pred);
  return b ? __builtin_ctzll(b) : 0;
}

// 32-bit max over lanes (DPP, one fused max per step); LANES = 8, 16 or 64
// (lanes beyond LANES must hold 0); uniform result.
template <int LANES>
__device__ __forceinline__ uint32_t MaxU32(uint32_t v) {
  auto step = [](uint32_t x, uint32_t t) { return x > t ? x : t; };
  v = step(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xb1, 0xf, 0xf, false)));
  v = step(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4e, 0xf, 0xf, false)));
  v = step(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xf, 0xf, false)));
  if constexpr (LANES == 8) return uint32_t(__builtin_amdgcn_readlane(int(v), 0));
  v = step(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x140, 0xf, 0xf, false)));
  if constexpr (LANES == 16) return uint32_t(__builtin_amdgcn_readlane(int(v), 0));
  v = step(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false)));
  v = step(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false)));
  return uint32_t(__builtin_amdgcn_readlane(int(v), 63));
}

// The largest 64-bit argmax key over lanes and its lane (the lowest lane
// holding it; lane 0 when every key is 0). The value word (high half) is
// reduced alone; the index word only settles exact value ties, which are
// rare (keys are unique per pixel, and a high word of 0 means a 0 key).
template <int LANES>
__device__ __forceinline__ uint64_t KeyMax(uint64_t key, int& lane_out) {
  const uint32_t hi = uint32_t(key >> 32);
  const uint32_t mh = MaxU32<LANES>(hi);
  if (mh == 0u) {
    lane_out = 0;
    return 0ull;
  }
  const uint64_t tie = __ballot(hi == mh);
  if ((tie & (tie - 1ull)) == 0ull) {
    lane_out = __builtin_ctzll(tie);
    return (uint64_t(mh) << 32) |
           uint32_t(__builtin_amdgcn_readlane(int(uint32_t(key)), lane_out));
  }
  const uint64_t k = hi == mh ? key : 0ull;
  const uint64_t m = LANES == 8 ? Max8U64(k) : LANES == 16 ? Max16U64(k) : Max64U64(k);
  lane_out = FirstLane(key == m);
  return m;
}

template <int NI>
struct RegSlot {
  uint64_t key;
  uint32_t pos;
  float r[NI];
};

__device__ __forceinline__ void StoreGranule(uint64_t* g, uint32_t epoch,
                                             uint32_t v) {
  __hip_atomic_store(g, (uint64_t(epoch) << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t LoadGranule(uint64_t* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// IntegratePixel over NI register-resident values, with every per-image
// decision (weight zero, polarization joined, i % n_pol) made once per
// launch: the same floating-point operations in the same order as
// IntegratePixel (rdl_internal.h), without its per-pixel index arithmetic
// and runtime-indexed weight reads.
template <int NI>
struct RegIntegration {
  uint32_t mode = 0, copy = 0, n_img = 0, n_ch = 0, np = 1;
  uint32_t incl = 0;     // LINEAR / SQUARED_JOINS: image k enters the sum
  uint32_t ch_live = 0;  // SQUARE, > 1 channel: channel ch has weight != 0
  uint32_t pol_mask = 0;
  float w[NI];           // weight of image k (SQUARE > 1 ch: of channel k)
  float factor = 1.0f;

  __device__ void Init(const rdl_integration& g) {
    mode = g.mode;
    copy = g.copy_fast_path;
    n_img = g.n_images;
    n_ch = g.n_channels;
    np = g.n_pol;
    pol_mask = g.pol_mask;
    factor = g.factor;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      w[k] = 0.0f;
      if (uint32_t(k) < n_img && mode != RDL_INTEGRATE_SQUARE) {
        w[k] = g.weights[k];
        if (w[k] != 0.0f && ((pol_mask >> (uint32_t(k) % np)) & 1u)) incl |= 1u << k;
      }
      if (mode == RDL_INTEGRATE_SQUARE && uint32_t(k) < n_ch && uint32_t(k) * np < n_img) {
        w[k] = g.weights[uint32_t(k) * np];
        if (w[k] != 0.0f) ch_live |= 1u << k;
      }
    }
  }

  __device__ float operator()(const float (&v)[NI]) const {
    if (copy) return v[0];
    if (mode == RDL_INTEGRATE_LINEAR) {
      float acc = 0.0f;
      bool first = true;
#pragma unroll
      for (int k = 0; k < NI; ++k)
        if ((incl >> k) & 1u) {
          acc = first ? v[k] * w[k] : __builtin_fmaf(v[k], w[k], acc);
          first = false;
        }
      return first ? 0.0f : acc * factor;
    }
    if (mode == RDL_INTEGRATE_SQUARE) {
      if (n_ch == 1) {
        float acc = 0.0f;
        bool first = true;
#pragma unroll
        for (int p = 0; p < NI; ++p)
          if (uint32_t(p) < np && ((pol_mask >> p) & 1u)) {
            acc = first ? v[p] * v[p] : __builtin_fmaf(v[p], v[p], acc);
            first = false;
          }
        return __builtin_sqrtf(acc) * factor;
      }
      float dest = 0.0f;
#pragma unroll
      for (int ch = 0; ch < NI; ++ch) {
        if (uint32_t(ch) >= n_ch) continue;
        float scratch = 0.0f;
        if ((ch_live >> ch) & 1u) {
          if (np == 1) {
            scratch = v[ch];
          } else {
            float acc = 0.0f;
            bool first = true;
#pragma unroll
            for (int q = 0; q < NI; ++q) {
              const uint32_t p = uint32_t(q) - uint32_t(ch) * np;  // image q = ch np + p
              if (uint32_t(q) >= uint32_t(ch) * np && p < np && ((pol_mask >> p) & 1u)) {
                acc = first ? v[q] * v[q] : __builtin_fmaf(v[q], v[q], acc);
                first = false;
              }
            }
            scratch = first ? 0.0f : __builtin_sqrtf(acc);
          }
        }
        dest = ch == 0 ? scratch * w[ch] : __builtin_fmaf(scratch, w[ch], dest);
      }
      return dest * factor;
    }
    float acc = 0.0f;  // RDL_INTEGRATE_SQUARED_JOINS
    bool first = true;
#pragma unroll
    for (int k = 0; k < NI; ++k)
      if ((incl >> k) & 1u) {
        acc = first ? v[k] * v[k] * w[k] : __builtin_fmaf(v[k] * v[k], w[k], acc);
        first = false;
      }
    return first ? 0.0f : __builtin_sqrtf(acc) * factor;
  }
};

// FAST: one image whose integration is the identity (ImageSet copy fast path,
// cpp/image_set.cc:425-430): the integrated value is the residual itself.
// THREADS = 512 (eight waves, one LDS barrier per iteration) or 64: the
// single-wave form for small selections, where the winner goes from the
// wave argmax straight to every lane by readlane (no LDS slot, no barrier).
template <int NI, int ITEMS, bool FAST, int THREADS = kRegThreads>
__global__ __launch_bounds__(THREADS) void SubminorLoopReg(LoopArgs a) {
  constexpr int REC = 3 + NI;  // granules per record: key hi, key lo, pos, r[NI]
  constexpr int WAVES = THREADS / 64;
  __shared__ RegSlot<NI> slots[2][WAVES];
  __shared__ RegSlot<NI> gwin;
  __shared__ uint32_t gflag;

  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t base = uint64_t(blockIdx.x) * a.per_block;
  const uint32_t cnt =
      base >= a.n_sel ? 0u : uint32_t(min<uint64_t>(a.per_block, a.n_sel - base));
  const int n_img = int(a.n_img);
  const int n_pol = int(a.n_pol);
  RegIntegration<NI> ri;
  if constexpr (!FAST) ri.Init(a.integ);

  uint32_t pos[ITEMS];
  float R[ITEMS][NI];
  float M[ITEMS][NI];
  float F[ITEMS];  // RMS factor of each pixel (1 without one)
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t j = tid + uint32_t(i) * THREADS;
    const bool valid = j < cnt;
    pos[i] = valid ? a.pos[base + j] : 0u;
    F[i] = (valid && a.rms)
               ? a.rms[size_t(pos[i] >> 16) * a.width + (pos[i] & 0xffffu)]
               : 1.0f;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      R[i][k] = (valid && k < n_img) ? a.r[size_t(k) * a.n_sel + base + j] : 0.0f;
      M[i][k] = 0.0f;
    }
  }

  const int W = int(a.width), H = int(a.height);
  const size_t plane = size_t(a.width) * a.height;
  float c[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) c[k] = 0.0f;
  uint32_t cp = 0;  // the component's selection index (its table row)
  int cx = 0, cy = 0;
  bool have_component = false;
  float start_abs = 0.0f;
  bool diverging = false;
  float flux = 0.0f;
  uint64_t iteration = a.iteration_start;
  float m = 0.0f;
  uint32_t epoch = 0;
  uint64_t* gran = reinterpret_cast<uint64_t*>(a.records);

  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
  const bool prof = a.prof && blockIdx.x == 0 && wave == 0;
  uint64_t t_prev = prof ? __builtin_amdgcn_s_memtime() : 0;
#define RDL_PHASE(i)                                       \
  if (prof) {                                              \
    const uint64_t t_now = __builtin_amdgcn_s_memtime();   \
    ph[i] += t_now - t_prev;                               \
    t_prev = t_now;                                        \
  }
  while (true) {
    // ---- subtract the current component: all gathers first, then FMAs
    if (have_component) {
      float pv[ITEMS][NI];
      bool in[ITEMS];
      if (a.table) {
        // the component's row of the pairwise table: contiguous over j
        const size_t sq = size_t(a.n_sel) * a.n_sel;
        const float* row = a.table + size_t(cp) * a.n_sel + base;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const uint32_t j = tid + uint32_t(i) * THREADS;
          const bool valid = j < cnt;
#pragma unroll
          for (int k = 0; k < NI; ++k)
            pv[i][k] = (valid && k < n_img) ? row[size_t(k / n_pol) * sq + j] : 0.0f;
          in[i] = valid && __float_as_uint(pv[i][0]) != kOutsideBits;
        }
      } else {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = tid + uint32_t(i) * THREADS;
        const int px = int(pos[i] & 0xffffu), py = int(pos[i] >> 16);
        const int dx = px - cx + W / 2, dy = py - cy + H / 2;
        in[i] = j < cnt && dx >= 0 && dx < W && dy >= 0 && dy < H;
        const size_t off = in[i] ? size_t(dy) * a.width + size_t(dx) : 0;
#pragma unroll
        for (int k = 0; k < NI; ++k)
          pv[i][k] = k < n_img ? a.psfs[size_t(k / n_pol) * plane + off] : 0.0f;
      }
      }
#pragma unroll
      for (int i = 0; i < ITEMS; ++i)
#pragma unroll
        for (int k = 0; k < NI; ++k)
          if (in[i] && k < n_img) R[i][k] = __builtin_fmaf(-pv[i][k], c[k], R[i][k]);
    }
    RDL_PHASE(0)
    // ---- integrate + per-thread argmax
    uint64_t best = 0;
    int best_i = 0;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t j = tid + uint32_t(i) * THREADS;
      if (j < cnt) {
        float integ = FAST ? R[i][0] : ri(R[i]);
        if (a.rms) integ *= F[i];  // scratch *= rms (subminor_loop.cc:16-18)
        uint64_t key = MaxKey(integ, a.allow_negative, base + j);
        if (base + j == 0 && integ != integ) key = ~0ull;  // scratch[0] is NaN
        if (key > best) {
          best = key;
          best_i = i;
        }
      }
    }
    // ---- wave argmax; the owner (or lane 0 when nothing qualifies, which
    // stands for selection index 0) writes the wave's slot
    RDL_PHASE(1)
    int owner_lane;
    const uint64_t wmax = KeyMax<64>(best, owner_lane);
    const uint32_t par = epoch & 1u;
    uint64_t gkey;
    uint32_t wpos;
    float wr[NI];
    if constexpr (WAVES == 1) {
      // every lane stages its own candidate; the owner's comes by readlane
      uint32_t pp = pos[0];
      float rr[NI];
#pragma unroll
      for (int k = 0; k < NI; ++k) rr[k] = R[0][k];
#pragma unroll
      for (int i = 1; i < ITEMS; ++i)
        if (i == best_i && wmax != 0) {
          pp = pos[i];
#pragma unroll
          for (int k = 0; k < NI; ++k) rr[k] = R[i][k];
        }
      gkey = wmax;
      wpos = uint32_t(__builtin_amdgcn_readlane(int(pp), owner_lane));
#pragma unroll
      for (int k = 0; k < NI; ++k)
        wr[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rr[k]), owner_lane));
      ++epoch;
      RDL_PHASE(2)
      RDL_PHASE(3)
    } else {
    if (int(lane) == owner_lane) {
      RegSlot<NI>& sl = slots[par][wave];
      sl.key = wmax;
      uint32_t pp = pos[0];
      float rr[NI];
#pragma unroll
      for (int k = 0; k < NI; ++k) rr[k] = R[0][k];
#pragma unroll
      for (int i = 1; i < ITEMS; ++i)
        if (i == best_i && wmax != 0) {
          pp = pos[i];
#pragma unroll
          for (int k = 0; k < NI; ++k) rr[k] = R[i][k];
        }
      sl.pos = pp;
#pragma unroll
      for (int k = 0; k < NI; ++k) sl.r[k] = rr[k];
    }
    RDL_PHASE(2)
    LdsBarrier();
    RDL_PHASE(3)
    // ---- block winner: every wave reduces the slots (ties -> lowest wave,
    // which only matters for the all-zero case)
    // lanes 0..7 read a whole slot each (one LDS round trip); the winner's
    // payload then comes from its lane by readlane
    uint64_t sk = 0ull;
    uint32_t spos = 0;
    float sr[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) sr[k] = 0.0f;
    if (lane < uint32_t(WAVES)) {
      const RegSlot<NI>& sl = slots[par][lane];
      sk = sl.key;
      spos = sl.pos;
#pragma unroll
      for (int k = 0; k < NI; ++k) sr[k] = sl.r[k];
    }
    int bw;
    const uint64_t bkey = KeyMax<(WAVES <= 8 ? 8 : 16)>(sk, bw);
    gkey = bkey;
    wpos = uint32_t(__builtin_amdgcn_readlane(int(spos), bw));
#pragma unroll
    for (int k = 0; k < NI; ++k)
      wr[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sr[k]), bw));

    if (a.n_blocks > 1) {
      ++epoch;  // 1, 2, ... (never 0: granules are zeroed per launch)
      uint64_t* mine = gran + (size_t(par) * a.n_blocks + blockIdx.x) * REC;
      // wave 1 publishes (its stores drain off wave 0's vmcnt) while wave 0
      // sweeps
      if (wave == 1 && lane < uint32_t(REC)) {
        uint32_t v;
        if (lane == 0) v = uint32_t(gkey >> 32);
        else if (lane == 1) v = uint32_t(gkey);
        else if (lane == 2) v = wpos;
        else {
          v = __float_as_uint(wr[0]);
#pragma unroll
          for (int k = 1; k < NI; ++k)
            if (int(lane) - 3 == k) v = __float_as_uint(wr[k]);
        }
        StoreGranule(mine + lane, epoch, v);
      }
      if (wave == 0) {
        // sweep: lane b handles blocks b, b+64, ...; all tags must match
        const uint32_t nb = a.n_blocks;
        uint64_t lk = 0;
        uint32_t lb = 0xffffffffu;
        uint32_t lrec[REC] = {};
        uint64_t spins = 0;
        bool failed = false;
        while (true) {
          bool ok = true;
          lk = 0;
          lb = 0xffffffffu;
          for (uint32_t b = lane; b < nb; b += 64) {
            uint64_t* rec = gran + (size_t(par) * nb + b) * REC;
            uint32_t v[REC];
#pragma unroll
            for (int w = 0; w < REC; ++w) {
              const uint64_t x = LoadGranule(rec + w);
              ok &= uint32_t(x >> 32) == epoch;
              v[w] = uint32_t(x);
            }
            const uint64_t key = (uint64_t(v[0]) << 32) | v[1];
            if (lb == 0xffffffffu || key > lk) {
              lk = key;
              lb = b;
#pragma unroll
              for (int w = 0; w < REC; ++w) lrec[w] = v[w];
            }
          }
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (uint64_t(1) << 26)) {
            failed = true;
            break;
          }
        }
        // wave argmax over (key, block): keys are unique unless 0, and 0
        // means block 0 (lane 0 holds it first)
        const uint64_t kmax = Max64U64(lk);
        const int src = kmax != 0 ? FirstLane(lk == kmax) : 0;
        uint32_t rec[REC];
#pragma unroll
        for (int w = 0; w < REC; ++w)
          rec[w] = uint32_t(__builtin_amdgcn_readlane(int(lrec[w]), src));
        if (lane == 0) {
          gwin.key = (uint64_t(rec[0]) << 32) | rec[1];
          gwin.pos = rec[2];
#pragma unroll
          for (int kk = 0; kk < NI; ++kk) gwin.r[kk] = __uint_as_float(rec[3 + kk]);
          gflag = failed ? 1u : 0u;
        }
      }
      LdsBarrier();
      if (gflag) {
        if (tid == 0) StoreSc1(&a.result[8], 1u);
        return;
      }
      gkey = gwin.key;
      wpos = gwin.pos;
#pragma unroll
      for (int k = 0; k < NI; ++k) wr[k] = gwin.r[k];
    } else {
      ++epoch;
    }
    }  // WAVES > 1

    RDL_PHASE(4)
    // ---- identical decisions everywhere (subminor_loop.cc:56-89)
    const uint64_t winner_p = (gkey == 0 || gkey == ~0ull)
                                  ? 0ull
                                  : uint64_t(0xffffffffu - uint32_t(gkey));
    m = FAST ? wr[0] : ri(wr);
    if (a.rms) {
      // the winner's integrated x factor is the value its key was made from
      // (with its sign from the integrated value, the factor being >= 0)
      const float kv = KeyValue(gkey);
      m = (gkey == 0 || gkey == ~0ull) ? __int_as_float(0x7fc00000)
          : a.allow_negative            ? copysignf(kv, m)
                                        : kv;
    }
    if (!have_component) {
      start_abs = fabsf(m);
    } else {
      if (a.divergence_limit != 0.0f)
        diverging = fabsf(m) > start_abs * a.divergence_limit;
      ++iteration;
    }
    const bool go = fabsf(m) > a.threshold && iteration < a.max_iterations &&
                    (!a.stop_on_negative || m >= 0.0f) && !diverging;
    if (!go) break;
    if (a.spectral) {
      // PerformSpectralFit of the gain-scaled values (subminor_loop.cc:66-76)
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < NI; ++q)
          if (k < n_img && q < n_img)
            acc = __builtin_fmaf(a.spectral[k * n_img + q], wr[q] * a.gain, acc);
        c[k] = acc;
      }
    } else {
#pragma unroll
      for (int k = 0; k < NI; ++k) c[k] = k < n_img ? wr[k] * a.gain : 0.0f;
    }
    flux += m * a.gain;
    cx = int(wpos & 0xffffu);
    cy = int(wpos >> 16);
    cp = uint32_t(winner_p);
    if (winner_p >= base && winner_p < base + cnt) {
      const uint32_t j = uint32_t(winner_p - base);
      if (j % THREADS == tid) {
        const int wi = int(j / THREADS);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
          if (i == wi)
#pragma unroll
            for (int k = 0; k < NI; ++k) M[i][k] += c[k];
      }
    }
    if (blockIdx.x == 0 && tid == 0 && a.trace) {
      const uint64_t t = iteration - a.iteration_start;
      if (t < a.trace_cap) {
        a.trace[2 * t] = uint32_t(cx);
        a.trace[2 * t + 1] = uint32_t(cy);
      }
    }
    have_component = true;
    RDL_PHASE(5)
  }
#undef RDL_PHASE
  if (prof && lane == 0) {
    uint64_t* out = reinterpret_cast<uint64_t*>(a.result + 16);
    for (int i = 0; i < 6; ++i) out[i] = ph[i];
  }

#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t j = tid + uint32_t(i) * THREADS;
    if (j < cnt)
#pragma unroll
      for (int k = 0; k < NI; ++k)
        if (k < n_img) a.m[size_t(k) * a.n_sel + base + j] = M[i][k];
  }
  if (blockIdx.x == 0 && tid == 0) {
    LoopResult* r = reinterpret_cast<LoopResult*>(a.result);
    r->iteration = iteration;
    r->peak = m;
    r->diverging = diverging ? 1 : 0;
    r->flux = flux;
  }
}

// ------------------------------------------------- pairwise-table loop
// SubminorLoopTab: SubminorLoopReg<1, ITEMS, true, THREADS> specialised for
// the multiscale hot path's common shape — one image whose integration is the
// identity, the pairwise PSF table, no RMS factor, spectral map or
// log-polynomial fit — with the per-iteration dependency chain cut to: the
// table row's loads, FMAs and 32-bit value keys, a DPP wave max whose owner
// is found by one ballot per item (the lowest selection index among equal
// values, as the 64-bit keys order them), one 16-byte LDS slot per wave and
// one LDS barrier, an 8/16-lane DPP max of the slots, scalar decisions.
//
// G > 1 participants split the selection; their block winners are exchanged
// through epoch-tagged 8-byte granules {epoch, word} every wave polls. The
// grid is launched as 8 G blocks of which blocks 0, 8, 16, ... participate
// (one XCD under the dispatcher's round-robin dealing; speed only): the
// participants first exchange their HW_REG_XCC_ID through the placement-
// independent protocol (sc1 stores and sc1 loads) and, only when all of them
// are on one XCD, exchange through that XCD's L2 (plain stores, which keep
// the line in L2, polled by sc1 loads, which bypass only L1); otherwise every
// granule goes through sc1 stores as well. RDL_TRACE_SUBMINOR=1 measured the
// sc1 exchange at ~4 700 of ~7 800 cycles per iteration.
//
// Same operations in the same order, same argmax order and tie rules as the
// generic kernels: traces and model values are identical.
constexpr uint32_t kTabParticipantStride = 8;  // blocks per participant (LoopArgs::part_stride)

// The "fast" exchange below publishes records with workgroup-scope stores
// that the other participants poll with agent-scope (L1-bypassing) loads:
// visible to them only because gfx950's vector L1 is write-through, so every
// store reaches the XCD's L2 the participants share (checked at run time:
// all participants on one XCC). A target whose L1 could hold such stores
// needs the agent-scope form, which RDL_SUBMINOR_EXCHANGE=agent selects (and
// tests/test_gpu_kernels.py compares with the fast one).
// Other targets always take the agent-scope form (kFastExchange false).
#if defined(__gfx950__) || !defined(__HIP_DEVICE_COMPILE__)
constexpr bool kFastExchange = true;
#else
constexpr bool kFastExchange = false;
#endif

__device__ __forceinline__ uint32_t XccId() {
  // HW_REG_XCC_ID (hwreg 20), bits [3:0]
  return uint32_t(__builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)));
}

template <int ITEMS, int THREADS, bool NEG>
__global__ __launch_bounds__(THREADS) void SubminorLoopTab(LoopArgs a) {
  constexpr int WAVES = THREADS / 64;
  constexpr int SLANES = WAVES <= 8 ? 8 : 16;
  // {key hi, key lo, value bits, -}, parity double-buffered
  __shared__ uint4 slots[2][WAVES];
  // the atomic form (G == 1): per iteration one 64-bit key cell and the
  // bits of selection index 0's value, triple-buffered (a cell is cleared
  // two iterations before its next use, after a barrier every reader of
  // its last use has passed)
  __shared__ unsigned long long cells[3];
  __shared__ uint32_t first_bits[3];
  const uint32_t G = a.n_blocks;
  if (G > 1 && blockIdx.x % a.part_stride != 0u) return;
  const uint32_t rank = G > 1 ? blockIdx.x / a.part_stride : 0u;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t n = uint32_t(a.n_sel), per = a.per_block;
  const uint32_t base = rank * per;
  const uint32_t cnt = base >= n ? 0u : min(per, n - base);
  const bool neg = a.allow_negative != 0;
  // exchange granules (zeroed per launch): [G] XCC ids, then [2][G][3] records
  uint64_t* gran = reinterpret_cast<uint64_t*>(a.records);
  uint64_t* recs = gran + G;
  float R[ITEMS], M[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t j = tid + uint32_t(i) * THREADS;
    // beyond the slice: NaN (key 0, never a winner; see the padded table)
    R[i] = j < cnt ? a.r[base + j] : __int_as_float(0x7fc00000);
    M[i] = 0.0f;
  }
  bool fast = true;  // G > 1: exchange through the one L2 of the participants
  bool failed = false;
  if (G > 1) {
    if (tid == 0)
      __hip_atomic_store(gran + rank, (uint64_t(1) << 32) | XccId(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t xcc = 0u;
    bool ok = false;
    for (uint64_t spins = 0; !failed; ++spins) {
      uint64_t v = 0;
      if (lane < G)
        v = __hip_atomic_load(gran + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = lane >= G || (v >> 32) == 1u;
      if (__all(ok)) {
        xcc = uint32_t(v);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      failed = spins > (uint64_t(1) << 24);
    }
    const uint32_t x0 = uint32_t(__builtin_amdgcn_readlane(int(xcc), 0));
    fast = kFastExchange && __all(lane >= G || xcc == x0) && !a.agent_exchange;
  }
  const float* table = a.table;
  float c = 0.0f, m = 0.0f, start_abs = 0.0f, flux = 0.0f;
  uint32_t cp = 0, par = 0, epoch = 0;
  uint32_t row_cp = 0xffffffffu;  // the component whose row pv holds
  float pv[ITEMS];
  uint32_t pend_pos = 0;
  bool pend = false;  // a trace entry waiting for its position's load
  bool have = false, diverging = false;
  uint64_t iteration = a.iteration_start;
  const bool tracer = rank == 0 && tid == 0 && a.trace;
  const bool atomic = G == 1 && a.atomic_reduce != 0;
  uint32_t cell = 0;  // iteration % 3
  if (atomic) {
    if (tid < 3u) cells[tid] = 0ull;
    LdsBarrier();
  }
  // the loop's comparisons as integer tests on float bits (see decisions)
  const uint32_t thr_bits = __float_as_uint(a.threshold) & 0x7fffffffu;
  const uint32_t thr_mode = a.threshold != a.threshold        ? 0u
                            : (__float_as_uint(a.threshold) >> 31) && thr_bits ? 1u
                                                                                : 2u;
  uint32_t lim_mode = 0u, lim_bits = 0u;
  const bool stop_neg = a.stop_on_negative != 0;
  uint64_t remaining =
      a.max_iterations > a.iteration_start ? a.max_iterations - a.iteration_start : 0u;
  // RDL_TRACE_SUBMINOR=1: per-phase cycles of participant 0, wave 0
  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
  const bool prof = a.prof && rank == 0 && wave == 0;
  uint64_t t_prev = prof ? __builtin_amdgcn_s_memtime() : 0;
#define RDL_TPHASE(i)                                      \
  if (prof) {                                              \
    const uint64_t t_now = __builtin_amdgcn_s_memtime();   \
    ph[i] += t_now - t_prev;                               \
    t_prev = t_now;                                        \
  }
  while (!failed) {
    if (have) {
      // the component's row of the pairwise table (contiguous over j), issued
      // before the previous iteration's decisions (a repeated component
      // reuses the row already in registers); the FMAs (subminor_loop.cc:
      // 93-108)
#pragma unroll
      for (int i = 0; i < ITEMS; ++i)
        if (__float_as_uint(pv[i]) != kOutsideBits) R[i] = __builtin_fmaf(-pv[i], c, R[i]);
      if (pend) {  // the previous component's position has arrived with the row
        const uint64_t t = iteration - a.iteration_start;
        if (t < a.trace_cap) {
          a.trace[2 * t] = pend_pos & 0xffffu;
          a.trace[2 * t + 1] = pend_pos >> 16;
        }
        pend = false;
      }
    }
    RDL_TPHASE(0)
    // ---- this thread's best: the largest key, then the lowest index
    // (MaxKey's high word; NaN 0, index 0's NaN ~0); compares and selects
    // only, no branch per item
    uint32_t bh = 0u, bj = 0xffffffffu, bv = __float_as_uint(R[0]);
    if constexpr (NEG) {
      // |R| keys: the largest |R| by a float max chain (the max skips NaN,
      // whose key is 0), then the lowest item holding it
      float tb = -1.0f;
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) tb = __builtin_fmaxf(tb, __builtin_fabsf(R[i]));
      bh = tb >= 0.0f ? (__float_as_uint(tb) | 0x80000000u) : 0u;
#pragma unroll
      for (int i = ITEMS - 1; i >= 0; --i) {
        const bool eq = __builtin_fabsf(R[i]) == tb;
        bj = eq ? base + tid + uint32_t(i) * THREADS : bj;
        bv = eq ? __float_as_uint(R[i]) : bv;
      }
      if (base == 0u && tid == 0u && cnt > 0u && R[0] != R[0]) {
        bh = 0xffffffffu;  // selection index 0 holding NaN outranks every key
        bj = 0u;
      }
    } else {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const float v = neg ? fabsf(R[i]) : R[i];
        const uint32_t u = __float_as_uint(v);
        uint32_t h = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        const uint32_t j = base + tid + uint32_t(i) * THREADS;
        if (v != v) h = (j == 0u && cnt > 0u) ? 0xffffffffu : 0u;
        const bool better = h > bh;  // items ascend in j: equal keys keep the first
        bh = better ? h : bh;
        bj = better ? j : bj;
        bv = better ? __float_as_uint(R[i]) : bv;
      }
    }
    RDL_TPHASE(1)
    uint32_t gh, gl, gv;
    if (atomic) {
      // ---- block winner: the 64-bit key (value word, then the lowest
      // selection index, then the value's sign bit to rebuild it) as one LDS
      // atomic max per 16-lane row after a DPP max within the row; the same
      // total order as the two-level (hi, ~j) reduction below. A key-0 lane
      // (every item NaN / beyond the slice) holds 0; selection index 0's
      // value bits stand for the all-zero (and the NaN-at-0) outcome.
      uint64_t key = 0ull;
      if (bh != 0u)
        key = (uint64_t(bh) << 32) | (uint64_t((0x7fffffffu - bj) << 1) | (bv >> 31));
      uint64_t t;
      t = DppU64<0xb1>(key);
      key = t > key ? t : key;
      t = DppU64<0x4e>(key);
      key = t > key ? t : key;
      t = DppU64<0x141>(key);
      key = t > key ? t : key;
      t = DppU64<0x140>(key);
      key = t > key ? t : key;
      if ((lane & 15u) == 0u && key != 0ull) atomicMax(&cells[cell], (unsigned long long)key);
      if (tid == 0) first_bits[cell] = __float_as_uint(R[0]);
      RDL_TPHASE(2)
      LdsBarrier();
      RDL_TPHASE(3)
      const uint64_t k = cells[cell];
      const uint32_t fb = first_bits[cell];
      if (tid == 0) cells[cell == 0u ? 2u : cell - 1u] = 0ull;  // used two iterations on
      cell = cell == 2u ? 0u : cell + 1u;
      gh = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(k >> 32))));
      const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(k))));
      const uint32_t fbs = uint32_t(__builtin_amdgcn_readfirstlane(int(fb)));
      const uint32_t j = 0x7fffffffu - (lo >> 1);
      gl = gh == 0u ? 0u : ~j;
      if (gh == 0u || gh == 0xffffffffu) {
        gv = fbs;  // selection index 0's value (all keys 0, or NaN at index 0)
      } else if (NEG || neg) {
        gv = (gh & 0x7fffffffu) | (lo << 31);  // |R| bits, R's sign
      } else {
        gv = (gh & 0x80000000u) ? (gh & 0x7fffffffu) : ~gh;  // the key transform inverted
      }
    } else {
    // ---- wave winner: DPP max of the keys; the lowest index on exact ties
    const uint32_t mh = MaxU32<64>(bh);
    const uint64_t tie = __ballot(bh == mh);
    int owner;
    if ((tie & (tie - 1ull)) == 0ull) {
      owner = __builtin_ctzll(tie);
    } else {  // several lanes: the largest ~j among them (0: a key-0 wave)
      const uint32_t ml = MaxU32<64>(bh == mh ? ~bj : 0u);
      owner = FirstLane(bh == mh && ~bj == ml);
    }
    // a key-0 wave stands for its first pixel (lane 0's item 0, as
    // SubminorLoopReg), whose value is lane 0's initial bv
    const uint32_t wl = mh == 0u ? 0u : ~uint32_t(__builtin_amdgcn_readlane(int(bj), owner));
    const uint32_t wv = uint32_t(__builtin_amdgcn_readlane(int(bv), mh == 0u ? 0 : owner));
    if (lane == 0) slots[par][wave] = make_uint4(mh, wl, wv, 0u);
    RDL_TPHASE(2)
    LdsBarrier();
    RDL_TPHASE(3)
    // ---- block winner over the wave slots
    const uint4 s4 = lane < uint32_t(WAVES) ? slots[par][lane] : make_uint4(0u, 0u, 0u, 0u);
    par ^= 1u;
    gh = MaxU32<SLANES>(s4.x);
    {
      const bool mine = lane < uint32_t(WAVES) && s4.x == gh;
      const uint64_t t2 = __ballot(mine);
      int win;
      if ((t2 & (t2 - 1ull)) == 0ull) {
        win = __builtin_ctzll(t2);
      } else {
        const uint32_t l2 = MaxU32<SLANES>(mine ? s4.y : 0u);
        win = FirstLane(mine && s4.y == l2);
      }
      owner = win;
    }
    gl = uint32_t(__builtin_amdgcn_readlane(int(s4.y), owner));
    gv = uint32_t(__builtin_amdgcn_readlane(int(s4.z), owner));
    if (G > 1) {
      // ---- exchange of the participants' winners
      ++epoch;  // 1, 2, ... (granules are zeroed per launch)
      uint64_t* mine_rec = recs + (size_t(epoch & 1u) * G + rank) * 3;
      if (wave == 0 && lane < 3u) {
        const uint32_t w = lane == 0 ? gh : lane == 1 ? gl : gv;
        const uint64_t g = (uint64_t(epoch) << 32) | w;
        if (fast)
          __hip_atomic_store(mine_rec + lane, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
          __hip_atomic_store(mine_rec + lane, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      uint32_t xh = 0u, xl = 0u, xv = 0u;
      for (uint64_t spins = 0;; ++spins) {
        bool ok = true;
        if (lane < G) {
          const uint64_t* rr = recs + (size_t(epoch & 1u) * G + lane) * 3;
          const uint64_t g0 = __hip_atomic_load(rr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint64_t g1 =
              __hip_atomic_load(rr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint64_t g2 =
              __hip_atomic_load(rr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = uint32_t(g0 >> 32) == epoch && uint32_t(g1 >> 32) == epoch &&
               uint32_t(g2 >> 32) == epoch;
          xh = uint32_t(g0);
          xl = uint32_t(g1);
          xv = uint32_t(g2);
        }
        if (__all(ok)) break;
        if (spins > (uint64_t(1) << 26)) {
          failed = true;
          break;
        }
      }
      if (failed) break;
      // lexicographic (hi, lo) max over the participants (lanes < G)
      gh = MaxU32<64>(lane < G ? xh : 0u);
      const bool mine = lane < G && xh == gh;
      const uint64_t t2 = __ballot(mine);
      int win;
      if ((t2 & (t2 - 1ull)) == 0ull) {
        win = __builtin_ctzll(t2);
      } else {
        const uint32_t l2 = MaxU32<64>(mine ? xl : 0u);
        win = FirstLane(mine && xl == l2);
      }
      gl = uint32_t(__builtin_amdgcn_readlane(int(xl), win));
      gv = uint32_t(__builtin_amdgcn_readlane(int(xv), win));
    }
    }  // the wave-slot reduction
    RDL_TPHASE(4)
    // ---- identical decisions everywhere (subminor_loop.cc:56-89), on the
    // bit patterns in scalar registers (exact: |x| > t for t >= 0 is the
    // integer order of the bits; NaN never passes a comparison)
    const bool none = gh == 0u || (gh == 0xffffffffu && gl == 0xffffffffu);
    const uint32_t wp = none ? 0u : 0xffffffffu - gl;
    // the winner's table row: in flight while the decisions run (a row the
    // loop then does not use is only read; wp < n_sel always)
    if (wp != row_cp) {
      const float* row = table + size_t(wp) * n + base;
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) pv[i] = row[tid + uint32_t(i) * THREADS];
      row_cp = wp;
    }
    m = __uint_as_float(gv);
    const uint32_t ab = gv & 0x7fffffffu;
    const bool is_nan = ab > 0x7f800000u;
    if (!have) {
      start_abs = __uint_as_float(ab);
      if (a.divergence_limit != 0.0f) {
        const float lim = start_abs * a.divergence_limit;
        lim_bits = __float_as_uint(lim) & 0x7fffffffu;
        lim_mode = lim != lim ? 0u : ((__float_as_uint(lim) >> 31) && lim_bits) ? 1u : 2u;
      }
    } else {
      // fabsf(m) > start_abs * divergence_limit
      diverging = lim_mode == 1u ? !is_nan : lim_mode == 2u ? (!is_nan && ab > lim_bits) : false;
      ++iteration;
      --remaining;
    }
    const bool above = thr_mode == 1u ? !is_nan : thr_mode == 2u ? (!is_nan && ab > thr_bits)
                                                               : false;
    // !stop_on_negative || m >= 0 (-0 included, NaN excluded)
    const bool non_negative = !is_nan && ((gv >> 31) == 0u || gv == 0x80000000u);
    const bool go = above && remaining != 0u && (!stop_neg || non_negative) && !diverging;
    if (!go) break;
    c = m * a.gain;
    flux += c;  // flux += m * gain (the same product)
    cp = wp;
    // the owner lane adds the component (scalar branches to its wave and item)
    {
      const uint32_t off = wp - base;
      if (off < cnt && (off % uint32_t(THREADS)) / 64u == wave) {
        const uint32_t wi = off / uint32_t(THREADS);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
          if (uint32_t(i) == wi && lane == (off & 63u)) M[i] += c;
      }
    }
    if (tracer) {  // the load lands with the next row's (one wait for both)
      pend_pos = a.pos[wp];
      pend = true;
    }
    have = true;
    RDL_TPHASE(5)
  }
#undef RDL_TPHASE
  if (prof && lane == 0) {
    uint64_t* out = reinterpret_cast<uint64_t*>(a.result + 16);
    for (int i = 0; i < 6; ++i) out[i] = ph[i];
  }
  if (pend) {
    const uint64_t t = iteration - a.iteration_start;
    if (t < a.trace_cap) {
      a.trace[2 * t] = pend_pos & 0xffffu;
      a.trace[2 * t + 1] = pend_pos >> 16;
    }
  }
  if (failed) {
    if (tid == 0) StoreSc1(&a.result[8], 1u);
    return;
  }
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t j = tid + uint32_t(i) * THREADS;
    if (j < cnt) a.m[base + j] = M[i];
  }
  if (rank == 0 && tid == 0) {
    LoopResult* r = reinterpret_cast<LoopResult*>(a.result);
    r->iteration = iteration;
    r->peak = m;
    r->diverging = diverging ? 1 : 0;
    r->flux = flux;
  }
}

// RegIntegration's RDL_INTEGRATE_LINEAR branch alone (SubminorLoopTabN's
// integrations): the same operations in the same order
template <int NI>
struct LinearIntegration {
  uint32_t incl = 0;
  float w[NI];
  float factor = 1.0f;
  __device__ void Init(const rdl_integration& g) {
    factor = g.factor;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      w[k] = uint32_t(k) < g.n_images ? g.weights[k] : 0.0f;
      if (uint32_t(k) < g.n_images && w[k] != 0.0f && ((g.pol_mask >> (uint32_t(k) % g.n_pol)) & 1u))
        incl |= 1u << k;
    }
  }
  __device__ float operator()(const float (&v)[NI]) const {
    float acc = 0.0f;
    bool first = true;
#pragma unroll
    for (int k = 0; k < NI; ++k)
      if ((incl >> k) & 1u) {
        acc = first ? v[k] * w[k] : __builtin_fmaf(v[k], w[k], acc);
        first = false;
      }
    return first ? 0.0f : acc * factor;
  }
};

// ------------------------------------------------- pairwise-table loop, N_img
// SubminorLoopTabN: SubminorLoopTab for joined images (NI = 2..8 images of
// one polarization, each with its own PSF, the linear integration; no RMS
// factor, spectral map or log-polynomial fit). Per iteration the component's table row of
// every PSF (FMAs into the register-resident images), the integrated value
// per pixel, the key argmax as SubminorLoopTab's (|integrated| max chain with
// allow_negative), the wave winner's image values through its LDS slot, and
// for G > 1 participants (one XCD, as SubminorLoopTab) records of 3 + N_img
// epoch-tagged granules. The same operations in the same order as
// SubminorLoopReg: traces and model values are identical.
template <int NI, int ITEMS, int THREADS, bool NEG>
__global__ __launch_bounds__(THREADS) void SubminorLoopTabN(LoopArgs a) {
  constexpr int WAVES = THREADS / 64;
  constexpr int SLANES = WAVES <= 8 ? 8 : 16;
  constexpr uint32_t REC = 3 + NI;
  __shared__ uint4 slots[2][WAVES];     // {key hi, key lo, integrated bits, -}
  __shared__ float slotv[2][WAVES][NI];  // the wave winner's image values
  const uint32_t G = a.n_blocks;
  if (G > 1 && blockIdx.x % a.part_stride != 0u) return;
  const uint32_t rank = G > 1 ? blockIdx.x / a.part_stride : 0u;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t n = uint32_t(a.n_sel), per = a.per_block;
  const uint32_t base = rank * per;
  const uint32_t cnt = base >= n ? 0u : min(per, n - base);
  const bool neg = a.allow_negative != 0;
  LinearIntegration<NI> ri;
  ri.Init(a.integ);
  // uniform values kept in VGPRs (one wave per SIMD leaves them free; as
  // SGPRs they spilled): weights, factor, and below the component values
#pragma unroll
  for (int k = 0; k < NI; ++k) asm volatile("" : "+v"(ri.w[k]));
  asm volatile("" : "+v"(ri.factor));
  uint64_t* gran = reinterpret_cast<uint64_t*>(a.records);
  uint64_t* recs = gran + G;
  float R[ITEMS][NI], M[ITEMS][NI];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t j = tid + uint32_t(i) * THREADS;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      // beyond the slice: NaN (never a winner; see the padded table)
      R[i][k] = j < cnt ? a.r[size_t(k) * n + base + j] : __int_as_float(0x7fc00000);
      M[i][k] = 0.0f;
    }
  }
  bool fast = true;
  bool failed = false;
  if (G > 1) {
    if (tid == 0)
      __hip_atomic_store(gran + rank, (uint64_t(1) << 32) | XccId(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t xcc = 0u;
    for (uint64_t spins = 0; !failed; ++spins) {
      uint64_t v = 0;
      if (lane < G)
        v = __hip_atomic_load(gran + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all(lane >= G || (v >> 32) == 1u)) {
        xcc = uint32_t(v);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      failed = spins > (uint64_t(1) << 24);
    }
    const uint32_t x0 = uint32_t(__builtin_amdgcn_readlane(int(xcc), 0));
    fast = kFastExchange && __all(lane >= G || xcc == x0) && !a.agent_exchange;
  }
  const size_t sq = size_t(n) * n;
  float c[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) c[k] = 0.0f;
  float m = 0.0f, start_abs = 0.0f, flux = 0.0f;
  uint32_t cp = 0, par = 0, epoch = 0;
  uint32_t row_cp = 0xffffffffu;
  float pv[ITEMS][NI];
  uint32_t pend_pos = 0;
  bool pend = false, have = false, diverging = false;
  uint64_t iteration = a.iteration_start;
  const bool tracer = rank == 0 && tid == 0 && a.trace;
  const uint32_t thr_bits = __float_as_uint(a.threshold) & 0x7fffffffu;
  const uint32_t thr_mode = a.threshold != a.threshold        ? 0u
                            : (__float_as_uint(a.threshold) >> 31) && thr_bits ? 1u
                                                                                : 2u;
  uint32_t lim_mode = 0u, lim_bits = 0u;
  const bool stop_neg = a.stop_on_negative != 0;
  uint64_t remaining =
      a.max_iterations > a.iteration_start ? a.max_iterations - a.iteration_start : 0u;
  while (!failed) {
    if (have) {
      // the component's row of every PSF (contiguous over j), issued before
      // the previous iteration's decisions
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const bool in = __float_as_uint(pv[i][0]) != kOutsideBits;
#pragma unroll
        for (int k = 0; k < NI; ++k) {
          const float t = __builtin_fmaf(-pv[i][k], c[k], R[i][k]);
          R[i][k] = in ? t : R[i][k];
        }
      }
      if (pend) {
        const uint64_t t = iteration - a.iteration_start;
        if (t < a.trace_cap) {
          a.trace[2 * t] = pend_pos & 0xffffu;
          a.trace[2 * t + 1] = pend_pos >> 16;
        }
        pend = false;
      }
    }
    // ---- integrated values and this thread's best (as SubminorLoopTab)
    float iv[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) iv[i] = ri(R[i]);
    uint32_t bh = 0u, bj = 0xffffffffu, bv = __float_as_uint(iv[0]), li = 0u;
    if constexpr (NEG) {
      float tb = -1.0f;
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) tb = __builtin_fmaxf(tb, __builtin_fabsf(iv[i]));
      bh = tb >= 0.0f ? (__float_as_uint(tb) | 0x80000000u) : 0u;
#pragma unroll
      for (int i = ITEMS - 1; i >= 0; --i) {
        const bool eq = __builtin_fabsf(iv[i]) == tb;
        bj = eq ? base + tid + uint32_t(i) * THREADS : bj;
        bv = eq ? __float_as_uint(iv[i]) : bv;
        li = eq ? uint32_t(i) : li;
      }
      if (base == 0u && tid == 0u && cnt > 0u && iv[0] != iv[0]) {
        bh = 0xffffffffu;
        bj = 0u;
        li = 0u;
      }
    } else {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const float v = neg ? fabsf(iv[i]) : iv[i];
        const uint32_t u = __float_as_uint(v);
        uint32_t h = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        const uint32_t j = base + tid + uint32_t(i) * THREADS;
        if (v != v) h = (j == 0u && cnt > 0u) ? 0xffffffffu : 0u;
        const bool better = h > bh;
        bh = better ? h : bh;
        bj = better ? j : bj;
        bv = better ? __float_as_uint(iv[i]) : bv;
        li = better ? uint32_t(i) : li;
      }
    }
    // ---- wave winner and its image values
    const uint32_t mh = MaxU32<64>(bh);
    const uint64_t tie = __ballot(bh == mh);
    int owner;
    if (mh == 0u) {
      owner = 0;  // a key-0 wave stands for lane 0's item 0
    } else if ((tie & (tie - 1ull)) == 0ull) {
      owner = __builtin_ctzll(tie);
    } else {
      const uint32_t ml = MaxU32<64>(bh == mh ? ~bj : 0u);
      owner = FirstLane(bh == mh && ~bj == ml);
    }
    const uint32_t wl = mh == 0u ? 0u : ~uint32_t(__builtin_amdgcn_readlane(int(bj), owner));
    const uint32_t wv = uint32_t(__builtin_amdgcn_readlane(int(bv), owner));
    if (lane == 0) slots[par][wave] = make_uint4(mh, wl, wv, 0u);
    // the owner lane stores its candidate's image values (a key-0 wave: lane
    // 0's item 0, li = 0)
    if (int(lane) == owner) {
      float v[NI];
#pragma unroll
      for (int k = 0; k < NI; ++k) v[k] = R[0][k];
#pragma unroll
      for (int i = 1; i < ITEMS; ++i)
#pragma unroll
        for (int k = 0; k < NI; ++k) v[k] = li == uint32_t(i) ? R[i][k] : v[k];
#pragma unroll
      for (int k = 0; k < NI; ++k) slotv[par][wave][k] = v[k];
    }
    LdsBarrier();
    // ---- block winner over the wave slots
    const uint4 s4 = lane < uint32_t(WAVES) ? slots[par][lane] : make_uint4(0u, 0u, 0u, 0u);
    uint32_t gh = MaxU32<SLANES>(s4.x);
    {
      const bool mine = lane < uint32_t(WAVES) && s4.x == gh;
      const uint64_t t2 = __ballot(mine);
      if ((t2 & (t2 - 1ull)) == 0ull) {
        owner = __builtin_ctzll(t2);
      } else {
        const uint32_t l2 = MaxU32<SLANES>(mine ? s4.y : 0u);
        owner = FirstLane(mine && s4.y == l2);
      }
    }
    uint32_t gl = uint32_t(__builtin_amdgcn_readlane(int(s4.y), owner));
    uint32_t gv = uint32_t(__builtin_amdgcn_readlane(int(s4.z), owner));
    float wr[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      wr[k] = slotv[par][owner][k];
      asm volatile("" : "+v"(wr[k]));
    }
    par ^= 1u;
    if (G > 1) {
      ++epoch;
      uint64_t* mine_rec = recs + (size_t(epoch & 1u) * G + rank) * REC;
      if (wave == 0 && lane < REC) {
        uint32_t w = lane == 0 ? gh : lane == 1 ? gl : gv;
#pragma unroll
        for (int k = 0; k < NI; ++k)
          if (lane == 3u + uint32_t(k)) w = __float_as_uint(wr[k]);
        const uint64_t g = (uint64_t(epoch) << 32) | w;
        if (fast)
          __hip_atomic_store(mine_rec + lane, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
          __hip_atomic_store(mine_rec + lane, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      uint32_t xr[REC];
#pragma unroll
      for (uint32_t w = 0; w < REC; ++w) xr[w] = 0u;
      for (uint64_t spins = 0;; ++spins) {
        bool ok = true;
        if (lane < G) {
          const uint64_t* rr = recs + (size_t(epoch & 1u) * G + lane) * REC;
#pragma unroll
          for (uint32_t w = 0; w < REC; ++w) {
            const uint64_t g = __hip_atomic_load(rr + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = ok && uint32_t(g >> 32) == epoch;
            xr[w] = uint32_t(g);
          }
        }
        if (__all(ok)) break;
        if (spins > (uint64_t(1) << 26)) {
          failed = true;
          break;
        }
      }
      if (failed) break;
      gh = MaxU32<64>(lane < G ? xr[0] : 0u);
      const bool mine = lane < G && xr[0] == gh;
      const uint64_t t2 = __ballot(mine);
      int win;
      if ((t2 & (t2 - 1ull)) == 0ull) {
        win = __builtin_ctzll(t2);
      } else {
        const uint32_t l2 = MaxU32<64>(mine ? xr[1] : 0u);
        win = FirstLane(mine && xr[1] == l2);
      }
      gl = uint32_t(__builtin_amdgcn_readlane(int(xr[1]), win));
      gv = uint32_t(__builtin_amdgcn_readlane(int(xr[2]), win));
#pragma unroll
      for (int k = 0; k < NI; ++k)
        wr[k] = __uint_as_float(uint32_t(__builtin_amdgcn_readlane(int(xr[3 + k]), win)));
    }
    // ---- decisions (as SubminorLoopTab, on the integrated value's bits)
    const bool none = gh == 0u || (gh == 0xffffffffu && gl == 0xffffffffu);
    const uint32_t wp = none ? 0u : 0xffffffffu - gl;
    if (wp != row_cp) {
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const float* row = a.table + size_t(q) * sq + size_t(wp) * n + base;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) pv[i][q] = row[tid + uint32_t(i) * THREADS];
      }
      row_cp = wp;
    }
    m = __uint_as_float(gv);
    const uint32_t ab = gv & 0x7fffffffu;
    const bool is_nan = ab > 0x7f800000u;
    if (!have) {
      start_abs = __uint_as_float(ab);
      if (a.divergence_limit != 0.0f) {
        const float lim = start_abs * a.divergence_limit;
        lim_bits = __float_as_uint(lim) & 0x7fffffffu;
        lim_mode = lim != lim ? 0u : ((__float_as_uint(lim) >> 31) && lim_bits) ? 1u : 2u;
      }
    } else {
      diverging = lim_mode == 1u ? !is_nan : lim_mode == 2u ? (!is_nan && ab > lim_bits) : false;
      ++iteration;
      --remaining;
    }
    const bool above = thr_mode == 1u ? !is_nan : thr_mode == 2u ? (!is_nan && ab > thr_bits)
                                                               : false;
    const bool non_negative = !is_nan && ((gv >> 31) == 0u || gv == 0x80000000u);
    const bool go = above && remaining != 0u && (!stop_neg || non_negative) && !diverging;
    if (!go) break;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      c[k] = wr[k] * a.gain;
      asm volatile("" : "+v"(c[k]));
    }
    flux += m * a.gain;
    cp = wp;
    {
      const uint32_t off = wp - base;
      if (off < cnt && (off % uint32_t(THREADS)) / 64u == wave) {
        const uint32_t oi = off / uint32_t(THREADS);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
          if (uint32_t(i) == oi && lane == (off & 63u))
#pragma unroll
            for (int k = 0; k < NI; ++k) M[i][k] += c[k];
      }
    }
    if (tracer) {
      pend_pos = a.pos[wp];
      pend = true;
    }
    have = true;
  }
  if (pend) {
    const uint64_t t = iteration - a.iteration_start;
    if (t < a.trace_cap) {
      a.trace[2 * t] = pend_pos & 0xffffu;
      a.trace[2 * t + 1] = pend_pos >> 16;
    }
  }
  if (failed) {
    if (tid == 0) StoreSc1(&a.result[8], 1u);
    return;
  }
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t j = tid + uint32_t(i) * THREADS;
    if (j < cnt)
#pragma unroll
      for (int k = 0; k < NI; ++k) a.m[size_t(k) * n + base + j] = M[i][k];
  }
  if (rank == 0 && tid == 0) {
    LoopResult* r = reinterpret_cast<LoopResult*>(a.result);
    r->iteration = iteration;
    r->peak = m;
    r->diverging = diverging ? 1 : 0;
    r->flux = flux;
  }
}

template <int NI, bool NEG>
auto TabNKernel(uint32_t items) {
  return items <= 1   ? SubminorLoopTabN<NI, 1, 256, NEG>
         : items <= 2 ? SubminorLoopTabN<NI, 2, 256, NEG>
                      : SubminorLoopTabN<NI, 4, 256, NEG>;
}

template <int NI>
int LaunchTabN(const LoopArgs& a, uint32_t items, hipStream_t stream) {
  auto k = a.allow_negative ? TabNKernel<NI, true>(items) : TabNKernel<NI, false>(items);
  if (a.n_blocks > 1) {
    void* args[] = {const_cast<LoopArgs*>(&a)};
    RDL_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k),
                                             dim3(a.n_blocks * a.part_stride),
                                             dim3(256), args, 0, stream));
  } else {
    k<<<1, 256, 0, stream>>>(a);
    RDL_HIP_CHECK(hipGetLastError());
  }
  return RDL_OK;
}

template <int THREADS, bool NEG>
auto TabKernel(uint32_t items) {
  return items <= 1    ? SubminorLoopTab<1, THREADS, NEG>
         : items <= 2  ? SubminorLoopTab<2, THREADS, NEG>
         : items <= 4  ? SubminorLoopTab<4, THREADS, NEG>
         : items <= 8  ? SubminorLoopTab<8, THREADS, NEG>
         : items <= 16 ? SubminorLoopTab<16, THREADS, NEG>
                       : SubminorLoopTab<(THREADS <= 256 ? 32 : 16), THREADS, NEG>;
}

template <int THREADS>
int LaunchTab(const LoopArgs& a, uint32_t items, hipStream_t stream) {
  auto k = a.allow_negative ? TabKernel<THREADS, true>(items) : TabKernel<THREADS, false>(items);
  if (a.n_blocks > 1) {
    void* args[] = {const_cast<LoopArgs*>(&a)};
    RDL_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k),
                                             dim3(a.n_blocks * a.part_stride),
                                             dim3(THREADS), args, 0, stream));
  } else {
    k<<<1, THREADS, 0, stream>>>(a);
    RDL_HIP_CHECK(hipGetLastError());
  }
  return RDL_OK;
}

template <int NI, int ITEMS>
int LaunchWave(const LoopArgs& a, hipStream_t stream) {
  auto kernel = (NI == 1 && a.integ.copy_fast_path)
                    ? SubminorLoopReg<NI, ITEMS, NI == 1, 64>
                    : SubminorLoopReg<NI, ITEMS, false, 64>;
  kernel<<<1, 64, 0, stream>>>(a);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

// Single-wave register budget: ITEMS x N_img residuals + model values +
// gathers per lane.
constexpr uint32_t WaveMaxItems(uint32_t ni) {
  return ni <= 1 ? 16 : ni <= 2 ? 8 : ni <= 4 ? 4 : 2;
}

template <int NI>
int LaunchWaveItems(const LoopArgs& a, uint32_t items, hipStream_t stream) {
  constexpr uint32_t kMax = WaveMaxItems(NI);
  if (items <= 1) return LaunchWave<NI, 1>(a, stream);
  if (items <= 2) return LaunchWave<NI, 2>(a, stream);
  if (items <= 4 || kMax <= 4) return LaunchWave<NI, (kMax >= 4 ? 4 : 2)>(a, stream);
  if (items <= 8 || kMax <= 8) return LaunchWave<NI, (kMax >= 8 ? 8 : 2)>(a, stream);
  return LaunchWave<NI, (kMax >= 16 ? 16 : 2)>(a, stream);
}

// One 1024-thread workgroup (sixteen waves): selections too large for one
// 512-thread workgroup's registers that would otherwise pay the
// cross-workgroup exchange every iteration.
template <int NI, int ITEMS>
int LaunchBig(const LoopArgs& a, hipStream_t stream) {
  auto kernel = (NI == 1 && a.integ.copy_fast_path)
                    ? SubminorLoopReg<NI, ITEMS, NI == 1, 1024>
                    : SubminorLoopReg<NI, ITEMS, false, 1024>;
  if (a.n_blocks > 1) {
    void* args[] = {const_cast<LoopArgs*>(&a)};
    RDL_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kernel),
                                             dim3(a.n_blocks), dim3(1024), args, 0,
                                             stream));
  } else {
    kernel<<<1, 1024, 0, stream>>>(a);
    RDL_HIP_CHECK(hipGetLastError());
  }
  return RDL_OK;
}

template <int NI>
int LaunchBigItems(const LoopArgs& a, uint32_t items, hipStream_t stream) {
  if (items <= 1) return LaunchBig<NI, 1>(a, stream);
  if (items <= 2) return LaunchBig<NI, 2>(a, stream);
  if (items <= 4 || NI > 2) return LaunchBig<NI, 4>(a, stream);
  return LaunchBig<NI, 8>(a, stream);
}

template <int NI, int ITEMS>
int LaunchReg(const LoopArgs& a, hipStream_t stream) {
  auto kernel = (NI == 1 && a.integ.copy_fast_path) ? SubminorLoopReg<NI, ITEMS, NI == 1>
                                                    : SubminorLoopReg<NI, ITEMS, false>;
  if (a.n_blocks > 1) {
    void* args[] = {const_cast<LoopArgs*>(&a)};
    RDL_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kernel),
                                             dim3(a.n_blocks), dim3(kRegThreads),
                                             args, 0, stream));
  } else {
    kernel<<<1, kRegThreads, 0, stream>>>(a);
    RDL_HIP_CHECK(hipGetLastError());
  }
  return RDL_OK;
}

// Register budget: ITEMS x N_img residuals + model values + gathers per lane.
constexpr uint32_t RegMaxItems(uint32_t ni) {
  return ni <= 2 ? 8 : ni <= 4 ? 4 : 2;
}

template <int NI>
int LaunchRegItems(const LoopArgs& a, uint32_t items, hipStream_t stream) {
  constexpr uint32_t kMax = RegMaxItems(NI);
  if (items <= 1) return LaunchReg<NI, 1>(a, stream);
  if (items <= 2 || kMax == 2) return LaunchReg<NI, 2>(a, stream);
  if (items <= 4 || kMax == 4) return LaunchReg<NI, (kMax >= 4 ? 4 : 2)>(a, stream);
  return LaunchReg<NI, (kMax >= 8 ? 8 : 2)>(a, stream);
}

int Grow(void** p, size_t* have, size_t need, hipStream_t stream) {
  if (*have >= need) return RDL_OK;
  if (*p) {
    RDL_HIP_CHECK(hipStreamSynchronize(stream));
    RDL_HIP_CHECK(rdl::DevFree(*p));
    *p = nullptr;
    *have = 0;
  }
  RDL_HIP_CHECK(rdl::DevMalloc(p, need));
  *have = need;
  // RDL_POISON=1: NaN bytes in every fresh buffer (uninitialised reads show)
  if (PoisonOn()) RDL_HIP_CHECK(hipMemsetAsync(*p, 0xff, need, stream));
  return RDL_OK;
}

template <int NI>
int LaunchLoop(const LoopArgs& a, size_t lds_bytes, hipStream_t stream) {
  auto kernel = SubminorLoop<NI>;
  if (lds_bytes > 0)
    RDL_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kernel),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_bytes)));
  if (a.n_blocks > 1) {
    void* args[] = {const_cast<LoopArgs*>(&a)};
    RDL_HIP_CHECK(hipLaunchCooperativeKernel(
        reinterpret_cast<const void*>(kernel), dim3(a.n_blocks),
        dim3(kLoopThreads), args, unsigned(lds_bytes), stream));
  } else {
    kernel<<<1, kLoopThreads, lds_bytes, stream>>>(a);
    RDL_HIP_CHECK(hipGetLastError());
  }
  return RDL_OK;
}

}  // namespace rdl

extern "C" {

int rdl_subminor_create(rdl_session* s, rdl_subminor** out) {
  RDL_ARG_CHECK(s && out, "NULL argument");
  auto h = new rdl_subminor();
  h->s = s;
  // experiments: RDL_SUBMINOR_WAVE_MAX=0 disables the single-wave kernel
  if (const char* e = std::getenv("RDL_SUBMINOR_WAVE_MAX"))
    h->wave_max = uint32_t(std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("RDL_SUBMINOR_BIG_MAX"))
    h->big_max = uint32_t(std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("RDL_SUBMINOR_TARGET"))  // pixels x images per workgroup
    h->target_per_block = uint32_t(std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("RDL_SUBMINOR_BIG_TARGET"))
    h->big_target = uint32_t(std::strtoul(e, nullptr, 10));
  // RDL_SUBMINOR_SELECT=1 (2): the single-pass look-back selection (chunks
  // in ticket / blockIdx order); 3: count + scan + scatter (comparisons)
  if (const char* e = std::getenv("RDL_SUBMINOR_SELECT")) {
    const int v = std::atoi(e);
    h->select_passes = v == 3 ? 3 : v == 1 || v == 2 ? 1 : 0;
    h->select_ticket = v == 2 ? 0 : 1;
    h->select_quad = v == 4 ? 0 : 1;  // 4: the sparse selection's scalar loads
  }
  if (const char* e = std::getenv("RDL_SUBMINOR_TAB")) h->tab = std::atoi(e);
  if (const char* e = std::getenv("RDL_SUBMINOR_TAB_TARGET"))
    h->tab_target = uint32_t(std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("RDL_SUBMINOR_TAB_SINGLE"))
    h->tab_single = uint32_t(std::min<unsigned long>(std::strtoul(e, nullptr, 10), 16384));
  if (const char* e = std::getenv("RDL_SUBMINOR_TAB_THREADS"))
    h->tab_threads = uint32_t(std::strtoul(e, nullptr, 10));
  // test hook: RDL_SELECT_SPIN_LIMIT=0 makes any look-back wait fail
  if (const char* e = std::getenv("RDL_SELECT_SPIN_LIMIT"))
    h->select_spin_limit = std::strtoull(e, nullptr, 10);
  // RDL_SUBMINOR_TABLE_MAX=0 keeps the per-iteration PSF gathers
  if (const char* e = std::getenv("RDL_SUBMINOR_TABLE_MAX"))
    h->table_max = uint32_t(std::strtoul(e, nullptr, 10));
  *out = h;
  return RDL_OK;
}

int rdl_subminor_destroy(rdl_subminor* h) {
  if (!h) return RDL_OK;
  if (rdl::ShutDown()) return RDL_OK;  // rdl_shutdown released everything
  if (h->s->loop_owner == h) h->s->loop_owner = nullptr;
  (void)hipStreamSynchronize(h->s->stream);
  if (h->counts) (void)rdl::DevFree(h->counts);
  if (h->sel) (void)rdl::DevFree(h->sel);
  if (h->pos_buf) (void)rdl::DevFree(h->pos_buf);
  if (h->local_buf) (void)rdl::DevFree(h->local_buf);
  if (h->stamp_mark) (void)rdl::DevFree(h->stamp_mark);
  if (h->sync) (void)rdl::DevFree(h->sync);
  if (h->table) (void)rdl::DevFree(h->table);
  delete h;
  return RDL_OK;
}

namespace {
int SubminorLaunch(rdl_subminor* h, const float* d_residuals, const float* d_psfs,
                   const rdl_subminor_params* p, rdl_subminor_result* out, uint64_t trace_cap,
                   uint32_t** trace_dev);
int SubminorCollect(rdl_subminor* h, rdl_subminor_result* out, uint32_t* h_trace,
                    uint64_t trace_cap, const uint32_t* trace_dev);
}  // namespace

int rdl_subminor_run(rdl_subminor* h, const float* d_residuals,
                     const float* d_psfs, const rdl_subminor_params* p,
                     rdl_subminor_result* out, uint32_t* h_trace,
                     uint64_t trace_cap) {
  RDL_ARG_CHECK(h && d_residuals && d_psfs && p && out, "NULL argument");
  RDL_ARG_CHECK(!h->pending, "rdl_subminor_run: the previous loop was not collected");
  uint32_t* trace_dev = nullptr;
  const uint64_t cap = h_trace ? trace_cap : 0;
  RDL_TRY(SubminorLaunch(h, d_residuals, d_psfs, p, out, cap, &trace_dev));
  if (!h->pending) return RDL_OK;  // nothing selected: no loop
  return SubminorCollect(h, out, h_trace, cap, trace_dev);
}

int rdl_subminor_launch(rdl_subminor* h, const float* d_residuals, const float* d_psfs,
                        const rdl_subminor_params* p, rdl_subminor_result* out) {
  RDL_ARG_CHECK(h && d_residuals && d_psfs && p && out, "NULL argument");
  RDL_ARG_CHECK(!h->pending, "rdl_subminor_launch: the previous loop was not collected");
  uint32_t* trace_dev = nullptr;
  return SubminorLaunch(h, d_residuals, d_psfs, p, out, 0, &trace_dev);
}

int rdl_subminor_collect(rdl_subminor* h, rdl_subminor_result* out) {
  RDL_ARG_CHECK(h && out, "NULL argument");
  if (!h->pending) return RDL_OK;  // nothing was launched (no selection)
  return SubminorCollect(h, out, nullptr, 0, nullptr);
}

namespace {
int SubminorLaunch(rdl_subminor* h, const float* d_residuals, const float* d_psfs,
                   const rdl_subminor_params* p, rdl_subminor_result* out, uint64_t trace_cap,
                   uint32_t** trace_dev) {
  uint32_t* h_trace = nullptr;  // (the trace is read by SubminorCollect)
  RDL_ARG_CHECK(h && d_residuals && d_psfs && p && out, "NULL argument");
  RDL_ARG_CHECK(p->n_images >= 1 && p->n_images <= RDL_MAX_IMAGES,
                "n_images out of range");
  RDL_ARG_CHECK(p->n_pol >= 1 && p->n_images % p->n_pol == 0, "bad n_pol");
  RDL_ARG_CHECK(!p->logpoly || (p->logpoly->n_channels * p->n_pol == p->n_images &&
                                p->logpoly->n_channels <= RDL_LOGPOLY_MAX_CHANNELS &&
                                p->logpoly->n_terms >= 1 &&
                                p->logpoly->n_terms <= RDL_LOGPOLY_MAX_TERMS),
                "log-polynomial fit does not match the images");
  RDL_ARG_CHECK(p->width > 0 && p->height > 0 && p->width <= 65535 &&
                    p->height <= 65535,
                "image size out of range (1..65535)");
  rdl_session* s = h->s;
  // one mapped result slot per session (kMappedLoop): a second handle's
  // launch would overwrite a result that is still to be collected
  RDL_ARG_CHECK(!s->loop_owner || s->loop_owner == h,
                "another rdl_subminor handle of this session has a launched loop that was "
                "not collected (rdl_subminor_collect it first)");
  hipStream_t st = s->stream;
  h->width = p->width;
  h->height = p->height;
  h->n_images = p->n_images;

  // ---------------- selection (subminor_loop.cc:143-184)
  rdl::SelArgs sa{};
  sa.residuals = d_residuals;
  sa.mask = p->d_mask;
  sa.width = p->width;
  sa.height = p->height;
  sa.n = p->width * p->height;
  sa.xs = p->h_border;
  sa.xe = std::max<int64_t>(sa.xs, int64_t(p->width) - int64_t(p->h_border));
  sa.ys = p->v_border;
  sa.ye = std::max<int64_t>(sa.ys, int64_t(p->height) - int64_t(p->v_border));
  sa.xe = std::min(sa.xe, p->width);
  sa.ye = std::min(sa.ye, p->height);
  sa.xs = std::min(sa.xs, sa.xe);
  sa.ys = std::min(sa.ys, sa.ye);
  sa.bw = std::max<uint32_t>(1, sa.xe - sa.xs);
  sa.box_pixels = uint64_t(sa.xe - sa.xs) * (sa.ye - sa.ys);
  sa.integ = p->integ;
  sa.threshold = p->threshold;
  sa.allow_negative = p->allow_negative;
  sa.rms = p->d_rms;
  // the sparse selection's 16-byte-load variant: rows of whole float4
  // (width % 4 == 0), at most 16 items of 512 float4 per row
  const uint32_t quads_per_row = ((sa.xe + 3) >> 2) - (sa.xs >> 2);
  const uint32_t quad_ipr = std::max<uint32_t>(1, rdl::DivUp(quads_per_row, rdl::kSpThreads));
  const bool quad = h->select_passes == 0 && h->select_quad && p->width % 4 == 0 &&
                    p->integ.copy_fast_path && !p->d_rms && sa.box_pixels > 0 &&
                    quad_ipr <= rdl::kQuadItems;
  const uint32_t quad_rpb = rdl::kQuadItems / quad_ipr;
  const uint32_t n_chunks =
      quad ? rdl::DivUp(sa.ye - sa.ys, quad_rpb)
           : std::max<uint32_t>(1, rdl::DivUp(sa.box_pixels, h->select_passes == 3
                                                                 ? rdl::kChunk
                                                                 : rdl::kSpChunk));
  const uint32_t chunk_slots = quad ? rdl::kQuadChunk : rdl::kSpChunk;
  uint64_t* d_total = reinterpret_cast<uint64_t*>(s->d_small);
  // the count the host reads: SelScan also stores it in the mapped buffer
  uint64_t* m_total = static_cast<uint64_t*>(rdl::MappedResult(s, rdl::kMappedSelTotal));
  const double sel_bytes = double(sa.box_pixels) * 4.0 * p->n_images;
  // positions of up to the whole box (single pass) or the counts (three
  // kernels: RDL_SUBMINOR_SELECT=3, for comparison)
  uint32_t* counts = nullptr;
  uint32_t* sel_failed = nullptr;  // single pass: set by a timed-out look-back
  if (h->select_passes == 0) {
    // counts (then offsets), the chunks' local lists, the placed positions
    const size_t slots = size_t(n_chunks) * chunk_slots;
    RDL_TRY(rdl::Grow(&h->counts, &h->counts_bytes,
                      size_t(n_chunks) * sizeof(uint32_t) + 64, st));
    RDL_TRY(rdl::Grow(&h->local_buf, &h->local_bytes, slots * sizeof(uint32_t), st));
    RDL_TRY(rdl::Grow(&h->pos_buf, &h->pos_bytes,
                      std::max<size_t>(sa.box_pixels, 1) * sizeof(uint32_t), st));
    counts = static_cast<uint32_t*>(h->counts);
    rdl::ScopedTiming t(s, "subminor_select", sel_bytes);
    if (quad)
      rdl::SelLocalQuad<<<n_chunks, rdl::kSpThreads, 0, st>>>(
          sa, quad_ipr, quad_rpb, counts, static_cast<uint32_t*>(h->local_buf));
    else
      rdl::SelLocal<<<n_chunks, rdl::kSpThreads, 0, st>>>(
          sa, counts, static_cast<uint32_t*>(h->local_buf));
    rdl::SelScan<<<1, 1024, 0, st>>>(counts, n_chunks, d_total, m_total);
    rdl::SelPlace<<<n_chunks, 256, 0, st>>>(counts, n_chunks, d_total,
                                            static_cast<const uint32_t*>(h->local_buf),
                                            chunk_slots, static_cast<uint32_t*>(h->pos_buf));
  } else if (h->select_passes == 1) {
    RDL_TRY(rdl::Grow(&h->counts, &h->counts_bytes,
                      size_t(n_chunks) * sizeof(uint64_t) + 64, st));
    RDL_TRY(rdl::Grow(&h->pos_buf, &h->pos_bytes,
                      std::max<size_t>(sa.box_pixels, 1) * sizeof(uint32_t), st));
    uint64_t* status = static_cast<uint64_t*>(h->counts);
    uint32_t* ticket = reinterpret_cast<uint32_t*>(status + n_chunks);
    sel_failed = ticket + 1;
    RDL_HIP_CHECK(hipMemsetAsync(status, 0, size_t(n_chunks) * sizeof(uint64_t) + 64, st));
    rdl::ScopedTiming t(s, "subminor_select", sel_bytes);
    rdl::SelSinglePass<<<n_chunks, rdl::kSpThreads, 0, st>>>(
        sa, h->select_ticket ? ticket : nullptr, status, n_chunks,
        static_cast<uint32_t*>(h->pos_buf), d_total, sel_failed, h->select_spin_limit);
  } else {
    RDL_TRY(rdl::Grow(&h->counts, &h->counts_bytes,
                      size_t(n_chunks) * sizeof(uint32_t) + 64, st));
    counts = static_cast<uint32_t*>(h->counts);
    rdl::ScopedTiming t(s, "subminor_select", 2.0 * sel_bytes);
    rdl::SelCount<<<n_chunks, rdl::kSelThreads, 0, st>>>(sa, counts);
    rdl::SelScan<<<1, 1024, 0, st>>>(counts, n_chunks, d_total, m_total);
  }
  RDL_HIP_CHECK(hipGetLastError());
  uint64_t n_sel = 0;
  uint32_t failed = 0;
  {
    // RDL_SEL_COUNT_COPY=1: read the count back by a copy (r04 form; bisect)
    static const bool count_copy = [] {
      const char* e = std::getenv("RDL_SEL_COUNT_COPY");
      return e && e[0] == '1';
    }();
    const rdl::SmallRead r[2] = {{&n_sel, h->select_passes == 1 || count_copy ? d_total : m_total,
                                  sizeof(n_sel)},
                                 {&failed, sel_failed, sizeof(failed)}};
    RDL_TRY(rdl::ReadSmall(s, r, sel_failed ? 2 : 1));
  }
  if (failed) {
    rdl::SetError("rdl_subminor_run: selection look-back timed out");
    return RDL_ERR_TIMEOUT;
  }
  h->n_selected = n_sel;
  out->n_selected = n_sel;
  out->iteration = p->iteration_start;
  out->diverging = 0;
  out->flux_cleaned = 0.0f;
  if (n_sel == 0) {  // subminor_loop.cc:52-54
    out->has_peak = 0;
    out->peak = 0.0f;
    return RDL_OK;
  }
  const uint32_t ni = p->n_images;
  if (h->select_passes != 3) {
    RDL_TRY(rdl::Grow(&h->sel, &h->sel_bytes, 2 * n_sel * ni * sizeof(float) + 256, st));
    h->d_pos = static_cast<uint32_t*>(h->pos_buf);
    h->d_r = static_cast<float*>(h->sel);
    h->d_m = h->d_r + n_sel * ni;
    rdl::ScopedTiming t(s, "subminor_select", 12.0 * n_sel * ni);
    const unsigned grid = unsigned(std::min<uint64_t>(rdl::DivUp(n_sel, 256), 4096));
    rdl::SelGather<<<grid, 256, 0, st>>>(d_residuals, p->width, p->width * p->height,
                                         h->d_pos, n_sel, ni, h->d_r);
  } else {
    const size_t sel_need =
        n_sel * sizeof(uint32_t) + 2 * n_sel * ni * sizeof(float) + 256;
    RDL_TRY(rdl::Grow(&h->sel, &h->sel_bytes, sel_need, st));
    h->d_pos = static_cast<uint32_t*>(h->sel);
    h->d_r = reinterpret_cast<float*>(
        static_cast<char*>(h->sel) + (n_sel * sizeof(uint32_t) + 15) / 16 * 16);
    h->d_m = h->d_r + n_sel * ni;
    rdl::ScopedTiming t(s, "subminor_select", sel_bytes + 8.0 * n_sel * ni);
    rdl::SelScatter<<<n_chunks, rdl::kSelThreads, 0, st>>>(
        sa, counts, ni, n_sel, h->d_pos, h->d_r);
  }
  RDL_HIP_CHECK(hipGetLastError());

  // ---------------- partition and loop
  uint32_t max_blocks = uint32_t(std::max(1, std::min(s->n_cus, 256)));
  if (s->coop_limit) max_blocks = std::min(max_blocks, s->coop_limit);
  // register kernel: N_img <= 8, <= 4096 pixels per workgroup
  uint32_t ni_t = ni <= 1 ? 1 : ni <= 2 ? 2 : ni <= 4 ? 4 : 8;
  uint32_t g = 1;
  uint64_t per = n_sel;
  // the log-polynomial fit runs in the LDS-resident loop only
  const bool lpfit = p->logpoly != nullptr;
  const bool reg_ok = ni <= 8 && !lpfit;
  bool use_reg = reg_ok && h->mode != 1;
  const uint64_t reg_cap = uint64_t(rdl::kRegThreads) * rdl::RegMaxItems(ni_t);
  // the size limits count PSF gathers per iteration (pixels x images): with
  // joined channels one workgroup's memory pipe, not the exchange, bounds an
  // iteration (8 channels x 3000 pixels on one CU: 26 us per component)
  const uint64_t work = n_sel * ni;
  // with the pairwise table an iteration reads one contiguous row per PSF:
  // one workgroup (up to 1024 threads) then holds selections that would
  // otherwise pay a cross-workgroup exchange per component
  const uint64_t big_cap = 1024ull * (ni_t <= 2 ? 8 : 4);
  const bool want_table = (h->mode == 0 || h->mode == 6) && reg_ok && n_sel >= 2 && n_sel <= h->table_max &&
                          uint64_t(ni / p->n_pol) * n_sel * n_sel <=
                              (uint64_t(1) << (ni > 1 ? 29 : 28));  // 1 / 2 GiB
  // (one CU's memory pipe streams those rows: at most 8192 values per
  // iteration, so joined channels keep the grid above 8192 / N_img pixels)
  const bool table_single = want_table && n_sel <= big_cap && work <= 8192;
  if (use_reg) {
    if (!table_single && (n_sel > reg_cap || work > h->single_max)) {
      const uint64_t target = std::max<uint64_t>(
          std::max<uint32_t>(h->target_per_block, 512) / ni, 64);
      g = uint32_t(std::min<uint64_t>(max_blocks, (n_sel + target - 1) / target));
      g = std::max<uint32_t>(g, std::min<uint32_t>(2, max_blocks));
      per = (n_sel + g - 1) / g;
      use_reg = per <= reg_cap;
    }
  }
  if (!use_reg && (h->mode == 2 || h->mode == 3)) {
    rdl::SetError("register sub-minor kernel cannot hold this selection");
    return RDL_ERR_ARG;
  }
  // single wave: no barrier and no LDS exchange per iteration
  const uint64_t wave_cap = 64ull * rdl::WaveMaxItems(ni_t);
  const bool use_wave =
      use_reg && g == 1 &&
      ((h->mode == 0 && n_sel <= wave_cap && work <= h->wave_max) ||
       (h->mode == 3 && n_sel <= wave_cap));
  if (h->mode == 3 && !use_wave) {
    rdl::SetError("single-wave sub-minor kernel cannot hold this selection");
    return RDL_ERR_ARG;
  }
  // one sixteen-wave workgroup (mode 4 forces it)
  bool use_big =
      !use_wave && reg_ok && h->mode != 1 && h->mode != 2 &&
      ((h->mode == 0 && n_sel <= big_cap &&
        ((work <= h->big_max && work > 1024) || (table_single && n_sel > 1024))) ||
       (h->mode == 4 && n_sel <= big_cap));
  // 1024-thread workgroups on a cooperative grid (mode 5, target pixels per
  // workgroup from set_tuning; mode 0 when big_target is set)
  bool use_big_grid = false;
  if (!use_wave && !use_big && reg_ok &&
      ((h->mode == 5) || (h->mode == 0 && h->big_target > 0 && n_sel > h->big_max))) {
    const uint64_t target = h->mode == 5 ? std::max<uint32_t>(h->target_per_block, 1024)
                                         : h->big_target;
    uint32_t gb = uint32_t(std::min<uint64_t>(max_blocks, (n_sel + target - 1) / target));
    gb = std::max<uint32_t>(gb, 1);
    const uint64_t pb = (n_sel + gb - 1) / gb;
    if (pb <= big_cap) {
      use_big_grid = true;
      g = gb;
      per = pb;
      use_reg = true;
    }
  }
  if (h->mode == 4 && !use_big) {
    rdl::SetError("1024-thread sub-minor kernel cannot hold this selection");
    return RDL_ERR_ARG;
  }
  if (use_big) {
    g = 1;
    per = n_sel;
    use_reg = true;
  }
  if (use_big_grid) use_big = true;
  uint32_t items = 0;
  bool use_lds = false;
  size_t lds_bytes = 0;
  if (use_reg) {
    const uint64_t need = (per + rdl::kRegThreads - 1) / rdl::kRegThreads;
    items = need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : 8;
  } else {
    const size_t bytes_per_px = 4 + 8 * size_t(ni);
    const size_t lds_cap = 150 * 1024;
    if (n_sel <= 4096)
      g = 1;
    else
      g = std::min<uint64_t>(max_blocks, (n_sel + 4095) / 4096);
    per = (n_sel + g - 1) / g;
    use_lds = per * bytes_per_px <= lds_cap;
    if (!use_lds) {
      g = max_blocks;
      per = (n_sel + g - 1) / g;
      use_lds = per * bytes_per_px <= lds_cap;
    }
    lds_bytes = use_lds ? per * bytes_per_px : 0;
  }
  // the pairwise-table loop (mode 6 forces it): one image, identity
  // integration, no RMS / spectral / log-polynomial fit; participants of
  // about tab_target pixels each (one workgroup up to tab_target)
  const bool tab_shape = want_table && ni == 1 && p->integ.copy_fast_path && !p->d_rms &&
                         !p->d_spectral && !lpfit;
  const bool use_tab = tab_shape && ((h->mode == 0 && h->tab) || h->mode == 6) &&
                       !(h->mode == 0 && use_wave);
  if (h->mode == 6 && !use_tab) {
    rdl::SetError("table sub-minor kernel does not apply to this selection");
    return RDL_ERR_ARG;
  }
  // joined images (2..8, no RMS / spectral / log-polynomial fit):
  // SubminorLoopTabN, participants of up to 1024 pixels (a row of every PSF
  // per pixel: 1024 x 8 PSFs is the 32 KiB an iteration of one workgroup
  // streams), at most 32 (one XCD)
  const bool tabn_shape = want_table && ni > 1 && ni <= 8 && !p->d_rms && !p->d_spectral &&
                          !lpfit && h->tab && h->mode == 0 && !use_wave &&
                          p->integ.mode == RDL_INTEGRATE_LINEAR && !p->integ.copy_fast_path &&
                          p->n_pol == 1;
  uint32_t tabn_g = 0, tabn_items = 0;
  if (tabn_shape) {
    const uint64_t target = std::max<uint64_t>(256, 8192 / std::max<uint32_t>(ni / p->n_pol, 1));
    const uint64_t tgt = std::min<uint64_t>(target, 1024);
    const uint64_t gg = (n_sel + tgt - 1) / tgt;
    if (gg <= std::min<uint32_t>(32, max_blocks)) {
      tabn_g = uint32_t(std::max<uint64_t>(gg, 1));
      const uint64_t pp = (n_sel + tabn_g - 1) / tabn_g;
      const uint64_t need = (pp + 255) / 256;
      tabn_items = need <= 1 ? 1 : need <= 2 ? 2 : 4;
      g = tabn_g;
      per = pp;
    }
  }
  const bool use_tabn = tabn_g > 0;
  uint32_t tab_g = 1, tab_threads = 512, tab_items = 1;
  uint64_t tab_per = n_sel;
  if (use_tab) {
    // one workgroup up to 8192 pixels (measured on MI355X: an exchange costs
    // more than the row it splits below that; tools/bench_subminor.py), then
    // participants of tab_target pixels; mode 6 always splits by tab_target
    const uint64_t target = h->mode == 6 || n_sel > h->tab_single
                                ? std::max<uint32_t>(h->tab_target, 256)
                                : std::max<uint64_t>(n_sel, 1);
    tab_g = uint32_t(std::min<uint64_t>({(n_sel + target - 1) / target, 32, max_blocks}));
    tab_g = std::max<uint32_t>(tab_g, 1);
    tab_per = (n_sel + tab_g - 1) / tab_g;
    // measured on MI355X (tools/bench_subminor.py, RDL_BENCH_TAB): four
    // waves up to 2048 pixels and for grid participants, eight to 8192
    tab_threads = h->tab_threads == 256 || h->tab_threads == 512 || h->tab_threads == 1024
                      ? h->tab_threads
                      : (tab_g > 1 || tab_per <= 2048 ? 256u : 512u);
    const uint64_t need = (tab_per + tab_threads - 1) / tab_threads;
    const uint32_t cap = tab_threads == 256 ? 32 : 16;
    if (need > cap) tab_threads = 1024;
    const uint64_t need2 = (tab_per + tab_threads - 1) / tab_threads;
    tab_items = need2 <= 1 ? 1 : need2 <= 2 ? 2 : need2 <= 4 ? 4 : need2 <= 8 ? 8
                : need2 <= 16 ? 16 : 32;
    if (need2 > (tab_threads == 256 ? 32u : 16u)) {
      rdl::SetError("table sub-minor kernel: too many pixels per participant");
      return RDL_ERR_ARG;
    }
    g = tab_g;
    per = tab_per;
  }
  rdl::LoopArgs la{};
  la.pos = h->d_pos;
  la.r = h->d_r;
  la.m = h->d_m;
  la.psfs = d_psfs;
  la.n_sel = n_sel;
  la.per_block = uint32_t(per);
  la.n_blocks = g;
  la.rec_words = (4 + ni + 3) / 4 * 4;
  la.width = p->width;
  la.height = p->height;
  la.n_img = ni;
  la.n_pol = p->n_pol;
  la.integ = p->integ;
  la.threshold = p->threshold;
  la.gain = p->gain;
  la.spectral = lpfit ? nullptr : p->d_spectral;
  la.rms = p->d_rms;
  if (lpfit) {
    la.lp = *p->logpoly;
    la.has_lp = 1;
  }
  la.divergence_limit = p->divergence_limit;
  la.iteration_start = p->iteration_start;
  la.max_iterations = p->max_iterations;
  la.allow_negative = p->allow_negative;
  la.stop_on_negative = p->stop_on_negative;
  la.use_lds = use_lds ? 1 : 0;
  la.prof = s->trace_subminor_phases ? 1 : 0;
  // a pooled session (coop_limit: its share of the CUs) launches only as
  // many blocks as its share; the participants then spread over XCDs and
  // exchange through agent-scope stores (the kernel sees the XCC ids)
  la.part_stride = rdl::kTabParticipantStride;
  if ((use_tab || use_tabn) && g > 1 && s->coop_limit &&
      uint64_t(g) * rdl::kTabParticipantStride > s->coop_limit)
    la.part_stride = 1;
  {
    const char* e = std::getenv("RDL_SUBMINOR_EXCHANGE");  // read per run (tests toggle it)
    la.agent_exchange = e && std::strcmp(e, "agent") == 0 ? 1 : 0;
    const char* at = std::getenv("RDL_SUBMINOR_ATOMIC");  // read per run (A/B in one job)
    la.atomic_reduce = at && at[0] == '0' ? 0 : 1;
  }
  const uint64_t n_trace = trace_cap;
  (void)h_trace;
  const size_t rec_bytes =
      use_tab    ? (size_t(7) * g * sizeof(uint64_t) + 15) / 16 * 16
      : use_tabn ? ((size_t(1) + 2 * (3 + ni)) * g * sizeof(uint64_t) + 15) / 16 * 16
      : use_reg ? (size_t(2) * g * (3 + ni_t) * sizeof(uint64_t) + 15) / 16 * 16
                : size_t(2) * g * la.rec_words * sizeof(uint32_t);
  const size_t sync_need = 256 + 256 + rec_bytes + n_trace * 8;
  RDL_TRY(rdl::Grow(&h->sync, &h->sync_bytes, sync_need, st));
  char* sb = static_cast<char*>(h->sync);
  la.counter = reinterpret_cast<uint32_t*>(sb);
  // the result (and the timeout flag, word 8) goes straight to the mapped
  // buffer: no read-back copy; the previous run's words are cleared here (the
  // stream is idle: every run ends in ReadSmall's sync)
  la.result = static_cast<uint32_t*>(rdl::MappedResult(s, rdl::kMappedLoop));
  if (rdl::ZeroCopyOn())
    std::memset(static_cast<char*>(s->m_small) + rdl::kMappedLoop, 0, 256);
  else
    RDL_HIP_CHECK(hipMemsetAsync(la.result, 0, 256, st));
  la.records = reinterpret_cast<uint32_t*>(sb + 512);
  la.trace = n_trace ? reinterpret_cast<uint32_t*>(sb + 512 + rec_bytes) : nullptr;
  la.trace_cap = n_trace;
  // zero counter, result and (register kernel) the epoch-tagged granules:
  // with a pairwise table, by BuildPairTable
  const size_t zero_bytes = (use_reg || use_tab || use_tabn) ? 512 + rec_bytes : 512;
  // RDL_TABLE_ZERO=0: a separate memset of the exchange area (r04 form; bisect)
  static const bool table_zero_on = [] {
    const char* e = std::getenv("RDL_TABLE_ZERO");
    return !(e && e[0] == '0');
  }();
  const bool build_table = (use_reg || use_tab || use_tabn) && want_table;
  const bool table_zeroes = build_table && table_zero_on;
  if (!table_zeroes) RDL_HIP_CHECK(hipMemsetAsync(sb, 0, zero_bytes, st));
  la.table = nullptr;
  const uint32_t n_psf = ni / p->n_pol;
  if (build_table) {
    // (+ 32 KiB: the table loop reads whole workgroup-sized slices of a row)
    const size_t table_bytes = size_t(n_psf) * n_sel * n_sel * sizeof(float) + (32 << 10);
    RDL_TRY(rdl::Grow(&h->table, &h->table_bytes, table_bytes, st));
    rdl::ScopedTiming t(s, "subminor_table", 8.0 * double(n_psf) * n_sel * n_sel);
    rdl::BuildPairTable<<<dim3(rdl::DivUp(n_sel, 256), uint32_t(n_sel)), 256, 0, st>>>(
        h->d_pos, d_psfs, uint32_t(n_sel), n_psf, p->width, p->height,
        static_cast<float*>(h->table), reinterpret_cast<uint64_t*>(sb),
        table_zeroes ? uint32_t((zero_bytes + 7) / 8) : 0u);
    RDL_HIP_CHECK(hipGetLastError());
    la.table = static_cast<const float*>(h->table);
  }
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  if (s->trace_subminor) {
    ev0 = s->GetEvent();
    ev1 = s->GetEvent();
    RDL_HIP_CHECK(hipEventRecord(ev0, st));
  }
  {
    rdl::ScopedTiming t(s, "subminor_loop", 0.0);
    if (use_tab) {
      if (tab_threads == 256)
        RDL_TRY(rdl::LaunchTab<256>(la, tab_items, st));
      else if (tab_threads == 512)
        RDL_TRY(rdl::LaunchTab<512>(la, tab_items, st));
      else
        RDL_TRY(rdl::LaunchTab<1024>(la, tab_items, st));
    } else if (use_tabn) {
      switch (ni) {
        case 2: RDL_TRY(rdl::LaunchTabN<2>(la, tabn_items, st)); break;
        case 3: RDL_TRY(rdl::LaunchTabN<3>(la, tabn_items, st)); break;
        case 4: RDL_TRY(rdl::LaunchTabN<4>(la, tabn_items, st)); break;
        case 5: RDL_TRY(rdl::LaunchTabN<5>(la, tabn_items, st)); break;
        case 6: RDL_TRY(rdl::LaunchTabN<6>(la, tabn_items, st)); break;
        case 7: RDL_TRY(rdl::LaunchTabN<7>(la, tabn_items, st)); break;
        default: RDL_TRY(rdl::LaunchTabN<8>(la, tabn_items, st)); break;
      }
    } else if (use_big) {
      const uint64_t bi = (per + 1023) / 1024;
      const uint32_t bitems = bi <= 1 ? 1 : bi <= 2 ? 2 : bi <= 4 ? 4 : 8;
      if (ni_t == 1)
        RDL_TRY(rdl::LaunchBigItems<1>(la, bitems, st));
      else if (ni_t == 2)
        RDL_TRY(rdl::LaunchBigItems<2>(la, bitems, st));
      else if (ni_t == 4)
        RDL_TRY(rdl::LaunchBigItems<4>(la, bitems, st));
      else
        RDL_TRY(rdl::LaunchBigItems<8>(la, bitems, st));
    } else if (use_wave) {
      const uint64_t wi = (n_sel + 63) / 64;
      const uint32_t witems = wi <= 1 ? 1 : wi <= 2 ? 2 : wi <= 4 ? 4 : wi <= 8 ? 8 : 16;
      if (ni_t == 1)
        RDL_TRY(rdl::LaunchWaveItems<1>(la, witems, st));
      else if (ni_t == 2)
        RDL_TRY(rdl::LaunchWaveItems<2>(la, witems, st));
      else if (ni_t == 4)
        RDL_TRY(rdl::LaunchWaveItems<4>(la, witems, st));
      else
        RDL_TRY(rdl::LaunchWaveItems<8>(la, witems, st));
    } else if (use_reg) {
      if (ni_t == 1)
        RDL_TRY(rdl::LaunchRegItems<1>(la, items, st));
      else if (ni_t == 2)
        RDL_TRY(rdl::LaunchRegItems<2>(la, items, st));
      else if (ni_t == 4)
        RDL_TRY(rdl::LaunchRegItems<4>(la, items, st));
      else
        RDL_TRY(rdl::LaunchRegItems<8>(la, items, st));
    } else if (ni == 1) {
      RDL_TRY(rdl::LaunchLoop<1>(la, lds_bytes, st));
    } else if (ni <= 2) {
      RDL_TRY(rdl::LaunchLoop<2>(la, lds_bytes, st));
    } else if (ni <= 4) {
      RDL_TRY(rdl::LaunchLoop<4>(la, lds_bytes, st));
    } else if (ni <= 8) {
      RDL_TRY(rdl::LaunchLoop<8>(la, lds_bytes, st));
    } else if (ni <= 16) {
      RDL_TRY(rdl::LaunchLoop<16>(la, lds_bytes, st));
    } else {
      RDL_TRY(rdl::LaunchLoop<RDL_MAX_IMAGES>(la, lds_bytes, st));
    }
  }
  if (s->trace_subminor) RDL_HIP_CHECK(hipEventRecord(ev1, st));
  out->has_peak = 1;  // a selection: the loop's first component exists
  h->pending = true;
  s->loop_owner = h;
  h->pending_start = p->iteration_start;
  h->pending_bytes_per_it = 12.0 * double(ni) * double(n_sel);
  h->pending_result = la.result;
  h->pending_ev0 = ev0;
  h->pending_ev1 = ev1;
  h->pending_n_sel = n_sel;
  h->pending_g = g;
  h->pending_kind = use_tab ? 30 + int(tab_items) : use_tabn ? 50 + int(tabn_items)
                    : use_reg ? 10 + int(items) : int(use_lds);
  h->pending_threads = use_tab ? int(tab_threads) : use_tabn ? 256
                       : use_wave ? 64 : use_big ? 1024 : use_reg ? int(rdl::kRegThreads) : 512;
  h->pending_table = la.table ? 1 : 0;
  *trace_dev = la.trace;
  return RDL_OK;
}

int SubminorCollect(rdl_subminor* h, rdl_subminor_result* out, uint32_t* h_trace,
                    uint64_t trace_cap, const uint32_t* trace_dev) {
  rdl_session* s = h->s;
  hipStream_t st = s->stream;
  h->pending = false;
  if (s->loop_owner == h) s->loop_owner = nullptr;
  rdl::LoopResult res{};
  uint32_t err = 0;
  {
    // the result (words 0-5) and the exchange's timeout flag (word 8) in ONE
    // read: each read-back is a blit launch plus host latency per component run
    static_assert(sizeof(rdl::LoopResult) <= 8 * sizeof(uint32_t), "result before word 8");
    uint32_t raw[9];
    const rdl::SmallRead r{raw, h->pending_result, sizeof(raw)};
    RDL_TRY(rdl::ReadSmall(s, &r, 1));
    std::memcpy(&res, raw, sizeof(res));
    err = raw[8];
  }
  if (err) {
    rdl::SetError("sub-minor loop: grid exchange timed out");
    return RDL_ERR_TIMEOUT;
  }
  // algorithmic bytes: 12 B x N_img x N_sel per iteration
  rdl::AddTimingBytes(s, "subminor_loop",
                      h->pending_bytes_per_it * double(res.iteration - h->pending_start));
  if (s->trace_subminor) {
    const hipEvent_t ev0 = h->pending_ev0, ev1 = h->pending_ev1;
    float ms = 0.0f;
    RDL_HIP_CHECK(hipEventElapsedTime(&ms, ev0, ev1));
    {
      const std::lock_guard<std::recursive_mutex> lock(s->timing_mutex);
      s->event_pool.push_back(ev0);
      s->event_pool.push_back(ev1);
    }
    uint64_t ph[6] = {};
    const rdl::SmallRead r{ph, h->pending_result + 16, sizeof(ph)};
    RDL_TRY(rdl::ReadSmall(s, &r, 1));
    std::fprintf(stderr,
                 "[subminor] n_sel=%llu g=%u kind=%d threads=%d table=%d iters=%llu us=%.1f "
                 "gather=%llu integ=%llu wred=%llu bar=%llu xchg=%llu dec=%llu\n",
                 (unsigned long long)h->pending_n_sel, h->pending_g, h->pending_kind,
                 h->pending_threads, h->pending_table,
                 (unsigned long long)(res.iteration - h->pending_start),
                 double(ms) * 1e3, (unsigned long long)ph[0], (unsigned long long)ph[1],
                 (unsigned long long)ph[2], (unsigned long long)ph[3],
                 (unsigned long long)ph[4], (unsigned long long)ph[5]);
  }
  out->n_selected = h->pending_n_sel;
  out->iteration = res.iteration;
  out->has_peak = 1;
  out->peak = res.peak;
  out->diverging = res.diverging;
  out->flux_cleaned = res.flux;
  if (h_trace && trace_cap && trace_dev) {
    const uint64_t n = std::min<uint64_t>(res.iteration - h->pending_start, trace_cap);
    RDL_HIP_CHECK(hipMemcpyAsync(h_trace, trace_dev, n * 8,
                                 hipMemcpyDeviceToHost, st));
    RDL_HIP_CHECK(hipStreamSynchronize(st));
  }
  return RDL_OK;
}
}  // namespace

int rdl_subminor_set_tuning(rdl_subminor* h, int mode,
                            uint32_t target_per_block) {
  RDL_ARG_CHECK(h, "NULL argument");
  RDL_ARG_CHECK(mode >= 0 && mode <= 6, "mode must be 0 to 6");
  h->mode = mode;
  if (mode == 6) {  // the table kernel: target_per_block = pixels per participant
    if (target_per_block) h->tab_target = target_per_block;
    return RDL_OK;
  }
  if (target_per_block) h->target_per_block = target_per_block;
  return RDL_OK;
}

int rdl_subminor_model(rdl_subminor* h, uint32_t image_index, float* d_dest,
                       uint32_t dest_w, uint32_t dest_h, uint32_t ox,
                       uint32_t oy, int mode) {
  RDL_ARG_CHECK(h && d_dest, "NULL argument");
  RDL_ARG_CHECK(image_index < h->n_images || h->n_selected == 0,
                "image index out of range");
  RDL_ARG_CHECK(dest_w >= h->width + ox && dest_h >= h->height + oy,
                "destination too small");
  rdl_session* s = h->s;
  if (mode == 0)
    RDL_HIP_CHECK(hipMemsetAsync(d_dest, 0, size_t(dest_w) * dest_h * sizeof(float),
                                 s->stream));
  if (h->n_selected == 0) return RDL_OK;
  const unsigned grid = std::min<uint64_t>(4096, rdl::DivUp(h->n_selected, 256));
  rdl::ScatterModel<float><<<grid, 256, 0, s->stream>>>(
      h->d_pos, h->d_m + size_t(image_index) * h->n_selected, h->n_selected,
      d_dest, dest_w, ox, oy, mode == 1);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_subminor_model_masked(rdl_subminor* h, uint32_t image_index, float* d_dest,
                              uint32_t dest_w, uint32_t dest_h, const uint8_t* d_rows,
                              uint32_t oy) {
  RDL_ARG_CHECK(h && d_dest && d_rows, "NULL argument");
  RDL_ARG_CHECK(image_index < h->n_images || h->n_selected == 0,
                "image index out of range");
  RDL_ARG_CHECK(dest_w >= h->width && dest_h >= h->height, "destination too small");
  if (h->n_selected == 0) return RDL_OK;
  rdl_session* s = h->s;
  rdl::ZeroMarkedRows<<<std::min<uint32_t>(dest_h, 4096), 256, 0, s->stream>>>(
      d_dest, dest_w, dest_h, d_rows, oy);
  RDL_HIP_CHECK(hipGetLastError());
  const unsigned grid = std::min<uint64_t>(4096, rdl::DivUp(h->n_selected, 256));
  rdl::ScatterModel<float><<<grid, 256, 0, s->stream>>>(
      h->d_pos, h->d_m + size_t(image_index) * h->n_selected, h->n_selected, d_dest,
      dest_w, 0, 0, false);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_subminor_add_shape_model(rdl_subminor* h, uint32_t image_index,
                                 const float* d_kernel, uint32_t n, float* d_model,
                                 uint32_t width, uint32_t height) {
  RDL_ARG_CHECK(h && d_kernel && d_model, "NULL argument");
  RDL_ARG_CHECK(image_index < h->n_images || h->n_selected == 0,
                "image index out of range");
  RDL_ARG_CHECK(width == h->width && height == h->height, "model size differs");
  RDL_ARG_CHECK(n >= 1 && n % 2 == 1 && n <= width && n <= height,
                "shape kernel must be odd and no larger than the image");
  if (h->n_selected == 0) return RDL_OK;
  rdl_session* s = h->s;
  const uint32_t tiles_x = rdl::DivUp(width, rdl::kStampTile);
  const uint32_t tiles_y = rdl::DivUp(height, rdl::kStampTile);
  {
    // algorithmic bytes: the selection read per tile is cached; count the
    // model read-modify-write of the whole plane
    rdl::ScopedTiming t(s, "stamp_model", 8.0 * double(width) * height);
    const size_t n_tiles = size_t(tiles_x) * tiles_y;
    const size_t n_chunks = rdl::DivUp(h->n_selected, rdl::kStampThreads);
    const size_t mark_bytes = (n_tiles + 15) / 16 * 16;
    RDL_TRY(rdl::Grow(&h->stamp_mark, &h->stamp_mark_bytes,
                      mark_bytes + n_chunks * sizeof(int4), s->stream));
    uint8_t* mark = static_cast<uint8_t*>(h->stamp_mark);
    int4* bounds = reinterpret_cast<int4*>(mark + mark_bytes);
    RDL_HIP_CHECK(hipMemsetAsync(mark, 0, n_tiles, s->stream));
    const float* mi = h->d_m + size_t(image_index) * h->n_selected;
    static_assert(rdl::kStampThreads == 256, "one MarkStampTiles workgroup per chunk");
    rdl::MarkStampTiles<<<unsigned(n_chunks), 256, 0, s->stream>>>(
        h->d_pos, mi, h->n_selected, n, width, height, tiles_x, mark, bounds);
    // RDL_STAMP_BOUNDS=0: every tile walks every chunk (comparison)
    static const bool bounds_on = [] {
      const char* e = std::getenv("RDL_STAMP_BOUNDS");
      return !(e && e[0] == '0');
    }();
    rdl::StampShapeModel<<<tiles_x * tiles_y, rdl::kStampThreads, 0, s->stream>>>(
        h->d_pos, mi, h->n_selected, d_kernel, n, d_model, width, height, tiles_x, mark,
        bounds_on ? bounds : nullptr);
  }
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_subminor_model_rows(rdl_subminor* h, uint32_t image_index,
                            uint8_t* d_rows, uint32_t n_rows, uint32_t oy) {
  RDL_ARG_CHECK(h && d_rows, "NULL argument");
  RDL_ARG_CHECK(image_index < h->n_images || h->n_selected == 0,
                "image index out of range");
  RDL_ARG_CHECK(n_rows >= h->height + oy, "row mask too short");
  rdl_session* s = h->s;
  RDL_HIP_CHECK(hipMemsetAsync(d_rows, 0, n_rows, s->stream));
  if (h->n_selected == 0) return RDL_OK;
  const unsigned grid = std::min<uint64_t>(4096, rdl::DivUp(h->n_selected, 256));
  rdl::MarkModelRows<<<grid, 256, 0, s->stream>>>(
      h->d_pos, h->d_m + size_t(image_index) * h->n_selected, h->n_selected, d_rows,
      oy);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_subminor_model_f64(rdl_subminor* h, uint32_t image_index,
                           double* d_dest, uint32_t dest_w, uint32_t dest_h,
                           uint32_t ox, uint32_t oy) {
  RDL_ARG_CHECK(h && d_dest, "NULL argument");
  RDL_ARG_CHECK(image_index < h->n_images || h->n_selected == 0,
                "image index out of range");
  RDL_ARG_CHECK(dest_w >= h->width + ox && dest_h >= h->height + oy,
                "destination too small");
  rdl_session* s = h->s;
  RDL_HIP_CHECK(hipMemsetAsync(d_dest, 0, size_t(dest_w) * dest_h * sizeof(double),
                               s->stream));
  if (h->n_selected == 0) return RDL_OK;
  const unsigned grid = std::min<uint64_t>(4096, rdl::DivUp(h->n_selected, 256));
  rdl::ScatterModel<double><<<grid, 256, 0, s->stream>>>(
      h->d_pos, h->d_m + size_t(image_index) * h->n_selected, h->n_selected,
      d_dest, dest_w, ox, oy, 0);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_subminor_update_mask(rdl_subminor* h, uint8_t* d_mask) {
  RDL_ARG_CHECK(h && d_mask, "NULL argument");
  if (h->n_selected == 0) return RDL_OK;
  const uint32_t grid = uint32_t((h->n_selected + 255) / 256);
  rdl::UpdateMaskKernel<<<grid, 256, 0, h->s->stream>>>(h->d_pos, h->d_m, h->n_selected,
                                                       h->n_images, h->width, d_mask);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_subminor_get(rdl_subminor* h, uint32_t* h_positions, float* h_models,
                     uint64_t capacity) {
  RDL_ARG_CHECK(h, "NULL argument");
  const uint64_t n = std::min(capacity, h->n_selected);
  if (n == 0) return RDL_OK;
  if (h_positions)
    RDL_HIP_CHECK(hipMemcpyAsync(h_positions, h->d_pos, n * sizeof(uint32_t),
                                 hipMemcpyDeviceToHost, h->s->stream));
  if (h_models)
    for (uint32_t k = 0; k < h->n_images; ++k)
      RDL_HIP_CHECK(hipMemcpyAsync(h_models + k * n, h->d_m + k * h->n_selected,
                                   n * sizeof(float), hipMemcpyDeviceToHost,
                                   h->s->stream));
  RDL_HIP_CHECK(hipStreamSynchronize(h->s->stream));
  return RDL_OK;
}

}  // extern "C"
