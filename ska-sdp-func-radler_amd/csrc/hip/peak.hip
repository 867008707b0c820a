// Peak finding (argmax) and RMS: replaces math::peak_finder
// (cpp/math/peak_finder.cc) and ThreadedDeconvolutionTools::RMS.
//
// One streaming pass over the border box (4 B/px, +1 B/px with a mask):
// rows are dealt to 256-thread workgroups, each lane reads float4 (16 B)
// so a wave moves 1 KiB per load; the per-lane (value,index) max is packed in
// a 64-bit key (rdl::PeakKey) so the reduction is a plain integer max that
// reproduces the reference's "strict '>' from FLT_MIN, first index wins".
// A single-workgroup second stage reduces the per-block keys.
#include <cfloat>
#include <cstdlib>

#include "rdl_internal.h"

namespace rdl {

struct BoxArgs {
  const float* image;
  const uint8_t* mask;
  uint32_t width, height;
  uint32_t xs, xe, ys, ye;
  uint32_t rows_per_block;
  int allow_negative;
};

// kFinish: the last workgroup finishes the search (PeakArrive); without it
// the kernel carries none of that code (the two-launch form's register and
// LDS footprint)
template <bool kVec, bool kFinish>
__global__ __launch_bounds__(256) void FindPeakPartial(BoxArgs a,
                                                       uint64_t* partials, PeakFinish f) {
  __shared__ uint64_t lds[16];
  uint64_t best = 0;
  const uint32_t y0 = a.ys + blockIdx.x * a.rows_per_block;
  const uint32_t y1 = min(a.ye, y0 + a.rows_per_block);
  for (uint32_t y = y0; y < y1; ++y) {
    const float* row = a.image + size_t(y) * a.width;
    const uint8_t* mrow = a.mask ? a.mask + size_t(y) * a.width : nullptr;
    if constexpr (kVec) {
      const uint32_t q0 = a.xs >> 2, q1 = (a.xe + 3) >> 2;
      for (uint32_t q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
        const float4 v = reinterpret_cast<const float4*>(row)[q];
        uint32_t m4 = 0x01010101u;
        if (mrow) m4 = reinterpret_cast<const uint32_t*>(mrow)[q];
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t x = q * 4 + j;
          if (x >= a.xs && x < a.xe && ((m4 >> (8 * j)) & 0xffu)) {
            const uint64_t k =
                PeakKey(vv[j], a.allow_negative, y * a.width + x);
            best = k > best ? k : best;
          }
        }
      }
    } else {
      for (uint32_t x = a.xs + threadIdx.x; x < a.xe; x += blockDim.x) {
        if (mrow && !mrow[x]) continue;
        const uint64_t k = PeakKey(row[x], a.allow_negative, y * a.width + x);
        best = k > best ? k : best;
      }
    }
  }
  best = BlockMaxU64(best, lds);
  if constexpr (!kFinish) {
    if (threadIdx.x == 0) partials[blockIdx.x] = best;
  } else {
    if (threadIdx.x == 0)
      __hip_atomic_store(partials + blockIdx.x, best, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    PeakArrive(f, lds);
  }
}

__global__ __launch_bounds__(1024) void FindPeakFinal(
    const uint64_t* partials, uint32_t n, const float* image, uint32_t width,
    uint32_t height, int avx_semantics, int has_mask, PeakOut* out) {
  __shared__ uint64_t lds[16];
  uint64_t best = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    best = partials[i] > best ? partials[i] : best;
  best = BlockMaxU64(best, lds);
  if (threadIdx.x == 0) PeakOutOfKey(best, image, width, height, avx_semantics, has_mask, out);
}

__global__ __launch_bounds__(256) void SumSquaresPartial(const float* v,
                                                         size_t n,
                                                         double* partials) {
  __shared__ double lds[16];
  double acc = 0.0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n;
       i += size_t(gridDim.x) * blockDim.x) {
    const double x = v[i];
    acc += x * x;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (unsigned w = 0; w < blockDim.x / 64; ++w) s += lds[w];
    partials[blockIdx.x] = s;
  }
}

__global__ void SumSquaresFinal(const double* partials, uint32_t n, size_t count,
                                float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (uint32_t i = 0; i < n; ++i) s += partials[i];
    *out = float(std::sqrt(s / double(count)));
  }
}

int LaunchPeakFinal(rdl_session* s, const uint64_t* partials, uint32_t n,
                    const float* image, uint32_t width, uint32_t height, int avx_semantics,
                    int has_mask, void* d_out) {
  FindPeakFinal<<<1, 1024, 0, s->stream>>>(partials, n, image, width, height, avx_semantics,
                                           has_mask, static_cast<PeakOut*>(d_out));
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

void* PeakSlot(rdl_session* s, uint32_t slot) {
  return MappedResult(s, kMappedPeakSlots + size_t(slot) * sizeof(PeakOut));
}

uint32_t* PeakTicket(rdl_session* s, uint32_t slot) {
  return reinterpret_cast<uint32_t*>(static_cast<char*>(s->d_small) + kPeakTickets) + slot;
}

int LaunchFindPeak(rdl_session* s, const float* d_image, uint32_t width,
                   uint32_t height, uint32_t start_y, uint32_t end_y,
                   uint32_t h_border, uint32_t v_border, int allow_negative,
                   const uint8_t* d_mask, int avx_semantics, void* d_out, uint32_t ticket) {
  BoxArgs a;
  a.image = d_image;
  a.mask = d_mask;
  a.width = width;
  a.height = height;
  // peak_finder.cc:27-32 (unsigned wrap-around as in the reference)
  a.xs = h_border;
  a.xe = width - h_border;
  a.ys = start_y > v_border ? start_y : v_border;
  a.ye = end_y < height - v_border ? end_y : height - v_border;
  if (a.xe < a.xs) a.xe = a.xs;
  if (a.ye < a.ys) a.ye = a.ys;
  if (a.xe > width) a.xe = width;
  if (a.ye > height) a.ye = height;
  a.allow_negative = allow_negative;
  const uint32_t rows = a.ye - a.ys;
  const uint32_t target_blocks = 2048;
  a.rows_per_block = rows == 0 ? 1 : (rows + target_blocks - 1) / target_blocks;
  const uint32_t blocks =
      rows == 0 ? 1 : (rows + a.rows_per_block - 1) / a.rows_per_block;
  RDL_TRY(s->EnsureScratch(s->partials, size_t(blocks) * sizeof(uint64_t)));
  uint64_t* partials = static_cast<uint64_t*>(s->partials.ptr);
  const bool vec = (width % 4 == 0) &&
                   (reinterpret_cast<uintptr_t>(d_image) % 16 == 0) &&
                   (!d_mask || reinterpret_cast<uintptr_t>(d_mask) % 4 == 0);
  const double bytes = double(rows) * (a.xe - a.xs) * (d_mask ? 5.0 : 4.0);
  {
    ScopedTiming t(s, "find_peak", bytes);
    // the last workgroup finishes the search (PeakArrive); an empty box
    // keeps the two launches
    PeakFinish f;
    // RDL_PEAK_FINISH=0: the separate FindPeakFinal launch (comparison)
    static const bool finish_on = [] {
      const char* e = std::getenv("RDL_PEAK_FINISH");
      return !(e && e[0] == '0');
    }();
    if (rows != 0 && finish_on) {
      f.ticket = PeakTicket(s, ticket);
      f.out = static_cast<PeakOut*>(d_out);
      f.partials = partials;
      f.n_partials = blocks;
      f.image = d_image;
      f.width = width;
      f.height = height;
      f.avx_semantics = avx_semantics;
      f.has_mask = d_mask != nullptr;
    }
    if (rows == 0) {
      RDL_HIP_CHECK(hipMemsetAsync(partials, 0, sizeof(uint64_t), s->stream));
    } else if (vec) {
      if (f.ticket)
        FindPeakPartial<true, true><<<blocks, 256, 0, s->stream>>>(a, partials, f);
      else
        FindPeakPartial<true, false><<<blocks, 256, 0, s->stream>>>(a, partials, f);
    } else {
      if (f.ticket)
        FindPeakPartial<false, true><<<blocks, 256, 0, s->stream>>>(a, partials, f);
      else
        FindPeakPartial<false, false><<<blocks, 256, 0, s->stream>>>(a, partials, f);
    }
    if (!f.ticket)
      FindPeakFinal<<<1, 1024, 0, s->stream>>>(
          partials, blocks, d_image, width, height, avx_semantics,
          d_mask != nullptr, static_cast<PeakOut*>(d_out));
  }
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

}  // namespace rdl

extern "C" {

int rdl_find_peak(rdl_session* s, const float* d_image, uint32_t width,
                  uint32_t height, uint32_t start_y, uint32_t end_y,
                  uint32_t h_border, uint32_t v_border, int allow_negative,
                  const uint8_t* d_mask, int avx_semantics, rdl_peak* out) {
  RDL_ARG_CHECK(s && d_image && out, "NULL argument");
  RDL_ARG_CHECK(width > 0 && height > 0, "empty image");
  RDL_ARG_CHECK(uint64_t(width) * height < 0xffffffffull,
                "image too large for 32-bit pixel index");
  void* d_out = rdl::MappedResult(s, rdl::kMappedPeak);
  RDL_TRY(rdl::LaunchFindPeak(s, d_image, width, height, start_y, end_y,
                              h_border, v_border, allow_negative, d_mask,
                              avx_semantics, d_out, RDL_PEAK_SLOTS));
  rdl::PeakOut o;
  const rdl::SmallRead r{&o, d_out, sizeof(o)};
  RDL_TRY(rdl::ReadSmall(s, &r, 1));
  out->value = o.value;
  out->x = o.x;
  out->y = o.y;
  out->found = o.found;
  return RDL_OK;
}

}  // extern "C"

namespace {
// the deferred peak slots: the upper half of the session's small buffer
rdl::PeakOut* PeakSlots(rdl_session* s) {
  return static_cast<rdl::PeakOut*>(rdl::PeakSlot(s, 0));
}
static_assert(RDL_PEAK_SLOTS * sizeof(rdl::PeakOut) <= 32 * 1024, "peak slots");
}  // namespace

extern "C" {

int rdl_find_peak_enqueue(rdl_session* s, const float* d_image, uint32_t width,
                          uint32_t height, uint32_t start_y, uint32_t end_y,
                          uint32_t h_border, uint32_t v_border, int allow_negative,
                          const uint8_t* d_mask, int avx_semantics, uint32_t slot) {
  RDL_ARG_CHECK(s && d_image, "NULL argument");
  RDL_ARG_CHECK(width > 0 && height > 0, "empty image");
  RDL_ARG_CHECK(uint64_t(width) * height < 0xffffffffull,
                "image too large for 32-bit pixel index");
  RDL_ARG_CHECK(slot < RDL_PEAK_SLOTS, "peak slot out of range");
  return rdl::LaunchFindPeak(s, d_image, width, height, start_y, end_y, h_border, v_border,
                             allow_negative, d_mask, avx_semantics, PeakSlots(s) + slot, slot);
}

int rdl_find_peak_collect(rdl_session* s, uint32_t n, rdl_peak* out) {
  RDL_ARG_CHECK(s && (out || n == 0), "NULL argument");
  RDL_ARG_CHECK(n <= RDL_PEAK_SLOTS, "peak slot out of range");
  if (n == 0) return RDL_OK;
  rdl::PeakOut o[RDL_PEAK_SLOTS];
  const rdl::SmallRead r{o, PeakSlots(s), n * sizeof(rdl::PeakOut)};
  RDL_TRY(rdl::ReadSmall(s, &r, 1));
  for (uint32_t i = 0; i < n; ++i) {
    out[i].value = o[i].value;
    out[i].x = o[i].x;
    out[i].y = o[i].y;
    out[i].found = o[i].found;
  }
  return RDL_OK;
}

int rdl_rms(rdl_session* s, const float* d_image, size_t n, float* out) {
  RDL_ARG_CHECK(s && d_image && out, "NULL argument");
  RDL_ARG_CHECK(n > 0, "empty image");
  const uint32_t blocks = std::min<size_t>(1024, rdl::DivUp(n, 256));
  RDL_TRY(s->EnsureScratch(s->partials, blocks * sizeof(double)));
  double* partials = static_cast<double*>(s->partials.ptr);
  float* d_out = static_cast<float*>(rdl::MappedResult(s, rdl::kMappedRms));
  {
    rdl::ScopedTiming t(s, "rms", double(n) * 4.0);
    rdl::SumSquaresPartial<<<blocks, 256, 0, s->stream>>>(d_image, n,
                                                           partials);
    rdl::SumSquaresFinal<<<1, 64, 0, s->stream>>>(partials, blocks, n, d_out);
  }
  RDL_HIP_CHECK(hipGetLastError());
  const rdl::SmallRead r{out, d_out, sizeof(float)};
  RDL_TRY(rdl::ReadSmall(s, &r, 1));
  return RDL_OK;
}

}  // extern "C"
