// Internal declarations of librdl_hip.so (HIP for gfx950 / MI355X).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rdl_hip.h"

namespace rdl {

void SetError(const std::string& msg);

#define RDL_HIP_CHECK(expr)                                               \
  do {                                                                    \
    hipError_t _e = (expr);                                               \
    if (_e != hipSuccess) {                                               \
      ::rdl::SetError(std::string(#expr) + ": " + hipGetErrorString(_e)); \
      return RDL_ERR_HIP;                                                 \
    }                                                                     \
  } while (0)

#define RDL_ARG_CHECK(cond, msg)      \
  do {                                \
    if (!(cond)) {                    \
      ::rdl::SetError(msg);           \
      return RDL_ERR_ARG;             \
    }                                 \
  } while (0)

#define RDL_TRY(expr)         \
  do {                        \
    int _rc = (expr);         \
    if (_rc != RDL_OK) return _rc; \
  } while (0)

// Kernel-family timing with HIP events on the session stream (bench.py's
// roofline reads it; off by default).
struct TimingEntry {
  double ms = 0.0;
  uint64_t launches = 0;
  double bytes = 0.0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
};

// A reusable device scratch buffer that only grows.
struct Scratch {
  void* ptr = nullptr;
  size_t bytes = 0;
};

// Live-block registry for the RDL_SEGV_REPORT crash report: every device
// block (hipMalloc) and pinned host block (hipHostMalloc) this library holds,
// in a fixed lock-free table the signal handler can read (session.hip).
// kind: 'd' device, 'h' pinned host.
void TrackBlock(const void* p, size_t bytes, char kind);
void UntrackBlock(const void* p);

template <typename T>
hipError_t DevMalloc(T** p, size_t bytes) {
  const hipError_t e = hipMalloc(reinterpret_cast<void**>(p), bytes);
  if (e == hipSuccess) TrackBlock(*p, bytes, 'd');
  return e;
}
inline hipError_t DevFree(void* p) {
  UntrackBlock(p);
  return hipFree(p);
}
// RDL_POISON=1 (debug): fresh device buffers are filled with 0xff bytes
// (NaN floats) so reads of memory nothing wrote show up in results
inline bool PoisonOn() {
  static const bool on = [] {
    const char* e = std::getenv("RDL_POISON");
    return e && e[0] == '1';
  }();
  return on;
}
template <typename T>
hipError_t HostMalloc(T** p, size_t bytes) {
  const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(p), bytes, hipHostMallocDefault);
  if (e == hipSuccess) TrackBlock(*p, bytes, 'h');
  return e;
}
inline hipError_t HostFree(void* p) {
  UntrackBlock(p);
  return hipHostFree(p);
}
// A host->device upload on `stream`, waited for: never the null stream.
// Synchronous null-stream calls (hipMemset / hipMemcpy) made once per
// session left the 16-stream subimage pool ~21 % slower for the rest of the
// process (r06 bisection of r05's split joined regression).
inline hipError_t UploadSync(void* d, const void* h, size_t bytes, hipStream_t stream) {
  hipError_t e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(stream);
}
// Coherent pinned host memory the device writes directly (zero-copy): the
// results a host waits for (peaks, selection counts, loop results) are
// stored there by the kernel that makes them, so reading one back costs a
// stream sync and no copy launch. *d is the device's address of it.
inline hipError_t MappedMalloc(void** h, void** d, size_t bytes) {
  hipError_t e = hipHostMalloc(h, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return e;
  TrackBlock(*h, bytes, 'h');
  e = hipHostGetDevicePointer(d, *h, 0);
  if (e != hipSuccess) {
    UntrackBlock(*h);
    (void)hipHostFree(*h);
    *h = nullptr;
  }
  return e;
}

}  // namespace rdl

struct rdl_session {
  int device = 0;
  hipStream_t stream = nullptr;  // the current lane's stream (launchers use this)
  // two-lane chains (rdl_session_fork / _lane / _join): `home` is the
  // session's own stream, `aux` the second lane's; `lane` selects `stream`
  hipStream_t home = nullptr;
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int lane = 0;
  int n_cus = 256;
  uint32_t coop_limit = 0;       // cap on cooperative grids (0: n_cus)
  bool timing = false;
  // timings and event_pool are written by the thread driving this session
  // (ScopedTiming) and read by rdl_timing_*_all from any thread
  std::recursive_mutex timing_mutex;
  std::map<std::string, rdl::TimingEntry> timings;
  std::vector<hipEvent_t> event_pool;
  // small device/host scratch used by reductions
  void* d_small = nullptr;       // 64 KiB device
  void* h_small = nullptr;       // 64 KiB pinned host
  // 64 KiB coherent host memory written by kernels (MappedMalloc): [0, 4K)
  // single results (rdl_find_peak, rdl_rms, the selection count), [4K, 8K)
  // the sub-minor loop result, [32K, 64K) the deferred peak slots
  void* m_small = nullptr;       // host address
  void* m_small_dev = nullptr;   // device address of the same bytes
  rdl::Scratch partials;         // per-block partial keys
  rdl::Scratch radix;            // radix-select histograms
  bool poison = false;                 // RDL_POISON=1: NaN-fill fresh allocations
  bool trace_subminor_phases = false;  // RDL_TRACE_SUBMINOR=1 (2: timing only)
  bool trace_subminor = false;         // RDL_TRACE_SUBMINOR=1/2: per-launch stats
  rdl::Scratch kernel;           // host-provided kernels (H2D destination)
  rdl::Scratch loop_state;       // Högbom loop state / partials / trace
  rdl::Scratch iuwt;             // IUWT i0 / recompose accumulator plane
  void* comm = nullptr;          // ncclComm_t when initialised
  // the rdl_subminor handle whose launched loop has not been collected: its
  // result lives in the session's one mapped loop slot (kMappedLoop), so no
  // other handle of this session may launch until it is collected
  const void* loop_owner = nullptr;
  // rdl_malloc / rdl_free block cache: a freed block is kept for reuse by a
  // later allocation of this session (stream-ordered on `stream`), so the
  // per-Perform buffers cost no hipFree (which idles the device) and no
  // hipMalloc; RDL_ALLOC_CACHE=0 frees immediately
  std::mutex cache_mutex;
  std::multimap<size_t, void*> cache_free;      // size -> block
  std::map<void*, size_t> cache_live;           // block -> size
  size_t cache_bytes = 0;                       // bytes held in cache_free
  size_t cache_cap = size_t(96) << 30;          // min(96 GiB, device memory / 4)
  bool cache_on = true;
  int FlushCache();

  hipEvent_t GetEvent();
  void BeginTiming(const char* family, hipEvent_t* start);
  void EndTiming(const char* family, hipEvent_t start, double bytes);
  int CollectTimings();
  int EnsureScratch(rdl::Scratch& s, size_t bytes);
};

namespace rdl {
// hands every cached block of every session on `device` back (out of memory)
int FlushDeviceCaches(int device);
// rdl_shutdown has run: every block, stream and plan of this library is
// released, and the destroy/free entry points are no-ops from then on
extern std::atomic<bool> g_shutdown;
inline bool ShutDown() { return g_shutdown.load(std::memory_order_acquire); }
// rocFFT plans of the live rdl_fft objects (fftconv.hip), for rdl_shutdown
void ReleaseFftPlans();
// destroys a session's RCCL communicator (comm.hip)
void CommRelease(rdl_session* s);
// rdl_timing_enable_all: time every session of the process
extern std::atomic<bool> g_timing_all;
inline bool TimingOn(const rdl_session* s) {
  return s->timing || g_timing_all.load(std::memory_order_relaxed);
}
// rdl_timing_filter_all: when set, only this family records events (the
// event pairs of every other launch are skipped, so a timed region can keep
// the dominant family's HIP-event timing without the per-launch overhead of
// all the others); empty = every family
extern char g_timing_family[64];
inline bool FamilyOn(const char* family) {
  return g_timing_family[0] == 0 || std::strcmp(family, g_timing_family) == 0;
}
// Adds algorithmic bytes to a family after the fact (e.g. the sub-minor loop,
// whose iteration count is known only when it returns).
inline void AddTimingBytes(rdl_session* s, const char* family, double bytes) {
  if (TimingOn(s) && FamilyOn(family)) {
    const std::lock_guard<std::recursive_mutex> lock(s->timing_mutex);
    s->timings[family].bytes += bytes;
  }
}

// Records start/end events around a launcher's kernels when timing.
struct ScopedTiming {
  rdl_session* s;
  const char* family;
  double bytes;
  hipEvent_t start = nullptr;
  ScopedTiming(rdl_session* s_, const char* f, double b)
      : s(s_), family(f), bytes(b) {
    if (TimingOn(s) && FamilyOn(family)) s->BeginTiming(family, &start);
  }
  ~ScopedTiming() {
    if (start) s->EndTiming(family, start, bytes);
  }
};

// Integration of one pixel across the image set, bit-for-bit the reference's
// ImageSet::Get{Linear,Square}Integrated* (cpp/image_set.cc:309-462).
// `get(i)` returns image i's value at this pixel.
template <typename Get>
__device__ __forceinline__ float IntegratePixel(const rdl_integration& g,
                                                Get get) {
  if (g.copy_fast_path) return get(0);
  const uint32_t np = g.n_pol;
  if (g.mode == RDL_INTEGRATE_LINEAR) {
    // image_set.cc:432-460: AssignMultiply, then AddWithFactor (FMA), then *=
    float acc = 0.0f;
    bool first = true;
    for (uint32_t i = 0; i < g.n_images; ++i) {
      const float w = g.weights[i];
      if (w != 0.0f && ((g.pol_mask >> (i % np)) & 1u)) {
        const float v = get(i);
        acc = first ? v * w : __builtin_fmaf(v, w, acc);
        first = false;
      }
    }
    return first ? 0.0f : acc * g.factor;
  }
  if (g.mode == RDL_INTEGRATE_SQUARE) {
    if (g.n_channels == 1) {  // image_set.cc:361-386
      float acc = 0.0f;
      bool first = true;
      for (uint32_t p = 0; p < np; ++p) {
        if ((g.pol_mask >> p) & 1u) {
          const float v = get(p);
          acc = first ? v * v : __builtin_fmaf(v, v, acc);
          first = false;
        }
      }
      return __builtin_sqrtf(acc) * g.factor;
    }
    float dest = 0.0f;  // image_set.cc:388-421
    for (uint32_t ch = 0; ch < g.n_channels; ++ch) {
      const float w = g.weights[ch * np];
      float scratch = 0.0f;
      if (w != 0.0f) {
        if (np == 1) {
          scratch = get(ch);
        } else {
          float acc = 0.0f;
          bool first = true;
          for (uint32_t p = 0; p < np; ++p) {
            if ((g.pol_mask >> p) & 1u) {
              const float v = get(ch * np + p);
              acc = first ? v * v : __builtin_fmaf(v, v, acc);
              first = false;
            }
          }
          scratch = first ? 0.0f : __builtin_sqrtf(acc);
        }
      }
      dest = ch == 0 ? scratch * w : __builtin_fmaf(scratch, w, dest);
    }
    return dest * g.factor;
  }
  // RDL_INTEGRATE_SQUARED_JOINS, image_set.cc:429-455 (aocommon SquareWithFactor
  // / AddSquared operation order is not in /root/reference: parity unpinned)
  float acc = 0.0f;
  bool first = true;
  for (uint32_t i = 0; i < g.n_images; ++i) {
    const float w = g.weights[i];
    if (w != 0.0f && ((g.pol_mask >> (i % np)) & 1u)) {
      const float v = get(i);
      acc = first ? v * v * w : __builtin_fmaf(v * v, w, acc);
      first = false;
    }
  }
  return first ? 0.0f : __builtin_sqrtf(acc) * g.factor;
}

// Orderable 64-bit argmax key: larger key = larger value, ties -> smaller
// index. Values that do not qualify (<= FLT_MIN, NaN, sign filtered) get 0.
__device__ __forceinline__ uint64_t PeakKey(float v, bool allow_negative,
                                            uint32_t index) {
  uint32_t u = __float_as_uint(v);
  if (allow_negative) u &= 0x7fffffffu;
  // qualify: FLT_MIN < value <= +inf (sign bit set -> fails the <= test)
  const bool q = (u > 0x00800000u) && (u <= 0x7f800000u);
  return q ? ((uint64_t(u) << 32) | uint64_t(0xffffffffu - index)) : 0ull;
}

__device__ __forceinline__ uint64_t WaveMaxU64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// peak.hip: the second stage of a peak search over per-block/per-row keys,
// and the deferred result slots of rdl_find_peak_enqueue / _collect
int LaunchPeakFinal(rdl_session* s, const uint64_t* partials, uint32_t n,
                    const float* image, uint32_t width, uint32_t height, int avx_semantics,
                    int has_mask, void* d_out);
void* PeakSlot(rdl_session* s, uint32_t slot);
// the arrival ticket of peak slot `slot` (RDL_PEAK_SLOTS: rdl_find_peak's)
uint32_t* PeakTicket(rdl_session* s, uint32_t slot);

// Block-wide max of a uint64 (blockDim multiple of 64, <= 1024).
__device__ __forceinline__ uint64_t BlockMaxU64(uint64_t v, uint64_t* lds) {
  v = WaveMaxU64(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n_waves = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  if (wave == 0) {
    uint64_t w = lane < n_waves ? lds[lane] : 0ull;
    w = WaveMaxU64(w);
    if (lane == 0) lds[0] = w;
  }
  __syncthreads();
  const uint64_t r = lds[0];
  return r;
}

// A peak search's result (rdl_find_peak / _collect read it from the
// session's mapped buffer).
struct PeakOut {
  uint64_t key;
  float value;
  uint32_t x, y;
  int32_t found;
};

// The result of the best key (peak_finder.cc:202,250-252: with the AVX
// semantics and no mask an empty box reports pixel 0).
__device__ __forceinline__ void PeakOutOfKey(uint64_t best, const float* image, uint32_t width,
                                             uint32_t height, int avx_semantics, int has_mask,
                                             PeakOut* out) {
  PeakOut o;
  o.key = best;
  if (best != 0) {
    const uint32_t idx = 0xffffffffu - uint32_t(best & 0xffffffffu);
    o.x = idx % width;
    o.y = idx / width;
    o.value = image[idx];
    o.found = 1;
  } else if (avx_semantics && !has_mask) {
    o.x = 0;
    o.y = 0;
    o.value = image[0];
    o.found = 1;
  } else {
    o.x = width;
    o.y = height;
    o.value = 0.0f;
    o.found = 0;
  }
  *out = o;
}

// In-kernel second stage of a peak search over an image an earlier launch
// wrote: every workgroup arrives once, after thread 0 stored its partial key
// with an agent-scope (write-through) store; the last to arrive reduces the
// n_partials keys and writes the PeakOut (no FindPeakFinal launch). No
// fences: the partials travel by write-through stores and agent-scope loads
// (a release fence here writes back the whole L2). The ticket is 0 between
// launches (the last workgroup resets it); one per concurrently pending
// search (PeakTicket).
struct PeakFinish {
  uint32_t* ticket = nullptr;  // nullptr: the caller launches FindPeakFinal
  PeakOut* out = nullptr;
  const uint64_t* partials = nullptr;
  uint32_t n_partials = 0;
  const float* image = nullptr;
  uint32_t width = 0, height = 0;
  int avx_semantics = 0, has_mask = 0;
};

// Every thread of every workgroup calls this once (it holds barriers).
// lds: >= 16 uint64 of the caller's shared memory.
__device__ __forceinline__ void PeakArrive(const PeakFinish& f, uint64_t* lds) {
  __shared__ uint32_t last;
  if (threadIdx.x == 0) {
#if defined(__gfx950__) || !defined(__HIP_DEVICE_COMPILE__)
    // gfx950: the vector L1 is write-through, so once vmcnt(0) has retired
    // the partial's agent-scope store it is in the L2 every workgroup reads
    // (the loads below bypass L1); the ticket needs no release/acquire
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial has landed
    last = atomicAdd(f.ticket, 1u) == gridDim.x - 1u ? 1u : 0u;
#else
    // other targets: the C++ memory model's ordering (release of the
    // partial, acquire of the others' before the last workgroup reads them)
    last = __hip_atomic_fetch_add(f.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                   gridDim.x - 1u
               ? 1u
               : 0u;
#endif
  }
  __syncthreads();
  if (!last) return;
  uint64_t best = 0;
  for (uint32_t i = threadIdx.x; i < f.n_partials; i += blockDim.x) {
    const uint64_t v = __hip_atomic_load(f.partials + i, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    best = v > best ? v : best;
  }
  best = BlockMaxU64(best, lds);
  if (threadIdx.x == 0) {
    PeakOutOfKey(best, f.image, f.width, f.height, f.avx_semantics, f.has_mask, f.out);
    __hip_atomic_store(f.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

inline unsigned DivUp(size_t a, size_t b) { return unsigned((a + b - 1) / b); }

}  // namespace rdl

namespace rdl {
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (call site,
// device): the call can stall, and the attribute is per device, so a pool
// of workers on several GPUs needs it on each. `done` is the call site's
// device bitmask.
inline int SetMaxLdsOnce(const void* fn, int bytes, int device,
                         std::atomic<uint64_t>& done) {
  const uint64_t bit = uint64_t(1) << (device & 63);
  if (done.load(std::memory_order_acquire) & bit) return RDL_OK;
  RDL_HIP_CHECK(
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.fetch_or(bit, std::memory_order_acq_rel);
  return RDL_OK;
}
}  // namespace rdl

namespace rdl {
// Small device->host reads go through the session's pinned 64 KiB buffer:
// one DMA straight into pinned memory instead of the runtime's pageable
// staging path (lower latency per outer iteration, and no shared staging
// buffer between the worker threads of a subimage pool). Copies `n` regions
// (device src, bytes) back to back, syncs the stream, then scatters them.
struct SmallRead {
  void* h_dst;
  const void* d_src;
  size_t bytes;
};
// A region inside the session's mapped buffer (m_small) is read in place
// after the sync: no copy.
inline const char* MappedHost(const rdl_session* s, const void* d_src, size_t bytes) {
  const char* d = static_cast<const char*>(d_src);
  const char* m = static_cast<const char*>(s->m_small_dev);
  if (!m || d < m || d + bytes > m + (size_t(1) << 16)) return nullptr;
  return static_cast<const char*>(s->m_small) + (d - m);
}
inline int ReadSmall(rdl_session* s, const SmallRead* reads, int n) {
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    if (MappedHost(s, reads[i].d_src, reads[i].bytes)) continue;
    const size_t b = (reads[i].bytes + 15) / 16 * 16;
    if (off + b > (size_t(1) << 16)) {
      SetError("ReadSmall: more than 64 KiB");
      return RDL_ERR_ARG;
    }
    RDL_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(s->h_small) + off, reads[i].d_src,
                                 reads[i].bytes, hipMemcpyDeviceToHost, s->stream));
    off += b;
  }
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  off = 0;
  for (int i = 0; i < n; ++i) {
    if (const char* m = MappedHost(s, reads[i].d_src, reads[i].bytes)) {
      std::memcpy(reads[i].h_dst, m, reads[i].bytes);
      continue;
    }
    std::memcpy(reads[i].h_dst, static_cast<const char*>(s->h_small) + off,
                reads[i].bytes);
    off += (reads[i].bytes + 15) / 16 * 16;
  }
  return RDL_OK;
}
// the mapped buffer's regions (device addresses); RDL_ZERO_COPY=0 keeps
// the results in device memory and reads them back by copies (comparison)
inline bool ZeroCopyOn() {
  static const bool on = [] {
    const char* e = std::getenv("RDL_ZERO_COPY");
    return !(e && e[0] == '0');
  }();
  return on;
}
inline void* MappedResult(rdl_session* s, size_t offset) {
  return static_cast<char*>(ZeroCopyOn() ? s->m_small_dev : s->d_small) + offset;
}
constexpr size_t kMappedSelTotal = 0;      // uint64_t selection count
constexpr size_t kMappedPeak = 64;         // PeakOut of rdl_find_peak
constexpr size_t kMappedRms = 128;         // float of rdl_rms
constexpr size_t kMappedLoop = 4096;       // sub-minor LoopResult (+ phase probes)
constexpr size_t kMappedPeakSlots = 32 * 1024;
// the device small buffer's last 1 KiB: peak search tickets (PeakTicket),
// zeroed at session creation
constexpr size_t kPeakTickets = 63 * 1024;
}  // namespace rdl
