// Session / runtime part of the C-ABI (rdl_hip.h "runtime" section).
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rdl_internal.h"

namespace rdl {
namespace {
thread_local std::string g_last_error;

// Process-wide timing (rdl_timing_*_all): every live session, plus the
// collected totals of sessions destroyed since the last reset.
std::mutex g_registry_mutex;
std::vector<rdl_session*> g_sessions;
std::map<std::string, TimingEntry> g_retired;

// Diagnostics for crashes outside our code (RDL_SEGV_REPORT=<file>): the
// signal, the faulting pc with the module holding it (dladdr), a native
// backtrace, every live block of this library (device and pinned host, with
// the block holding or nearest to the fault address), and the process's whole
// module map (/proc/self/maps), appended to <file>; then the default action
// runs (the process dies as it would have). Only async-signal-safe calls
// after the first line (open/write/read/close; the integer formatting is our
// own); dladdr and backtrace are warmed up when the handler is installed.
char g_segv_path[512] = {0};

// Live-block registry: open addressing over a fixed table, one CAS per
// insert, a relaxed store per removal; readers (the handler) take whatever is
// there. Full table: the block is simply not listed.
constexpr size_t kBlockSlots = 8192;
struct BlockSlot {
  std::atomic<uintptr_t> base{0};
  std::atomic<size_t> bytes{0};
  std::atomic<char> kind{0};
};
BlockSlot g_blocks[kBlockSlots];

size_t SlotOf(uintptr_t p) { return size_t((p >> 12) * 0x9E3779B97F4A7C15ull >> 51) % kBlockSlots; }

void WriteAll(int fd, const char* p, size_t n) {
  while (n > 0) {
    const ssize_t w = write(fd, p, n);
    if (w <= 0) return;
    p += w;
    n -= size_t(w);
  }
}
void WriteStr(int fd, const char* p) { WriteAll(fd, p, strlen(p)); }
void WriteHex(int fd, uintptr_t v) {
  char b[19] = "0x";
  int n = 2;
  for (int sh = 60; sh >= 0; sh -= 4) {
    const unsigned d = unsigned(v >> sh) & 15u;
    if (n > 2 || d || sh == 0) b[n++] = char(d < 10 ? '0' + d : 'a' + d - 10);
  }
  WriteAll(fd, b, size_t(n));
}
void WriteDec(int fd, uint64_t v) {
  char b[21];
  int n = 20;
  b[n] = 0;
  do {
    b[--n] = char('0' + v % 10);
    v /= 10;
  } while (v);
  WriteAll(fd, b + n, size_t(20 - n));
}

void WriteBlocks(int fd, uintptr_t fault) {
  WriteStr(fd, "--- live blocks of librdl_hip (kind base bytes end)\n");
  uintptr_t best_base = 0, best_end = 0;
  uintptr_t best_dist = ~uintptr_t(0);
  char best_kind = 0;
  uint64_t n = 0, dev = 0, host = 0;
  for (size_t i = 0; i != kBlockSlots; ++i) {
    const uintptr_t b = g_blocks[i].base.load(std::memory_order_relaxed);
    if (!b) continue;
    const size_t bytes = g_blocks[i].bytes.load(std::memory_order_relaxed);
    const char k = g_blocks[i].kind.load(std::memory_order_relaxed);
    const uintptr_t e = b + bytes;
    ++n;
    (k == 'h' ? host : dev) += bytes;
    char kb[3] = {k ? k : '?', ' ', 0};
    WriteStr(fd, kb);
    WriteHex(fd, b);
    WriteStr(fd, " ");
    WriteDec(fd, bytes);
    WriteStr(fd, " ");
    WriteHex(fd, e);
    WriteStr(fd, "\n");
    const uintptr_t d = fault < b ? b - fault : fault >= e ? fault - e + 1 : 0;
    if (d < best_dist) {
      best_dist = d;
      best_base = b;
      best_end = e;
      best_kind = k;
    }
  }
  WriteStr(fd, "blocks ");
  WriteDec(fd, n);
  WriteStr(fd, ", device bytes ");
  WriteDec(fd, dev);
  WriteStr(fd, ", pinned host bytes ");
  WriteDec(fd, host);
  WriteStr(fd, "\nfault address ");
  WriteHex(fd, fault);
  if (best_dist == ~uintptr_t(0)) {
    WriteStr(fd, ": no live block\n");
    return;
  }
  WriteStr(fd, best_dist == 0 ? ": INSIDE " : ": nearest ");
  char kb[2] = {best_kind ? best_kind : '?', 0};
  WriteStr(fd, kb);
  WriteStr(fd, " block ");
  WriteHex(fd, best_base);
  WriteStr(fd, "..");
  WriteHex(fd, best_end);
  if (best_dist) {
    WriteStr(fd, " at distance ");
    WriteDec(fd, best_dist);
  }
  WriteStr(fd, "\n");
}

void SegvReport(int sig, siginfo_t* info, void* ctx) {
  const int fd = open(g_segv_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (fd >= 0) {
    void* pc = nullptr;
#if defined(__x86_64__)
    const ucontext_t* uc = static_cast<const ucontext_t*>(ctx);
    pc = reinterpret_cast<void*>(uc->uc_mcontext.gregs[REG_RIP]);
#else
    (void)ctx;
#endif
    Dl_info d{};
    const bool known = pc && dladdr(pc, &d) != 0;
    WriteStr(fd, "signal ");
    WriteDec(fd, uint64_t(sig));
    WriteStr(fd, " (code ");
    WriteDec(fd, uint64_t(uint32_t(info->si_code)));
    WriteStr(fd, ") address ");
    WriteHex(fd, reinterpret_cast<uintptr_t>(info->si_addr));
    WriteStr(fd, " pc ");
    WriteHex(fd, reinterpret_cast<uintptr_t>(pc));
    WriteStr(fd, " module ");
    WriteStr(fd, known && d.dli_fname ? d.dli_fname : "?");
    WriteStr(fd, " +");
    WriteHex(fd, known && d.dli_fbase ? uintptr_t((char*)pc - (char*)d.dli_fbase) : 0);
    WriteStr(fd, " symbol ");
    WriteStr(fd, known && d.dli_sname ? d.dli_sname : "?");
    WriteStr(fd, "\n");
    void* frames[64];
    backtrace_symbols_fd(frames, backtrace(frames, 64), fd);
    WriteBlocks(fd, reinterpret_cast<uintptr_t>(info->si_addr));
    WriteStr(fd, "--- /proc/self/maps\n");
    const int maps = open("/proc/self/maps", O_RDONLY);
    if (maps >= 0) {
      char buf[4096];
      ssize_t r;
      while ((r = read(maps, buf, sizeof buf)) > 0) WriteAll(fd, buf, size_t(r));
      close(maps);
    }
    close(fd);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

void InstallSegvReport() {
  const char* path = std::getenv("RDL_SEGV_REPORT");
  if (!path || !path[0]) return;
  snprintf(g_segv_path, sizeof g_segv_path, "%s", path);
  // load libgcc's unwinder and resolve dladdr now, not inside the handler
  void* frames[4];
  (void)backtrace(frames, 4);
  Dl_info d{};
  (void)dladdr(reinterpret_cast<void*>(&InstallSegvReport), &d);
  struct sigaction sa {};
  sa.sa_sigaction = SegvReport;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
}
std::once_flag g_segv_once;

// rdl_shutdown at process exit (RDL_EXIT_SHUTDOWN=0: leave everything to the
// runtime's own teardown, as before r06). Registered by the first
// rdl_session_create, after HIP has initialised, so it runs BEFORE the HIP
// runtime's exit handlers (atexit order is the reverse of registration): the
// process-lifetime sessions (one per GPU, the subimage pool's workers), their
// block caches, plans, mapped host buffers and streams are released while the
// runtime is still whole.
std::once_flag g_exit_once;
void ExitShutdown() { (void)rdl_shutdown(); }
void RegisterExitShutdown() {
  const char* e = std::getenv("RDL_EXIT_SHUTDOWN");
  if (e && e[0] == '0') return;
  std::atexit(ExitShutdown);
}

void Fold(std::map<std::string, TimingEntry>& into,
          const std::map<std::string, TimingEntry>& from) {
  for (const auto& [name, t] : from) {
    TimingEntry& e = into[name];
    e.ms += t.ms;
    e.launches += t.launches;
    e.bytes += t.bytes;
  }
}
}  // namespace
std::atomic<bool> g_timing_all{false};
std::atomic<bool> g_shutdown{false};
char g_timing_family[64] = {0};
void SetError(const std::string& msg) { g_last_error = msg; }

void TrackBlock(const void* p, size_t bytes, char kind) {
  const uintptr_t b = reinterpret_cast<uintptr_t>(p);
  if (!b) return;
  for (size_t i = 0, k = SlotOf(b); i != kBlockSlots; ++i, k = (k + 1) % kBlockSlots) {
    uintptr_t empty = 0;
    if (g_blocks[k].base.load(std::memory_order_relaxed) == 0 &&
        g_blocks[k].base.compare_exchange_strong(empty, b, std::memory_order_relaxed)) {
      g_blocks[k].bytes.store(bytes, std::memory_order_relaxed);
      g_blocks[k].kind.store(kind, std::memory_order_relaxed);
      return;
    }
  }
}

void UntrackBlock(const void* p) {
  const uintptr_t b = reinterpret_cast<uintptr_t>(p);
  if (!b) return;
  for (size_t i = 0, k = SlotOf(b); i != kBlockSlots; ++i, k = (k + 1) % kBlockSlots)
    if (g_blocks[k].base.load(std::memory_order_relaxed) == b) {
      g_blocks[k].bytes.store(0, std::memory_order_relaxed);
      g_blocks[k].kind.store(0, std::memory_order_relaxed);
      g_blocks[k].base.store(0, std::memory_order_relaxed);
      return;
    }
}
}  // namespace rdl

hipEvent_t rdl_session::GetEvent() {
  const std::lock_guard<std::recursive_mutex> lock(timing_mutex);
  if (!event_pool.empty()) {
    hipEvent_t e = event_pool.back();
    event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void rdl_session::BeginTiming(const char* family, hipEvent_t* start) {
  (void)family;
  *start = GetEvent();
  (void)hipEventRecord(*start, stream);
}

void rdl_session::EndTiming(const char* family, hipEvent_t start,
                            double bytes) {
  hipEvent_t end = GetEvent();
  (void)hipEventRecord(end, stream);
  const std::lock_guard<std::recursive_mutex> lock(timing_mutex);
  rdl::TimingEntry& t = timings[family];
  t.pending.emplace_back(start, end);
  t.launches += 1;
  t.bytes += bytes;
}

int rdl_session::CollectTimings() {
  const std::lock_guard<std::recursive_mutex> lock(timing_mutex);
  for (auto& [name, t] : timings) {
    for (auto& [a, b] : t.pending) {
      RDL_HIP_CHECK(hipEventSynchronize(b));
      float ms = 0.0f;
      RDL_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
      t.ms += ms;
      event_pool.push_back(a);
      event_pool.push_back(b);
    }
    t.pending.clear();
  }
  return RDL_OK;
}

int rdl_session::EnsureScratch(rdl::Scratch& s, size_t bytes) {
  if (s.bytes >= bytes) return RDL_OK;
  if (s.ptr) {
    RDL_HIP_CHECK(hipStreamSynchronize(home));
    if (aux) RDL_HIP_CHECK(hipStreamSynchronize(aux));
    RDL_HIP_CHECK(rdl::DevFree(s.ptr));
    s.ptr = nullptr;
    s.bytes = 0;
  }
  RDL_HIP_CHECK(rdl::DevMalloc(&s.ptr, bytes));
  s.bytes = bytes;
  if (poison) RDL_HIP_CHECK(hipMemsetAsync(s.ptr, 0xff, bytes, stream));
  return RDL_OK;
}

namespace rdl {
int FlushDeviceCaches(int device) {
  // Under the registry lock (rdl_session_destroy takes it before deleting a
  // session, so no session listed here can go away meanwhile): take every
  // cached block of the device's sessions, wait for the whole device once
  // (no other session's streams are touched: one may be forking its second
  // lane concurrently), then free them. The caller has made `device` current.
  std::vector<void*> blocks;
  const std::lock_guard<std::mutex> lock(g_registry_mutex);
  for (rdl_session* o : g_sessions) {
    if (o->device != device) continue;
    const std::lock_guard<std::mutex> clock(o->cache_mutex);
    for (auto& [bytes, p] : o->cache_free) blocks.push_back(p);
    o->cache_free.clear();
    o->cache_bytes = 0;
  }
  if (blocks.empty()) return RDL_OK;
  RDL_HIP_CHECK(hipDeviceSynchronize());
  for (void* p : blocks) RDL_HIP_CHECK(rdl::DevFree(p));
  return RDL_OK;
}
}  // namespace rdl

extern "C" {

const char* rdl_last_error(void) { return rdl::g_last_error.c_str(); }

const char* rdl_version(void) { return "rdl_hip 0.1.0 (gfx950)"; }

int rdl_device_count(int* count) {
  RDL_ARG_CHECK(count, "count is NULL");
  RDL_HIP_CHECK(hipGetDeviceCount(count));
  return RDL_OK;
}

namespace rdl {
// Streams come from a per-device pool created with the device's first
// session (RDL_STREAM_POOL streams, default 40; 0: one fresh stream per
// request, the earlier behaviour). HIP binds a stream to one of its few
// hardware queues (GPU_MAX_HW_QUEUES, 4) when the stream is created; the
// subimage pool's 16 worker sessions created after a long run of another
// session measured 1.3-2x slower per pass than the same workers created
// early (r06: bench_legs.py joined,joined_split 9.4 s against 4.7 s), so
// every session's streams are created together, up front, in one order.
std::mutex g_stream_mutex;
std::map<int, std::vector<hipStream_t>> g_stream_free;  // device -> FIFO
std::map<int, bool> g_stream_made;
int StreamPoolSize() {
  const char* e = std::getenv("RDL_STREAM_POOL");
  return e ? std::max(0, std::atoi(e)) : 40;
}
int TakeStream(int device, hipStream_t* out) {
  const std::lock_guard<std::mutex> lock(g_stream_mutex);
  auto& v = g_stream_free[device];
  if (!g_stream_made[device]) {
    g_stream_made[device] = true;
    for (int i = 0, n = StreamPoolSize(); i < n; ++i) {
      hipStream_t st = nullptr;
      RDL_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      v.push_back(st);
    }
  }
  if (v.empty()) {
    RDL_HIP_CHECK(hipStreamCreateWithFlags(out, hipStreamNonBlocking));
    return RDL_OK;
  }
  *out = v.front();
  v.erase(v.begin());
  return RDL_OK;
}
// back to the pool (idle: the caller synchronized it), or destroyed
void GiveStream(int device, hipStream_t st) {
  if (!st) return;
  if (StreamPoolSize() == 0) {
    (void)hipStreamDestroy(st);
    return;
  }
  (void)hipStreamSynchronize(st);
  const std::lock_guard<std::mutex> lock(g_stream_mutex);
  g_stream_free[device].push_back(st);
}
void DestroyStreamPools() {
  const std::lock_guard<std::mutex> lock(g_stream_mutex);
  for (auto& [device, v] : g_stream_free) {
    (void)hipSetDevice(device);
    for (hipStream_t st : v) (void)hipStreamDestroy(st);
    v.clear();
  }
}
}  // namespace rdl

int rdl_session_create(int device, rdl_session** out) {
  RDL_ARG_CHECK(out, "out is NULL");
  RDL_ARG_CHECK(!rdl::ShutDown(), "rdl_shutdown has run");
  std::call_once(rdl::g_segv_once, rdl::InstallSegvReport);
  int n = 0;
  RDL_HIP_CHECK(hipGetDeviceCount(&n));
  std::call_once(rdl::g_exit_once, rdl::RegisterExitShutdown);
  RDL_ARG_CHECK(device >= 0 && device < n, "invalid device index");
  // leave the caller's current device as it was (a pool creates sessions
  // for other GPUs from the main thread)
  int prev = 0;
  RDL_HIP_CHECK(hipGetDevice(&prev));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  RDL_HIP_CHECK(hipSetDevice(device));
  auto s = std::make_unique<rdl_session>();
  s->device = device;
  RDL_TRY(rdl::TakeStream(device, &s->stream));
  s->home = s->stream;
  hipDeviceProp_t prop;
  RDL_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  s->n_cus = prop.multiProcessorCount;
  s->cache_cap = std::min(s->cache_cap, size_t(prop.totalGlobalMem) / 4);
  // debug aid: fill every fresh allocation with NaN bytes (0xff)
  const char* poison = std::getenv("RDL_POISON");
  s->poison = poison && poison[0] == '1';
  const char* trace = std::getenv("RDL_TRACE_SUBMINOR");
  s->trace_subminor = trace && (trace[0] == '1' || trace[0] == '2');
  const char* cache = std::getenv("RDL_ALLOC_CACHE");
  s->cache_on = !(cache && cache[0] == '0');
  s->trace_subminor_phases = trace && trace[0] == '1';  // 2: timing only
  RDL_HIP_CHECK(rdl::DevMalloc(&s->d_small, 1 << 16));
  // the peak tickets start at 0. On the session's own stream: a synchronous
  // hipMemset here (the null stream, once per session) made the 16-worker
  // pool's passes 21 % slower for the rest of the process (r05's split joined
  // regression, 4.6 -> 5.6 s; bisected in r06 to this one call)
  RDL_HIP_CHECK(hipMemsetAsync(s->d_small, 0, 1 << 16, s->stream));
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  RDL_HIP_CHECK(rdl::HostMalloc(&s->h_small, 1 << 16));
  if (rdl::ZeroCopyOn()) {  // RDL_ZERO_COPY=0: no mapped host memory at all
    RDL_HIP_CHECK(rdl::MappedMalloc(&s->m_small, &s->m_small_dev, 1 << 16));
    std::memset(s->m_small, 0, 1 << 16);
  }
  {
    const std::lock_guard<std::mutex> lock(rdl::g_registry_mutex);
    rdl::g_sessions.push_back(s.get());
  }
  *out = s.release();
  return RDL_OK;
}

int rdl_session::FlushCache() {
  std::multimap<size_t, void*> blocks;
  {
    const std::lock_guard<std::mutex> lock(cache_mutex);
    blocks.swap(cache_free);
    cache_bytes = 0;
  }
  if (blocks.empty()) return RDL_OK;
  RDL_HIP_CHECK(hipStreamSynchronize(home));
  if (aux) RDL_HIP_CHECK(hipStreamSynchronize(aux));
  for (auto& [bytes, p] : blocks) RDL_HIP_CHECK(rdl::DevFree(p));
  return RDL_OK;
}

int rdl_session_destroy(rdl_session* s) {
  if (!s) return RDL_OK;
  if (rdl::ShutDown()) return RDL_OK;  // released by rdl_shutdown
  (void)hipSetDevice(s->device);
  if (s->aux) (void)hipStreamSynchronize(s->aux);
  s->stream = s->home;
  s->lane = 0;
  (void)hipStreamSynchronize(s->stream);
  (void)s->FlushCache();
  {
    const std::lock_guard<std::mutex> lock(rdl::g_registry_mutex);
    auto& v = rdl::g_sessions;
    v.erase(std::remove(v.begin(), v.end(), s), v.end());
    const std::lock_guard<std::recursive_mutex> tlock(s->timing_mutex);
    if (s->CollectTimings() == RDL_OK) rdl::Fold(rdl::g_retired, s->timings);
  }
  for (auto& [name, t] : s->timings)
    for (auto& [a, b] : t.pending) {
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
    }
  for (hipEvent_t e : s->event_pool) (void)hipEventDestroy(e);
  if (s->partials.ptr) (void)rdl::DevFree(s->partials.ptr);
  if (s->radix.ptr) (void)rdl::DevFree(s->radix.ptr);
  if (s->kernel.ptr) (void)rdl::DevFree(s->kernel.ptr);
  if (s->loop_state.ptr) (void)rdl::DevFree(s->loop_state.ptr);
  if (s->iuwt.ptr) (void)rdl::DevFree(s->iuwt.ptr);
  if (s->d_small) (void)rdl::DevFree(s->d_small);
  if (s->h_small) (void)rdl::HostFree(s->h_small);
  if (s->m_small) (void)rdl::HostFree(s->m_small);
  if (s->comm) rdl_comm_destroy(s);
  rdl::GiveStream(s->device, s->aux);
  if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
  if (s->ev_join) (void)hipEventDestroy(s->ev_join);
  rdl::GiveStream(s->device, s->home);
  delete s;
  return RDL_OK;
}

int rdl_shutdown(void) {
  bool expected = false;
  if (!rdl::g_shutdown.compare_exchange_strong(expected, true)) return RDL_OK;
  std::vector<rdl_session*> sessions;
  {
    const std::lock_guard<std::mutex> lock(rdl::g_registry_mutex);
    sessions.swap(rdl::g_sessions);
  }
  // drain every stream before anything is released
  for (rdl_session* s : sessions) {
    (void)hipSetDevice(s->device);
    if (s->aux) (void)hipStreamSynchronize(s->aux);
    (void)hipStreamSynchronize(s->home);
  }
  for (rdl_session* s : sessions) {
    (void)hipSetDevice(s->device);
    rdl::CommRelease(s);
    {
      const std::lock_guard<std::recursive_mutex> tlock(s->timing_mutex);
      for (auto& [name, t] : s->timings) {
        for (auto& [a, b] : t.pending) {
          (void)hipEventDestroy(a);
          (void)hipEventDestroy(b);
        }
        t.pending.clear();
      }
      for (hipEvent_t e : s->event_pool) (void)hipEventDestroy(e);
      s->event_pool.clear();
    }
    if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
    if (s->ev_join) (void)hipEventDestroy(s->ev_join);
    rdl::GiveStream(s->device, s->aux);
    rdl::GiveStream(s->device, s->home);
    s->ev_fork = s->ev_join = nullptr;
    s->aux = s->home = s->stream = nullptr;
    const std::lock_guard<std::mutex> clock(s->cache_mutex);
    s->cache_free.clear();
    s->cache_live.clear();
    s->cache_bytes = 0;
    // the session structs stay allocated (the host wrappers may still hold
    // them; every destroy/free entry point is a no-op from here on)
  }
  rdl::ReleaseFftPlans();
  rdl::DestroyStreamPools();
  // every device block, pinned and mapped host block this library holds:
  // the sessions' caches and scratch, plans' work buffers, sub-minor handles,
  // and the buffers of host objects that outlive the process's last call
  size_t n = 0;
  for (rdl::BlockSlot& b : rdl::g_blocks) {
    const uintptr_t p = b.base.load(std::memory_order_relaxed);
    if (!p) continue;
    const char kind = b.kind.load(std::memory_order_relaxed);
    b.base.store(0, std::memory_order_relaxed);
    b.bytes.store(0, std::memory_order_relaxed);
    b.kind.store(0, std::memory_order_relaxed);
    if (kind == 'h')
      (void)hipHostFree(reinterpret_cast<void*>(p));
    else
      (void)hipFree(reinterpret_cast<void*>(p));
    ++n;
  }
  if (const char* e = std::getenv("RDL_SHUTDOWN_LOG"); e && e[0] == '1')
    std::fprintf(stderr, "[rdl] shutdown: %zu sessions, %zu blocks released\n",
                 sessions.size(), n);
  return RDL_OK;
}

int rdl_session_fork(rdl_session* s) {
  RDL_ARG_CHECK(s, "session is NULL");
  RDL_ARG_CHECK(s->lane == 0, "fork from lane 1");
  if (!s->aux) {
    RDL_HIP_CHECK(hipSetDevice(s->device));
    RDL_TRY(rdl::TakeStream(s->device, &s->aux));
    RDL_HIP_CHECK(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
    RDL_HIP_CHECK(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming));
  }
  RDL_HIP_CHECK(hipEventRecord(s->ev_fork, s->home));
  RDL_HIP_CHECK(hipStreamWaitEvent(s->aux, s->ev_fork, 0));
  return RDL_OK;
}

int rdl_session_lane(rdl_session* s, int lane) {
  RDL_ARG_CHECK(s, "session is NULL");
  RDL_ARG_CHECK(lane == 0 || (lane == 1 && s->aux), "lane 1 needs rdl_session_fork");
  s->lane = lane;
  s->stream = lane ? s->aux : s->home;
  return RDL_OK;
}

int rdl_session_join(rdl_session* s) {
  RDL_ARG_CHECK(s, "session is NULL");
  s->lane = 0;
  s->stream = s->home;
  if (!s->aux) return RDL_OK;
  RDL_HIP_CHECK(hipEventRecord(s->ev_join, s->aux));
  RDL_HIP_CHECK(hipStreamWaitEvent(s->home, s->ev_join, 0));
  return RDL_OK;
}

int rdl_session_sync(rdl_session* s) {
  RDL_ARG_CHECK(s, "session is NULL");
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

void* rdl_session_stream(rdl_session* s) { return s ? s->stream : nullptr; }

int rdl_session_bind(rdl_session* s) {
  RDL_ARG_CHECK(s, "NULL session");
  RDL_HIP_CHECK(hipSetDevice(s->device));
  return RDL_OK;
}

int rdl_session_set_concurrency(rdl_session* s, uint32_t n_sharing) {
  RDL_ARG_CHECK(s, "NULL session");
  s->coop_limit =
      n_sharing <= 1 ? 0 : std::max<uint32_t>(1, uint32_t(s->n_cus) / n_sharing);
  return RDL_OK;
}

int rdl_malloc(rdl_session* s, size_t bytes, void** d_out) {
  RDL_ARG_CHECK(s && d_out, "NULL argument");
  *d_out = nullptr;
  if (bytes == 0) return RDL_OK;
  if (s->cache_on) {
    // best fit among cached blocks of at most 1.25x the request
    const std::lock_guard<std::mutex> lock(s->cache_mutex);
    auto it = s->cache_free.lower_bound(bytes);
    if (it != s->cache_free.end() && it->first <= bytes + bytes / 4) {
      *d_out = it->second;
      s->cache_bytes -= it->first;
      s->cache_live[it->second] = it->first;
      s->cache_free.erase(it);
    }
  }
  if (!*d_out) {
    int prev = 0;
    RDL_HIP_CHECK(hipGetDevice(&prev));
    if (prev != s->device) RDL_HIP_CHECK(hipSetDevice(s->device));
    hipError_t e = rdl::DevMalloc(d_out, bytes);
    if (e == hipErrorOutOfMemory) {
      // give back every cached block on this device (the main session's and
      // every worker's: a pool's sessions live for the process), then retry
      (void)hipGetLastError();
      RDL_TRY(rdl::FlushDeviceCaches(s->device));
      e = rdl::DevMalloc(d_out, bytes);
    }
    if (prev != s->device) (void)hipSetDevice(prev);
    RDL_HIP_CHECK(e);
    if (s->cache_on) {
      const std::lock_guard<std::mutex> lock(s->cache_mutex);
      s->cache_live[*d_out] = bytes;
    }
  }
  if (s->poison) {
    RDL_HIP_CHECK(hipMemsetAsync(*d_out, 0xff, bytes, s->stream));
    RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  }
  return RDL_OK;
}

// Blocks this session allocated go back to its cache (reused in stream order
// on the session's stream: every buffer is used on its owner's stream, or by
// other streams only between host synchronisations); anything else, and
// everything beyond the cache cap, is freed after the stream drains.
int rdl_free(rdl_session* s, void* d_ptr) {
  RDL_ARG_CHECK(s, "NULL session");
  if (!d_ptr || rdl::ShutDown()) return RDL_OK;
  if (s->cache_on) {
    const std::lock_guard<std::mutex> lock(s->cache_mutex);
    auto it = s->cache_live.find(d_ptr);
    if (it != s->cache_live.end()) {
      const size_t bytes = it->second;
      s->cache_live.erase(it);
      if (s->cache_bytes + bytes <= s->cache_cap) {
        s->cache_free.emplace(bytes, d_ptr);
        s->cache_bytes += bytes;
        return RDL_OK;
      }
    }
  }
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  RDL_HIP_CHECK(rdl::DevFree(d_ptr));
  return RDL_OK;
}

int rdl_memcpy_h2d(rdl_session* s, void* d_dst, const void* h_src,
                   size_t bytes) {
  RDL_ARG_CHECK(s, "NULL session");
  if (bytes == 0) return RDL_OK;
  RDL_HIP_CHECK(
      hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, s->stream));
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

int rdl_memcpy_d2h(rdl_session* s, void* h_dst, const void* d_src,
                   size_t bytes) {
  RDL_ARG_CHECK(s, "NULL session");
  if (bytes == 0) return RDL_OK;
  RDL_HIP_CHECK(
      hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, s->stream));
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  return RDL_OK;
}

int rdl_host_alloc(size_t bytes, void** h_out) {
  RDL_ARG_CHECK(h_out, "NULL argument");
  *h_out = nullptr;
  RDL_HIP_CHECK(rdl::HostMalloc(h_out, std::max<size_t>(bytes, 64)));
  return RDL_OK;
}

int rdl_host_free(void* h_ptr) {
  if (rdl::ShutDown()) return RDL_OK;
  if (h_ptr) RDL_HIP_CHECK(rdl::HostFree(h_ptr));
  return RDL_OK;
}

int rdl_memcpy_d2d(rdl_session* s, void* d_dst, const void* d_src,
                   size_t bytes) {
  RDL_ARG_CHECK(s, "NULL session");
  if (bytes == 0) return RDL_OK;
  RDL_HIP_CHECK(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice,
                               s->stream));
  return RDL_OK;
}

int rdl_memcpy_peer(rdl_session* s, void* d_dst, int dst_device,
                    const void* d_src, int src_device, size_t bytes) {
  RDL_ARG_CHECK(s, "NULL session");
  if (bytes == 0) return RDL_OK;
  if (dst_device == src_device)
    RDL_HIP_CHECK(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice,
                                 s->stream));
  else
    RDL_HIP_CHECK(hipMemcpyPeerAsync(d_dst, dst_device, d_src, src_device, bytes,
                                     s->stream));
  return RDL_OK;
}

int rdl_memset_zero(rdl_session* s, void* d_dst, size_t bytes) {
  RDL_ARG_CHECK(s, "NULL session");
  if (bytes == 0) return RDL_OK;
  RDL_HIP_CHECK(hipMemsetAsync(d_dst, 0, bytes, s->stream));
  return RDL_OK;
}

int rdl_timing_enable(rdl_session* s, int enable) {
  RDL_ARG_CHECK(s, "NULL session");
  s->timing = enable != 0;
  return RDL_OK;
}

int rdl_timing_get(rdl_session* s, const char* family, double* ms,
                   uint64_t* launches, double* bytes) {
  RDL_ARG_CHECK(s && family, "NULL argument");
  const std::lock_guard<std::recursive_mutex> lock(s->timing_mutex);
  RDL_TRY(s->CollectTimings());
  auto it = s->timings.find(family);
  if (it == s->timings.end()) {
    if (ms) *ms = 0.0;
    if (launches) *launches = 0;
    if (bytes) *bytes = 0.0;
    return RDL_OK;
  }
  if (ms) *ms = it->second.ms;
  if (launches) *launches = it->second.launches;
  if (bytes) *bytes = it->second.bytes;
  return RDL_OK;
}

int rdl_timing_reset(rdl_session* s) {
  RDL_ARG_CHECK(s, "NULL session");
  const std::lock_guard<std::recursive_mutex> lock(s->timing_mutex);
  RDL_TRY(s->CollectTimings());
  s->timings.clear();
  return RDL_OK;
}

int rdl_timing_filter_all(const char* family) {
  const std::lock_guard<std::mutex> lock(rdl::g_registry_mutex);
  std::memset(rdl::g_timing_family, 0, sizeof(rdl::g_timing_family));
  if (family) std::strncpy(rdl::g_timing_family, family, sizeof(rdl::g_timing_family) - 1);
  return RDL_OK;
}

int rdl_timing_enable_all(int enable) {
  rdl::g_timing_all.store(enable != 0, std::memory_order_relaxed);
  return RDL_OK;
}

int rdl_timing_get_all(const char* family, double* ms, uint64_t* launches,
                       double* bytes) {
  RDL_ARG_CHECK(family, "NULL family");
  const std::lock_guard<std::mutex> lock(rdl::g_registry_mutex);
  std::map<std::string, rdl::TimingEntry> total;
  rdl::Fold(total, rdl::g_retired);
  for (rdl_session* s : rdl::g_sessions) {
    const std::lock_guard<std::recursive_mutex> tlock(s->timing_mutex);
    RDL_TRY(s->CollectTimings());
    rdl::Fold(total, s->timings);
  }
  const auto it = total.find(family);
  const bool found = it != total.end();
  if (ms) *ms = found ? it->second.ms : 0.0;
  if (launches) *launches = found ? it->second.launches : 0;
  if (bytes) *bytes = found ? it->second.bytes : 0.0;
  return RDL_OK;
}

int rdl_timing_reset_all(void) {
  const std::lock_guard<std::mutex> lock(rdl::g_registry_mutex);
  rdl::g_retired.clear();
  for (rdl_session* s : rdl::g_sessions) {
    const std::lock_guard<std::recursive_mutex> tlock(s->timing_mutex);
    RDL_TRY(s->CollectTimings());
    s->timings.clear();
  }
  return RDL_OK;
}

}  // extern "C"
