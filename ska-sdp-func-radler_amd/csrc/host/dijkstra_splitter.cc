#include "dijkstra_splitter.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <cmath>
#include <cstdint>
#include <limits>
#include <memory>
#include <queue>
#include <cstdlib>
#include <stdexcept>
#include <system_error>
#include <thread>

namespace radler::math {

namespace {

// The open list: libstdc++'s std::priority_queue algorithm (push_heap's
// sift-up, pop_heap's hole walk to a leaf then sift-up: bits/stl_heap.h) over
// the comparator "later first" (a.cost > b.cost, the reference's Visit
// order, dijkstra_splitter.h:24-29), restated on split arrays: the costs the
// comparisons read are packed 4 bytes apart and the payload (target and
// predecessor as (u, v), 8 bytes) moves alongside. The same comparisons and
// moves as the reference's queue, so equal costs pop in its order.
class OpenList {
 public:
  explicit OpenList(size_t reserve) {
    cost_.reserve(reserve);
    load_.reserve(reserve);
  }
  bool Empty() const { return cost_.empty(); }
  float TopCost() const { return cost_[0]; }
  uint64_t TopLoad() const { return load_[0]; }
  void Push(float c, uint64_t l) {
    cost_.push_back(c);
    load_.push_back(l);
    SiftUp(cost_.size() - 1, 0, c, l);
  }
  void Pop() {
    const size_t last = cost_.size() - 1;
    const float vc = cost_[last];
    const uint64_t vl = load_[last];
    cost_[last] = cost_[0];
    load_[last] = load_[0];
    // __adjust_heap(first, 0, len = last, value)
    const size_t len = last;
    size_t hole = 0, child = 0;
    while (len > 0 && child < (len - 1) / 2) {
      child = 2 * (child + 1);
      if (cost_[child] > cost_[child - 1]) --child;  // comp(child, child - 1)
      cost_[hole] = cost_[child];
      load_[hole] = load_[child];
      hole = child;
    }
    if (len > 0 && (len & 1) == 0 && child == (len - 2) / 2) {
      child = 2 * (child + 1);
      cost_[hole] = cost_[child - 1];
      load_[hole] = load_[child - 1];
      hole = child - 1;
    }
    SiftUp(hole, 0, vc, vl);
    cost_.pop_back();
    load_.pop_back();
  }

 private:
  // __push_heap(first, hole, top, value): while comp(parent, value)
  void SiftUp(size_t hole, size_t top, float c, uint64_t l) {
    size_t parent = (hole - 1) / 2;
    while (hole > top && cost_[parent] > c) {
      cost_[hole] = cost_[parent];
      load_[hole] = load_[parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    cost_[hole] = c;
    load_[hole] = l;
  }
  std::vector<float> cost_;
  std::vector<uint64_t> load_;
};

// The same heap on one array of 8-byte items (cost bits << 32 | payload):
// the comparisons read only the cost half, so equal costs pop exactly as in
// OpenList (the pushed costs are finite and non-negative, where the float
// order and the bit order agree), and a comparison and its move touch one
// cache line instead of two. The pop's walk to a leaf takes two levels a
// round with the grandchildren prefetched.
class PackedOpenList {
 public:
  explicit PackedOpenList(size_t reserve) : item_(std::max<size_t>(reserve, 64)) {}
  bool Empty() const { return n_ == 0; }
  uint64_t Top() const { return item_[0]; }
  void Push(uint64_t x) {
    if (n_ == item_.size()) item_.resize(2 * n_);
    uint64_t* a = item_.data();
    size_t hole = n_++;
    const uint32_t c = Key(x);
    while (hole > 0) {  // __push_heap
      const size_t parent = (hole - 1) / 2;
      if (!(Key(a[parent]) > c)) break;
      a[hole] = a[parent];
      hole = parent;
    }
    a[hole] = x;
  }
  void Pop() {
    const size_t len = --n_;
    uint64_t* a = item_.data();
    const uint64_t v = a[len];
    size_t hole = 0, child = 0;
    if (len > 2) {  // __adjust_heap: the hole walks to a leaf
      const size_t lim = (len - 1) / 2;
      while (child < lim) {
        const size_t c0 = 2 * child + 1;
        __builtin_prefetch(a + 2 * c0 + 1);
        child = c0 + 1 - (Key(a[c0 + 1]) > Key(a[c0]));
        a[hole] = a[child];
        hole = child;
        if (!(child < lim)) break;
        const size_t d0 = 2 * child + 1;
        child = d0 + 1 - (Key(a[d0 + 1]) > Key(a[d0]));
        a[hole] = a[child];
        hole = child;
      }
    }
    if (len > 0 && (len & 1) == 0 && child == (len - 2) / 2) {
      child = 2 * child + 2;
      a[hole] = a[child - 1];
      hole = child - 1;
    }
    const uint32_t c = Key(v);
    while (hole > 0) {  // __push_heap of the former last item
      const size_t parent = (hole - 1) / 2;
      if (!(Key(a[parent]) > c)) break;
      a[hole] = a[parent];
      hole = parent;
    }
    a[hole] = v;
  }

 private:
  static uint32_t Key(uint64_t x) { return uint32_t(x >> 32); }
  std::vector<uint64_t> item_;
  size_t n_ = 0;
};

// payload: target (u, v) and predecessor (pu, pv), 16 bits each
inline uint64_t Load(uint32_t u, uint32_t v, uint32_t pu, uint32_t pv) {
  return uint64_t(u) | (uint64_t(v) << 16) | (uint64_t(pu) << 32) | (uint64_t(pv) << 48);
}


// The radix heap of a monotone search (keys never below the last popped one):
// non-negative float keys compare as their bit patterns, bucket b holds the
// keys whose highest bit differing from the last popped key is bit b - 1.
// Items are (key << 32 | payload) words. Pops come in key order; equal keys
// in no particular order.
class RadixQueue {
 public:
  bool Empty() const { return size_ == 0; }
  void Push(uint64_t item) {
    bucket_[Bucket(uint32_t(item >> 32))].push_back(item);
    ++size_;
  }
  uint64_t Pop() {  // the queue must not be empty
    if (bucket_[0].empty()) {
      size_t b = 1;
      while (bucket_[b].empty()) ++b;
      uint64_t lowest = UINT64_MAX;
      for (uint64_t it : bucket_[b]) lowest = std::min(lowest, it);
      last_ = uint32_t(lowest >> 32);
      for (uint64_t it : bucket_[b]) bucket_[Bucket(uint32_t(it >> 32))].push_back(it);
      bucket_[b].clear();
    }
    const uint64_t item = bucket_[0].back();
    bucket_[0].pop_back();
    --size_;
    return item;
  }

 private:
  size_t Bucket(uint32_t key) const {
    return key == last_ ? 0 : size_t(32 - __builtin_clz(key ^ last_));
  }
  std::vector<uint64_t> bucket_[33];
  uint32_t last_ = 0;
  size_t size_ = 0;
};

inline uint32_t KeyBits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}
inline float KeyFloat(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

std::atomic<uint64_t> g_fast_divides{0}, g_exact_divides{0}, g_hybrid_divides{0};

enum : uint32_t {  // predecessor of target (u, v)
  kFromUpNext = 0,   // (u - 1, v + 1)
  kFromNext = 1,     // (u, v + 1)
  kFromUp = 2,       // (u - 1, v)
  kFromUpPrev = 3,   // (u - 1, v - 1)
  kFromPrev = 4,     // (u, v - 1)
  kFromStart = 5,    // (u, v) itself
};

// band-local index of the predecessor a code names
inline size_t PredOf(size_t at, uint32_t code, size_t band) {
  switch (code) {
    case kFromUpNext: return at - band + 1;
    case kFromNext: return at + 1;
    case kFromUp: return at - band;
    case kFromUpPrev: return at - band - 1;
    case kFromPrev: return at - 1;
    default: return at;
  }
}

// A prefix of the exact search that a key-order search can use (the race
// in DijkstraSplitter::Divide): when the key-order divider is decided by ties
// only at pixels settled at keys <= k (see DivideByKeyOrder), the exact
// search is stopped once every entry of key <= k has popped (stop_key = the
// bits of k), and its predecessor codes for those pixels complete the
// divider: above k the key-order search's predecessors are the unique ones.
}  // namespace

struct DivideReplay {
  std::atomic<uint32_t> stop_key{UINT32_MAX};
  std::atomic<int> stopped{0};  // the exact search stopped at stop_key (back is valid there)
  std::atomic<int> done{0};     // the exact search has returned (any way)
  std::unique_ptr<uint8_t[]> back;
};

namespace {

// The reference's search visits pixels in key order (the key of an entry is
// its predecessor's path cost) and keeps, per pixel, the predecessor of the
// first entry popped; only entries with EQUAL keys to the same pixel pop in
// an order that depends on the heap's history. This search settles the same
// pixels at the same costs in key order with any tie order (a radix heap),
// and marks every pixel that a second entry reaches with its settling key.
// The divider it traces is the reference's when no pixel whose predecessor
// the trace reads is marked, none was settled at the final key, and no other
// last-row pixel ends at the final cost: then every predecessor on the path
// and the end pixel are the unique minimum, whatever the pop order among
// equal keys. With `replay` (the exact search running alongside), a path
// whose first marked pixel from the end was settled at key k < the final key
// is completed from the exact search stopped after key k: keys never rise
// along the path towards its start, so every predecessor the trace reads
// from there on is final in that prefix. Returns false (output untouched)
// when neither applies, or when the exact search finished first.
template <bool kVertical>
bool DivideByKeyOrder(const float* image, float* output, size_t width, size_t height,
                      size_t lo, size_t hi, std::atomic<int>* race, DivideReplay* replay = nullptr) {
  const size_t n_u = kVertical ? height : width;
  const size_t band = hi - lo;
  auto pixel = [&](size_t u, size_t v) -> size_t {
    return kVertical ? u * width + v : v * width + u;
  };
  const float unset = std::numeric_limits<float>::max();
  // key_of and back are written when a pixel settles, before any read
  std::unique_ptr<float[]> weight(new float[band * n_u]), key_of(new float[band * n_u]);
  std::unique_ptr<uint32_t[]> back(new uint32_t[band * n_u]);
  std::vector<float> dist(band * n_u, unset);
  std::vector<uint8_t> tied(band * n_u, 0);
  for (size_t u = 0; u != n_u; ++u)
    for (size_t v = lo; v != hi; ++v) weight[u * band + (v - lo)] = std::fabs(image[pixel(u, v)]);
  // The queue holds settled pixels, keyed by their cost: popping one at key
  // k pops, in the reference's terms, its (up to five) entries of key k;
  // every entry of a smaller key has been popped, so a target still
  // unsettled settles at k, and a settled one reached at its own settling
  // key is a tie. Payload: the pixel as u << vbits | v - lo.
  unsigned vbits = 1, ubits = 1;
  while ((size_t(1) << vbits) < band) ++vbits;
  while ((size_t(1) << ubits) <= n_u) ++ubits;
  if (ubits + vbits > 32) return false;
  const uint32_t vmask = (1u << vbits) - 1;
  RadixQueue open;
  // settle (u, v) from (pu, pv) at key k, or mark the tie
  auto reach = [&](uint32_t k, uint32_t u, uint32_t v, uint32_t pu, uint32_t pv) {
    const size_t at = size_t(u) * band + (v - lo);
    if (dist[at] != unset) {
      if (KeyBits(key_of[at]) == k) tied[at] = 1;
      return;
    }
    const float cost = KeyFloat(k) + weight[at];
    if (!(cost < unset)) return;  // NaN / inf: never settles (as there)
    dist[at] = cost;
    key_of[at] = KeyFloat(k);
    back[at] = (pu << 16) | pv;
    open.Push((uint64_t(KeyBits(cost)) << 32) | (u << vbits) | (v - uint32_t(lo)));
  };
  for (size_t v = lo; v != hi; ++v) reach(0u, 0, uint32_t(v), 0, uint32_t(v));
  uint32_t end_key = 0, end_pu = 0, end_pv = 0;
  bool ended = false;
  while (!open.Empty()) {
    const uint64_t top = open.Pop();
    const uint32_t k = uint32_t(top >> 32);
    if (ended && k != end_key) break;  // drained the final key
    const uint32_t cu = uint32_t(top) >> vbits, cv = (uint32_t(top) & vmask) + uint32_t(lo);
    const uint32_t u1 = cu + 1;
    if (u1 == n_u) {  // its entries past the last row end the search
      if (!ended) {
        ended = true;
        end_key = k;
        end_pu = cu;
        end_pv = cv;
      }
      if (cv > lo) reach(k, cu, cv - 1, cu, cv);
      if (cv + 1u < hi) reach(k, cu, cv + 1, cu, cv);
      continue;
    }
    if (cv > lo) {
      reach(k, u1, cv - 1, cu, cv);
      reach(k, cu, cv - 1, cu, cv);
    }
    reach(k, u1, cv, cu, cv);
    if (cv + 1u < hi) {
      reach(k, u1, cv + 1, cu, cv);
      reach(k, cu, cv + 1, cu, cv);
    }
  }
  if (!ended) return false;
  // another last-row pixel at the final cost: the end is a tie
  const size_t last = (n_u - 1) * band;
  for (size_t v = 0; v != band; ++v)
    if (v + lo != end_pv && KeyBits(dist[last + v]) == end_key) return false;
  // the first marked pixel from the end (keys only fall towards the start)
  uint32_t split_key = UINT32_MAX;
  for (uint32_t pu = end_pu, pv = end_pv; pu > 0;) {
    const size_t at = size_t(pu) * band + (pv - lo);
    if (KeyBits(key_of[at]) >= end_key) return false;
    if (tied[at]) {
      if (!replay) return false;
      split_key = KeyBits(key_of[at]);
      break;
    }
    pu = back[at] >> 16;
    pv = back[at] & 0xffffu;
  }
  if (split_key != UINT32_MAX) {
    // the exact search's prefix up to split_key decides the rest
    replay->stop_key.store(split_key, std::memory_order_release);
    // (sleeping, not spinning: the exact searches of other bands may need
    // this core)
    while (!replay->done.load(std::memory_order_acquire))
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (!replay->stopped.load(std::memory_order_acquire)) return false;  // it finished first
  }
  // racing the exact search: the first to claim the band writes it (the
  // two dividers are then identical)
  int running = 0;
  if (race && !race->compare_exchange_strong(running, split_key == UINT32_MAX ? 1 : 3))
    return split_key == UINT32_MAX;
  for (size_t u = 0; u != n_u; ++u)
    for (size_t v = lo; v != hi; ++v) output[pixel(u, v)] = 0.0f;
  size_t at = size_t(end_pu) * band + (end_pv - lo);
  while (at >= band) {  // u > 0
    output[pixel(at / band, at % band + lo)] = 1.0f;
    if (KeyBits(key_of[at]) > split_key || split_key == UINT32_MAX) {
      const uint32_t p = back[at];
      at = size_t(p >> 16) * band + ((p & 0xffffu) - lo);
    } else {
      at = PredOf(at, replay->back[at], band);
    }
  }
  output[pixel(0, at + lo)] = 1.0f;
  return true;
}

// The reference's search (dijkstra_splitter.cc:34-86 / :88-142) with its
// heap's exact pop order, on PackedOpenList. An entry's payload is its
// target as a band-local index (u * band + v - lo; u = n_u past the last
// row) times 8 plus a code for the predecessor, which is always the target
// itself (a start entry) or one of five neighbours; the settled pixels keep
// the code (one byte) instead of the predecessor's coordinates. Needs
// (n_u + 1) * band < 2^29; false (output untouched) otherwise.
template <bool kVertical>
bool DivideExactPacked(const float* image, float* output, size_t width, size_t height,
                       size_t lo, size_t hi, std::atomic<int>* race, DivideReplay* replay) {
  const size_t n_u = kVertical ? height : width;
  const size_t band = hi - lo;
  if (band == 0 || (n_u + 1) * band >= (size_t(1) << 29)) return false;
  auto pixel = [&](size_t u, size_t v) -> size_t {
    return kVertical ? u * width + v : v * width + u;
  };
  std::vector<float> weight(band * n_u);
  std::vector<float> dist(band * n_u, std::numeric_limits<float>::max());
  for (size_t u = 0; u != n_u; ++u)
    for (size_t v = lo; v != hi; ++v) weight[u * band + (v - lo)] = std::fabs(image[pixel(u, v)]);
  // predecessor codes, written when a pixel settles (the replay's own
  // array when a key-order search may read a prefix of them)
  std::unique_ptr<uint8_t[]> own;
  if (!replay) own.reset(new uint8_t[band * n_u]);
  uint8_t* const back = replay ? replay->back.get() : own.get();
  PackedOpenList open(8 * band);
  for (size_t v = 0; v != band; ++v) open.Push(uint64_t(v) << 3 | kFromStart);
  const size_t n_settle = n_u * band;
  // the last entry popped: its predecessor starts the trace (the entry past
  // the last row, or, when none gets there, the last one the queue held)
  size_t end_at = 0;
  uint32_t end_code = kFromStart;
  for (uint32_t poll = 0; !open.Empty();) {
    if (race && ++poll == 0x1000u) {  // cancelled by a key-order result
      poll = 0;
      if (race->load(std::memory_order_relaxed) == 1) return true;
      // or stopped after the prefix a key-order divider needs
      if (replay && uint32_t(open.Top() >> 32) > replay->stop_key.load(std::memory_order_acquire)) {
        replay->stopped.store(1, std::memory_order_release);
        return true;
      }
    }
    const uint64_t top = open.Top();
    open.Pop();
    const size_t at = size_t(uint32_t(top) >> 3);
    const uint32_t code = uint32_t(top) & 7u;
    end_at = at;
    end_code = code;
    if (at >= n_settle) break;  // an entry past the last row ends the search
    const float cost = KeyFloat(uint32_t(top >> 32)) + weight[at];
    if (!(cost < dist[at])) continue;
    dist[at] = cost;
    back[at] = uint8_t(code);
    const uint64_t key = uint64_t(KeyBits(cost)) << 32;
    const size_t v = at % band;
    const uint64_t down = uint64_t(at + band) << 3;
    if (v > 0) {
      open.Push(key | (down - 8) | kFromUpNext);
      open.Push(key | (uint64_t(at - 1) << 3) | kFromNext);
    }
    open.Push(key | down | kFromUp);
    if (v + 1 < band) {
      open.Push(key | (down + 8) | kFromUpPrev);
      open.Push(key | (uint64_t(at + 1) << 3) | kFromPrev);
    }
  }
  int running = 0;
  if (race && !race->compare_exchange_strong(running, 2)) return true;
  for (size_t u = 0; u != n_u; ++u)
    for (size_t v = lo; v != hi; ++v) output[pixel(u, v)] = 0.0f;
  size_t p = PredOf(end_at, end_code, band);
  for (; p >= band; p = PredOf(p, back[p], band)) output[pixel(p / band, p % band + lo)] = 1.0f;
  output[pixel(0, p + lo)] = 1.0f;
  return true;
}

}  // namespace

DivideStats DijkstraSplitter::Stats() {
  return {g_fast_divides.load(), g_exact_divides.load(), g_hybrid_divides.load()};
}

template <bool kVertical>
void DijkstraSplitter::Divide(const float* image, float* output, size_t lo,
                              size_t hi) const {
  if (width_ >= 65535 || height_ >= 65535)
    throw std::runtime_error("DijkstraSplitter: image side of 65535 pixels or more");
  static const bool exact_only = [] {
    const char* e = std::getenv("RDL_SPLIT_EXACT");
    return e && e[0] == '1';
  }();
  static const bool race_on = [] {
    const char* e = std::getenv("RDL_SPLIT_RACE");
    return !(e && e[0] == '0');
  }();
  if (exact_only) {
    ++g_exact_divides;
    DivideExact<kVertical>(image, output, lo, hi, nullptr);
    return;
  }
  if (!race_on) {
    if (DivideByKeyOrder<kVertical>(image, output, width_, height_, lo, hi, nullptr)) {
      ++g_fast_divides;
      return;
    }
    ++g_exact_divides;
    DivideExact<kVertical>(image, output, lo, hi, nullptr);
    return;
  }
  // Race: the exact search runs on its own thread from the start; a
  // key-order result (about a fifth of its time) cancels it, else it
  // finishes. The divider costs max(key order, exact) at worst instead of
  // their sum.
  // 0 running, 1 key order wrote, 2 exact wrote, 3 key order wrote with the
  // exact search's prefix (DivideReplay)
  std::atomic<int> race{0};
  // the replay prefix only exists for bands the packed exact search holds
  // (the OpenList fallback never honours stop_key)
  const size_t n_u = kVertical ? height_ : width_;
  const bool packed = hi > lo && (n_u + 1) * (hi - lo) < (size_t(1) << 29);
  DivideReplay replay;
  if (packed) replay.back.reset(new uint8_t[(hi - lo) * n_u]);
  DivideReplay* const with_replay = packed ? &replay : nullptr;
  std::exception_ptr exact_error;
  std::thread exact;
  try {
    exact = std::thread([&] {
      try {
        DivideExact<kVertical>(image, output, lo, hi, &race, with_replay);
      } catch (...) {
        exact_error = std::current_exception();
      }
      replay.done.store(1, std::memory_order_release);
    });
  } catch (const std::system_error&) {
    // no thread to be had: the two searches in turn
    if (DivideByKeyOrder<kVertical>(image, output, width_, height_, lo, hi, nullptr)) {
      ++g_fast_divides;
      return;
    }
    ++g_exact_divides;
    DivideExact<kVertical>(image, output, lo, hi, nullptr);
    return;
  }
  try {
    (void)DivideByKeyOrder<kVertical>(image, output, width_, height_, lo, hi, &race,
                                      with_replay);
  } catch (...) {
    // the exact search still decides
  }
  exact.join();
  // the search that claimed the band wrote it (DivideByKeyOrder also returns
  // true when it lost the claim to an exact result)
  const int writer = race.load();
  if (writer != 1 && exact_error) std::rethrow_exception(exact_error);
  if (writer == 0)
    throw std::logic_error("DijkstraSplitter: neither divider search wrote the band");
  ++(writer == 1 ? g_fast_divides : writer == 3 ? g_hybrid_divides : g_exact_divides);
}

template <bool kVertical>
void DijkstraSplitter::DivideExact(const float* image, float* output, size_t lo,
                                   size_t hi, std::atomic<int>* race,
                                   DivideReplay* replay) const {
  if (DivideExactPacked<kVertical>(image, output, width_, height_, lo, hi, race, replay)) return;
  // (bands of 2^29 pixels or more) the same search on OpenList
  const size_t n_u = kVertical ? height_ : width_;  // path length axis
  const size_t band = hi - lo;
  auto pixel = [&](size_t u, size_t v) -> size_t {
    return kVertical ? u * width_ + v : v * width_ + u;
  };
  // the search runs on band-local copies laid out [u][v - lo] (|pixel| and
  // the settled costs): the frontier then walks neighbouring cache lines
  // instead of image rows a full width apart (a horizontal band is
  // transposed). Same pushes and pops in the same order, same result.
  std::vector<float> weight(band * n_u);
  std::vector<float> dist(band * n_u, std::numeric_limits<float>::max());
  for (size_t u = 0; u != n_u; ++u)
    for (size_t v = lo; v != hi; ++v) weight[u * band + (v - lo)] = std::fabs(image[pixel(u, v)]);
  OpenList open(8 * band);
  for (size_t v = lo; v != hi; ++v) open.Push(0.0f, Load(0, uint32_t(v), 0, uint32_t(v)));
  // predecessor of each settled pixel (pu << 16 | pv), band-local layout
  std::vector<uint32_t> back(band * n_u);
  uint32_t end_pu = 0, end_pv = 0;
  for (uint32_t poll = 0; !open.Empty();) {
    if (race && ++poll == 0x1000u) {  // cancelled by a key-order result
      poll = 0;
      if (race->load(std::memory_order_relaxed) == 1) return;
    }
    const float top_cost = open.TopCost();
    const uint64_t top = open.TopLoad();
    open.Pop();
    const uint32_t cu = uint32_t(top & 0xffffu), cv = uint32_t((top >> 16) & 0xffffu);
    end_pu = uint32_t((top >> 32) & 0xffffu);
    end_pv = uint32_t(top >> 48);
    if (cu == n_u) break;
    const size_t at = size_t(cu) * band + (cv - lo);
    const float cost = top_cost + weight[at];
    if (!(cost < dist[at])) continue;
    dist[at] = cost;
    back[at] = (end_pu << 16) | end_pv;
    const uint32_t u1 = cu + 1;
    if (cv > lo) {
      open.Push(cost, Load(u1, cv - 1, cu, cv));
      open.Push(cost, Load(cu, cv - 1, cu, cv));
    }
    open.Push(cost, Load(u1, cv, cu, cv));
    if (cv + 1u < hi) {
      open.Push(cost, Load(u1, cv + 1, cu, cv));
      open.Push(cost, Load(cu, cv + 1, cu, cv));
    }
  }
  int running = 0;
  if (race && !race->compare_exchange_strong(running, 2)) return;
  for (size_t u = 0; u != n_u; ++u)
    for (size_t v = lo; v != hi; ++v) output[pixel(u, v)] = 0.0f;
  uint32_t pu = end_pu, pv = end_pv;
  for (; pu > 0;) {
    output[pixel(pu, pv)] = 1.0f;
    const uint32_t p = back[size_t(pu) * band + (pv - lo)];
    pu = p >> 16;
    pv = p & 0xffffu;
  }
  output[pixel(0, pv)] = 1.0f;
}

void DijkstraSplitter::AddVerticalDivider(const float* image, float* scratch,
                                          float* output, size_t x1, size_t x2) const {
  DivideVertically(image, scratch, x1, x2);
  for (size_t y = 0; y != height_; ++y)
    for (size_t i = y * width_ + x1; i != y * width_ + x2; ++i) output[i] += scratch[i];
}

void DijkstraSplitter::AddHorizontalDivider(const float* image, float* scratch,
                                            float* output, size_t y1, size_t y2) const {
  DivideHorizontally(image, scratch, y1, y2);
  for (size_t i = y1 * width_; i != y2 * width_; ++i) output[i] += scratch[i];
}

void DijkstraSplitter::DivideVertically(const float* image, float* output,
                                        size_t x1, size_t x2) const {
  Divide<true>(image, output, x1, x2);
}

void DijkstraSplitter::DivideHorizontally(const float* image, float* output,
                                          size_t y1, size_t y2) const {
  Divide<false>(image, output, y1, y2);
}

void DijkstraSplitter::FloodVerticalArea(const float* subdivision,
                                         size_t subimage_x, bool* mask, size_t& x,
                                         size_t& subwidth) const {
  std::fill(mask, mask + width_ * height_, false);
  size_t left = width_, right = 0;
  for (size_t y = 0; y != height_; ++y) {
    const float* row = subdivision + y * width_;
    bool* mrow = mask + y * width_;
    int64_t i = int64_t(subimage_x);
    for (; i >= 0 && row[i] == 0.0f; --i) mrow[i] = true;  // up to the border
    for (; i >= 0 && row[i] != 0.0f; --i) mrow[i] = true;  // and through it
    left = std::min(left, size_t(i + 1));
    i = int64_t(subimage_x) + 1;
    for (; size_t(i) < width_ && row[i] == 0.0f; ++i) mrow[i] = true;
    right = std::max(right, size_t(i));
  }
  x = left;
  subwidth = right < left ? 0 : right - left;
}

void DijkstraSplitter::FloodHorizontalArea(const float* subdivision,
                                           size_t subimage_y, bool* mask,
                                           size_t& y, size_t& subheight) const {
  std::fill(mask, mask + width_ * height_, false);
  size_t top = height_, bottom = 0;
  for (size_t x = 0; x != width_; ++x) {
    int64_t i = int64_t(subimage_y);
    for (; i >= 0 && subdivision[i * width_ + x] == 0.0f; --i)
      mask[i * width_ + x] = true;
    for (; i >= 0 && subdivision[i * width_ + x] != 0.0f; --i)
      mask[i * width_ + x] = true;
    top = std::min(top, size_t(i + 1));
    i = int64_t(subimage_y) + 1;
    for (; size_t(i) < height_ && subdivision[i * width_ + x] == 0.0f; ++i)
      mask[i * width_ + x] = true;
    bottom = std::max(bottom, size_t(i));
  }
  y = top;
  subheight = bottom < top ? 0 : bottom - top;
}

void DijkstraSplitter::GetBoundingMask(const bool* vertical_mask,
                                       size_t vertical_mask_x,
                                       size_t vertical_mask_width,
                                       const bool* horizontal_mask, bool* mask,
                                       size_t& sub_x, size_t& sub_y,
                                       size_t& subwidth, size_t& subheight) const {
  size_t x_lo = vertical_mask_width + vertical_mask_x, y_lo = height_;
  size_t x_hi = 0, y_hi = 0;
  for (size_t y = 0; y != height_; ++y) {
    for (size_t x = 0; x != vertical_mask_width; ++x) {
      const size_t gx = x + vertical_mask_x;
      const bool inside = vertical_mask[y * vertical_mask_width + x] &&
                          horizontal_mask[y * width_ + gx];
      mask[y * width_ + gx] = inside;
      if (inside) {
        x_lo = std::min(x_lo, gx);
        x_hi = std::max(x_hi, gx);
        y_lo = std::min(y_lo, y);
        y_hi = y;
      }
    }
  }
  if (x_hi < x_lo) {
    subwidth = subheight = 0;
  } else {
    subwidth = x_hi + 1 - x_lo;
    subheight = y_hi + 1 - y_lo;
  }
  // even images keep even subimages: grow by one column/row (to the left/top
  // when the right/bottom edge would leave the image) that is masked out
  if (width_ % 2 == 0 && subwidth % 2 != 0) {
    ++subwidth;
    size_t col;
    if (subwidth + x_lo >= width_)
      col = --x_lo;
    else
      col = x_lo + subwidth - 1;
    for (size_t y = y_lo; y != y_lo + subheight; ++y) mask[col + y * width_] = false;
  }
  if (height_ % 2 == 0 && subheight % 2 != 0) {
    ++subheight;
    size_t row;
    if (subheight + y_lo >= height_)
      row = --y_lo;
    else
      row = y_lo + subheight - 1;
    std::fill_n(mask + row * width_ + x_lo, subwidth, false);
  }
  sub_x = x_lo;
  sub_y = y_lo;
}

}  // namespace radler::math
