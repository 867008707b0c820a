#include "host_profile.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

namespace radler::prof {
namespace {
struct Store {
  std::mutex mutex;
  std::map<std::string, std::pair<uint64_t, uint64_t>> sections;
  ~Store() {
    if (!Enabled() || sections.empty()) return;
    std::vector<Entry> v;
    for (const auto& [name, cn] : sections) v.push_back({name, cn.first, cn.second});
    std::sort(v.begin(), v.end(), [](const Entry& a, const Entry& b) { return a.ns > b.ns; });
    std::fprintf(stderr, "[host-profile] %-34s %10s %12s %10s\n", "section", "count",
                 "total ms", "avg us");
    for (const Entry& e : v)
      std::fprintf(stderr, "[host-profile] %-34s %10llu %12.2f %10.2f\n", e.name.c_str(),
                   (unsigned long long)e.count, e.ns * 1e-6,
                   e.count ? e.ns * 1e-3 / e.count : 0.0);
  }
};
Store& TheStore() {
  static Store s;
  return s;
}
}  // namespace

std::atomic<bool>& Flag() {
  static std::atomic<bool> on{[] {
    const char* e = std::getenv("RADLER_HOST_PROFILE");
    return e && e[0] == '1';
  }()};
  return on;
}

bool Enabled() { return Flag().load(std::memory_order_relaxed); }

void SetEnabled(bool on) { Flag().store(on, std::memory_order_relaxed); }

void Add(const char* name, uint64_t ns) {
  Store& s = TheStore();
  const std::lock_guard<std::mutex> lock(s.mutex);
  auto& e = s.sections[name];
  ++e.first;
  e.second += ns;
}

std::vector<Entry> Snapshot() {
  Store& s = TheStore();
  const std::lock_guard<std::mutex> lock(s.mutex);
  std::vector<Entry> v;
  for (const auto& [name, cn] : s.sections) v.push_back({name, cn.first, cn.second});
  return v;
}

void Reset() {
  Store& s = TheStore();
  const std::lock_guard<std::mutex> lock(s.mutex);
  s.sections.clear();
}

}  // namespace radler::prof
