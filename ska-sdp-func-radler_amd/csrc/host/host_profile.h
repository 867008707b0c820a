// Host-side wall-clock sections (RADLER_HOST_PROFILE=1): where a major
// iteration's host time goes — device waits (syncs, blocking copies),
// allocations and the algorithm's phases. Printed to stderr at process exit,
// or read with radler.gpu.host_profile(). Off by default: one getenv check.
#pragma once

#include <chrono>
#include <cstdint>
#include <string>
#include <vector>

namespace radler::prof {

bool Enabled();
/// Turns the sections on or off at run time (bench.py's reference legs).
void SetEnabled(bool on);
void Add(const char* name, uint64_t ns);
struct Entry {
  std::string name;
  uint64_t count, ns;
};
std::vector<Entry> Snapshot();
void Reset();

class Section {
 public:
  explicit Section(const char* name)
      : name_(Enabled() ? name : nullptr),
        t0_(name_ ? std::chrono::steady_clock::now()
                  : std::chrono::steady_clock::time_point()) {}
  ~Section() {
    if (name_)
      Add(name_, uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0_)
                              .count()));
  }
  Section(const Section&) = delete;
  Section& operator=(const Section&) = delete;

 private:
  const char* name_;
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace radler::prof
