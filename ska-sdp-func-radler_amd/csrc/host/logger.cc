#include "logger.h"

#include <atomic>
#include <cstdlib>

namespace radler::log {
namespace {
std::atomic<int> g_level{-1};
}
int Verbosity() {
  int v = g_level.load();
  if (v < 0) {
    const char* e = std::getenv("RADLER_VERBOSE");
    v = e ? std::atoi(e) : 0;
    g_level.store(v);
  }
  return v;
}
void SetVerbosity(int level) { g_level.store(level); }
}  // namespace radler::log
