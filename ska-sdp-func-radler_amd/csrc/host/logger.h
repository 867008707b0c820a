// Thin logger standing in for aocommon::Logger (the reference logs through
// it everywhere; cpp/logging/ forwards per-subimage logs). Quiet unless
// RADLER_VERBOSE is set or SetVerbosity(>0) is called.
#pragma once

#include <iostream>
#include <sstream>

namespace radler::log {

int Verbosity();
void SetVerbosity(int level);

class Line {
 public:
  explicit Line(int level) : on_(Verbosity() >= level) {}
  ~Line() {
    if (on_) std::cout << s_.str() << std::flush;
  }
  template <typename T>
  Line& operator<<(const T& v) {
    if (on_) s_ << v;
    return *this;
  }

 private:
  bool on_;
  std::ostringstream s_;
};

inline Line Info() { return Line(1); }
inline Line Debug() { return Line(2); }
inline Line Warn() { return Line(0); }

}  // namespace radler::log
