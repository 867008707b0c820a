// radler::PsfOffset (reference: cpp/psf_offset.h:10-31).
#pragma once

#include <cstddef>
#include <ostream>

namespace radler {

class PsfOffset {
 public:
  PsfOffset() = default;
  explicit PsfOffset(size_t x_offset, size_t y_offset) : x(x_offset), y(y_offset) {}
  /// Offset in pixels from the corner position.
  size_t x{0};
  size_t y{0};
  friend std::ostream& operator<<(std::ostream& out, const PsfOffset& p) {
    return out << "[x: " << p.x << ", y: " << p.y << ']';
  }
};

}  // namespace radler
