// radler::math::DijkstraSplitter (reference: cpp/math/dijkstra_splitter.{h,cc}):
// minimum-|flux| paths that split the integrated image into subimages for
// ParallelDeconvolution. Runs on the host (a priority-queue search, not
// data-parallel); the image comes from the device once per major iteration.
#pragma once

#include <atomic>
#include <cstddef>
#include <vector>

namespace radler::math {

/// Divider searches so far (process-wide): settled by the key-order search
/// with a unique minimum path, run through the reference's heap order, or
/// the key-order path completed from a prefix of that heap order (ties only
/// below some key; DivideReplay).
struct DivideStats {
  unsigned long long key_order, exact, hybrid;
};

struct DivideReplay;  // a prefix of the exact search shared with the key-order search

class DijkstraSplitter {
 public:
  DijkstraSplitter(size_t width, size_t height) : width_(width), height_(height) {}

  /// Process-wide counts of the two divider searches (see Divide).
  static DivideStats Stats();

  /// Shortest top-to-bottom path of sum |image| inside columns [x1, x2);
  /// output (a width x height plane) gets 1 on the path, 0 elsewhere in the
  /// band, untouched outside it (dijkstra_splitter.cc:32-84).
  void DivideVertically(const float* image, float* output, size_t x1,
                        size_t x2) const;
  /// DivideVertically into `scratch`, then output += scratch over the band
  /// (dijkstra_splitter.cc:14-23).
  void AddVerticalDivider(const float* image, float* scratch, float* output,
                          size_t x1, size_t x2) const;
  /// The same for a horizontal divider (dijkstra_splitter.cc:25-32).
  void AddHorizontalDivider(const float* image, float* scratch, float* output,
                            size_t y1, size_t y2) const;
  /// Left-to-right path inside rows [y1, y2) (dijkstra_splitter.cc:86-136).
  void DivideHorizontally(const float* image, float* output, size_t y1,
                          size_t y2) const;
  /// Area between the dividers around column subimage_x
  /// (dijkstra_splitter.cc:138-172).
  void FloodVerticalArea(const float* subdivision, size_t subimage_x, bool* mask,
                         size_t& x, size_t& subwidth) const;
  /// Area between the dividers around row subimage_y (:174-208).
  void FloodHorizontalArea(const float* subdivision, size_t subimage_y,
                           bool* mask, size_t& y, size_t& subheight) const;
  /// Overlap of a vertical area (trimmed to its columns) and a horizontal
  /// area; bounding box kept even when the image is (:210-285).
  void GetBoundingMask(const bool* vertical_mask, size_t vertical_mask_x,
                       size_t vertical_mask_width, const bool* horizontal_mask,
                       bool* mask, size_t& sub_x, size_t& sub_y, size_t& subwidth,
                       size_t& subheight) const;

 private:
  /// Divider search: the key-order search (a radix heap) when its path is
  /// provably the reference's (no tie decides it), else DivideExact; the two
  /// race on two threads (RDL_SPLIT_RACE=0: one after the other).
  /// RDL_SPLIT_EXACT=1 always runs DivideExact.
  template <bool kVertical>
  void Divide(const float* image, float* output, size_t lo, size_t hi) const;
  /// The reference's search with its binary heap's exact pop order. With
  /// `race`, it returns without writing once a key-order result claimed the
  /// band (race == 1), and claims it (race = 2) before writing.
  /// With `replay`, it also stops (without writing) once every entry of key
  /// <= replay's stop key has popped, leaving its predecessors there.
  template <bool kVertical>
  void DivideExact(const float* image, float* output, size_t lo, size_t hi,
                   std::atomic<int>* race, DivideReplay* replay = nullptr) const;

  size_t width_, height_;
};

}  // namespace radler::math
