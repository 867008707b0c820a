#include "dijkstra_splitter.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <queue>
#include <stdexcept>

namespace radler::math {

namespace {

// One heap entry: the cost of the path up to the predecessor, the target and
// the predecessor as (u, v) — u runs along the path, v across the band.
// 12 bytes (images up to 65535 pixels a side); the heap order depends only
// on `cost`, like the reference's Visit (dijkstra_splitter.h:24-29), so
// equal costs pop in the same heap order as the reference's queue.
struct Node {
  float cost;
  uint16_t u, v, pu, pv;
};
struct LaterFirst {
  bool operator()(const Node& a, const Node& b) const { return a.cost > b.cost; }
};

}  // namespace

template <bool kVertical>
void DijkstraSplitter::Divide(const float* image, float* output, size_t lo,
                              size_t hi) const {
  const size_t n_u = kVertical ? height_ : width_;  // path length axis
  if (width_ >= 65535 || height_ >= 65535)
    throw std::runtime_error("DijkstraSplitter: image side of 65535 pixels or more");
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
  std::vector<Node> heap_store;
  heap_store.reserve(8 * band);
  std::priority_queue<Node, std::vector<Node>, LaterFirst> open(LaterFirst(),
                                                                std::move(heap_store));
  for (size_t v = lo; v != hi; ++v)
    open.push(Node{0.0f, 0, uint16_t(v), 0, uint16_t(v)});
  // predecessor of each settled pixel (pu << 16 | pv), band-local layout
  std::vector<uint32_t> back(band * n_u);
  Node cur{};
  while (!open.empty()) {
    cur = open.top();
    open.pop();
    if (cur.u == n_u) break;
    const size_t at = size_t(cur.u) * band + (cur.v - lo);
    const float cost = cur.cost + weight[at];
    if (!(cost < dist[at])) continue;
    dist[at] = cost;
    back[at] = (uint32_t(cur.pu) << 16) | cur.pv;
    const uint16_t u = cur.u, v = cur.v;
    const uint16_t u1 = uint16_t(u + 1);
    if (v > lo) {
      open.push(Node{cost, u1, uint16_t(v - 1), u, v});
      open.push(Node{cost, u, uint16_t(v - 1), u, v});
    }
    open.push(Node{cost, u1, v, u, v});
    if (v + 1u < hi) {
      open.push(Node{cost, u1, uint16_t(v + 1), u, v});
      open.push(Node{cost, u, uint16_t(v + 1), u, v});
    }
  }
  for (size_t u = 0; u != n_u; ++u)
    for (size_t v = lo; v != hi; ++v) output[pixel(u, v)] = 0.0f;
  uint32_t pu = cur.pu, pv = cur.pv;
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
