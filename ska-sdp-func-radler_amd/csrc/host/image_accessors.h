// In-memory accessors over caller-owned pixel buffers (reference:
// cpp/utils/load_image_accessor.h:28-56, load_and_store_image_accessor.h:28-56).
// The caller keeps the buffers alive while Radler uses them.
#pragma once

#include <algorithm>
#include <stdexcept>
#include <thread>
#include <vector>

#include "aocommon_compat.h"

namespace radler::utils {

/// std::copy_n split over a few host threads for whole images: one thread
/// copies ~10 GB/s, so a 256 MiB plane took ~25 ms of every accessor load
/// and store of a Perform (the page-locked staging buffer and the link
/// itself are ~5x faster).
inline void ParallelCopy(const float* src, size_t n, float* dst) {
  constexpr size_t kMinPerThread = size_t(1) << 22;  // 16 MiB
  const size_t hw = std::max<size_t>(1, std::thread::hardware_concurrency());
  const size_t threads = std::min<size_t>({hw, 8, std::max<size_t>(1, n / kMinPerThread)});
  if (threads <= 1) {
    std::copy_n(src, n, dst);
    return;
  }
  const size_t chunk = (n + threads - 1) / threads;
  std::vector<std::thread> pool;
  pool.reserve(threads - 1);
  for (size_t t = 1; t < threads; ++t) {
    const size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b < e) pool.emplace_back([=] { std::copy(src + b, src + e, dst + b); });
  }
  std::copy(src, src + std::min(n, chunk), dst);
  for (std::thread& th : pool) th.join();
}

class LoadOnlyImageAccessor final : public aocommon::ImageAccessor {
 public:
  explicit LoadOnlyImageAccessor(const aocommon::Image& image)
      : data_(image.Data()), width_(image.Width()), height_(image.Height()) {}
  size_t Width() const override { return width_; }
  size_t Height() const override { return height_; }
  void Load(float* data) const override { ParallelCopy(data_, width_ * height_, data); }
  void Store(const float*) override {
    throw std::logic_error("Unexpected LoadOnlyImageAccessor::Store() call");
  }

 private:
  const float* data_;
  size_t width_, height_;
};

class LoadAndStoreImageAccessor final : public aocommon::ImageAccessor {
 public:
  explicit LoadAndStoreImageAccessor(aocommon::Image& image)
      : data_(image.Data()), width_(image.Width()), height_(image.Height()) {}
  size_t Width() const override { return width_; }
  size_t Height() const override { return height_; }
  void Load(float* data) const override { ParallelCopy(data_, width_ * height_, data); }
  void Store(const float* data) override { ParallelCopy(data, width_ * height_, data_); }

 private:
  float* data_;
  size_t width_, height_;
};

}  // namespace radler::utils
