// In-memory accessors over caller-owned pixel buffers (reference:
// cpp/utils/load_image_accessor.h:28-56, load_and_store_image_accessor.h:28-56).
// The caller keeps the buffers alive while Radler uses them.
#pragma once

#include <algorithm>
#include <stdexcept>

#include "aocommon_compat.h"

namespace radler::utils {

class LoadOnlyImageAccessor final : public aocommon::ImageAccessor {
 public:
  explicit LoadOnlyImageAccessor(const aocommon::Image& image)
      : data_(image.Data()), width_(image.Width()), height_(image.Height()) {}
  size_t Width() const override { return width_; }
  size_t Height() const override { return height_; }
  void Load(float* data) const override {
    std::copy_n(data_, width_ * height_, data);
  }
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
  void Load(float* data) const override {
    std::copy_n(data_, width_ * height_, data);
  }
  void Store(const float* data) override {
    std::copy_n(data, width_ * height_, data_);
  }

 private:
  float* data_;
  size_t width_, height_;
};

}  // namespace radler::utils
