// Minimal stand-ins for the aocommon / schaapcommon types that Radler's
// public headers use (cpp/settings.h, work_table_entry.h, radler.h). The
// reference takes them from the external/aocommon and external/schaapcommon
// submodules (empty in the snapshot). When this library is built inside a
// project that already provides the real aocommon (WSClean), define
// RADLER_AMD_USE_EXTERNAL_AOCOMMON and these definitions are skipped.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#ifndef RADLER_AMD_USE_EXTERNAL_AOCOMMON
namespace aocommon {

// Values follow aocommon/polarization.h (FITS / casacore codes).
enum PolarizationEnum {
  StokesI = 1,
  StokesQ = 2,
  StokesU = 3,
  StokesV = 4,
  RR = -1,
  LL = -2,
  RL = -3,
  LR = -4,
  XX = -5,
  YY = -6,
  XY = -7,
  YX = -8,
  FullStokes = 10,
  DiagonalInstrumental = 11,
  Instrumental = 12,
  Diagonal = 13
};

struct Polarization {
  static bool IsStokes(PolarizationEnum p) {
    return p == StokesI || p == StokesQ || p == StokesU || p == StokesV;
  }
  static bool HasDualPolarization(const std::set<PolarizationEnum>& p) {
    return (p.count(XX) && p.count(YY)) || (p.count(RR) && p.count(LL));
  }
  static bool HasFullLinearPolarization(const std::set<PolarizationEnum>& p) {
    return p.count(XX) && p.count(XY) && p.count(YX) && p.count(YY);
  }
  static bool HasFullCircularPolarization(const std::set<PolarizationEnum>& p) {
    return p.count(RR) && p.count(RL) && p.count(LR) && p.count(LL);
  }
  static std::string TypeToShortString(PolarizationEnum p) {
    switch (p) {
      case StokesI: return "I";
      case StokesQ: return "Q";
      case StokesU: return "U";
      case StokesV: return "V";
      case RR: return "RR";
      case LL: return "LL";
      case RL: return "RL";
      case LR: return "LR";
      case XX: return "XX";
      case YY: return "YY";
      case XY: return "XY";
      case YX: return "YX";
      default: return "?";
    }
  }
};

namespace system {
inline size_t ProcessorCount() {
  const unsigned n = std::thread::hardware_concurrency();
  return n == 0 ? 1 : n;
}
}  // namespace system

// A row-major float image, owning or viewing (aocommon::Image subset).
class Image {
 public:
  Image() = default;
  Image(size_t width, size_t height)
      : width_(width), height_(height), owned_(width * height) {
    data_ = owned_.data();
  }
  Image(size_t width, size_t height, float value)
      : width_(width), height_(height), owned_(width * height, value) {
    data_ = owned_.data();
  }
  // Non-owning view (aocommon::Image(float*, w, h)).
  Image(float* data, size_t width, size_t height)
      : width_(width), height_(height), data_(data) {}
  Image(const Image& o) : width_(o.width_), height_(o.height_) {
    owned_.assign(o.data_, o.data_ + o.Size());
    data_ = owned_.data();
  }
  Image(Image&& o) noexcept { *this = std::move(o); }
  Image& operator=(const Image& o) {
    if (this != &o) {
      width_ = o.width_;
      height_ = o.height_;
      owned_.assign(o.data_, o.data_ + o.Size());
      data_ = owned_.data();
    }
    return *this;
  }
  Image& operator=(Image&& o) noexcept {
    width_ = o.width_;
    height_ = o.height_;
    const bool owns = o.data_ == o.owned_.data() && !o.owned_.empty();
    owned_ = std::move(o.owned_);
    data_ = owns ? owned_.data() : o.data_;
    o.data_ = nullptr;
    o.width_ = o.height_ = 0;
    return *this;
  }
  Image& operator=(float v) {
    std::fill_n(data_, Size(), v);
    return *this;
  }
  size_t Width() const { return width_; }
  size_t Height() const { return height_; }
  size_t Size() const { return width_ * height_; }
  bool Empty() const { return Size() == 0; }
  float* Data() { return data_; }
  const float* Data() const { return data_; }
  float& operator[](size_t i) { return data_[i]; }
  const float& operator[](size_t i) const { return data_[i]; }
  float* begin() { return data_; }
  float* end() { return data_ + Size(); }
  const float* begin() const { return data_; }
  const float* end() const { return data_ + Size(); }
  void Reset() {
    owned_.clear();
    owned_.shrink_to_fit();
    data_ = nullptr;
    width_ = height_ = 0;
  }

 private:
  size_t width_ = 0, height_ = 0;
  std::vector<float> owned_;
  float* data_ = nullptr;
};

// aocommon/imageaccessor.h
class ImageAccessor {
 public:
  virtual ~ImageAccessor() = default;
  virtual size_t Width() const = 0;
  virtual size_t Height() const = 0;
  virtual void Load(float* data) const = 0;
  virtual void Store(const float* data) = 0;
};

}  // namespace aocommon

namespace schaapcommon::fitters {
// schaapcommon/fitters/spectralfitter.h
enum class SpectralFittingMode {
  kNoFitting,
  kPolynomial,
  kLogPolynomial,
  kForcedTerms
};
}  // namespace schaapcommon::fitters
#endif  // RADLER_AMD_USE_EXTERNAL_AOCOMMON
