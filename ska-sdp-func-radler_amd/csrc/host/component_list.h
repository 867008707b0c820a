// radler::ComponentList (reference: cpp/component_list.{h,cc}): per-scale
// component positions with one value per image. Built from the model images
// for single-scale algorithms; recorded by MultiScaleAlgorithm otherwise.
#pragma once

#include <cstddef>
#include <utility>
#include <vector>

namespace radler {

class ImageSet;

class ComponentList {
 public:
  ComponentList() = default;
  ComponentList(size_t width, size_t height, size_t n_scales,
                size_t n_frequencies)
      : width_(width),
        height_(height),
        n_frequencies_(n_frequencies),
        list_per_scale_(n_scales) {}
  /// Every non-zero model pixel becomes a scale-0 component
  /// (component_list.h:46-55 LoadFromImageSet).
  ComponentList(size_t width, size_t height, const ImageSet& model_set);

  struct Position {
    size_t x, y;
  };

  void Add(size_t x, size_t y, size_t scale_index, const float* values);
  void Add(const ComponentList& other, int offset_x, int offset_y);
  void MergeDuplicates();
  void Clear();
  size_t Width() const { return width_; }
  size_t Height() const { return height_; }
  size_t NScales() const { return list_per_scale_.size(); }
  void SetNScales(size_t n) { list_per_scale_.resize(n); }
  size_t NFrequencies() const { return n_frequencies_; }
  size_t ComponentCount(size_t scale_index) const {
    return list_per_scale_[scale_index].positions.size();
  }
  void GetComponent(size_t scale_index, size_t index, size_t& x, size_t& y,
                    float* values) const;
  std::pair<size_t, size_t> GetComponentPosition(size_t scale_index, size_t index) const {
    const auto& p = list_per_scale_[scale_index].positions[index];
    return {p.x, p.y};
  }
  /// GetSingleValue (component_list.h): value of image `image_index`
  float& Value(size_t scale_index, size_t index, size_t image_index) {
    return list_per_scale_[scale_index].values[index * n_frequencies_ + image_index];
  }
  /// component_list.h:157-164
  void SetValues(size_t scale_index, size_t index, const float* values);
  /// component_list.h:178-186 (primary-beam correction factors)
  void MultiplyScaleComponent(size_t scale_index, size_t position_index,
                              size_t channel, double correction_factor);
  /// component_list.h:191-194
  const std::vector<Position>& GetPositions(size_t scale_index) const {
    return list_per_scale_[scale_index].positions;
  }

 private:
  struct ScaleList {
    std::vector<Position> positions;
    std::vector<float> values;
  };
  void MergeDuplicates(size_t scale_index);
  size_t width_ = 0, height_ = 0, n_frequencies_ = 0;
  size_t added_since_merge_ = 0;
  std::vector<ScaleList> list_per_scale_;
};

}  // namespace radler
