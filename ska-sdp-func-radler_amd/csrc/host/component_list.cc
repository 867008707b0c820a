#include "component_list.h"

#include <algorithm>
#include <numeric>

#include "image_set.h"

namespace radler {

ComponentList::ComponentList(size_t width, size_t height,
                             const ImageSet& model_set)
    : width_(width),
      height_(height),
      n_frequencies_(model_set.Size()),
      list_per_scale_(1) {
  const size_t n = width * height;
  std::vector<float> host(n * model_set.Size());
  model_set.Session().D2H(host.data(), model_set.Base(),
                          host.size() * sizeof(float));
  std::vector<float> values(n_frequencies_);
  for (size_t p = 0; p != n; ++p) {
    bool nonzero = false;
    for (size_t i = 0; i != n_frequencies_; ++i) {
      values[i] = host[i * n + p];
      nonzero = nonzero || values[i] != 0.0f;
    }
    if (nonzero) Add(p % width, p / width, 0, values.data());
  }
}

void ComponentList::Add(size_t x, size_t y, size_t scale_index,
                        const float* values) {
  ScaleList& l = list_per_scale_[scale_index];
  l.positions.push_back({x, y});
  l.values.insert(l.values.end(), values, values + n_frequencies_);
  if (++added_since_merge_ >= 100000) MergeDuplicates();
}

void ComponentList::Add(const ComponentList& other, int offset_x,
                        int offset_y) {
  if (other.NScales() > NScales()) SetNScales(other.NScales());
  for (size_t s = 0; s != other.NScales(); ++s) {
    const ScaleList& l = other.list_per_scale_[s];
    for (size_t i = 0; i != l.positions.size(); ++i)
      Add(l.positions[i].x + offset_x, l.positions[i].y + offset_y, s,
          &l.values[i * n_frequencies_]);
  }
}

void ComponentList::MergeDuplicates() {
  if (added_since_merge_ == 0) return;
  for (size_t s = 0; s != list_per_scale_.size(); ++s) MergeDuplicates(s);
  added_since_merge_ = 0;
}

void ComponentList::MergeDuplicates(size_t scale_index) {
  // component_list.h:222-263: the reference accumulates the values into one
  // image per frequency (in list order), then emits, frequency by frequency,
  // every raster position whose value in that frequency is non-zero (with
  // all its frequencies, which are then cleared). Positions whose summed
  // values are zero in every frequency disappear. Here a stable raster sort
  // sums duplicates in the same order; the emission passes follow.
  ScaleList& l = list_per_scale_[scale_index];
  std::vector<size_t> order(l.positions.size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    const Position& pa = l.positions[a];
    const Position& pb = l.positions[b];
    return pa.y != pb.y ? pa.y < pb.y : pa.x < pb.x;
  });
  ScaleList merged;
  for (size_t idx : order) {
    const Position& p = l.positions[idx];
    if (!merged.positions.empty() && merged.positions.back().x == p.x &&
        merged.positions.back().y == p.y) {
      float* dst = &merged.values[merged.values.size() - n_frequencies_];
      for (size_t f = 0; f != n_frequencies_; ++f)
        dst[f] += l.values[idx * n_frequencies_ + f];
    } else {
      merged.positions.push_back(p);
      merged.values.insert(merged.values.end(),
                           l.values.begin() + idx * n_frequencies_,
                           l.values.begin() + (idx + 1) * n_frequencies_);
    }
  }
  ScaleList out;
  std::vector<char> emitted(merged.positions.size(), 0);
  for (size_t f = 0; f != n_frequencies_; ++f)
    for (size_t i = 0; i != merged.positions.size(); ++i) {
      if (emitted[i] || merged.values[i * n_frequencies_ + f] == 0.0f) continue;
      emitted[i] = 1;
      out.positions.push_back(merged.positions[i]);
      out.values.insert(out.values.end(), merged.values.begin() + i * n_frequencies_,
                        merged.values.begin() + (i + 1) * n_frequencies_);
    }
  l = std::move(out);
}

void ComponentList::MultiplyScaleComponent(size_t scale_index, size_t position_index,
                                           size_t channel, double correction_factor) {
  float& value =
      list_per_scale_[scale_index].values[channel + position_index * n_frequencies_];
  value *= correction_factor;  // component_list.h:178-186 (float *= double)
}

void ComponentList::SetValues(size_t scale_index, size_t index, const float* values) {
  std::copy_n(values, n_frequencies_,
              &list_per_scale_[scale_index].values[index * n_frequencies_]);
}

void ComponentList::Clear() {
  for (ScaleList& l : list_per_scale_) {
    l.positions.clear();
    l.values.clear();
  }
  added_since_merge_ = 0;
}

void ComponentList::GetComponent(size_t scale_index, size_t index, size_t& x,
                                 size_t& y, float* values) const {
  const ScaleList& l = list_per_scale_[scale_index];
  x = l.positions[index].x;
  y = l.positions[index].y;
  std::copy_n(&l.values[index * n_frequencies_], n_frequencies_, values);
}

}  // namespace radler
