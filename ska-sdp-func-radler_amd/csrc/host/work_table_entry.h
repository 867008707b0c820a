// radler::WorkTableEntry (reference: cpp/work_table_entry.h:16-94): one
// channel x polarization entry with borrowed image accessors.
#pragma once

#include <cmath>
#include <memory>
#include <ostream>
#include <vector>

#include "aocommon_compat.h"

namespace radler {

struct WorkTableEntry {
  double CentralFrequency() const {
    return 0.5 * (band_start_frequency + band_end_frequency);
  }
  size_t index = 0;
  double band_start_frequency = 0.0;
  double band_end_frequency = 0.0;
  aocommon::PolarizationEnum polarization = aocommon::PolarizationEnum::StokesI;
  size_t original_channel_index = 0;
  size_t original_interval_index = 0;
  size_t mask_channel_index = 0;
  double image_weight = 0.0;
  std::vector<std::unique_ptr<aocommon::ImageAccessor>> psf_accessors{};
  std::unique_ptr<aocommon::ImageAccessor> model_accessor;
  std::unique_ptr<aocommon::ImageAccessor> residual_accessor;

  friend std::ostream& operator<<(std::ostream& out, const WorkTableEntry& e) {
    return out << "  " << e.index << " "
               << aocommon::Polarization::TypeToShortString(e.polarization)
               << " " << e.original_channel_index << " " << e.mask_channel_index
               << " " << e.original_interval_index << " " << e.image_weight
               << " " << std::round(e.band_start_frequency * 1e-6) << "-"
               << std::round(e.band_end_frequency * 1e-6) << '\n';
  }
};

}  // namespace radler
