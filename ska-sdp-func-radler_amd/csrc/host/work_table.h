// radler::WorkTable (reference: cpp/work_table.h:73-158, work_table.cc):
// entries grouped by original channel; original groups mapped onto
// deconvolution groups; direction-dependent PSF offsets.
#pragma once

#include <memory>
#include <ostream>
#include <vector>

#include "psf_offset.h"
#include "work_table_entry.h"

namespace radler {

class WorkTable {
 public:
  using Entries = std::vector<std::unique_ptr<WorkTableEntry>>;
  using Group = std::vector<const WorkTableEntry*>;

  class EntryIteratorLite {
    using Base = Entries::const_iterator;

   public:
    explicit EntryIteratorLite(Base b) : b_(b) {}
    const WorkTableEntry& operator*() const { return **b_; }
    EntryIteratorLite& operator++() {
      ++b_;
      return *this;
    }
    bool operator!=(const EntryIteratorLite& o) const { return b_ != o.b_; }
    bool operator==(const EntryIteratorLite& o) const { return b_ == o.b_; }

   private:
    Base b_;
  };

  explicit WorkTable(std::vector<PsfOffset> psf_offsets,
                     std::size_t n_original_groups,
                     std::size_t n_deconvolution_groups,
                     std::size_t channel_index_offset = 0);
  WorkTable(WorkTable&&) = default;

  const std::vector<Group>& OriginalGroups() const { return original_groups_; }
  const std::vector<std::vector<std::size_t>>& DeconvolutionGroups() const {
    return deconvolution_groups_;
  }
  const Group& FirstOriginalGroup(size_t deconvolution_index) const {
    return original_groups_[deconvolution_groups_[deconvolution_index].front()];
  }
  Group GetOriginalSamePolarizationGroup(
      aocommon::PolarizationEnum polarization) const;
  EntryIteratorLite Begin() const { return EntryIteratorLite(entries_.begin()); }
  EntryIteratorLite End() const { return EntryIteratorLite(entries_.end()); }
  void AddEntry(std::unique_ptr<WorkTableEntry> entry);
  const WorkTableEntry& Front() const { return *entries_.front(); }
  size_t Size() const { return entries_.size(); }
  size_t GetChannelIndexOffset() const { return channel_index_offset_; }
  const std::vector<PsfOffset>& PsfOffsets() const noexcept {
    return psf_offsets_;
  }
  /// @throw std::runtime_error if the PSF accessors are inconsistent.
  void ValidatePsfs() const;

  friend EntryIteratorLite begin(const WorkTable& t) { return t.Begin(); }
  friend EntryIteratorLite end(const WorkTable& t) { return t.End(); }
  friend std::ostream& operator<<(std::ostream& out, const WorkTable& t);

 private:
  Entries entries_;
  std::vector<PsfOffset> psf_offsets_;
  std::size_t channel_index_offset_;
  std::vector<Group> original_groups_;
  std::vector<std::vector<std::size_t>> deconvolution_groups_;
};

}  // namespace radler
