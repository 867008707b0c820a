// reference: cpp/work_table.cc:13-98
#include "work_table.h"

#include <cassert>
#include <sstream>
#include <stdexcept>

namespace radler {

WorkTable::WorkTable(std::vector<PsfOffset> psf_offsets,
                     std::size_t n_original_groups,
                     std::size_t n_deconvolution_groups,
                     std::size_t channel_index_offset)
    : psf_offsets_(std::move(psf_offsets)),
      channel_index_offset_(channel_index_offset),
      original_groups_(std::max<std::size_t>(n_original_groups, 1)) {
  const size_t n_orig = original_groups_.size();
  const size_t n_deconv = n_deconvolution_groups == 0
                              ? n_orig
                              : std::min(n_orig, n_deconvolution_groups);
  deconvolution_groups_.resize(n_deconv);
  for (size_t i = 0; i != n_orig; ++i)
    deconvolution_groups_[i * n_deconv / n_orig].push_back(i);
}

WorkTable::Group WorkTable::GetOriginalSamePolarizationGroup(
    aocommon::PolarizationEnum polarization) const {
  Group g;
  for (const auto& e : entries_)
    if (e->polarization == polarization) g.push_back(e.get());
  return g;
}

void WorkTable::AddEntry(std::unique_ptr<WorkTableEntry> entry) {
  const size_t ch = entry->original_channel_index;
  if (ch >= original_groups_.size())
    throw std::runtime_error("WorkTable: original channel index out of range");
  entry->index = entries_.size();
  entries_.push_back(std::move(entry));
  original_groups_[ch].push_back(entries_.back().get());
}

namespace {
template <typename... T>
[[noreturn]] void Throw(const T&... parts) {
  std::ostringstream s;
  (s << ... << parts);
  throw std::runtime_error(s.str());
}
}  // namespace

void WorkTable::ValidatePsfs() const {
  if (entries_.empty()) return;
  const size_t n_psfs = std::max<size_t>(1, psf_offsets_.size());
  if (Front().psf_accessors.size() != n_psfs)
    Throw("WorkTable: Expected ", n_psfs,
          " PSF accessors in the first entry, but found ",
          Front().psf_accessors.size(), " PSF accessors.");
  for (const Group& group : original_groups_) {
    for (size_t i = 0; i < group.size(); ++i) {
      const WorkTableEntry& e = *group[i];
      if (i == 0) {
        if (e.psf_accessors.size() != n_psfs)
          Throw("WorkTable: Expected ", n_psfs,
                " PSF accessors per entry, but found an entry with ",
                e.psf_accessors.size(), " PSF accessors.");
        for (size_t p = 0; p < n_psfs; ++p) {
          const size_t w = e.psf_accessors[p]->Width();
          const size_t h = e.psf_accessors[p]->Height();
          if (w == 0 || h == 0)
            Throw("WorkTable: Found an entry with an empty image for PSF "
                  "accessor ", p, ".");
          if (w != Front().psf_accessors[p]->Width() ||
              h != Front().psf_accessors[p]->Height())
            Throw("WorkTable: Found an entry with a different size for PSF "
                  "accessor ", p, ".");
        }
      } else if (!e.psf_accessors.empty()) {
        throw std::runtime_error(
            "WorkTable: Only the first entry for a channel may have PSF "
            "accessors.");
      }
    }
  }
}

std::ostream& operator<<(std::ostream& out, const WorkTable& t) {
  out << "=== IMAGING TABLE ===\nOriginal groups       "
      << t.original_groups_.size() << "\nDeconvolution groups  "
      << t.deconvolution_groups_.size() << "\nChannel index         "
      << t.channel_index_offset_ << '\n';
  if (!t.entries_.empty()) {
    out << "   # Pol Ch Mask Interval Weight Freq(MHz)\n";
    for (const auto& e : t.entries_) out << *e;
  }
  if (!t.psf_offsets_.empty()) {
    out << "=== PSFs ===\n";
    for (const auto& p : t.psf_offsets_) out << p << '\n';
  }
  return out;
}

}  // namespace radler
