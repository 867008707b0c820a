// radler::ImageSet, device-resident: the [channel][pol] image stack lives in
// one contiguous HBM allocation (image i at Data(i) = Base() + i*W*H).
// Reference: cpp/image_set.{h,cc}. Integration, PSF averaging and the
// weighted loads run as HIP kernels with the reference's summation order;
// host memory is touched only through the WorkTable's image accessors.
#pragma once

#include <memory>
#include <set>
#include <vector>

#include "device.h"
#include "spectral_fitter.h"
#include "rdl_hip.h"
#include "work_table.h"

namespace radler {

class ImageSet {
 public:
  ImageSet(const WorkTable& table, bool squared_joins,
           const std::set<aocommon::PolarizationEnum>& linked_polarizations,
           size_t width, size_t height, gpu::Session& session);
  /// Same configuration, different image size (image_set.cc:448-450).
  ImageSet(const ImageSet& like, size_t width, size_t height);
  /// Same configuration, planes allocated on another session (a subimage
  /// worker's device/stream).
  ImageSet(const ImageSet& like, size_t width, size_t height,
           gpu::Session& session);
  ImageSet(const ImageSet&) = delete;
  ImageSet& operator=(const ImageSet&) = delete;

  /// image_set.cc:105-140 (use_residual_images: residual vs model accessors)
  void LoadAndAverage(bool use_residual_images);
  /// image_set.cc:142-207: result[psf_index] holds NDeconvolutionChannels()
  /// planes.
  std::vector<gpu::Planes> LoadAndAveragePsfs() const;
  /// image_set.cc:290-307
  void AssignAndStoreResidual();
  /// image_set.cc:209-288. With a polynomial fitter and fewer deconvolution
  /// than original channels, every original channel receives the fit over
  /// the deconvolution channels evaluated at its central frequency
  /// (rdl_spectral_interpolate); without one (kNoFitting), the model of the
  /// deconvolution channel it was averaged into.
  void InterpolateAndStoreModel(
      const schaapcommon::fitters::SpectralFitter* fitter = nullptr);

  void GetLinearIntegrated(float* d_dest) const;
  void GetSquareIntegrated(float* d_dest) const;
  void GetIntegratedPsf(float* d_dest, const gpu::Planes& psfs) const;
  /// Integration descriptor for the device kernels.
  rdl_integration Integration(bool square) const;

  size_t NOriginalChannels() const { return table_.OriginalGroups().size(); }
  size_t NDeconvolutionChannels() const {
    return table_.DeconvolutionGroups().size();
  }
  size_t PsfCount() const { return NDeconvolutionChannels(); }
  size_t NPolarizations() const { return n_pol_; }
  size_t Size() const { return n_images_; }
  size_t Width() const { return width_; }
  size_t Height() const { return height_; }
  size_t PlaneSize() const { return width_ * height_; }
  size_t PsfIndex(size_t image_index) const {
    return image_index_to_psf_index_[image_index];
  }
  float* Data(size_t index) const { return planes_.Plane(index); }
  float* Base() const { return planes_.Base(); }
  const gpu::Planes& Planes() const { return planes_; }
  gpu::Session& Session() const { return *session_; }
  const WorkTable& Table() const { return table_; }
  const std::vector<float>& Weights() const { return weights_; }
  bool SquareJoinedChannels() const { return square_joined_channels_; }

  void Fill(float value);
  void CopyFrom(const ImageSet& other);
  /// Replace the image planes (sizes may differ; image_set.cc:69-72).
  void SetPlanes(gpu::Planes planes);

  static void CalculateDeconvolutionFrequencies(const WorkTable& table,
                                                std::vector<double>& frequencies,
                                                std::vector<float>& weights);

 private:
  void InitializePolFactor();
  void InitializeIndices();

  const WorkTable& table_;
  gpu::Session* session_;
  size_t width_, height_, n_images_, n_pol_;
  bool square_joined_channels_;
  std::set<aocommon::PolarizationEnum> linked_polarizations_;
  gpu::Planes planes_;
  std::vector<float> weights_;
  std::vector<size_t> entry_index_to_image_index_;
  std::vector<size_t> image_index_to_psf_index_;
  float polarization_normalization_factor_ = 1.0f;
};

}  // namespace radler
