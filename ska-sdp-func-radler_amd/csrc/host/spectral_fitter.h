// Spectral fitting of CLEAN components and model images (SURVEY.md §8(f)
// row 1): schaapcommon::fitters::SpectralFitter, which the reference takes
// from its external/schaapcommon submodule (not vendored in the snapshot),
// restated from its published behaviour for the modes the MI355X build
// runs:
//   kNoFitting     FitAndEvaluate leaves the values as they are;
//   kPolynomial    a weighted least-squares polynomial of NTerms() terms in
//                  x = frequency / reference_frequency - 1 over the channels
//                  with weight > 0 (at most one term per such channel), then
//                  evaluated at every channel frequency.
//   kLogPolynomial S = t0 10^(t1 lg + t2 lg^2 + ...), lg = log10(f / ref),
//                  a non-linear least-squares fit over the same channels
//                  (csrc/hip/logpoly.h states it; the same code runs in the
//                  device loops, so host and device fits agree).
// kForcedTerms (terms read from a FITS cube) stays unavailable: Radler
// rejects it with an error.
//
// Fitting then evaluating a polynomial at fixed frequencies and weights is a
// linear map of the channel values, independent of the pixel. SpectralMaps
// turns a fitter into those maps so the device applies them inside the
// sub-minor and Högbom loops (per component) and in
// ImageSet::InterpolateAndStoreModel (per pixel), instead of a host
// callback per component.
#pragma once

#include <cstddef>
#include <vector>

#include "aocommon_compat.h"
#include "rdl_hip.h"

#ifndef RADLER_AMD_USE_EXTERNAL_AOCOMMON
namespace schaapcommon::fitters {

class SpectralFitter {
 public:
  SpectralFitter(SpectralFittingMode mode, size_t n_terms,
                 std::vector<double> frequencies = {},
                 std::vector<float> weights = {});

  SpectralFittingMode Mode() const { return mode_; }
  size_t NTerms() const { return n_terms_; }
  const std::vector<double>& Frequencies() const { return frequencies_; }
  const std::vector<float>& Weights() const { return weights_; }
  /// Weighted mean of the channel frequencies (unweighted mean when every
  /// weight is zero).
  double ReferenceFrequency() const { return reference_frequency_; }

  /// terms (NTerms() values) of the fit to values[0..n_channels).
  /// x, y are the pixel (used by forced fitting only).
  void Fit(std::vector<float>& terms, const float* values, size_t x,
           size_t y) const;
  /// values[ch] = the fitted function at channel ch's frequency.
  void Evaluate(float* values, const std::vector<float>& terms) const;
  float Evaluate(const std::vector<float>& terms, double frequency) const;
  void FitAndEvaluate(float* values, size_t x, size_t y,
                      std::vector<float>& scratch) const;

 private:
  SpectralFittingMode mode_;
  size_t n_terms_;
  std::vector<double> frequencies_;
  std::vector<float> weights_;
  double reference_frequency_ = 0.0;
  // kPolynomial: terms = fit_ * values (n_terms_ x n_channels, row-major)
  std::vector<double> fit_;
};

}  // namespace schaapcommon::fitters
#endif  // RADLER_AMD_USE_EXTERNAL_AOCOMMON

namespace radler {

/// The linear maps of a polynomial fitter (empty when the fitter needs none:
/// kNoFitting, or no channel frequencies).
struct SpectralMaps {
  size_t n_channels = 0;
  /// fit[t * n_channels + c]: term t of the fit to unit value in channel c.
  std::vector<double> fit;
  size_t n_terms = 0;
  double reference_frequency = 0.0;  // x = frequency / this - 1
  bool Empty() const { return n_channels == 0; }
  /// Coefficients of the fit-and-evaluate map: row ch gives the fitted
  /// value at frequencies[ch] (n_channels x n_channels).
  std::vector<double> FitAndEvaluate(const std::vector<double>& frequencies) const;
  /// Row of the fitted value at `frequency` (n_channels values).
  std::vector<double> EvaluateAt(double frequency) const;
};

/// kPolynomial: weighted least squares through a pseudo-inverse (one-sided
/// Jacobi SVD of the column-balanced, weight-scaled design matrix; singular
/// values below DBL_EPSILON of the largest are dropped).
SpectralMaps MakeSpectralMaps(const schaapcommon::fitters::SpectralFitter& f);

/// Pseudo-inverse of the m x p matrix a (row-major, m >= 1, p >= 1) by a
/// one-sided Jacobi SVD, singular values below DBL_EPSILON of the largest
/// dropped; returns p x m (row-major).
std::vector<double> PseudoInverse(std::vector<double> a, size_t m, size_t p);

/// The per-component map of DeconvolutionAlgorithm::PerformSpectralFit
/// (deconvolution_algorithm.cc:29-46) over an image set of n_images =
/// n_channels * n_pol images (index ch * n_pol + p): block-diagonal per
/// polarization, row-major float, for the device loops. Empty when the
/// fitter leaves values unchanged.
std::vector<float> ComponentFitMatrix(
    const schaapcommon::fitters::SpectralFitter& f, size_t n_pol);

/// The device description of a kLogPolynomial fitter (false for the other
/// modes); throws when the channel or term count exceeds the device limits.
bool MakeLogPoly(const schaapcommon::fitters::SpectralFitter& f, rdl_logpoly* out);

}  // namespace radler
