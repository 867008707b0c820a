// TEST INFRASTRUCTURE — CPU oracle, used only by tests/, smoke() and the
// bench's cpu_baseline; never by the product.
//
// schaapcommon::fitters::SpectralFitter (the reference's external/schaapcommon
// submodule, not vendored in /root/reference) restated for kNoFitting,
// kPolynomial and kLogPolynomial, and DeconvolutionAlgorithm::PerformSpectralFit
// (cpp/algorithms/deconvolution_algorithm.cc:29-46) which applies it to a
// component. Parity anchors: the reference's own tests
// (python/test/test_radler.py:474-576 test_ndeconvolution_lt_noriginal /
// test_image_cube_joined; cpp/test/test_image_set.cc:622-670
// interpolate_and_store_model), pinned in tests/test_spectral.py.
// kLogPolynomial (schaapcommon's NonLinearPowerLawFitter) has no fixture or
// test in the reference: its restatement here is PARITY UNPINNED — the
// LogarithmicSI model S = t0 10^(t1 lg + t2 lg^2 + ...), lg = log10(f/ref),
// fitted by least squares in linear space (start: the log-space linear fit;
// then Gauss-Newton with step halving), as described in DESIGN.md.
#pragma once

#include <cstddef>
#include <vector>

namespace oracle {

struct SpectralFit {
  int mode = 0;  // 0 kNoFitting, 1 kPolynomial, 2 kLogPolynomial
  size_t n_terms = 0;
  std::vector<double> frequencies;  // per deconvolution channel
  std::vector<float> weights;
  double reference = 0.0;           // weighted mean frequency

  SpectralFit() = default;
  SpectralFit(int mode, size_t n_terms, std::vector<double> frequencies,
              std::vector<float> weights);
  // PolynomialFitter: weighted least squares over channels with weight > 0
  // in x = f / reference - 1, min(n_terms, #points) terms (the rest zero),
  // solved from the normal equations in long double.
  void Fit(std::vector<float>& terms, const float* values) const;
  // kLogPolynomial: see the header comment
  void FitLogPolynomial(std::vector<float>& terms, const float* values) const;
  float Evaluate(const std::vector<float>& terms, double frequency) const;
  void FitAndEvaluate(float* values) const;
};

// deconvolution_algorithm.cc:29-46: values ordered [channel][pol]; fit each
// polarization's channel spectrum in place.
void PerformSpectralFit(const SpectralFit* fit, size_t n_pol, float* values);

}  // namespace oracle
