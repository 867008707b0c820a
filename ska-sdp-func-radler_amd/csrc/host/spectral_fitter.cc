#include "spectral_fitter.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <mutex>
#include <stdexcept>
#include <string>

#include "logger.h"
#include "logpoly.h"

namespace radler {
namespace {

double ReferenceOf(const std::vector<double>& frequencies,
                   const std::vector<float>& weights) {
  double sum = 0.0, weight_sum = 0.0, plain = 0.0;
  for (size_t i = 0; i != frequencies.size(); ++i) {
    const double w = i < weights.size() ? double(weights[i]) : 1.0;
    sum += frequencies[i] * w;
    weight_sum += w;
    plain += frequencies[i];
  }
  if (weight_sum > 0.0) return sum / weight_sum;
  return frequencies.empty() ? 0.0 : plain / double(frequencies.size());
}

}  // namespace

std::vector<double> PseudoInverse(std::vector<double> a, size_t m, size_t p) {
  std::vector<double> v(p * p, 0.0);
  for (size_t j = 0; j != p; ++j) v[j * p + j] = 1.0;
  for (int sweep = 0; sweep != 80; ++sweep) {
    bool rotated = false;
    for (size_t j = 0; j + 1 < p; ++j) {
      for (size_t k = j + 1; k != p; ++k) {
        double alpha = 0.0, beta = 0.0, gamma = 0.0;
        for (size_t i = 0; i != m; ++i) {
          alpha += a[i * p + j] * a[i * p + j];
          beta += a[i * p + k] * a[i * p + k];
          gamma += a[i * p + j] * a[i * p + k];
        }
        if (gamma == 0.0 || std::fabs(gamma) <= DBL_EPSILON * std::sqrt(alpha * beta))
          continue;
        rotated = true;
        const double zeta = (beta - alpha) / (2.0 * gamma);
        const double t = (zeta >= 0.0 ? 1.0 : -1.0) /
                         (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
        for (size_t i = 0; i != m; ++i) {
          const double x = a[i * p + j], y = a[i * p + k];
          a[i * p + j] = c * x - s * y;
          a[i * p + k] = s * x + c * y;
        }
        for (size_t i = 0; i != p; ++i) {
          const double x = v[i * p + j], y = v[i * p + k];
          v[i * p + j] = c * x - s * y;
          v[i * p + k] = s * x + c * y;
        }
      }
    }
    if (!rotated) break;
  }
  std::vector<double> sigma(p, 0.0);
  double sigma_max = 0.0;
  for (size_t k = 0; k != p; ++k) {
    double n2 = 0.0;
    for (size_t i = 0; i != m; ++i) n2 += a[i * p + k] * a[i * p + k];
    sigma[k] = std::sqrt(n2);
    sigma_max = std::max(sigma_max, sigma[k]);
  }
  std::vector<double> pinv(p * m, 0.0);
  for (size_t k = 0; k != p; ++k) {
    if (!(sigma[k] > DBL_EPSILON * sigma_max)) continue;
    const double inv2 = 1.0 / (sigma[k] * sigma[k]);  // U_k = A_k / sigma_k
    for (size_t j = 0; j != p; ++j) {
      const double vj = v[j * p + k] * inv2;
      if (vj == 0.0) continue;
      for (size_t i = 0; i != m; ++i) pinv[j * m + i] += vj * a[i * p + k];
    }
  }
  return pinv;
}


SpectralMaps MakeSpectralMaps(const schaapcommon::fitters::SpectralFitter& f) {
  SpectralMaps maps;
  if (f.Mode() != schaapcommon::fitters::SpectralFittingMode::kPolynomial ||
      f.Frequencies().empty() || f.NTerms() == 0)
    return maps;
  const std::vector<double>& freqs = f.Frequencies();
  const std::vector<float>& weights = f.Weights();
  const size_t n = freqs.size();
  const double ref = ReferenceOf(freqs, weights);
  maps.n_channels = n;
  maps.n_terms = f.NTerms();
  maps.reference_frequency = ref;
  maps.fit.assign(maps.n_terms * n, 0.0);
  std::vector<size_t> points;
  for (size_t i = 0; i != n; ++i)
    if (i < weights.size() && weights[i] > 0.0f) points.push_back(i);
  const size_t m = points.size();
  const size_t p = std::min(maps.n_terms, m);
  if (p == 0) return maps;
  // design matrix sqrt(w_i) x_i^j, columns balanced to unit norm
  std::vector<double> a(m * p), norm(p, 0.0);
  for (size_t i = 0; i != m; ++i) {
    const double x = freqs[points[i]] / ref - 1.0;
    const double sw = std::sqrt(double(weights[points[i]]));
    double xp = 1.0;
    for (size_t j = 0; j != p; ++j) {
      a[i * p + j] = sw * xp;
      norm[j] += a[i * p + j] * a[i * p + j];
      xp *= x;
    }
  }
  for (size_t j = 0; j != p; ++j) {
    norm[j] = norm[j] > 0.0 ? std::sqrt(norm[j]) : 1.0;
    for (size_t i = 0; i != m; ++i) a[i * p + j] /= norm[j];
  }
  const std::vector<double> pinv = PseudoInverse(std::move(a), m, p);
  for (size_t j = 0; j != p; ++j)
    for (size_t i = 0; i != m; ++i)
      maps.fit[j * n + points[i]] = pinv[j * m + i] *
                                    std::sqrt(double(weights[points[i]])) /
                                    norm[j];
  return maps;
}

std::vector<double> SpectralMaps::EvaluateAt(double frequency) const {
  std::vector<double> row(n_channels, 0.0);
  const double x = frequency / reference_frequency - 1.0;
  double xp = 1.0;
  for (size_t t = 0; t != n_terms; ++t) {
    for (size_t c = 0; c != n_channels; ++c) row[c] += xp * fit[t * n_channels + c];
    xp *= x;
  }
  return row;
}

std::vector<double> SpectralMaps::FitAndEvaluate(
    const std::vector<double>& frequencies) const {
  std::vector<double> h;
  h.reserve(n_channels * n_channels);
  for (size_t ch = 0; ch != n_channels; ++ch) {
    const std::vector<double> row = EvaluateAt(frequencies[ch]);
    h.insert(h.end(), row.begin(), row.end());
  }
  return h;
}

std::vector<float> ComponentFitMatrix(
    const schaapcommon::fitters::SpectralFitter& f, size_t n_pol) {
  const SpectralMaps maps = MakeSpectralMaps(f);
  if (maps.Empty()) return {};
  const size_t n_ch = maps.n_channels, n_img = n_ch * n_pol;
  const std::vector<double> h = maps.FitAndEvaluate(f.Frequencies());
  std::vector<float> g(n_img * n_img, 0.0f);
  for (size_t ch = 0; ch != n_ch; ++ch)
    for (size_t c = 0; c != n_ch; ++c)
      for (size_t p = 0; p != n_pol; ++p)
        g[(ch * n_pol + p) * n_img + c * n_pol + p] = float(h[ch * n_ch + c]);
  return g;
}

bool MakeLogPoly(const schaapcommon::fitters::SpectralFitter& f, rdl_logpoly* out) {
  if (f.Mode() != schaapcommon::fitters::SpectralFittingMode::kLogPolynomial) return false;
  const std::vector<double>& freqs = f.Frequencies();
  const std::vector<float>& weights = f.Weights();
  if (freqs.empty() || freqs.size() > RDL_LOGPOLY_MAX_CHANNELS)
    throw std::runtime_error("Log-polynomial spectral fitting supports 1 to " +
                             std::to_string(RDL_LOGPOLY_MAX_CHANNELS) + " channels");
  if (f.NTerms() < 1 || f.NTerms() > RDL_LOGPOLY_MAX_TERMS)
    throw std::runtime_error("Log-polynomial spectral fitting supports 1 to " +
                             std::to_string(RDL_LOGPOLY_MAX_TERMS) + " terms");
  rdl_logpoly lp{};
  lp.n_channels = uint32_t(freqs.size());
  lp.n_terms = uint32_t(f.NTerms());
  for (size_t c = 0; c != freqs.size(); ++c) {
    if (c < weights.size() && weights[c] > 0.0f) lp.fit_mask |= 1u << c;
    lp.lg[c] = std::log10(freqs[c] / f.ReferenceFrequency());
  }
  *out = lp;
  return true;
}

}  // namespace radler

#ifndef RADLER_AMD_USE_EXTERNAL_AOCOMMON
namespace schaapcommon::fitters {

SpectralFitter::SpectralFitter(SpectralFittingMode mode, size_t n_terms,
                               std::vector<double> frequencies,
                               std::vector<float> weights)
    : mode_(mode),
      n_terms_(n_terms),
      frequencies_(std::move(frequencies)),
      weights_(std::move(weights)) {
  if (weights_.size() < frequencies_.size())
    weights_.resize(frequencies_.size(), 1.0f);
  reference_frequency_ = radler::ReferenceOf(frequencies_, weights_);
  if (mode_ == SpectralFittingMode::kPolynomial)
    fit_ = radler::MakeSpectralMaps(*this).fit;
  if (mode_ == SpectralFittingMode::kLogPolynomial) {
    // schaapcommon's NonLinearPowerLawFitter is not vendored with the
    // reference: the restated fitter (csrc/hip/logpoly.h) is unpinned
    static std::once_flag warned;
    std::call_once(warned, [] {
      radler::log::Warn()
          << "Warning: log-polynomial spectral fitting uses a restated "
             "Gauss-Newton power-law fitter; its parity with schaapcommon's "
             "NonLinearPowerLawFitter is unverified (term convention and "
             "convergence criteria are assumptions).\n";
    });
  }
}

void SpectralFitter::Fit(std::vector<float>& terms, const float* values, size_t,
                         size_t) const {
  switch (mode_) {
    case SpectralFittingMode::kNoFitting:
      return;
    case SpectralFittingMode::kPolynomial: {
      const size_t n = frequencies_.size();
      terms.assign(n_terms_, 0.0f);
      if (fit_.empty()) return;
      for (size_t t = 0; t != n_terms_; ++t) {
        double sum = 0.0;
        for (size_t c = 0; c != n; ++c)
          if (weights_[c] > 0.0f) sum += fit_[t * n + c] * double(values[c]);
        terms[t] = float(sum);
      }
      return;
    }
    case SpectralFittingMode::kLogPolynomial: {
      rdl_logpoly lp;
      radler::MakeLogPoly(*this, &lp);
      terms.assign(n_terms_, 0.0f);
      rdl::lp::Fit(lp, values, terms.data());
      return;
    }
    case SpectralFittingMode::kForcedTerms:
      break;
  }
  throw std::runtime_error(
      "SpectralFitter: forced-term fitting is not available in the MI355X build");
}

float SpectralFitter::Evaluate(const std::vector<float>& terms,
                               double frequency) const {
  if (terms.empty()) return 0.0f;
  if (mode_ == SpectralFittingMode::kLogPolynomial)
    return rdl::lp::Evaluate(terms.data(), int(terms.size()),
                             std::log10(frequency / reference_frequency_));
  const float x = float(frequency / reference_frequency_ - 1.0);
  float value = terms[0], power = 1.0f;
  for (size_t i = 1; i != terms.size(); ++i) {
    power *= x;
    value += power * terms[i];
  }
  return value;
}

void SpectralFitter::Evaluate(float* values, const std::vector<float>& terms) const {
  if (mode_ == SpectralFittingMode::kNoFitting) return;
  for (size_t ch = 0; ch != frequencies_.size(); ++ch)
    values[ch] = Evaluate(terms, frequencies_[ch]);
}

void SpectralFitter::FitAndEvaluate(float* values, size_t x, size_t y,
                                    std::vector<float>& scratch) const {
  if (mode_ == SpectralFittingMode::kNoFitting) return;
  Fit(scratch, values, x, y);
  Evaluate(values, scratch);
}

}  // namespace schaapcommon::fitters
#endif  // RADLER_AMD_USE_EXTERNAL_AOCOMMON
