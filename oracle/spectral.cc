// TEST INFRASTRUCTURE — see spectral.h.
#include "spectral.h"

#include <algorithm>
#include <cmath>
#include <utility>

namespace oracle {

SpectralFit::SpectralFit(int m, size_t n, std::vector<double> f, std::vector<float> w)
    : mode(m), n_terms(n), frequencies(std::move(f)), weights(std::move(w)) {
  weights.resize(frequencies.size(), 1.0f);
  double sum = 0.0, wsum = 0.0;
  for (size_t i = 0; i != frequencies.size(); ++i) {
    sum += frequencies[i] * weights[i];
    wsum += weights[i];
  }
  if (wsum > 0.0) {
    reference = sum / wsum;
  } else if (!frequencies.empty()) {
    for (double v : frequencies) reference += v;
    reference /= double(frequencies.size());
  }
}

void SpectralFit::Fit(std::vector<float>& terms, const float* values) const {
  terms.assign(n_terms, 0.0f);
  std::vector<long double> xs, ys, ws;
  for (size_t i = 0; i != frequencies.size(); ++i) {
    if (weights[i] > 0.0f) {
      xs.push_back((long double)(frequencies[i] / reference - 1.0));
      ys.push_back(values[i]);
      ws.push_back(weights[i]);
    }
  }
  const size_t p = std::min(n_terms, xs.size());
  if (p == 0) return;
  // normal equations  (X^T W X) c = X^T W y
  std::vector<long double> a(p * (p + 1), 0.0L);
  for (size_t i = 0; i != xs.size(); ++i) {
    std::vector<long double> pw(2 * p, 1.0L);
    for (size_t k = 1; k != 2 * p; ++k) pw[k] = pw[k - 1] * xs[i];
    for (size_t r = 0; r != p; ++r) {
      for (size_t c = 0; c != p; ++c) a[r * (p + 1) + c] += ws[i] * pw[r + c];
      a[r * (p + 1) + p] += ws[i] * pw[r] * ys[i];
    }
  }
  for (size_t col = 0; col != p; ++col) {  // Gauss-Jordan, partial pivoting
    size_t piv = col;
    for (size_t r = col + 1; r != p; ++r)
      if (std::fabs(a[r * (p + 1) + col]) > std::fabs(a[piv * (p + 1) + col])) piv = r;
    for (size_t c = 0; c != p + 1; ++c) std::swap(a[col * (p + 1) + c], a[piv * (p + 1) + c]);
    const long double d = a[col * (p + 1) + col];
    if (d == 0.0L) continue;
    for (size_t r = 0; r != p; ++r) {
      if (r == col) continue;
      const long double f = a[r * (p + 1) + col] / d;
      for (size_t c = col; c != p + 1; ++c) a[r * (p + 1) + c] -= f * a[col * (p + 1) + c];
    }
  }
  for (size_t k = 0; k != p; ++k) {
    const long double d = a[k * (p + 1) + k];
    terms[k] = d == 0.0L ? 0.0f : float(a[k * (p + 1) + p] / d);
  }
}

float SpectralFit::Evaluate(const std::vector<float>& terms, double frequency) const {
  if (terms.empty()) return 0.0f;
  const float x = float(frequency / reference - 1.0);
  float value = terms[0], power = 1.0f;
  for (size_t i = 1; i != terms.size(); ++i) {
    power *= x;
    value += power * terms[i];
  }
  return value;
}

void SpectralFit::FitAndEvaluate(float* values) const {
  if (mode == 0) return;
  std::vector<float> terms;
  Fit(terms, values);
  for (size_t ch = 0; ch != frequencies.size(); ++ch)
    values[ch] = Evaluate(terms, frequencies[ch]);
}

void PerformSpectralFit(const SpectralFit* fit, size_t n_pol, float* values) {
  if (!fit) return;
  const size_t n = fit->frequencies.size();
  for (size_t p = 0; p != n_pol; ++p) {
    // gather the polarization's channels to the front (an in-place
    // single-column transpose), fit, and undo the moves in reverse order
    for (size_t ch = 0; ch != n; ++ch) std::swap(values[ch * n_pol + p], values[ch]);
    fit->FitAndEvaluate(values);
    for (size_t i = 0; i != n; ++i) {
      const size_t ch = n - i - 1;
      std::swap(values[ch * n_pol + p], values[ch]);
    }
  }
}

}  // namespace oracle
