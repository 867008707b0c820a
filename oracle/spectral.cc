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

namespace {

// x of (a + ridge * max diag) x = b by Gauss-Jordan elimination with partial
// pivoting; false when singular
bool SolveNormal(std::vector<double> a, std::vector<double>& b, size_t n) {
  double big = 0.0;
  for (size_t i = 0; i != n; ++i) big = std::max(big, a[i * n + i]);
  if (!(big > 0.0)) return false;
  for (size_t i = 0; i != n; ++i) a[i * n + i] += 1e-14 * big;
  for (size_t col = 0; col != n; ++col) {
    size_t piv = col;
    for (size_t r = col + 1; r != n; ++r)
      if (std::fabs(a[r * n + col]) > std::fabs(a[piv * n + col])) piv = r;
    if (a[piv * n + col] == 0.0) return false;
    for (size_t c = 0; c != n; ++c) std::swap(a[col * n + c], a[piv * n + c]);
    std::swap(b[col], b[piv]);
    for (size_t r = 0; r != n; ++r) {
      if (r == col) continue;
      const double f = a[r * n + col] / a[col * n + col];
      for (size_t c = col; c != n; ++c) a[r * n + c] -= f * a[col * n + c];
      b[r] -= f * b[col];
    }
  }
  for (size_t i = 0; i != n; ++i) b[i] /= a[i * n + i];
  return true;
}

// s 10^(a0 + a1 lg + a2 lg^2 + ...)
double PowerLaw(const std::vector<double>& a, double s, double lg) {
  double e = 0.0, p = 1.0;
  for (size_t k = 0; k != a.size(); ++k) {
    e += a[k] * p;
    p *= lg;
  }
  return s * std::pow(10.0, e);
}

}  // namespace

void SpectralFit::FitLogPolynomial(std::vector<float>& terms, const float* values) const {
  terms.assign(n_terms, 0.0f);
  std::vector<double> lg, y;
  for (size_t i = 0; i != frequencies.size(); ++i)
    if (weights[i] > 0.0f) {
      lg.push_back(std::log10(frequencies[i] / reference));
      y.push_back(values[i]);
    }
  const size_t m = lg.size();
  if (m == 0 || n_terms == 0) return;
  double mean = 0.0;
  for (double v : y) mean += v;
  mean /= double(m);
  if (n_terms == 1) {
    terms[0] = float(mean);
    return;
  }
  const double s = mean >= 0.0 ? 1.0 : -1.0;
  std::vector<size_t> pos;
  for (size_t i = 0; i != m; ++i)
    if (s * y[i] > 0.0) pos.push_back(i);
  if (pos.empty()) {
    terms[0] = float(mean);
    return;
  }
  // log-space start: least squares of log10(s y) on powers of lg
  std::vector<double> a(n_terms, 0.0);
  size_t d = std::min(n_terms, pos.size());
  for (;; --d) {
    std::vector<double> g(d * d, 0.0), b(d, 0.0);
    for (size_t i : pos) {
      const double ly = std::log10(s * y[i]);
      for (size_t r = 0; r != d; ++r) {
        b[r] += std::pow(lg[i], double(r)) * ly;
        for (size_t c = 0; c != d; ++c) g[r * d + c] += std::pow(lg[i], double(r + c));
      }
    }
    if (d == 1) {
      double acc = 0.0;
      for (size_t i : pos) acc += std::log10(s * y[i]);
      a[0] = acc / double(pos.size());
      break;
    }
    if (SolveNormal(g, b, d)) {
      for (size_t k = 0; k != d; ++k) a[k] = b[k];
      break;
    }
  }
  // Gauss-Newton in linear space with step halving
  auto sse_of = [&](const std::vector<double>& p) {
    double e = 0.0;
    for (size_t i = 0; i != m; ++i) {
      const double r = y[i] - PowerLaw(p, s, lg[i]);
      e += r * r;
    }
    return e;
  };
  double sse = sse_of(a);
  const size_t n = n_terms;
  for (int it = 0; it != 32; ++it) {
    std::vector<double> g(n * n, 0.0), b(n, 0.0);
    for (size_t i = 0; i != m; ++i) {
      const double f = PowerLaw(a, s, lg[i]);
      for (size_t r = 0; r != n; ++r) {
        const double jr = f * std::log(10.0) * std::pow(lg[i], double(r));
        b[r] += jr * (y[i] - f);
        for (size_t c = 0; c != n; ++c)
          g[r * n + c] += jr * f * std::log(10.0) * std::pow(lg[i], double(c));
      }
    }
    if (!SolveNormal(g, b, n)) break;
    std::vector<double> trial(n);
    double step = 1.0, next = sse;
    bool accepted = false;
    for (int h = 0; h != 24 && !accepted; ++h, step *= 0.5) {
      for (size_t k = 0; k != n; ++k) trial[k] = a[k] + step * b[k];
      next = sse_of(trial);
      accepted = next <= sse;
    }
    if (!accepted) break;
    a = trial;
    const double change = sse - next;
    sse = next;
    if (!(change > 1e-13 * sse) || sse == 0.0) break;
  }
  terms[0] = float(s * std::pow(10.0, a[0]));
  for (size_t k = 1; k != n; ++k) terms[k] = float(a[k]);
}

void SpectralFit::Fit(std::vector<float>& terms, const float* values) const {
  if (mode == 2) {
    FitLogPolynomial(terms, values);
    return;
  }
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
  if (mode == 2) {
    const double lg = std::log10(frequency / reference);
    double e = 0.0, p = lg;
    for (size_t k = 1; k != terms.size(); ++k) {
      e += double(terms[k]) * p;
      p *= lg;
    }
    return float(double(terms[0]) * std::pow(10.0, e));
  }
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
