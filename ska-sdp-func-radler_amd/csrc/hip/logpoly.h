// Log-polynomial spectral fitting (schaapcommon::fitters::SpectralFitter in
// kLogPolynomial mode: NonLinearPowerLawFitter; the reference's
// external/schaapcommon submodule is not vendored in /root/reference, so the
// algorithm below is a restatement and its parity is unpinned — DESIGN.md).
// The reference calls it from DeconvolutionAlgorithm::PerformSpectralFit
// (cpp/algorithms/deconvolution_algorithm.cc:29-46) for every component, from
// ImageSet::InterpolateAndStoreModel (cpp/image_set.cc:238-285) for every
// non-zero model pixel, and from ComponentList::Write
// (cpp/component_list.cc:80-117, LogarithmicSI=true).
//
// Model (the LogarithmicSI convention of the component list):
//   S(nu) = t0 * 10^( t1 lg + t2 lg^2 + ... ),  lg = log10(nu / nu_ref)
// fitted by least squares in linear space over the channels with weight > 0:
//   1. s = sign of the mean (+1 for zero); one term: t0 = the mean;
//   2. start: linear least squares of log10(s y) on 1, lg, lg^2, ... over the
//      points with s y > 0 (as many terms as such points, at most n_terms);
//   3. Gauss-Newton on (log10|t0|, t1, ...) for S = s 10^(a0 + sum a_k lg^k),
//      step halved until the squared error does not grow, at most 32 steps,
//      stopping when a step changes the error by less than 1e-13 relative.
// Every step runs in double in a fixed order, so every thread that evaluates
// it on the same values gets the same bits (the loops use it redundantly).
// Terms are returned as float (the reference's std::vector<float>) and the
// evaluation starts from them, as SpectralFitter::FitAndEvaluate does.
#pragma once

#include <cmath>
#include <cstdint>

#include "rdl_hip.h"

#if defined(__HIPCC__)
#define RDL_HD __host__ __device__
#else
#define RDL_HD
#endif

namespace rdl {
namespace lp {

constexpr int kMaxCh = RDL_LOGPOLY_MAX_CHANNELS;
constexpr int kMaxTerms = RDL_LOGPOLY_MAX_TERMS;
constexpr double kLn10 = 2.302585092994045684;

// Solves the symmetric positive (semi-)definite n x n system g x = b in place
// (Cholesky with a relative ridge on the diagonal for rank-deficient sets);
// returns false when it is singular even so.
RDL_HD inline bool SolveSpd(double (&g)[kMaxTerms][kMaxTerms], double (&b)[kMaxTerms],
                            int n) {
  double scale = 0.0;
  for (int i = 0; i < n; ++i) scale = g[i][i] > scale ? g[i][i] : scale;
  if (!(scale > 0.0)) return false;
  for (int i = 0; i < n; ++i) g[i][i] += 1e-14 * scale;
  for (int j = 0; j < n; ++j) {
    double d = g[j][j];
    for (int k = 0; k < j; ++k) d -= g[j][k] * g[j][k];
    if (!(d > 0.0)) return false;
    d = sqrt(d);
    g[j][j] = d;
    for (int i = j + 1; i < n; ++i) {
      double v = g[i][j];
      for (int k = 0; k < j; ++k) v -= g[i][k] * g[j][k];
      g[i][j] = v / d;
    }
  }
  for (int i = 0; i < n; ++i) {  // L z = b
    double v = b[i];
    for (int k = 0; k < i; ++k) v -= g[i][k] * b[k];
    b[i] = v / g[i][i];
  }
  for (int i = n - 1; i >= 0; --i) {  // L^T x = z
    double v = b[i];
    for (int k = i + 1; k < n; ++k) v -= g[k][i] * b[k];
    b[i] = v / g[i][i];
  }
  return true;
}

// exponent sum_{k>=1} a_k lg^k (Horner)
RDL_HD inline double Exponent(const double* a, int n, double lg) {
  double e = 0.0;
  for (int k = n - 1; k >= 1; --k) e = (e + a[k]) * lg;
  return e;
}

RDL_HD inline double SquaredError(const double* a, int n, double s, const double* lg,
                                  const double* y, int m) {
  double sse = 0.0;
  for (int i = 0; i < m; ++i) {
    const double r = y[i] - s * exp(kLn10 * (a[0] + Exponent(a, n, lg[i])));
    sse += r * r;
  }
  return sse;
}

// terms[0..f.n_terms) of the channel spectrum y[0..f.n_channels)
RDL_HD inline void Fit(const rdl_logpoly& f, const float* values, float* terms) {
  const int n_terms = int(f.n_terms);
  for (int k = 0; k < n_terms; ++k) terms[k] = 0.0f;
  double lg[kMaxCh], y[kMaxCh];
  int m = 0;
  double sum = 0.0;
  for (int c = 0; c < int(f.n_channels); ++c)
    if ((f.fit_mask >> c) & 1u) {
      lg[m] = f.lg[c];
      y[m] = double(values[c]);
      sum += y[m];
      ++m;
    }
  if (m == 0 || n_terms == 0) return;
  const double mean = sum / double(m);
  if (n_terms == 1) {
    terms[0] = float(mean);
    return;
  }
  const double s = mean >= 0.0 ? 1.0 : -1.0;
  // 2. log-space start over the points on the mean's side of zero
  double a[kMaxTerms];
  for (int k = 0; k < kMaxTerms; ++k) a[k] = 0.0;
  int q = 0;
  for (int i = 0; i < m; ++i) q += s * y[i] > 0.0 ? 1 : 0;
  if (q == 0) {
    terms[0] = float(mean);
    return;
  }
  int d = q < n_terms ? q : n_terms;
  {
    double g[kMaxTerms][kMaxTerms], b[kMaxTerms];
    for (int r = 0; r < d; ++r) {
      b[r] = 0.0;
      for (int c = 0; c < d; ++c) g[r][c] = 0.0;
    }
    for (int i = 0; i < m; ++i) {
      if (!(s * y[i] > 0.0)) continue;
      const double ly = log10(s * y[i]);
      double pr = 1.0;
      for (int r = 0; r < d; ++r) {
        double pc = 1.0;
        for (int c = 0; c < d; ++c) {
          g[r][c] += pr * pc;
          pc *= lg[i];
        }
        b[r] += pr * ly;
        pr *= lg[i];
      }
    }
    while (d > 1 && !SolveSpd(g, b, d)) {  // degenerate: fewer terms
      --d;
      for (int r = 0; r < d; ++r) {
        b[r] = 0.0;
        for (int c = 0; c < d; ++c) g[r][c] = 0.0;
      }
      for (int i = 0; i < m; ++i) {
        if (!(s * y[i] > 0.0)) continue;
        const double ly = log10(s * y[i]);
        double pr = 1.0;
        for (int r = 0; r < d; ++r) {
          double pc = 1.0;
          for (int c = 0; c < d; ++c) {
            g[r][c] += pr * pc;
            pc *= lg[i];
          }
          b[r] += pr * ly;
          pr *= lg[i];
        }
      }
    }
    if (d == 1) {
      double acc = 0.0;
      for (int i = 0; i < m; ++i)
        if (s * y[i] > 0.0) acc += log10(s * y[i]);
      b[0] = acc / double(q);
    }
    for (int k = 0; k < d; ++k) a[k] = b[k];
  }
  // 3. Gauss-Newton in linear space on all n_terms parameters
  double sse = SquaredError(a, n_terms, s, lg, y, m);
  for (int it = 0; it < 32; ++it) {
    double g[kMaxTerms][kMaxTerms], b[kMaxTerms];
    for (int r = 0; r < n_terms; ++r) {
      b[r] = 0.0;
      for (int c = 0; c < n_terms; ++c) g[r][c] = 0.0;
    }
    for (int i = 0; i < m; ++i) {
      const double fi = s * exp(kLn10 * (a[0] + Exponent(a, n_terms, lg[i])));
      const double r_i = y[i] - fi;
      double jr = fi * kLn10;  // d f / d a_k = f ln10 lg^k
      double jv[kMaxTerms];
      for (int k = 0; k < n_terms; ++k) {
        jv[k] = jr;
        jr *= lg[i];
      }
      for (int r = 0; r < n_terms; ++r) {
        for (int c = 0; c < n_terms; ++c) g[r][c] += jv[r] * jv[c];
        b[r] += jv[r] * r_i;
      }
    }
    if (!SolveSpd(g, b, n_terms)) break;
    double step = 1.0, next = sse;
    double trial[kMaxTerms];
    bool accepted = false;
    for (int h = 0; h < 24; ++h) {
      for (int k = 0; k < n_terms; ++k) trial[k] = a[k] + step * b[k];
      next = SquaredError(trial, n_terms, s, lg, y, m);
      if (next <= sse) {
        accepted = true;
        break;
      }
      step *= 0.5;
    }
    if (!accepted) break;
    for (int k = 0; k < n_terms; ++k) a[k] = trial[k];
    const double change = sse - next;
    sse = next;
    if (!(change > 1e-13 * sse) || sse == 0.0) break;
  }
  terms[0] = float(s * exp(kLn10 * a[0]));
  for (int k = 1; k < n_terms; ++k) terms[k] = float(a[k]);
}

// S(nu) for lg = log10(nu / nu_ref) from float terms
RDL_HD inline float Evaluate(const float* terms, int n_terms, double lg) {
  if (n_terms <= 0) return 0.0f;
  double e = 0.0;
  for (int k = n_terms - 1; k >= 1; --k) e = (e + double(terms[k])) * lg;
  return float(double(terms[0]) * exp(kLn10 * e));
}

// SpectralFitter::FitAndEvaluate on one channel spectrum, in place
RDL_HD inline void FitAndEvaluate(const rdl_logpoly& f, float* values) {
  float terms[kMaxTerms];
  Fit(f, values, terms);
  for (int c = 0; c < int(f.n_channels); ++c)
    values[c] = Evaluate(terms, int(f.n_terms), f.lg[c]);
}

// PerformSpectralFit: values ordered [channel][pol]; each polarization's
// channel spectrum is fitted and evaluated in place
RDL_HD inline void PerformSpectralFit(const rdl_logpoly& f, uint32_t n_pol, float* values) {
  for (uint32_t p = 0; p < n_pol; ++p) {
    float ch[kMaxCh];
    for (uint32_t c = 0; c < f.n_channels; ++c) ch[c] = values[c * n_pol + p];
    FitAndEvaluate(f, ch);
    for (uint32_t c = 0; c < f.n_channels; ++c) values[c * n_pol + p] = ch[c];
  }
}

}  // namespace lp
}  // namespace rdl
