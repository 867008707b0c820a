// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Double-precision FFT used by the CPU restatement of Radler's convolutions.
// Radler itself calls schaapcommon::math::Convolve (FFTW 3.3.8 float, not
// present in /root/reference: external/schaapcommon is an empty submodule).
// Its contract, inferred from the call sites
//   cpp/algorithms/multiscale/multiscale_transforms.cc:16-20
//   cpp/algorithms/subminor_loop.cc:201-211
// is a circular convolution at the given size of `image` with a kernel whose
// origin is index 0, normalised so a unit delta kernel is the identity.
// This oracle computes that convolution in double precision (more accurate
// than FFTW float); GPU results (rocFFT float) are compared within tolerance.
#pragma once

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstddef>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace oracle {

using cplx = std::complex<double>;

size_t NThreads();
void SetNThreads(size_t n);

// Static partition of [begin,end) over NThreads() std::threads, like
// aocommon::StaticFor (cpp/algorithms/threaded_deconvolution_tools.cc:22).
inline void ParallelFor(size_t begin, size_t end,
                        const std::function<void(size_t, size_t)>& fn) {
  const size_t n = end > begin ? end - begin : 0;
  const size_t nt = std::min(NThreads(), std::max<size_t>(n, 1));
  if (nt <= 1 || n < 2) {
    fn(begin, end);
    return;
  }
  std::vector<std::thread> threads;
  threads.reserve(nt);
  for (size_t t = 0; t != nt; ++t) {
    const size_t s = begin + n * t / nt;
    const size_t e = begin + n * (t + 1) / nt;
    threads.emplace_back([&fn, s, e] { fn(s, e); });
  }
  for (auto& th : threads) th.join();
}

class FftPlan {
 public:
  explicit FftPlan(size_t n) : n_(n) {
    size_t m = n;
    for (size_t p : {4, 2, 3, 5, 7}) {
      while (m % p == 0) {
        factors_.push_back(p);
        m /= p;
      }
    }
    for (size_t p = 11; m > 1 && p * p <= m; p += 2) {
      while (m % p == 0) {
        factors_.push_back(p);
        m /= p;
      }
    }
    if (m > 1) factors_.push_back(m);
    size_t max_p = 1;
    for (size_t p : factors_) max_p = std::max(max_p, p);
    twiddles_.resize(n);
    for (size_t k = 0; k != n; ++k)
      twiddles_[k] = std::polar(1.0, -2.0 * M_PI * double(k) / double(n));
    if (max_p > 13) {
      // Bluestein (chirp-z) for sizes with a large prime factor.
      bluestein_ = true;
      size_t m2 = 1;
      while (m2 < 2 * n - 1) m2 *= 2;
      bs_size_ = m2;
      bs_plan_ = std::make_unique<FftPlan>(m2);
      chirp_.resize(n);
      for (size_t k = 0; k != n; ++k) {
        const unsigned long long kk = (unsigned long long)k * k % (2 * n);
        chirp_[k] = std::polar(1.0, -M_PI * double(kk) / double(n));
      }
      std::vector<cplx> b(m2, cplx(0, 0));
      b[0] = std::conj(chirp_[0]);
      for (size_t k = 1; k != n; ++k) {
        b[k] = std::conj(chirp_[k]);
        b[m2 - k] = std::conj(chirp_[k]);
      }
      std::vector<cplx> scratch(m2);
      bs_plan_->Forward(b.data(), scratch.data());
      bs_kernel_ = std::move(b);
    }
  }

  size_t Size() const { return n_; }
  size_t ScratchSize() const { return bluestein_ ? 3 * bs_size_ : n_; }

  // In-place forward transform (sign -1). scratch: ScratchSize() elements.
  void Forward(cplx* data, cplx* scratch) const {
    if (bluestein_) {
      BluesteinForward(data, scratch);
      return;
    }
    std::copy_n(data, n_, scratch);
    Recurse(scratch, data, n_, 1, 0, 1);
  }

  // In-place inverse transform (sign +1, unnormalised).
  void Inverse(cplx* data, cplx* scratch) const {
    for (size_t i = 0; i != n_; ++i) data[i] = std::conj(data[i]);
    Forward(data, scratch);
    for (size_t i = 0; i != n_; ++i) data[i] = std::conj(data[i]);
  }

 private:
  // kissfft-style recursive decimation in time.
  void Recurse(const cplx* in, cplx* out, size_t n, size_t stride,
               size_t factor_index, size_t tw_step) const {
    const size_t p = factors_[factor_index];
    const size_t m = n / p;
    if (m == 1) {
      for (size_t r = 0; r != p; ++r) out[r] = in[r * stride];
    } else {
      for (size_t r = 0; r != p; ++r)
        Recurse(in + r * stride, out + r * m, m, stride * p, factor_index + 1,
                tw_step * p);
    }
    Butterfly(out, m, p, tw_step);
  }

  void Butterfly(cplx* out, size_t m, size_t p, size_t tw_step) const {
    cplx t[64];
    std::vector<cplx> tbig;
    cplx* tp = t;
    if (p > 64) {
      tbig.resize(p);
      tp = tbig.data();
    }
    const size_t n = n_;
    if (p == 2) {
      for (size_t k = 0; k != m; ++k) {
        const cplx a0 = out[k];
        const cplx a1 = out[k + m] * twiddles_[(k * tw_step) % n];
        out[k] = a0 + a1;
        out[k + m] = a0 - a1;
      }
      return;
    }
    if (p == 4) {
      for (size_t k = 0; k != m; ++k) {
        const cplx a0 = out[k];
        const cplx a1 = out[k + m] * twiddles_[(k * tw_step) % n];
        const cplx a2 = out[k + 2 * m] * twiddles_[(2 * k * tw_step) % n];
        const cplx a3 = out[k + 3 * m] * twiddles_[(3 * k * tw_step) % n];
        const cplx t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
        const cplx mit3(t3.imag(), -t3.real());  // -i * t3
        out[k] = t0 + t2;
        out[k + 2 * m] = t0 - t2;
        out[k + m] = t1 + mit3;
        out[k + 3 * m] = t1 - mit3;
      }
      return;
    }
    for (size_t k = 0; k != m; ++k) {
      for (size_t r = 0; r != p; ++r) {
        const size_t idx = (r * k * tw_step) % n;
        tp[r] = out[k + r * m] * twiddles_[idx];
      }
      // size-p DFT with twiddle W_p^{rq} = W_n^{rq n/p}
      const size_t wstep = n / p;
      for (size_t q = 0; q != p; ++q) {
        cplx acc = tp[0];
        for (size_t r = 1; r != p; ++r) {
          const size_t idx = ((r * q) % p) * wstep;
          acc += tp[r] * twiddles_[idx];
        }
        out[k + q * m] = acc;
      }
    }
  }

  void BluesteinForward(cplx* data, cplx* scratch) const {
    cplx* a = scratch;
    cplx* sc = scratch + bs_size_;
    std::fill_n(a, bs_size_, cplx(0, 0));
    for (size_t k = 0; k != n_; ++k) a[k] = data[k] * chirp_[k];
    bs_plan_->Forward(a, sc);
    for (size_t k = 0; k != bs_size_; ++k) a[k] *= bs_kernel_[k];
    bs_plan_->Inverse(a, sc);
    const double inv = 1.0 / double(bs_size_);
    for (size_t k = 0; k != n_; ++k) data[k] = a[k] * chirp_[k] * inv;
  }

  size_t n_;
  std::vector<size_t> factors_;
  std::vector<cplx> twiddles_;
  bool bluestein_ = false;
  size_t bs_size_ = 0;
  std::unique_ptr<FftPlan> bs_plan_;
  std::vector<cplx> chirp_;
  std::vector<cplx> bs_kernel_;
};

const FftPlan& GetPlan(size_t n);

// 2-D in-place complex FFT of a height x width row-major array.
void Fft2d(cplx* data, size_t width, size_t height, bool inverse);

// Circular convolution of `image` (width x height, float) with `kernel`
// (same size, origin at index 0). Result is normalised like
// schaapcommon::math::Convolve and rounded to float.
void ConvolveCircular(float* image, const float* kernel, size_t width,
                      size_t height);

}  // namespace oracle
