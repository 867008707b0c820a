// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
// See fft.h for what this restates and why it is double precision.
#include "fft.h"

#include <atomic>

namespace oracle {

namespace {
std::atomic<size_t> g_nthreads{1};
std::mutex g_plan_mutex;
std::map<size_t, std::unique_ptr<FftPlan>> g_plans;
}  // namespace

size_t NThreads() { return g_nthreads.load(); }
void SetNThreads(size_t n) { g_nthreads.store(n == 0 ? 1 : n); }

const FftPlan& GetPlan(size_t n) {
  std::lock_guard<std::mutex> lock(g_plan_mutex);
  auto it = g_plans.find(n);
  if (it == g_plans.end())
    it = g_plans.emplace(n, std::make_unique<FftPlan>(n)).first;
  return *it->second;
}

void Fft2d(cplx* data, size_t width, size_t height, bool inverse) {
  const FftPlan& row_plan = GetPlan(width);
  const FftPlan& col_plan = GetPlan(height);
  ParallelFor(0, height, [&](size_t y0, size_t y1) {
    std::vector<cplx> scratch(row_plan.ScratchSize());
    for (size_t y = y0; y != y1; ++y) {
      if (inverse)
        row_plan.Inverse(data + y * width, scratch.data());
      else
        row_plan.Forward(data + y * width, scratch.data());
    }
  });
  constexpr size_t kBlock = 8;
  const size_t n_blocks = (width + kBlock - 1) / kBlock;
  ParallelFor(0, n_blocks, [&](size_t b0, size_t b1) {
    std::vector<cplx> scratch(col_plan.ScratchSize());
    std::vector<cplx> cols(kBlock * height);
    for (size_t b = b0; b != b1; ++b) {
      const size_t x0 = b * kBlock;
      const size_t nx = std::min(kBlock, width - x0);
      for (size_t y = 0; y != height; ++y)
        for (size_t i = 0; i != nx; ++i)
          cols[i * height + y] = data[y * width + x0 + i];
      for (size_t i = 0; i != nx; ++i) {
        if (inverse)
          col_plan.Inverse(cols.data() + i * height, scratch.data());
        else
          col_plan.Forward(cols.data() + i * height, scratch.data());
      }
      for (size_t y = 0; y != height; ++y)
        for (size_t i = 0; i != nx; ++i)
          data[y * width + x0 + i] = cols[i * height + y];
    }
  });
}

void ConvolveCircular(float* image, const float* kernel, size_t width,
                      size_t height) {
  const size_t n = width * height;
  // Pack image into the real part and kernel into the imaginary part: one
  // forward complex FFT yields both spectra via Hermitian symmetry.
  std::vector<cplx> z(n);
  ParallelFor(0, n, [&](size_t a, size_t b) {
    for (size_t i = a; i != b; ++i) z[i] = cplx(image[i], kernel[i]);
  });
  Fft2d(z.data(), width, height, false);
  std::vector<cplx> c(n);
  ParallelFor(0, height, [&](size_t y0, size_t y1) {
    for (size_t y = y0; y != y1; ++y) {
      const size_t ny = (height - y) % height;
      for (size_t x = 0; x != width; ++x) {
        const size_t nx = (width - x) % width;
        const cplx zk = z[y * width + x];
        const cplx zn = std::conj(z[ny * width + nx]);
        const cplx a = 0.5 * (zk + zn);
        const cplx bb = (zk - zn) * cplx(0.0, -0.5);
        c[y * width + x] = a * bb;
      }
    }
  });
  Fft2d(c.data(), width, height, true);
  const double norm = 1.0 / double(n);
  ParallelFor(0, n, [&](size_t a, size_t b) {
    for (size_t i = a; i != b; ++i) image[i] = float(c[i].real() * norm);
  });
}

}  // namespace oracle
