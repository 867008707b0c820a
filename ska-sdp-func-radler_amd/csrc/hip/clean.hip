// PSF subtraction and the device-resident Högbom loop.
//
// rdl_subtract_psf replaces ThreadedDeconvolutionTools::SubtractImage ->
// simple_clean::PartialSubtractImage (cpp/algorithms/simple_clean.cc:96-131):
// the window is x in [max(x-W/2,0), min(x+W/2,W)), y in [max(y-H/2,0),
// min(y+H/2,H)) and every pixel gets one fused multiply-add, exactly what GCC
// -O3 -march=native emits for `img - psf*factor`.
//
// rdl_hogbom_run replaces the Högbom branch of
// GenericClean::ExecuteMajorIteration (cpp/algorithms/generic_clean.cc:163-207).
// Each iteration is two launches on one stream: a grid-wide fused
// "subtract PSF_i(window) + square-integrate + argmax partial" pass over the
// image (12 B/px inside the window, 4 B/px outside it, per image) and a
// one-workgroup "reduce + bookkeeping" step that updates the model, the loop
// state and the next component's factors. Loop control lives in device
// memory, so the host enqueues batches of iterations without synchronising;
// launches after the loop ended return immediately.
#include "rdl_internal.h"
#include "logpoly.h"

namespace rdl {

struct Window {
  uint32_t x0, x1, y0, y1;  // image coordinates, half-open
  int32_t off_x, off_y;     // psf(x - off_x, y - off_y)
};

__host__ __device__ inline Window SubtractWindow(uint32_t width,
                                                 uint32_t height, uint32_t x,
                                                 uint32_t y) {
  Window w;
  w.off_x = int32_t(x) - int32_t(width / 2);
  w.off_y = int32_t(y) - int32_t(height / 2);
  w.x0 = w.off_x > 0 ? uint32_t(w.off_x) : 0u;
  w.y0 = w.off_y > 0 ? uint32_t(w.off_y) : 0u;
  w.x1 = x + width / 2;
  if (w.x1 > width) w.x1 = width;
  w.y1 = y + height / 2;
  if (w.y1 > height) w.y1 = height;
  return w;
}

__global__ __launch_bounds__(256) void SubtractKernel(float* image,
                                                      const float* psf,
                                                      uint32_t width, Window w,
                                                      float factor) {
  const uint32_t y = w.y0 + blockIdx.y;
  const size_t row = size_t(y) * width;
  const size_t prow = size_t(int64_t(y) - w.off_y) * width;
  for (uint32_t x = w.x0 + blockIdx.x * blockDim.x + threadIdx.x; x < w.x1;
       x += gridDim.x * blockDim.x) {
    const float p = psf[prow + size_t(int64_t(x) - w.off_x)];
    image[row + x] = __builtin_fmaf(-p, factor, image[row + x]);
  }
}

// ---------------------------------------------------------------- Högbom
struct HogbomState {
  uint64_t iteration;
  uint64_t first_iteration;
  uint32_t done;
  uint32_t peak_index;
  float peak_value;
  int32_t found;
  int32_t diverging;
  uint32_t pad;
  float factors[RDL_MAX_IMAGES];
};

struct HogbomArgs {
  float* residuals;
  float* models;
  const float* psfs;
  const uint8_t* mask;
  const float* spectral;  // n_images x n_images spectral-fit map, or nullptr
  const float* rms;       // RMS factor image, or nullptr
  HogbomState* state;
  uint64_t* partials;
  uint32_t* trace;
  uint64_t trace_cap;
  uint32_t width, height, n_images, n_pol;
  uint32_t bx0, bx1, by0, by1;  // peak-finder border box
  uint32_t rows_per_block;
  uint32_t n_blocks;
  rdl_integration integ;
  float gain, threshold, initial_max, divergence_limit;
  uint64_t max_iterations;
  int32_t allow_negative, stop_on_negative;
  rdl_logpoly lp;  // log-polynomial fit (has_lp), instead of spectral
  int32_t has_lp;
};

// Iteration pass: subtract the current component from every image inside its
// window, square-integrate, per-block argmax key.
template <int NI>
__global__ __launch_bounds__(256) void HogbomPass(HogbomArgs a) {
  __shared__ uint64_t lds[16];
  const HogbomState& st = *a.state;
  if (st.done) return;
  const uint32_t n = a.width * a.height;
  const uint32_t px = st.peak_index % a.width, py = st.peak_index / a.width;
  const Window w = SubtractWindow(a.width, a.height, px, py);
  float f[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) f[i] = i < int(a.n_images) ? st.factors[i] : 0.0f;
  uint64_t best = 0;
  const uint32_t y0 = blockIdx.x * a.rows_per_block;
  const uint32_t y1 = min(a.height, y0 + a.rows_per_block);
  for (uint32_t y = y0; y < y1; ++y) {
    const bool in_wy = y >= w.y0 && y < w.y1;
    const bool in_by = y >= a.by0 && y < a.by1;
    if (!in_wy && !in_by) continue;
    for (uint32_t x = threadIdx.x; x < a.width; x += blockDim.x) {
      const uint32_t idx = y * a.width + x;
      const bool in_w = in_wy && x >= w.x0 && x < w.x1;
      float v[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if (i >= int(a.n_images)) {
          v[i] = 0.0f;
          continue;
        }
        float r = a.residuals[size_t(i) * n + idx];
        if (in_w) {
          const float* psf = a.psfs + size_t(i / a.n_pol) * n;
          const float pv = psf[size_t(int64_t(y) - w.off_y) * a.width +
                               size_t(int64_t(x) - w.off_x)];
          r = __builtin_fmaf(-pv, f[i], r);
          a.residuals[size_t(i) * n + idx] = r;
        }
        v[i] = r;
      }
      if (in_by && x >= a.bx0 && x < a.bx1 && (!a.mask || a.mask[idx])) {
        float integ = IntegratePixel(a.integ, [&](uint32_t k) {
          float r = v[0];
#pragma unroll
          for (int j = 1; j < NI; ++j) r = (uint32_t(j) == k) ? v[j] : r;
          return r;
        });
        if (a.rms) integ *= a.rms[idx];  // GenericClean::FindPeak (:258-264)
        const uint64_t k = PeakKey(integ, a.allow_negative, idx);
        best = k > best ? k : best;
      }
    }
  }
  best = BlockMaxU64(best, lds);
  if (threadIdx.x == 0) a.partials[blockIdx.x] = best;
}

__device__ float IntegratedAt(const HogbomArgs& a, uint32_t idx) {
  const uint32_t n = a.width * a.height;
  return IntegratePixel(a.integ,
                        [&](uint32_t k) { return a.residuals[size_t(k) * n + idx]; });
}

// Prepares the next component: evaluates the loop condition
// (generic_clean.cc:169-171) and, if it holds, computes the N_img factors,
// updates the model (generic_clean.cc:182-192) and records the trace.
__device__ void HogbomPrepare(const HogbomArgs& a, HogbomState& st) {
  const float m = st.peak_value;
  const bool go = st.found && fabsf(m) > a.threshold &&
                  st.iteration < a.max_iterations &&
                  !(m < 0.0f && a.stop_on_negative) && !st.diverging;
  if (!go) {
    st.done = 1;
    return;
  }
  const uint32_t n = a.width * a.height;
  const uint32_t idx = st.peak_index;
  if (a.has_lp) {  // log-polynomial PerformSpectralFit before the gain
    float v[RDL_MAX_IMAGES];
    for (uint32_t i = 0; i < a.n_images; ++i) v[i] = a.residuals[size_t(i) * n + idx];
    lp::PerformSpectralFit(a.lp, a.n_pol, v);
    for (uint32_t i = 0; i < a.n_images; ++i) {
      const float f = v[i] * a.gain;
      st.factors[i] = f;
      a.models[size_t(i) * n + idx] += f;
    }
  }
  for (uint32_t i = 0; i < a.n_images && !a.has_lp; ++i) {
    float v = a.residuals[size_t(i) * n + idx];
    if (a.spectral) {  // PerformSpectralFit before the gain (:186-189)
      v = 0.0f;
      for (uint32_t q = 0; q < a.n_images; ++q)
        v = __builtin_fmaf(a.spectral[i * a.n_images + q],
                           a.residuals[size_t(q) * n + idx], v);
    }
    v *= a.gain;
    st.factors[i] = v;
    a.models[size_t(i) * n + idx] += v;
  }
  const uint64_t t = st.iteration - st.first_iteration;
  if (a.trace && t < a.trace_cap) {
    a.trace[2 * t] = idx % a.width;
    a.trace[2 * t + 1] = idx / a.width;
  }
}

__global__ __launch_bounds__(1024) void HogbomStep(HogbomArgs a, int init) {
  __shared__ uint64_t lds[16];
  HogbomState& st = *a.state;
  if (st.done) return;
  if (!init) {
    uint64_t best = 0;
    for (uint32_t i = threadIdx.x; i < a.n_blocks; i += blockDim.x)
      best = a.partials[i] > best ? a.partials[i] : best;
    best = BlockMaxU64(best, lds);
    if (threadIdx.x != 0) return;
    // FindPeak (generic_clean.cc:199 -> Find / FindWithMask)
    if (best != 0) {
      st.peak_index = 0xffffffffu - uint32_t(best & 0xffffffffu);
      st.found = 1;
    } else if (!a.mask) {
      st.peak_index = 0;  // Avx<>: no qualifying pixel -> index 0
      st.found = 1;
    } else {
      st.found = 0;
    }
    if (st.found) {
      st.peak_value = IntegratedAt(a, st.peak_index);
      if (a.rms) st.peak_value *= a.rms[st.peak_index];
    }
    if (st.found && a.divergence_limit != 0.0f)
      st.diverging = fabsf(st.peak_value) > a.initial_max * a.divergence_limit;
    st.iteration += 1;
  } else if (threadIdx.x != 0) {
    return;
  }
  HogbomPrepare(a, st);
}

}  // namespace rdl

extern "C" {

int rdl_subtract_psf(rdl_session* s, float* d_image, const float* d_psf,
                     uint32_t width, uint32_t height, uint32_t x, uint32_t y,
                     float factor) {
  RDL_ARG_CHECK(s && d_image && d_psf, "NULL argument");
  RDL_ARG_CHECK(x < width && y < height, "component outside the image");
  const rdl::Window w = rdl::SubtractWindow(width, height, x, y);
  if (w.x1 <= w.x0 || w.y1 <= w.y0) return RDL_OK;
  const uint32_t nx = w.x1 - w.x0;
  dim3 grid(std::min<uint32_t>(rdl::DivUp(nx, 256), 8), w.y1 - w.y0);
  rdl::ScopedTiming t(s, "subtract_psf", double(nx) * (w.y1 - w.y0) * 12.0);
  rdl::SubtractKernel<<<grid, 256, 0, s->stream>>>(d_image, d_psf, width, w,
                                                   factor);
  RDL_HIP_CHECK(hipGetLastError());
  return RDL_OK;
}

int rdl_hogbom_run(rdl_session* s, float* d_residuals, float* d_models,
                   const float* d_psfs, const rdl_hogbom_params* p,
                   rdl_hogbom_result* out, uint32_t* h_trace,
                   uint64_t trace_cap) {
  RDL_ARG_CHECK(s && d_residuals && d_models && d_psfs && p && out,
                "NULL argument");
  RDL_ARG_CHECK(p->n_images >= 1 && p->n_images <= RDL_MAX_IMAGES,
                "n_images out of range");
  RDL_ARG_CHECK(p->n_pol >= 1 && p->n_images % p->n_pol == 0, "bad n_pol");
  RDL_ARG_CHECK(p->width > 0 && p->height > 0, "empty image");
  rdl::HogbomArgs a{};
  a.residuals = d_residuals;
  a.models = d_models;
  a.psfs = d_psfs;
  a.mask = p->d_mask;
  a.spectral = p->logpoly ? nullptr : p->d_spectral;
  a.rms = p->d_rms;
  if (p->logpoly) {
    RDL_ARG_CHECK(p->logpoly->n_channels * p->n_pol == p->n_images &&
                      p->logpoly->n_channels <= RDL_LOGPOLY_MAX_CHANNELS &&
                      p->logpoly->n_terms >= 1 &&
                      p->logpoly->n_terms <= RDL_LOGPOLY_MAX_TERMS,
                  "log-polynomial fit does not match the images");
    a.lp = *p->logpoly;
    a.has_lp = 1;
  }
  a.width = p->width;
  a.height = p->height;
  a.n_images = p->n_images;
  a.n_pol = p->n_pol;
  a.integ = p->integ;
  a.gain = p->gain;
  a.threshold = p->threshold;
  a.initial_max = p->initial_max;
  a.divergence_limit = p->divergence_limit;
  a.max_iterations = p->max_iterations;
  a.allow_negative = p->allow_negative;
  a.stop_on_negative = p->stop_on_negative;
  a.bx0 = p->h_border;
  a.bx1 = p->width - p->h_border;
  if (a.bx1 < a.bx0 || a.bx1 > p->width) a.bx1 = a.bx0;
  a.by0 = p->v_border;
  a.by1 = p->height - p->v_border;
  if (a.by1 < a.by0 || a.by1 > p->height) a.by1 = a.by0;
  const uint32_t target_blocks = 2048;
  a.rows_per_block = (p->height + target_blocks - 1) / target_blocks;
  a.n_blocks = (p->height + a.rows_per_block - 1) / a.rows_per_block;

  // device state + partials + trace
  const uint64_t n_trace = (h_trace && trace_cap) ? trace_cap : 0;
  const size_t state_bytes = (sizeof(rdl::HogbomState) + 255) / 256 * 256;
  const size_t part_bytes = size_t(a.n_blocks) * sizeof(uint64_t);
  const size_t trace_bytes = n_trace * 2 * sizeof(uint32_t);
  RDL_TRY(s->EnsureScratch(s->loop_state, state_bytes + part_bytes + trace_bytes));
  void* buf = s->loop_state.ptr;
  a.state = static_cast<rdl::HogbomState*>(buf);
  a.partials = reinterpret_cast<uint64_t*>(static_cast<char*>(buf) + state_bytes);
  a.trace = n_trace ? reinterpret_cast<uint32_t*>(static_cast<char*>(buf) +
                                                  state_bytes + part_bytes)
                    : nullptr;
  a.trace_cap = n_trace;
  rdl::HogbomState init{};
  init.iteration = p->iteration_start;
  init.first_iteration = p->iteration_start;
  init.done = 0;
  init.peak_index = p->start_y * p->width + p->start_x;
  init.peak_value = p->start_value;
  init.found = p->start_found;
  init.diverging = 0;
  RDL_HIP_CHECK(hipMemcpyAsync(a.state, &init, sizeof(init),
                               hipMemcpyHostToDevice, s->stream));
  const double pass_bytes = double(p->width) * p->height * p->n_images * 12.0;
  {
    rdl::ScopedTiming t(s, "hogbom_step", 0.0);
    rdl::HogbomStep<<<1, 1024, 0, s->stream>>>(a, 1);
  }
  rdl::HogbomState st{};
  const uint64_t batch = 32;
  while (true) {
    for (uint64_t b = 0; b < batch; ++b) {
      {
        rdl::ScopedTiming t(s, "hogbom_pass", pass_bytes);
        if (p->n_images == 1)
          rdl::HogbomPass<1><<<a.n_blocks, 256, 0, s->stream>>>(a);
        else if (p->n_images <= 4)
          rdl::HogbomPass<4><<<a.n_blocks, 256, 0, s->stream>>>(a);
        else if (p->n_images <= 16)
          rdl::HogbomPass<16><<<a.n_blocks, 256, 0, s->stream>>>(a);
        else
          rdl::HogbomPass<RDL_MAX_IMAGES><<<a.n_blocks, 256, 0, s->stream>>>(a);
      }
      {
        rdl::ScopedTiming t(s, "hogbom_step", 0.0);
        rdl::HogbomStep<<<1, 1024, 0, s->stream>>>(a, 0);
      }
    }
    RDL_HIP_CHECK(hipGetLastError());
    const rdl::SmallRead r{&st, a.state, sizeof(st)};
    RDL_TRY(rdl::ReadSmall(s, &r, 1));
    if (st.done) break;
  }
  if (n_trace) {
    const uint64_t n = std::min<uint64_t>(st.iteration - st.first_iteration,
                                          n_trace);
    RDL_HIP_CHECK(hipMemcpyAsync(h_trace, a.trace, n * 2 * sizeof(uint32_t),
                                 hipMemcpyDeviceToHost, s->stream));
  }
  RDL_HIP_CHECK(hipStreamSynchronize(s->stream));
  out->iteration = st.iteration;
  out->found = st.found;
  out->peak = st.peak_value;
  out->x = st.peak_index % p->width;
  out->y = st.peak_index / p->width;
  out->diverging = st.diverging;
  return RDL_OK;
}

}  // extern "C"
