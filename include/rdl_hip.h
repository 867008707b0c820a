/*
 * rdl_hip.h — C-ABI of the MI355X-native Radler CLEAN engine (librdl_hip.so).
 *
 * Plain pointers and sizes only: no C++ or torch types cross this boundary.
 * Device pointers ("d_" prefix) are addresses returned by rdl_malloc (or any
 * hipMalloc'd memory on the session's device). Every call is ordered on the
 * session's HIP stream; calls that return values to the host (peaks, loop
 * results) synchronise that stream. All functions return RDL_OK (0) or an
 * error code; rdl_last_error() gives the thread's last message. The host C++
 * library (libradler_amd) wraps these calls and rethrows std::runtime_error
 * where the reference throws.
 *
 * Each entry point cites the reference interface it replaces
 * (paths relative to ska-sdp-func-radler/, snapshot 2025-04-10).
 */
#ifndef RDL_HIP_H_
#define RDL_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RDL_OK 0
#define RDL_ERR_ARG 1
#define RDL_ERR_HIP 2
#define RDL_ERR_FFT 3
#define RDL_ERR_TIMEOUT 4
#define RDL_ERR_UNSUPPORTED 5

/* Maximum images in one ImageSet handled by the fused kernels
 * (channels x polarizations). */
#define RDL_MAX_IMAGES 64

typedef struct rdl_session rdl_session;
typedef struct rdl_fft rdl_fft;
typedef struct rdl_subminor rdl_subminor;

/* ---------------------------------------------------------------- runtime */
const char* rdl_last_error(void);
const char* rdl_version(void);
int rdl_device_count(int* count);
int rdl_session_create(int device, rdl_session** out);
int rdl_session_destroy(rdl_session* s);
/* Releases everything this library holds, process-wide: drains and destroys
 * every session's streams and events, its RCCL communicator, the rocFFT
 * plans, and frees every device, pinned and mapped host block (block caches,
 * scratch, plan work buffers, buffers of host objects still alive). Afterwards
 * every destroy/free entry point is a no-op and rdl_session_create fails.
 * Runs automatically at process exit (an atexit handler registered by the
 * first rdl_session_create, so it precedes the HIP runtime's own exit
 * handlers; RDL_EXIT_SHUTDOWN=0 disables it). The reference has no device
 * state to release (its images are host memory freed by their destructors,
 * cpp/radler.cc); this is the device-side counterpart of process teardown. */
int rdl_shutdown(void);
int rdl_session_sync(rdl_session* s);
/* hipStream_t of the session, for callers that record events on it. */
void* rdl_session_stream(rdl_session* s);
/* Two launch lanes on one session, for independent chains that overlap on
 * the device (the per-scale inverse transforms + peak searches of
 * FindActiveScaleConvolvedMaxima, multiscale_algorithm.cc:578-634 of the
 * reference, which runs them on threads). rdl_session_fork orders a second
 * stream after everything issued so far; rdl_session_lane(s, 1) sends the
 * following launches there (0: back to the session's stream);
 * rdl_session_join orders the session's stream after the second lane and
 * selects lane 0. Launchers that keep scratch (the four-step column
 * scratch) keep one per lane; fused peak searches keep one partials area
 * per peak slot. rdl_malloc / rdl_free (stream-ordered on lane 0) must not
 * be called while lane 1 is selected. */
int rdl_session_fork(rdl_session* s);
int rdl_session_lane(rdl_session* s, int lane);
int rdl_session_join(rdl_session* s);
/* Make the session's device current for the calling host thread (worker
 * threads of the subimage pool call this once before allocating). */
int rdl_session_bind(rdl_session* s);
/* `n_sharing` sessions run concurrently on this session's device: grids of
 * the workgroup-cooperative kernels (the multi-workgroup sub-minor loop) are
 * capped to n_cus / n_sharing so every concurrent loop stays co-resident.
 * The subimage pool of ParallelDeconvolution sets this
 * (cpp/algorithms/parallel_deconvolution.cc:583-616 runs subimages on
 * settings.parallel.max_threads threads). */
int rdl_session_set_concurrency(rdl_session* s, uint32_t n_sharing);

int rdl_malloc(rdl_session* s, size_t bytes, void** d_out);
int rdl_free(rdl_session* s, void* d_ptr);
int rdl_memcpy_h2d(rdl_session* s, void* d_dst, const void* h_src, size_t bytes);
int rdl_memcpy_d2h(rdl_session* s, void* h_dst, const void* d_src, size_t bytes);
int rdl_memcpy_d2d(rdl_session* s, void* d_dst, const void* d_src, size_t bytes);
int rdl_memset_zero(rdl_session* s, void* d_dst, size_t bytes);
/* Page-locked host memory (hipHostMalloc) for the accessor staging of
 * ImageSet::LoadAndAverage / Store (cpp/image_set.cc:105-140, 290-307):
 * copies from it run at the link rate instead of through pageable bounce
 * buffers. */
int rdl_host_alloc(size_t bytes, void** h_out);
int rdl_host_free(void* h_ptr);
/* Device-to-device copy between GPUs (xGMI peer copy when the devices
 * differ), ordered on the session's stream. */
int rdl_memcpy_peer(rdl_session* s, void* d_dst, int dst_device,
                    const void* d_src, int src_device, size_t bytes);

/* Per-kernel device timing (HIP events around every launch of a kernel
 * family on the session stream). Used by bench.py's roofline. */
int rdl_timing_enable(rdl_session* s, int enable);
/* Returns accumulated milliseconds and launch count for a kernel family name
 * ("find_peak", "subminor_loop", "fft", "spectrum_multiply", ...). */
int rdl_timing_get(rdl_session* s, const char* family, double* ms,
                   uint64_t* launches, double* bytes);
int rdl_timing_reset(rdl_session* s);
/* The same over EVERY session of the process (the main session, the worker
 * sessions of a subimage pool, sessions already destroyed since the last
 * reset): what one Radler::Perform launched, wherever it ran. Call get/reset
 * only while no other thread launches work. */
int rdl_timing_enable_all(int enable);
/* Record events for this family only (NULL or "": every family); applies to
 * every session. Lets a timed region keep one family's HIP-event timing
 * without the others' per-launch event overhead. */
int rdl_timing_filter_all(const char* family);
int rdl_timing_get_all(const char* family, double* ms, uint64_t* launches,
                       double* bytes);
int rdl_timing_reset_all(void);

/* ------------------------------------------------------------ peak finder */
typedef struct {
  float value;     /* signed image value at (x, y) */
  uint32_t x, y;
  int32_t found;   /* 0 = no qualifying pixel (Simple / FindWithMask) */
} rdl_peak;

/* Replaces math::peak_finder::Find / Avx<bool> / Simple / FindWithMask
 * (cpp/math/peak_finder.h:80-127, peak_finder.cc:19-56, 97-131, 199-253).
 * Box x in [h_border, w-h_border), y in [max(start_y,v_border),
 * min(end_y,h-v_border)); strict '>' from FLT_MIN, first row-major index on
 * ties, NaN never selected, value = signed pixel. d_mask (uint8, may be NULL)
 * selects FindWithMask. avx_semantics=1 reproduces the x86 default Avx<>
 * path: with no qualifying pixel it returns (0,0) and image[0] as found. */
int rdl_find_peak(rdl_session* s, const float* d_image, uint32_t width,
                  uint32_t height, uint32_t start_y, uint32_t end_y,
                  uint32_t h_border, uint32_t v_border, int allow_negative,
                  const uint8_t* d_mask, int avx_semantics, rdl_peak* out);

/* rdl_find_peak without the host round trip: the result goes to device
 * slot `slot` (< RDL_PEAK_SLOTS) and rdl_find_peak_collect reads slots
 * 0..n-1 with one synchronisation (the per-scale peak searches of
 * FindActiveScaleConvolvedMaxima, multiscale_algorithm.cc:578-634, queue
 * back to back instead of idling the device between scales). */
#define RDL_PEAK_SLOTS 64
int rdl_find_peak_enqueue(rdl_session* s, const float* d_image, uint32_t width,
                          uint32_t height, uint32_t start_y, uint32_t end_y,
                          uint32_t h_border, uint32_t v_border, int allow_negative,
                          const uint8_t* d_mask, int avx_semantics, uint32_t slot);
int rdl_find_peak_collect(rdl_session* s, uint32_t n, rdl_peak* out);

/* Sum of squares in double (ThreadedDeconvolutionTools::RMS,
 * cpp/algorithms/threaded_deconvolution_tools.h:40-44; logging only). */
int rdl_rms(rdl_session* s, const float* d_image, size_t n, float* out);

/* --------------------------------------------------------- PSF subtraction */
/* Replaces ThreadedDeconvolutionTools::SubtractImage ->
 * simple_clean::PartialSubtractImage (threaded_deconvolution_tools.cc:18-28,
 * simple_clean.cc:96-131): image -= psf(shifted to x,y) * factor over the
 * reference's window, one fused multiply-add per pixel. */
int rdl_subtract_psf(rdl_session* s, float* d_image, const float* d_psf,
                     uint32_t width, uint32_t height, uint32_t x, uint32_t y,
                     float factor);

/* ------------------------------------------------------ ImageSet integration */
#define RDL_INTEGRATE_LINEAR 0        /* GetLinearIntegratedWithNormalChannels */
#define RDL_INTEGRATE_SQUARE 1        /* GetSquareIntegratedWithNormalChannels */
#define RDL_INTEGRATE_SQUARED_JOINS 2 /* GetSquareIntegratedWithSquaredChannels */
typedef struct {
  uint32_t n_images;       /* images in the set, index = channel*n_pol + pol */
  uint32_t n_pol;
  uint32_t n_channels;
  uint32_t mode;           /* RDL_INTEGRATE_* */
  uint32_t copy_fast_path; /* image_set.cc:425-430 / :289-301 (1 image) */
  uint32_t pol_mask;       /* bit p: polarization p is joined (linked) */
  float weights[RDL_MAX_IMAGES]; /* channel weight of each image; 0 skips */
  /* LINEAR: float(pol_factor/sum w); SQUARE with 1 channel: sqrtf(pol_factor);
   * SQUARE with >1 channel: float(sqrtf(pol_factor)/sum w);
   * SQUARED_JOINS: float(sqrt(pol_factor/sum w)) (0 when sum w == 0). */
  float factor;
} rdl_integration;

/* Replaces ImageSet::GetLinearIntegrated / GetSquareIntegrated
 * (cpp/image_set.cc:309-462): images are n_images consecutive planes of
 * `n` floats each. Summation order and FMA placement follow the reference. */
int rdl_integrate(rdl_session* s, const rdl_integration* integ,
                  const float* d_images, size_t n, float* d_dest);

/* dest = a*alpha (assign=1) or dest = fma(a, alpha, dest) (assign=0);
 * aocommon Image::AddWithFactor / operator*= used by ImageSet::LoadAndAverage
 * and GetIntegratedPsf (cpp/image_set.cc:105-140, 499-530). */
int rdl_axpy(rdl_session* s, float* d_dest, const float* d_a, size_t n,
             float alpha, int assign);
int rdl_scale(rdl_session* s, float* d_dest, size_t n, float alpha);
/* Double-precision accumulation of ImageSet::LoadAndAveragePsfs
 * (cpp/image_set.cc:167-186): mode 0: dest = float(fma(double(a), alpha,
 * double(dest))); mode 1: dest = float(double(dest) * alpha) (d_a unused). */
int rdl_axpy_f64(rdl_session* s, float* d_dest, const float* d_a, size_t n,
                 double alpha, int mode);
/* dest += a (model accumulation, multiscale_algorithm.cc:457-460). */
int rdl_add(rdl_session* s, float* d_dest, const float* d_a, size_t n);

/* Exact median of values (or of |values - center| when use_center) by radix
 * select on the float order; aocommon Image::MedianAndStdDevFromMAD, used by
 * Radler::Perform (cpp/radler.cc:162-166). */
int rdl_median(rdl_session* s, const float* d_values, size_t n, int use_center,
               float center, float* out);

/* k-th smallest value (of |v - center| when use_center), exact: the
 * std::nth_element of IuwtDeconvolutionAlgorithm::Mad
 * (cpp/algorithms/iuwt_deconvolution_algorithm.cc:104-110, k = n/2). */
int rdl_select_kth(rdl_session* s, const float* d_values, size_t n, int use_center,
                   float center, size_t k, float* out);

/* ------------------------------------------------ IUWT deconvolution pieces */
/* IuwtDeconvolutionAlgorithm::GetMaxAbs (iuwt_deconvolution_algorithm.cc:
 * 112-167): strict '>' from numeric_limits<float>::lowest() over
 * [xb, W-xb) x [yb, H-yb) (and the mask), first index on ties; value is
 * |v| when allow_negative. Nothing qualifying: found = 0, x = W, y = H,
 * value = lowest(). */
int rdl_max_abs(rdl_session* s, const float* d_data, uint32_t width, uint32_t height,
                uint32_t x_border, uint32_t y_border, int allow_negative,
                const uint8_t* d_mask, rdl_peak* out);
/* image_analysis::SelectStructures (cpp/algorithms/iuwt/image_analysis.cc:
 * 227-259) as a per-pixel test: the flood fills it starts from every
 * exceeding pixel only ever reach exceeding pixels of the same box, scale
 * range and prior mask, so the resulting mask is exactly
 *   mask[s][p] = ExceedsThreshold(coeffs[s][p], thresholds[s])
 * for min_scale <= s < end_scale, p in the border box and the prior mask.
 * d_mask holds end_scale planes of width*height bytes; *area = its count
 * (the summed flood-fill area sizes). */
int rdl_iuwt_select(rdl_session* s, const float* d_coeffs, uint32_t width, uint32_t height,
                    uint32_t min_scale, uint32_t end_scale, const float* h_thresholds,
                    uint32_t x_border, uint32_t y_border, const uint8_t* d_prior,
                    uint8_t* d_mask, uint64_t* area);
/* IuwtDecomposition::ApplyMask for the n_scales coefficient planes
 * (iuwt_decomposition.h:284-291; the residual plane is not stored here). */
int rdl_iuwt_apply_mask(rdl_session* s, float* d_coeffs, const uint8_t* d_mask,
                        uint32_t width, uint32_t height, uint32_t n_scales);
/* DotProduct (iuwt_deconvolution_algorithm.cc:169-174) with a double sum. */
int rdl_dot(rdl_session* s, const float* d_a, const float* d_b, size_t n, double* out);
/* Snr's two sums over the coefficient planes (:308-321), double:
 * model_sum = sum m^2, noise_sum = sum (m - n)^2 (n = d_noisy, m = d_model). */
int rdl_iuwt_snr_sums(rdl_session* s, const float* d_noisy, const float* d_model, size_t n,
                      double* model_sum, double* noise_sum);
/* BoundingBox's scans (:180-214): with m = max |v| of the image, h_first[y]
 * and h_last[y] are the first and last x of row y with |v| > m * 0.01
 * (double compare), -1 for rows without any. */
int rdl_bbox_rows(rdl_session* s, const float* d_image, uint32_t width, uint32_t height,
                  int32_t* h_first, int32_t* h_last);
/* float <-> double planes (to_f64: float src -> double dst). */
int rdl_convert(rdl_session* s, const void* d_src, void* d_dst, size_t n, int to_f64);

/* ------------------------------------------------ spectral interpolation */
/* ImageSet::InterpolateAndStoreModel (cpp/image_set.cc:209-288) for a
 * polynomial SpectralFitter: out plane g (g < n_out, contiguous, n floats
 * apart) = sum_c h_coefficients[g * n_in + c] * in plane c, where in plane c
 * starts at d_in + c * in_stride floats. The coefficients are the fit over
 * the n_in deconvolution channels evaluated at original channel g's
 * frequency (a fixed linear map; zero pixels stay zero). n_in, n_out <=
 * RDL_MAX_IMAGES. */
int rdl_spectral_interpolate(rdl_session* s, const float* d_in, size_t in_stride,
                             uint32_t n_in, const float* h_coefficients,
                             uint32_t n_out, float* d_out, size_t n);

/* ------------------------------------------------------------ local RMS */
/* radler::math::rms_image (cpp/math/rms_image.cc:16-125) building blocks.
 * The Gaussian window convolution itself is an FFT convolution of the
 * squared image with the placed kernel (host: csrc/host/rms_image.cc). */
/* Image::Square: dst = src * src. */
int rdl_square(rdl_session* s, const float* d_src, float* d_dst, size_t n);
/* dst = a * b (the `scratch[i] = image[i] * rms_factor[i]` of every
 * RMS-weighted peak search, generic_clean.cc:258-264,
 * multiscale_algorithm.cc:707-713, threaded_deconvolution_tools.cc:84-87). */
int rdl_multiply(rdl_session* s, float* d_dst, const float* d_a, const float* d_b,
                 size_t n);
/* d = sqrt(d * norm) in double (rms_image.cc:32). */
int rdl_rms_finish(rdl_session* s, float* d, size_t n, double norm);
/* schaapcommon::math::RestoreImage's kernel: a box x box Gaussian of peak 1
 * (sigmas in the units of the pixel scales, major axis at `angle`) placed
 * with its centre (box/2, box/2) at the origin of a zeroed width x height
 * plane (PrepareSmallConvolutionKernel placement). */
int rdl_place_gaussian(rdl_session* s, float* d_dest, uint32_t width, uint32_t height,
                       uint32_t box, double pixel_scale_l, double pixel_scale_m,
                       double sigma_major, double sigma_minor, double angle);
/* rms_image::SlidingMinimum (rms_image.cc:35-68): row then column minimum
 * over [max(k, window/2) - window/2, min(k, len - window/2) + window/2).
 * d_scratch: 3 * width * height floats; 2 <= window, window/2 <= both sides. */
int rdl_sliding_min(rdl_session* s, const float* d_in, float* d_out, float* d_scratch,
                    uint32_t width, uint32_t height, uint64_t window);
/* rms = max<float>(rms, |min| * 0.3) (rms_image.cc:88-92). */
int rdl_rms_negativity_limit(rdl_session* s, float* d_rms, const float* d_min,
                             size_t n);
/* rms_image::MakeRmsFactorImage (rms_image.cc:95-125) in place; *lowest_rms
 * = the image minimum; RDL_ERR_ARG when it is negative. */
int rdl_rms_factor(rdl_session* s, float* d_rms, size_t n, double strength,
                   double* lowest_rms);

/* ------------------------------------------------ component optimisation */
/* math::GradientDescent (cpp/math/component_optimization.cc:100-177,
 * 265-321) on planes: the components are the model's non-zero pixels.
 * dst = model != 0 ? sign * src : 0 (CalculateDerivatives' gather). */
int rdl_masked_copy(rdl_session* s, const float* d_model, const float* d_src, float* d_dst,
                    size_t n, float sign);
/* model[i] += values[i] where model[i] != 0 (GradientDescent's update). */
int rdl_masked_add(rdl_session* s, float* d_model, const float* d_values, size_t n);
/* *ab = sum a*b, *aa = sum a*a in double (ApplyLineSearch's two sums). */
int rdl_dot_pair(rdl_session* s, const float* d_a, const float* d_b, size_t n,
                 double* ab, double* aa);

/* ------------------------------------------- log-polynomial spectral fit */
/* schaapcommon's SpectralFitter in kLogPolynomial mode (the fitter behind
 * DeconvolutionAlgorithm::PerformSpectralFit, cpp/algorithms/
 * deconvolution_algorithm.cc:29-46, and ImageSet::InterpolateAndStoreModel,
 * cpp/image_set.cc:238-285): S(nu) = t0 10^(t1 lg + t2 lg^2 + ...),
 * lg = log10(nu / nu_ref), least squares over the channels in fit_mask.
 * Non-linear, so it is passed as this description rather than as a matrix
 * (csrc/hip/logpoly.h states the algorithm). */
#define RDL_LOGPOLY_MAX_CHANNELS 16
#define RDL_LOGPOLY_MAX_TERMS 8
typedef struct {
  uint32_t n_channels;  /* deconvolution channels (per polarization) */
  uint32_t n_terms;     /* 1 .. RDL_LOGPOLY_MAX_TERMS */
  uint32_t fit_mask;    /* bit c: channel c has weight > 0 and is fitted */
  uint32_t reserved;
  double lg[RDL_LOGPOLY_MAX_CHANNELS]; /* log10(nu_c / nu_ref) per channel */
} rdl_logpoly;

/* ImageSet::InterpolateAndStoreModel for log-polynomial fitting, one
 * polarization: d_in holds n_channels planes of n_pixels (plane c at
 * d_in + c * in_stride); every pixel with a non-zero value is fitted and the
 * fit evaluated at out_lg[g] = log10(nu_g / nu_ref) into d_out + g * out_stride
 * (zero pixels give zero). */
int rdl_logpoly_interpolate(rdl_session* s, const float* d_in, size_t in_stride,
                            size_t n_pixels, const rdl_logpoly* fit,
                            const double* out_lg, uint32_t n_out, float* d_out,
                            size_t out_stride);

/* ---------------------------------------------------------------- Högbom */
typedef struct {
  uint32_t width, height;
  uint32_t n_images;
  uint32_t n_pol;          /* psf index of image i = i / n_pol */
  rdl_integration integ;   /* square integration used between iterations */
  float gain;              /* minor loop gain */
  float threshold;         /* first threshold (generic_clean.cc:99-112) */
  float initial_max;       /* |peak| at start, for the divergence test */
  float divergence_limit;
  uint64_t iteration_start, max_iterations;
  int32_t allow_negative, stop_on_negative;
  uint32_t h_border, v_border;
  const uint8_t* d_mask;   /* may be NULL */
  /* starting peak, from a prior rdl_find_peak on the integrated image */
  uint32_t start_x, start_y;
  float start_value;
  int32_t start_found;
  /* DeconvolutionAlgorithm::PerformSpectralFit (deconvolution_algorithm.cc:
   * 29-46) as a linear map: n_images x n_images row-major float matrix,
   * applied to the gathered peak values before the gain (generic_clean.cc:
   * 186); NULL = no fitting. See rdl_spectral_* below. */
  const float* d_spectral;
  /* DeconvolutionAlgorithm::RmsFactorImage (W x H factors multiplied into
   * every peak search, generic_clean.cc:255-264); NULL = none */
  const float* d_rms;
  /* log-polynomial PerformSpectralFit instead of d_spectral (host pointer,
   * copied at the call; NULL = none) */
  const rdl_logpoly* logpoly;
} rdl_hogbom_params;

typedef struct {
  uint64_t iteration;      /* IterationNumber() after the loop */
  float peak;              /* final signed integrated peak */
  uint32_t x, y;
  int32_t found;
  int32_t diverging;
} rdl_hogbom_result;

/* Replaces the Högbom branch of GenericClean::ExecuteMajorIteration
 * (cpp/algorithms/generic_clean.cc:163-207): per iteration gather N_img peak
 * values, model += gain*v, subtract PSF_i, square-integrate, find peak,
 * divergence test. The loop runs device-resident; h_trace (may be NULL)
 * receives x,y per component (2 x uint32 each, up to trace_cap). */
int rdl_hogbom_run(rdl_session* s, float* d_residuals, float* d_models,
                   const float* d_psfs, const rdl_hogbom_params* p,
                   rdl_hogbom_result* out, uint32_t* h_trace,
                   uint64_t trace_cap);

/* ------------------------------------------------------- sub-minor loop */
typedef struct {
  uint32_t width, height;  /* image size (psf size equals image size) */
  uint32_t n_images, n_pol;
  rdl_integration integ;   /* linear integration (subminor_loop.cc:17) */
  uint32_t h_border, v_border;
  int32_t allow_negative, stop_on_negative;
  float threshold;         /* SubMinorLoop::_threshold */
  float gain;
  float divergence_limit;
  uint64_t iteration_start, max_iterations;
  const uint8_t* d_mask;   /* may be NULL */
  /* PerformSpectralFit of each component's gain-scaled values
   * (subminor_loop.cc:64-76) as an n_images x n_images row-major linear map;
   * NULL = no fitting */
  const float* d_spectral;
  /* SubMinorLoop::SetRmsFactorImage: W x H factors multiplied into the
   * selection and the loop's argmax (subminor_loop.cc:13-36, 143-149);
   * NULL = none */
  const float* d_rms;
  /* log-polynomial PerformSpectralFit of each component's gain-scaled values
   * instead of d_spectral (host pointer, copied at the call; NULL = none) */
  const rdl_logpoly* logpoly;
} rdl_subminor_params;

typedef struct {
  uint64_t n_selected;
  uint64_t iteration;      /* CurrentIteration() after Run() */
  int32_t has_peak;        /* OptionalNumber set */
  float peak;              /* signed integrated value */
  int32_t diverging;
  float flux_cleaned;
} rdl_subminor_result;

int rdl_subminor_create(rdl_session* s, rdl_subminor** out);
int rdl_subminor_destroy(rdl_subminor* h);

/* Replaces SubMinorLoop::Run (cpp/algorithms/subminor_loop.cc:38-117) with
 * findPeakPositions/MakeSets (:119-184) and GetMaxComponent (:13-36):
 * stream-compaction of |integrated| >= threshold in the border box (and
 * mask), then a persistent device loop over the selected set.
 * d_residuals: n_images planes (the convolved residual set);
 * d_psfs: n_images/n_pol planes (twice convolved PSFs).
 * h_trace (may be NULL) receives x,y per component. */
int rdl_subminor_run(rdl_subminor* h, const float* d_residuals,
                     const float* d_psfs, const rdl_subminor_params* p,
                     rdl_subminor_result* out, uint32_t* h_trace,
                     uint64_t trace_cap);

/* rdl_subminor_run in two halves, so the host can queue the work that does
 * not depend on the loop's result (the residual correction, the model update,
 * the next peak searches: multiscale_algorithm.cc:436-462, 521-524) before it
 * waits for that result. _launch selects (reads the selection count) and
 * launches the loop; out->n_selected and out->has_peak are final, the other
 * fields are filled by _collect, which waits for the loop. The handle's
 * selection (positions, model values) may be used by other calls on the
 * session's stream in between. A second _launch before _collect fails, and
 * so does a _launch or _run of ANOTHER handle of the same session while this
 * one is uncollected (the session keeps one loop-result slot in mapped host
 * memory): collect first. */
int rdl_subminor_launch(rdl_subminor* h, const float* d_residuals, const float* d_psfs,
                        const rdl_subminor_params* p, rdl_subminor_result* out);
int rdl_subminor_collect(rdl_subminor* h, rdl_subminor_result* out);

/* Kernel choice for rdl_subminor_run (results are identical): mode 0 picks
 * automatically, 1 forces the LDS-resident loop, 2 the register-resident
 * loop, 3 the single-wave loop, 4 one 1024-thread workgroup, 5 a grid of
 * 1024-thread workgroups, 6 the single-workgroup pairwise-table loop (one
 * image, identity integration, no RMS / spectral / log-polynomial fit, at
 * most 8192 pixels); target_per_block (0 = keep) sets the selected pixels
 * per workgroup above which the register loop spreads over more workgroups
 * (mode 6: 512 or 1024 picks the workgroup size). */
int rdl_subminor_set_tuning(rdl_subminor* h, int mode, uint32_t target_per_block);

/* SubMinorLoop::GetFullIndividualModel (subminor_loop.cc:186-193), fused
 * with the caller's use: mode 0 writes the model of image `image_index` into
 * a zeroed dest (dest_w x dest_h, placed at offset ox,oy — Image::Untrim);
 * mode 1 adds it (model += scratch, generic_clean.cc:145-148). */
int rdl_subminor_model(rdl_subminor* h, uint32_t image_index, float* d_dest,
                       uint32_t dest_w, uint32_t dest_h, uint32_t ox,
                       uint32_t oy, int mode);
/* As mode 0 of rdl_subminor_model, into a zeroed float64 plane (input of the
 * double-precision residual correction, rdl_fft64_convolve). */
/* d_model += (that model convolved circularly with the odd n x n shape
 * kernel centred at (n/2, n/2)): the scale > 0 model update of the multiscale
 * fast sub-minor path (multiscale_algorithm.cc:442-460: GetFullIndividualModel,
 * Transform, AddWithFactor) by direct stamping in a fixed component order
 * instead of a pair of full-image FFTs. */
int rdl_subminor_add_shape_model(rdl_subminor* h, uint32_t image_index,
                                 const float* d_kernel, uint32_t n, float* d_model,
                                 uint32_t width, uint32_t height);
/* Row occupancy of that model in a plane with the model at row offset oy:
 * d_rows[y] = 1 where row y holds a non-zero model value, else 0 (n_rows
 * bytes). Lets the correction's transform skip the empty rows
 * (rdl_conv_rows_forward_masked / rdl_conv_columns_ex). */
int rdl_subminor_model_rows(rdl_subminor* h, uint32_t image_index,
                            uint8_t* d_rows, uint32_t n_rows, uint32_t oy);
int rdl_subminor_model_f64(rdl_subminor* h, uint32_t image_index,
                           double* d_dest, uint32_t dest_w, uint32_t dest_h,
                           uint32_t ox, uint32_t oy);
/* Mode 0 of rdl_subminor_model (at offset 0,0) restricted to the rows that
 * hold a non-zero model value: the rows y of d_dest marked d_rows[y + oy]
 * (rdl_subminor_model_rows' mask) are zeroed and every component is stored;
 * other rows keep their contents, which the masked correction transform
 * (rdl_conv_rows_forward_masked) never reads. Replaces a full-plane zero fill
 * per outer iteration. */
int rdl_subminor_model_masked(rdl_subminor* h, uint32_t image_index, float* d_dest,
                              uint32_t dest_w, uint32_t dest_h, const uint8_t* d_rows,
                              uint32_t oy);
/* Selected positions (packed y<<16|x) and per-image model values of the last
 * run, copied to host (UpdateComponentList / UpdateAutoMask inputs). */
/* SubMinorLoop::UpdateAutoMask (cpp/algorithms/subminor_loop.cc:220-228):
 * d_mask[y * width + x] = 1 for every selected pixel of the last run whose
 * model value is non-zero in any image (a width x height byte mask). */
int rdl_subminor_update_mask(rdl_subminor* h, uint8_t* d_mask);
int rdl_subminor_get(rdl_subminor* h, uint32_t* h_positions, float* h_models,
                     uint64_t capacity);

/* ---------------------------------------------------- FFT convolution */
/* Real 2-D transform pair at width x height (rocFFT, single precision).
 * Spectra are (width/2+1) x height complex float. */
int rdl_fft_create(rdl_session* s, uint32_t width, uint32_t height,
                   rdl_fft** out);
/* Same pair in double precision: spectra are (width/2+1) x height complex
 * double. Used for SubMinorLoop::CorrectResidualDirty (subminor_loop.cc:
 * 195-218), whose result feeds every later peak search: the float64 pass
 * keeps the corrected residual within float rounding of the exact
 * convolution (see DESIGN.md "Residual correction precision"). */
int rdl_fft_create_f64(rdl_session* s, uint32_t width, uint32_t height,
                       rdl_fft** out);
int rdl_fft_destroy(rdl_fft* f);
size_t rdl_fft_spectrum_bytes(const rdl_fft* f);
int rdl_fft_forward(rdl_fft* f, const float* d_in, void* d_spectrum);
/* Unnormalised inverse; d_spectrum is destroyed. */
int rdl_fft_inverse(rdl_fft* f, void* d_spectrum, float* d_out);
int rdl_fft64_forward(rdl_fft* f, const double* d_in, void* d_spectrum);
int rdl_fft64_inverse(rdl_fft* f, void* d_spectrum, double* d_out);
/* In-place circular convolution in double precision (see rdl_fft_convolve). */
int rdl_fft64_convolve(rdl_fft* f, double* d_image, const void* d_kernel_spectrum,
                       void* d_work);
/* ---------------------------------------- LDS-resident FFT convolution */
/* A width x height real 2-D transform pair built from three HBM passes
 * (rows / columns / rows, each transform held in LDS), replacing rocFFT for
 * the convolutions of multiscale_transforms.cc:9-21 and
 * subminor_loop.cc:195-218. Lengths must be 2^a 3^b 5^c 7^d and fit in LDS
 * (<= 20480 float, <= 10240 double); otherwise RDL_ERR_UNSUPPORTED.
 * Spectra are (width/2+1) x height complex (float or double) in natural
 * row-major order, like rocFFT's. Inputs and outputs are float images. */
typedef struct rdl_conv rdl_conv;
int rdl_conv_create(rdl_session* s, uint32_t width, uint32_t height, int f64,
                    rdl_conv** out);
/* As rdl_conv_create with an explicit column-pass strategy: AUTO (currently
 * the one-pass kernel), SINGLE forces the one-pass column kernel, SPLIT the
 * split (four-step, coalesced) passes (RDL_ERR_UNSUPPORTED
 * when the column length has no split into two factors >= 4). Spectra have
 * the same layout either way. rdl_conv_columns_split reports the choice. */
#define RDL_CONV_COLUMNS_AUTO 0
#define RDL_CONV_COLUMNS_SINGLE 1
#define RDL_CONV_COLUMNS_SPLIT 2
int rdl_conv_create_ex(rdl_session* s, uint32_t width, uint32_t height, int f64,
                       int columns, rdl_conv** out);
int rdl_conv_columns_split(const rdl_conv* c);
int rdl_conv_destroy(rdl_conv* c);
size_t rdl_conv_spectrum_bytes(const rdl_conv* c);
/* Row transforms of the plane holding the in_w x in_h image d_in at offset
 * (ox, oy) and zeros elsewhere (Image::Untrim fused). */
int rdl_conv_rows_forward(rdl_conv* c, const float* d_in, uint32_t in_w,
                          uint32_t in_h, uint32_t ox, uint32_t oy, void* d_spec);
/* Column transforms, in or out of place. mode 0: forward; mode 1: forward,
 * x kernel spectrum x scale, inverse; mode 2: input already column-
 * transformed: x kernel spectrum x scale, inverse. */
int rdl_conv_columns(rdl_conv* c, const void* d_in, void* d_out,
                     const void* d_kernel, int mode, double scale);
/* Inverse row transforms; the window (ox, oy, out_w, out_h) of the real plane
 * is written to d_out (out_w wide) or, with subtract != 0, subtracted from
 * it after rounding to float (Image::Trim + residual -= fused). */
int rdl_conv_rows_inverse(rdl_conv* c, const void* d_spec, float* d_out,
                          uint32_t out_w, uint32_t out_h, uint32_t ox,
                          uint32_t oy, int subtract);
/* rdl_conv_rows_inverse (write mode) of the out_w x out_h window at (ox, oy)
 * with the peak search of rdl_find_peak(start_y 0, end_y out_h,
 * avx_semantics 1) on that window fused into it: the result goes to peak
 * slot `slot` (rdl_find_peak_collect) without re-reading the image
 * (FindMultiScalePeak's per-scale search, threaded_deconvolution_tools.cc:
 * 52-107). Needs the compile-time-planned row kernels (RDL_ERR_UNSUPPORTED
 * otherwise). */
int rdl_conv_rows_inverse_peak(rdl_conv* c, const void* d_spec, float* d_out,
                               uint32_t out_w, uint32_t out_h, uint32_t ox, uint32_t oy,
                               uint32_t h_border, uint32_t v_border, int allow_negative,
                               const uint8_t* d_mask, uint32_t slot);
/* Full 2-D forward transform of a width x height float image. */
int rdl_conv_forward(rdl_conv* c, const float* d_in, void* d_spec);
/* Sparse / layout variants of the passes above.
 * rdl_conv_rows_forward_masked: d_row_mask[y] == 0 declares plane row y zero;
 * workgroups whose rows are all zero read and write nothing, so the column
 * pass must be given the same mask (it substitutes zeros for those rows).
 * rdl_conv_columns_ex: d_row_mask as above (NULL: dense); kernel_layout
 * RDL_CONV_COL_MAJOR reads the kernel spectrum as columns (column k at
 * d_kernel + k*height, contiguous: the strided kernel read of the row-major
 * layout is the column pass's costliest access); out_layout
 * RDL_CONV_COL_MAJOR writes a mode-0 spectrum that way (d_out != d_in). */
#define RDL_CONV_ROW_MAJOR 0
#define RDL_CONV_COL_MAJOR 1
int rdl_conv_rows_forward_masked(rdl_conv* c, const float* d_in, uint32_t in_w,
                                 uint32_t in_h, uint32_t ox, uint32_t oy,
                                 void* d_spec, const uint8_t* d_row_mask);
int rdl_conv_columns_ex(rdl_conv* c, const void* d_in, void* d_out,
                        const void* d_kernel, int mode, double scale,
                        const uint8_t* d_row_mask, int kernel_layout,
                        int out_layout);
/* rdl_conv_columns_ex mode 1 (row-major output) where only the output rows
 * [out_row0, out_row0 + out_rows) are needed (the inverse row pass of a
 * padded convolution reads the image window's rows only: Image::Trim,
 * subminor_loop.cc:213-215): the float64 convolution-column plans leave the
 * other rows unwritten; every other plan writes them all. */
int rdl_conv_columns_window(rdl_conv* c, const void* d_in, void* d_out,
                            const void* d_kernel, double scale, const uint8_t* d_row_mask,
                            int kernel_layout, uint32_t out_row0, uint32_t out_rows,
                            int kernel_f32);
/* kernel_f32 (float64 convolution-column plans only): d_kernel holds the
 * kernel spectrum as float complex (rdl_complex_narrow of the float64 one),
 * widened to double where it is multiplied. */
/* The padded convolve-and-subtract of CorrectResidualDirty
 * (subminor_loop.cc:199-216: Untrim, Convolve, Trim, residual -= result) as
 * one call: d_residual (img_w x img_h) -= the window (ox, oy) of
 * image (x) kernel, with d_image the window's content of a zero plane and
 * d_row_mask (optional) marking the plane rows that may be non-zero. Equal to
 * rdl_conv_rows_forward(_masked) + rdl_conv_columns_window + rdl_conv_rows_
 * inverse(subtract); the float64 convolution-column plans keep the
 * intermediate spectrum in the tiled layout (RDL_CONV_FAST_TILED's element
 * order, in double) so every pass moves whole cache lines. d_work holds
 * rdl_conv_convolve_subtract_bytes(c) bytes. */
size_t rdl_conv_convolve_subtract_bytes(const rdl_conv* c);
int rdl_conv_convolve_subtract(rdl_conv* c, const float* d_image, uint32_t img_w,
                               uint32_t img_h, uint32_t ox, uint32_t oy,
                               const void* d_kernel, int kernel_layout, int kernel_f32,
                               double scale, const uint8_t* d_row_mask, void* d_work,
                               float* d_residual);
/* d_dst[i] = (float complex) d_src[i], i < n_complex (double complex in). */
int rdl_complex_narrow(rdl_session* s, void* d_dst, const void* d_src, size_t n_complex);
/* As rdl_conv_columns_ex with the input layout too (in_layout
 * RDL_CONV_COL_MAJOR: a mode-2 spectrum stored as columns). Every layout
 * combination needs the compile-time-planned column kernels
 * (rdl_conv_fast(c) & RDL_CONV_FAST_COLUMNS); the runtime-plan kernels read
 * row-major input and write column-major output in mode 0 only. */
int rdl_conv_columns_layout(rdl_conv* c, const void* d_in, void* d_out,
                            const void* d_kernel, int mode, double scale,
                            const uint8_t* d_row_mask, int in_layout,
                            int kernel_layout, int out_layout);
/* Which passes of this plan use the compile-time-planned kernels
 * (csrc/hip/fft_fast.hip): a bitmask of the two flags. */
#define RDL_CONV_FAST_COLUMNS 1
#define RDL_CONV_FAST_ROWS 2
/* float planes with four-step column plans: every spectrum of this plan is
 * stored in tiles of 16 columns (complex element (y, k) at
 * ((k / 16) * height + y) * 16 + k % 16; rdl_conv_spectrum_bytes covers the
 * padded last tile) and the layout arguments do not apply. */
#define RDL_CONV_FAST_TILED 4
/* float64 plans whose convolution columns run ff::ColumnsConvD (the only
 * ones rdl_conv_columns_window's kernel_f32 applies to) */
#define RDL_CONV_FAST_CONVD 8
int rdl_conv_fast(const rdl_conv* c);

/* Several scale convolutions of ONE float plane (FindActiveScaleConvolvedMaxima
 * -> ThreadedDeconvolutionTools::FindMultiScalePeak, which convolves the same
 * integrated image with every active scale's kernel: multiscale_algorithm.cc:
 * 578-634, threaded_deconvolution_tools.cc:52-107, each a
 * MultiScaleTransforms::Transform, multiscale_transforms.cc:9-21), for plans
 * with RDL_CONV_FAST_TILED only (RDL_ERR_UNSUPPORTED otherwise):
 *   rdl_conv_forward_half: the row transforms of the plane (as
 *     rdl_conv_rows_forward) and the first column step, into d_half
 *     (rdl_conv_spectrum_bytes);
 *   rdl_conv_real_kernel: the scale kernel's spectrum: h_shape is the n x n
 *     shape function (MakeShapeFunction, n odd, symmetric in x and y) placed
 *     as PrepareSmallConvolutionKernel; such a kernel's spectrum is real and
 *     even, evaluated here in double and stored as float in the tiled layout
 *     (rdl_conv_real_kernel_bytes);
 *   rdl_conv_scales: for i < n_scales (<= 8): the rest of the forward column
 *     transform, x d_kernels[i] x scale, and the inner inverse column step,
 *     into d_outs[i] (spectrum-sized, distinct from d_half);
 *   rdl_conv_scale_finish: the outer inverse column step: d_in (one of
 *     d_outs) -> d_out (!= d_in), the column-inverted spectrum that
 *     rdl_conv_rows_inverse(_peak) turns into the convolved image.
 * The forward spectrum itself is never stored. */
size_t rdl_conv_real_kernel_bytes(const rdl_conv* c);
int rdl_conv_real_kernel(rdl_conv* c, const float* h_shape, uint32_t n, void* d_kernel);
int rdl_conv_forward_half(rdl_conv* c, const float* d_in, uint32_t in_w, uint32_t in_h,
                          uint32_t ox, uint32_t oy, void* d_half);
int rdl_conv_scales(rdl_conv* c, const void* d_half, uint32_t n_scales,
                    const void* const* d_kernels, void* const* d_outs, double scale);
int rdl_conv_scale_finish(rdl_conv* c, const void* d_in, void* d_out);

/* dst = a * b * scale, complex, n_complex elements. */
int rdl_spectrum_multiply(rdl_session* s, void* d_dst, const void* d_a,
                          const void* d_b, size_t n_complex, float scale);
/* Circular convolution of d_image (in place) with a kernel spectrum:
 * schaapcommon::math::Convolve contract (multiscale_transforms.cc:16-20,
 * subminor_loop.cc:210-211); normalised. d_work: spectrum-sized scratch. */
int rdl_fft_convolve(rdl_fft* f, float* d_image, const void* d_kernel_spectrum,
                     void* d_work);

/* schaapcommon::math::PrepareSmallConvolutionKernel: zero d_dest (w x h) and
 * wrap an n x n host kernel with its centre at the origin. */
int rdl_prepare_small_kernel(rdl_session* s, float* d_dest, uint32_t width,
                             uint32_t height, const float* h_kernel,
                             uint32_t n);
/* Image::Untrim + schaapcommon::math::PrepareConvolutionKernel fused
 * (subminor_loop.cc:199-202): centre a w x h image in a zeroed pw x ph
 * plane, then quadrant-shift so its (pw/2, ph/2) lands at the origin. */
int rdl_prepare_psf_kernel(rdl_session* s, float* d_dest, uint32_t pw,
                           uint32_t ph, const float* d_psf, uint32_t width,
                           uint32_t height);
/* rdl_prepare_psf_kernel into a float64 plane. */
int rdl_prepare_psf_kernel_f64(rdl_session* s, double* d_dest, uint32_t pw,
                               uint32_t ph, const float* d_psf, uint32_t width,
                               uint32_t height);
/* Image::Trim into float + `residual -= trimmed` from a float64 plane. */
int rdl_trim_subtract_f64(rdl_session* s, float* d_residual, uint32_t width,
                          uint32_t height, const double* d_padded, uint32_t pw,
                          uint32_t ph);
/* Image::Trim + `residual -= trimmed` (subminor_loop.cc:214-217). */
int rdl_trim_subtract(rdl_session* s, float* d_residual, uint32_t width,
                      uint32_t height, const float* d_padded, uint32_t pw,
                      uint32_t ph);
/* Image::Untrim / Trim as plain copies (ParallelDeconvolution PSF resize). */
int rdl_untrim(rdl_session* s, float* d_dest, uint32_t pw, uint32_t ph,
               const float* d_src, uint32_t width, uint32_t height);
int rdl_trim(rdl_session* s, float* d_dest, uint32_t width, uint32_t height,
             const float* d_src, uint32_t pw, uint32_t ph);
/* d_dest (pw x ph) = the w x h image repeated periodically and shifted by
 * (shift_x, shift_y): dest[y][x] = src[(y - sy) mod h][(x - sx) mod w].
 * Lets the multiscale transforms (multiscale_transforms.cc:9-21, circular at
 * W x H) run at an FFT-friendly size: a kernel of radius r <= shift convolved
 * with this plane and cropped at (shift_x, shift_y) is the circular
 * convolution at W x H, whatever prime factors W and H have. */
int rdl_periodic_extend(rdl_session* s, float* d_dest, uint32_t pw, uint32_t ph,
                        const float* d_src, uint32_t width, uint32_t height,
                        uint32_t shift_x, uint32_t shift_y);

/* multiscale::MultiScaleTransforms::AddShapeComponent
 * (multiscale_transforms.h:62-89): image += kernel(n x n host) * gain at x,y. */
int rdl_add_shape_component(rdl_session* s, float* d_image, uint32_t width,
                            uint32_t height, const float* h_kernel, uint32_t n,
                            uint32_t x, uint32_t y, float gain);

/* ------------------------------------------------------- box transfers */
/* w x h box from src (row stride src_w, origin src_x,src_y) to dst (stride
 * dst_w, origin dst_x,dst_y); d_mask (box-local w x h bytes, may be NULL):
 *   RDL_BOX_COPY         dst = src                 (ImageSet::Trim)
 *   RDL_BOX_COPY_MASKED  dst = src where mask      (ImageSet::CopyMasked)
 *   RDL_BOX_COPY_ZERO    dst = mask ? src : 0      (ImageSet::TrimMasked)
 *   RDL_BOX_ADD          dst += src                (ImageSet::AddSubImage)
 * (cpp/image_set.h:216-262, parallel_deconvolution.cc:308-318, 475-482). */
#define RDL_BOX_COPY 0
#define RDL_BOX_COPY_MASKED 1
#define RDL_BOX_COPY_ZERO 2
#define RDL_BOX_ADD 3
int rdl_box(rdl_session* s, float* d_dst, uint32_t dst_w, uint32_t dst_x,
            uint32_t dst_y, const float* d_src, uint32_t src_w, uint32_t src_x,
            uint32_t src_y, uint32_t w, uint32_t h, const uint8_t* d_mask, int op);

/* -------------------------------------------------- IUWT (à-trous) */
/* IuwtDecomposition::DecomposeMt (cpp/algorithms/iuwt/iuwt_decomposition.cc:
 * 9-54): d_coeffs receives n_scales detail planes and, as plane n_scales, the
 * approximation (zeroed unless include_largest). d_scratch is one plane; it
 * may be d_input itself, which reproduces the reference's Decompose(x, x, ..)
 * calls (iuwt_deconvolution_algorithm.cc:342, 385, 686, 785): the input is
 * overwritten and the first row pass runs in place. Bit-exact with the
 * reference build's tap order and FMA contraction. */
int rdl_iuwt_decompose(rdl_session* s, float* d_input, float* d_scratch,
                       uint32_t width, uint32_t height, uint32_t n_scales,
                       float* d_coeffs, int include_largest);
/* IuwtDecomposition::Recompose (iuwt_decomposition.h:121-146). */
int rdl_iuwt_recompose(rdl_session* s, const float* d_coeffs, uint32_t width,
                       uint32_t height, uint32_t n_scales, int include_largest,
                       float* d_out);

/* -------------------------------------------- multi-GPU (RCCL over xGMI) */
/* Size of an RCCL unique id blob; rank 0 creates it and the host side
 * distributes it (torch.distributed / MPI). */
int rdl_comm_id_size(void);
int rdl_comm_get_unique_id(void* h_id);
int rdl_comm_init(rdl_session* s, int n_ranks, int rank, const void* h_id);
int rdl_comm_destroy(rdl_session* s);
/* Signed max of one float over all ranks (ParallelDeconvolution start peak,
 * cpp/algorithms/parallel_deconvolution.cc:592-603). */
int rdl_comm_allreduce_max(rdl_session* s, float* value);
int rdl_comm_allreduce_sum_u64(rdl_session* s, uint64_t* value);
/* Element-wise max of n host floats over the ranks, in place (the
 * per-subimage peaks of the find-peak pass, which every rank needs for the
 * cost-ordered ownership of the cleaning pass). */
int rdl_comm_allreduce_max_n(rdl_session* s, float* values, size_t n);
/* In-place broadcast of a device buffer from `root`, stream ordered: the
 * owner rank's subimage residual/model boxes, which every rank then merges
 * in subimage order (ImageSet::CopyMasked / AddSubImage,
 * cpp/algorithms/parallel_deconvolution.cc:458-484). */
int rdl_comm_broadcast(rdl_session* s, void* d_buf, size_t bytes, int root);
/* This session's rank and the communicator size. */
int rdl_comm_rank(rdl_session* s, int* rank, int* n_ranks);

#ifdef __cplusplus
}
#endif

#endif /* RDL_HIP_H_ */
