"""ctypes bindings of the CPU restatement (oracle/build/liboracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg. Never by the product package.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_simple_clean.so")

f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
u8p = C.c_void_p


class SetDesc(C.Structure):
    _fields_ = [("width", C.c_uint64), ("height", C.c_uint64),
                ("n_channels", C.c_uint64), ("n_pol", C.c_uint64),
                ("weights", C.c_void_p), ("pol_factor", C.c_float),
                ("squared_joins", C.c_int32), ("fit_mode", C.c_int32),
                ("fit_terms", C.c_uint32), ("fit_frequencies", C.c_void_p),
                ("fit_weights", C.c_void_p)]


class AlgoSettings(C.Structure):
    _fields_ = [("threshold", C.c_double), ("major_iteration_threshold", C.c_double),
                ("minor_loop_gain", C.c_double), ("major_loop_gain", C.c_double),
                ("border_ratio", C.c_double), ("divergence_limit", C.c_double),
                ("max_iterations", C.c_uint64),
                ("allow_negative", C.c_int32), ("stop_on_negative", C.c_int32),
                ("use_sub_minor", C.c_int32), ("fast_sub_minor_loop", C.c_int32),
                ("sub_minor_loop_gain", C.c_double), ("scale_bias", C.c_double),
                ("max_scales", C.c_uint64), ("convolution_padding", C.c_double),
                ("shape", C.c_int32), ("pad0", C.c_int32),
                ("beam_size_in_pixels", C.c_double),
                ("scale_list", C.c_void_p), ("n_scale_list", C.c_uint64),
                ("clean_mask", C.c_void_p)]


class Result(C.Structure):
    _fields_ = [("has_starting_peak", C.c_int32), ("starting_peak", C.c_float),
                ("final_peak", C.c_float), ("another_iteration_required", C.c_int32),
                ("is_diverging", C.c_int32), ("pad0", C.c_int32),
                ("iteration_number", C.c_uint64), ("n_trace", C.c_uint64)]


def algo_settings(**kw):
    """Defaults of DeconvolutionAlgorithm (cpp/algorithms/deconvolution_algorithm.h:187-199)
    and Settings::Multiscale (cpp/settings.h:465-524)."""
    s = AlgoSettings()
    d = dict(threshold=0.0, major_iteration_threshold=0.0, minor_loop_gain=0.1,
             major_loop_gain=1.0, border_ratio=0.05, divergence_limit=4.0,
             max_iterations=500, allow_negative=1, stop_on_negative=0,
             use_sub_minor=1, fast_sub_minor_loop=1, sub_minor_loop_gain=0.2,
             scale_bias=0.6, max_scales=0, convolution_padding=1.1, shape=0,
             beam_size_in_pixels=1.0)
    d.update(kw)
    s._keep = []
    for k, v in d.items():
        if k == "clean_mask":
            continue
        setattr(s, k, v)
    mask = kw.get("clean_mask")
    if mask is not None:
        m = np.ascontiguousarray(mask, dtype=np.uint8)
        s._keep.append(m)
        s.clean_mask = m.ctypes.data
    return s


class Oracle:
    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run __graft_entry__.build())")
        L = self.lib = C.CDLL(path)
        L.orc_set_threads.argtypes = [C.c_uint64]
        L.orc_find_peak.argtypes = [f32p, C.c_uint64, C.c_uint64, C.c_int, C.c_uint64,
                                    C.c_uint64, C.c_uint64, C.c_uint64, u8p, C.c_int,
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_float)]
        L.orc_find_peak.restype = C.c_int
        L.orc_partial_subtract.argtypes = [f32p, f32p, C.c_uint64, C.c_uint64, C.c_uint64,
                                           C.c_uint64, C.c_float, C.c_uint64, C.c_uint64]
        L.orc_subtract.argtypes = [f32p, f32p, C.c_uint64, C.c_uint64, C.c_uint64,
                                   C.c_uint64, C.c_float]
        L.orc_good_fft_size.argtypes = [C.c_uint64]
        L.orc_good_fft_size.restype = C.c_uint64
        L.orc_convolution_size.argtypes = [C.c_double, C.c_uint64, C.c_double]
        L.orc_convolution_size.restype = C.c_uint64
        L.orc_convolve.argtypes = [f32p, f32p, C.c_uint64, C.c_uint64]
        L.orc_shape_function.argtypes = [C.c_float, C.c_uint64, C.c_int, C.c_void_p]
        L.orc_shape_function.restype = C.c_uint64
        L.orc_kernel_peak.argtypes = [C.c_double, C.c_uint64, C.c_int]
        L.orc_kernel_peak.restype = C.c_float
        L.orc_ms_transform.argtypes = [f32p, C.c_uint64, C.c_uint64, C.c_uint64,
                                       C.c_float, C.c_int]
        L.orc_add_shape_component.argtypes = [f32p, C.c_uint64, C.c_uint64, C.c_float,
                                              C.c_uint64, C.c_uint64, C.c_float, C.c_int]
        L.orc_integrate.argtypes = [C.POINTER(SetDesc), f32p, f32p, C.c_int]
        L.orc_algo_create.argtypes = [C.c_int, C.POINTER(AlgoSettings)]
        L.orc_algo_create.restype = C.c_void_p
        L.orc_algo_destroy.argtypes = [C.c_void_p]
        L.orc_algo_update.argtypes = [C.c_void_p, C.POINTER(AlgoSettings)]
        L.orc_algo_execute.argtypes = [C.c_void_p, C.POINTER(SetDesc), f32p, f32p, f32p,
                                       C.POINTER(Result), C.c_void_p, C.c_uint64]
        L.orc_algo_execute.restype = C.c_int
        L.orc_last_error.restype = C.c_char_p

    def set_threads(self, n):
        self.lib.orc_set_threads(n)

    def find_peak(self, img, allow_negative=True, start_y=0, end_y=None, hb=0, vb=0,
                  mask=None, simple=False):
        img = np.ascontiguousarray(img, dtype=np.float32)
        h, w = img.shape
        end_y = h if end_y is None else end_y
        x, y, v = C.c_uint64(), C.c_uint64(), C.c_float()
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        has = self.lib.orc_find_peak(img, w, h, int(allow_negative), start_y, end_y, hb, vb,
                                     None if m is None else m.ctypes.data, int(simple),
                                     C.byref(x), C.byref(y), C.byref(v))
        return bool(has), int(x.value), int(y.value), float(v.value)

    def subtract(self, img, psf, x, y, factor):
        h, w = img.shape
        self.lib.orc_subtract(img, psf, w, h, x, y, factor)

    def partial_subtract(self, img, psf, x, y, factor, start_y, end_y):
        h, w = img.shape
        self.lib.orc_partial_subtract(img, psf, w, h, x, y, factor, start_y, end_y)

    def good_fft_size(self, n):
        return self.lib.orc_good_fft_size(n)

    def convolution_size(self, scale, n, padding):
        return self.lib.orc_convolution_size(scale, n, padding)

    def convolve(self, img, kernel):
        h, w = img.shape
        self.lib.orc_convolve(img, np.ascontiguousarray(kernel, np.float32), w, h)

    def shape_function(self, scale, max_n, shape=0):
        n = self.lib.orc_shape_function(scale, max_n, shape, None)
        out = np.zeros((n, n), np.float32)
        self.lib.orc_shape_function(scale, max_n, shape, out.ctypes.data)
        return out

    def kernel_peak(self, scale, max_n, shape=0):
        return self.lib.orc_kernel_peak(scale, max_n, shape)

    def ms_transform(self, imgs, scale, shape=0):
        imgs = np.ascontiguousarray(imgs, np.float32)
        n = 1 if imgs.ndim == 2 else imgs.shape[0]
        h, w = imgs.shape[-2:]
        self.lib.orc_ms_transform(imgs, n, w, h, scale, shape)
        return imgs

    def add_shape_component(self, img, scale, x, y, gain, shape=0):
        h, w = img.shape
        self.lib.orc_add_shape_component(img, w, h, scale, x, y, gain, shape)

    @staticmethod
    def set_desc(width, height, n_channels=1, n_pol=1, weights=None, pol_factor=1.0,
                 squared_joins=False, spectral=None):
        """spectral: None or (mode, n_terms, frequencies, weights) of the
        algorithms' SpectralFitter (mode 1 = polynomial)."""
        d = SetDesc()
        w = np.ones(n_channels, np.float32) if weights is None else np.asarray(weights, np.float32)
        d._w = np.ascontiguousarray(w)
        d.width, d.height, d.n_channels, d.n_pol = width, height, n_channels, n_pol
        d.weights = d._w.ctypes.data
        d.pol_factor = pol_factor
        d.squared_joins = int(squared_joins)
        if spectral is not None:
            mode, terms, freqs, fw = spectral
            d._ff = np.ascontiguousarray(freqs, np.float64)
            d._fw = np.ascontiguousarray(fw, np.float32)
            assert d._ff.size == n_channels and d._fw.size == n_channels
            d.fit_mode, d.fit_terms = int(mode), int(terms)
            d.fit_frequencies, d.fit_weights = d._ff.ctypes.data, d._fw.ctypes.data
        return d

    def local_rms(self, integrated, method, window, beam, pixel_scale_x, pixel_scale_y,
                  strength=1.0):
        """Radler::Perform's local-RMS step (method 1 = rms_window, 2 =
        rms_and_minimum_window) -> (rms image, factor image, lowest rms)."""
        img = np.ascontiguousarray(integrated, np.float32)
        h, w = img.shape
        rms = np.zeros_like(img)
        factor = np.zeros_like(img)
        lowest = C.c_double()
        L = self.lib
        L.orc_local_rms.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_double,
                                    C.c_double, C.c_double, C.c_double, C.c_double,
                                    C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]
        if L.orc_local_rms(img.ctypes.data, w, h, int(method), float(window), float(beam),
                           float(pixel_scale_x), float(pixel_scale_y), float(strength),
                           rms.ctypes.data, factor.ctypes.data, C.byref(lowest)) != 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return rms, factor, lowest.value

    def gradient_descent(self, model, residual, psf):
        """GenericClean's kGradientDescent component optimisation of one
        image: returns model + the update."""
        m = np.ascontiguousarray(model, np.float32).copy()
        r = np.ascontiguousarray(residual, np.float32)
        p = np.ascontiguousarray(psf, np.float32)
        h, w = m.shape
        L = self.lib
        L.orc_gradient_descent.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                           C.c_uint64]
        L.orc_gradient_descent.restype = None
        L.orc_gradient_descent(m.ctypes.data, r.ctypes.data, p.ctypes.data, w, h)
        return m

    def ms_full_component_fitter(self, residual, model, psf, scales, lists, padding=1.1,
                                 shape=0):
        """RunFullComponentFitter for one image -> (residual, model)."""
        r = np.ascontiguousarray(residual, np.float32).copy()
        m = np.ascontiguousarray(model, np.float32).copy()
        p = np.ascontiguousarray(psf, np.float32)
        h, w = r.shape
        sc = np.ascontiguousarray(scales, np.float32)
        pos = np.ascontiguousarray([c for l in lists for xy in l for c in xy] or [0], np.uint32)
        counts = np.ascontiguousarray([len(l) for l in lists], np.uint64)
        L = self.lib
        L.orc_ms_full_component_fitter.argtypes = [C.c_void_p] * 3 + [C.c_uint64] * 2 + [
            C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_double, C.c_int]
        L.orc_ms_full_component_fitter.restype = None
        L.orc_ms_full_component_fitter(r.ctypes.data, m.ctypes.data, p.ctypes.data, w, h,
                                       sc.ctypes.data, sc.size, pos.ctypes.data,
                                       counts.ctypes.data, float(padding), int(shape))
        return r, m

    def linear_component_solve(self, model, image, psf):
        """math::LinearComponentSolve(model, image, psf): returns the new model."""
        m = np.ascontiguousarray(model, np.float32).copy()
        i = np.ascontiguousarray(image, np.float32)
        p = np.ascontiguousarray(psf, np.float32)
        h, w = m.shape
        L = self.lib
        L.orc_linear_component_solve.argtypes = [C.c_void_p] * 3 + [C.c_uint64] * 2
        L.orc_linear_component_solve.restype = None
        L.orc_linear_component_solve(m.ctypes.data, i.ctypes.data, p.ctypes.data, w, h)
        return m

    def gradient_descent_variable_psf(self, components, image, psfs, pw=0, ph=0):
        """math::GradientDescentWithVariablePsf (FFT convolutions) -> deltas."""
        img = np.ascontiguousarray(image, np.float32)
        h, w = img.shape
        ps = np.ascontiguousarray(np.stack(psfs), np.float32)
        pos = np.ascontiguousarray([c for l in components for xy in l for c in xy] or [0],
                                   np.uint32)
        counts = np.ascontiguousarray([len(l) for l in components], np.uint64)
        out = np.zeros((len(psfs), h, w), np.float32)
        L = self.lib
        L.orc_gradient_descent_variable_psf.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64,
                                                        C.c_void_p, C.c_void_p] + \
            [C.c_uint64] * 4 + [C.c_void_p]
        L.orc_gradient_descent_variable_psf.restype = None
        L.orc_gradient_descent_variable_psf(pos.ctypes.data, counts.ctypes.data, len(psfs),
                                            img.ctypes.data, ps.ctypes.data, w, h,
                                            pw or 2 * w, ph or 2 * h, out.ctypes.data)
        return list(out)

    def make_rms_factor_image(self, rms, strength):
        """math::rms_image::MakeRmsFactorImage -> (factor image, lowest rms)."""
        r = np.ascontiguousarray(rms, np.float32).copy()
        L = self.lib
        L.orc_make_rms_factor_image.argtypes = [C.c_void_p, C.c_uint64, C.c_double]
        L.orc_make_rms_factor_image.restype = C.c_double
        lowest = L.orc_make_rms_factor_image(r.ctypes.data, r.size, float(strength))
        return r, lowest

    def padded_convolution(self, image, psf, pw, ph):
        img = np.ascontiguousarray(image, np.float32).copy()
        p = np.ascontiguousarray(psf, np.float32)
        h, w = img.shape
        L = self.lib
        L.orc_padded_convolution.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                             C.c_uint64, C.c_uint64]
        L.orc_padded_convolution.restype = None
        L.orc_padded_convolution(img.ctypes.data, p.ctypes.data, w, h, pw, ph)
        return img

    def sliding_minimum(self, image, window):
        img = np.ascontiguousarray(image, np.float32)
        h, w = img.shape
        out = np.zeros_like(img)
        L = self.lib
        L.orc_sliding_minimum.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                          C.c_void_p]
        L.orc_sliding_minimum.restype = None
        L.orc_sliding_minimum(img.ctypes.data, w, h, int(window), out.ctypes.data)
        return out

    def spectral_fit(self, mode, n_terms, frequencies, weights, values):
        """SpectralFitter FitAndEvaluate -> (evaluated values, terms)."""
        f = np.ascontiguousarray(frequencies, np.float64)
        w = np.ascontiguousarray(weights, np.float32)
        v = np.ascontiguousarray(values, np.float32).copy()
        t = np.zeros(max(int(n_terms), 1), np.float32)
        L = self.lib
        L.orc_spectral_fit.argtypes = [C.c_int, C.c_uint32, C.c_void_p, C.c_void_p,
                                       C.c_uint64, C.c_void_p, C.c_void_p]
        L.orc_spectral_fit.restype = None
        L.orc_spectral_fit(int(mode), int(n_terms), f.ctypes.data, w.ctypes.data, f.size,
                           v.ctypes.data, t.ctypes.data)
        return v, t[:n_terms]

    def spectral_interpolate(self, mode, n_terms, frequencies, weights, planes,
                             out_frequencies):
        """ImageSet::InterpolateAndStoreModel for one polarization."""
        f = np.ascontiguousarray(frequencies, np.float64)
        w = np.ascontiguousarray(weights, np.float32)
        p = np.ascontiguousarray(planes, np.float32)
        of = np.ascontiguousarray(out_frequencies, np.float64)
        out = np.zeros((of.size,) + p.shape[1:], np.float32)
        L = self.lib
        L.orc_spectral_interpolate.argtypes = [C.c_int, C.c_uint32, C.c_void_p, C.c_void_p,
                                               C.c_uint64, C.c_void_p, C.c_uint64,
                                               C.c_void_p, C.c_uint64, C.c_void_p]
        L.orc_spectral_interpolate.restype = None
        L.orc_spectral_interpolate(int(mode), int(n_terms), f.ctypes.data, w.ctypes.data,
                                   f.size, p.ctypes.data, int(np.prod(p.shape[1:])),
                                   of.ctypes.data, of.size, out.ctypes.data)
        return out

    def integrate(self, images, weights=None, n_pol=1, pol_factor=1.0, square=False,
                  squared_joins=False):
        images = np.ascontiguousarray(images, np.float32)
        n, h, w = images.shape
        d = self.set_desc(w, h, n // n_pol, n_pol, weights, pol_factor, squared_joins)
        out = np.zeros((h, w), np.float32)
        self.lib.orc_integrate(C.byref(d), images, out, int(square))
        return out


class OracleAlgorithm:
    """A persistent DeconvolutionAlgorithm (GenericClean=0, MultiScale=1, IUWT=2)."""

    def __init__(self, oracle, kind, **settings):
        self.o = oracle
        self.settings = algo_settings(**settings)
        self.h = oracle.lib.orc_algo_create(kind, C.byref(self.settings))
        self.spectral = None

    def set_spectral_fitter(self, mode, n_terms, frequencies, weights):
        """DeconvolutionAlgorithm::SetSpectralFitter (polynomial: mode 1)."""
        self.spectral = (mode, n_terms, frequencies, weights)

    def set_component_optimization(self, algorithm):
        """SetComponentOptimizationAlgorithm: 0 clean, 2 gradient descent."""
        L = self.o.lib
        L.orc_algo_set_component_optimization.argtypes = [C.c_void_p, C.c_int]
        L.orc_algo_set_component_optimization.restype = None
        L.orc_algo_set_component_optimization(self.h, int(algorithm))

    def set_rms(self, factor):
        """DeconvolutionAlgorithm::SetRmsFactorImage (None clears it)."""
        L = self.o.lib
        L.orc_algo_set_rms.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_algo_set_rms.restype = None
        if factor is None:
            L.orc_algo_set_rms(self.h, None, 0)
        else:
            f = np.ascontiguousarray(factor, np.float32)
            L.orc_algo_set_rms(self.h, f.ctypes.data, f.size)

    def update(self, **settings):
        self.settings = algo_settings(**settings)
        self.o.lib.orc_algo_update(self.h, C.byref(self.settings))

    def execute(self, residual, model, psfs, weights=None, trace_cap=1 << 22):
        """residual/model: (n_img, h, w) float32 updated in place; psfs (n_ch, h, w)."""
        n, h, w = residual.shape
        d = Oracle.set_desc(w, h, psfs.shape[0], n // psfs.shape[0], weights,
                            spectral=self.spectral)
        r = Result()
        trace = np.zeros((trace_cap, 3), np.uint32)
        rc = self.o.lib.orc_algo_execute(self.h, C.byref(d), residual, model,
                                         np.ascontiguousarray(psfs, np.float32), C.byref(r),
                                         trace.ctypes.data, trace_cap)
        if rc != 0:
            raise RuntimeError(self.o.lib.orc_last_error().decode())
        return r, trace[: min(r.n_trace, trace_cap)].copy()

    def margins(self):
        """Decision margins of the last execute (oracle.h Component::margin):
        (margins [n_trace + 1], values [n_trace + 1]); the last entry is the
        end-of-run margin and the last component's |peak|."""
        L = self.o.lib
        L.orc_algo_margins.restype = C.c_uint64
        L.orc_algo_margins.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        n = L.orc_algo_margins(self.h, None, None, 0)
        m, v = np.zeros(n, np.float32), np.zeros(n, np.float32)
        L.orc_algo_margins(self.h, m.ctypes.data, v.ctypes.data, n)
        return m, v

    def set_clean_threads(self, n, after, stop=0):
        """Switch the multiscale outer loop to n threads after `after` outer
        iterations (n = 0: never) and stop after `stop` (0: never)."""
        L = self.o.lib
        L.orc_algo_set_clean_threads.restype = None
        L.orc_algo_set_clean_threads.argtypes = [C.c_void_p] + [C.c_uint64] * 3
        L.orc_algo_set_clean_threads(self.h, int(n), int(after), int(stop))

    def switch_info(self):
        """(seconds after the setup, components cleaned) at the thread switch."""
        L = self.o.lib
        L.orc_algo_switch_info.restype = None
        L.orc_algo_switch_info.argtypes = [C.c_void_p, C.POINTER(C.c_double),
                                           C.POINTER(C.c_uint64)]
        s, n = C.c_double(), C.c_uint64()
        L.orc_algo_switch_info(self.h, C.byref(s), C.byref(n))
        return s.value, int(n.value)

    def setup_seconds(self):
        """Wall seconds of the last multiscale execute's setup (scale-convolved
        PSFs and the first peak search, before the outer loop)."""
        L = self.o.lib
        L.orc_algo_setup_seconds.restype = C.c_double
        L.orc_algo_setup_seconds.argtypes = [C.c_void_p]
        return float(L.orc_algo_setup_seconds(self.h))

    def set_automask(self, track, use):
        """MultiScaleAlgorithm::SetAutoMaskMode (multiscale only)."""
        L = self.o.lib
        L.orc_algo_set_automask.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.orc_algo_set_automask.restype = None
        L.orc_algo_set_automask(self.h, int(track), int(use))

    def scale_masks(self, w, h):
        """The per-scale auto-masks as a (n_scales, h, w) uint8 array."""
        L = self.o.lib
        L.orc_algo_scale_mask.restype = C.c_uint64
        L.orc_algo_scale_mask.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]
        n = L.orc_algo_scale_mask(self.h, 0, None, 0)
        out = np.zeros((n, h, w), np.uint8)
        for i in range(n):
            L.orc_algo_scale_mask(self.h, i, out[i].ctypes.data, w * h)
        return out

    def iuwt_steps(self, cap=4096):
        """Steps of the last IUWT (kind 2) execute (oracle/iuwt_algorithm.h IuwtStep)."""
        out = np.zeros(cap, IUWT_STEP)
        L = self.o.lib
        L.orc_iuwt_steps.restype = C.c_uint64
        L.orc_iuwt_steps.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        n = L.orc_iuwt_steps(self.h, out.ctypes.data, cap)
        return out[: min(n, cap)].copy()

    def __del__(self):
        try:
            self.o.lib.orc_algo_destroy(self.h)
        except Exception:
            pass


# oracle/iuwt_algorithm.h IuwtStep (40 bytes)
IUWT_STEP = np.dtype([("succeeded", np.int32), ("scale", np.int32), ("x", np.uint32),
                      ("y", np.uint32), ("end_scale", np.int32), ("min_scale", np.int32),
                      ("area", np.uint64), ("max_value", np.float32),
                      ("trimmed_width", np.uint32)])


def iuwt_decompose(oracle, image, n_scales, aliased=False, include_largest=True):
    """oracle IUWT DecomposeMt: (coeffs [n_scales + 1, h, w], input after the
    call — overwritten when aliased, as in Decompose(x, x, ..))."""
    img = np.ascontiguousarray(image, np.float32).copy()
    h, w = img.shape
    coeffs = np.zeros((n_scales + 1, h, w), np.float32)
    L = oracle.lib
    L.orc_iuwt_decompose.argtypes = [f32p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                     C.c_int, f32p]
    if L.orc_iuwt_decompose(img, w, h, n_scales, int(aliased), int(include_largest),
                            coeffs) != 0:
        raise RuntimeError(L.orc_last_error().decode())
    return coeffs, img


def iuwt_recompose(oracle, coeffs, n_scales, include_largest=True):
    coeffs = np.ascontiguousarray(coeffs, np.float32)
    _, h, w = coeffs.shape
    out = np.zeros((h, w), np.float32)
    L = oracle.lib
    L.orc_iuwt_recompose.argtypes = [f32p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, f32p]
    L.orc_iuwt_recompose(coeffs, w, h, n_scales, int(include_largest), out)
    return out


def make_subimages(oracle, image, grid_w, grid_h):
    """oracle MakeSubImages: (boxes [n, 4] x,y,w,h; labels [h, w])."""
    image = np.ascontiguousarray(image, np.float32)
    h, w = image.shape
    boxes = np.zeros((grid_w * grid_h, 4), np.uint32)
    labels = np.zeros((h, w), np.uint16)
    L = oracle.lib
    L.orc_make_subimages.argtypes = [f32p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                     C.c_void_p, C.c_void_p]
    if L.orc_make_subimages(image, w, h, grid_w, grid_h, boxes.ctypes.data,
                            labels.ctypes.data) != 0:
        raise RuntimeError(L.orc_last_error().decode())
    return boxes, labels


class ParallelResult(C.Structure):
    _fields_ = [("another_iteration_required", C.c_int32), ("n_subimages", C.c_int32),
                ("start_peak", C.c_double), ("end_peak", C.c_double),
                ("first_iteration_number", C.c_uint64), ("total_iterations", C.c_uint64),
                ("n_trace", C.c_uint64)]


class OracleParallel:
    """ParallelDeconvolution tiling restatement (oracle/tiling.cc): a grid of
    per-subimage algorithms (GenericClean=0, MultiScale=1)."""

    def __init__(self, oracle, kind, grid_w, grid_h, **settings):
        self.o = oracle
        self.settings = algo_settings(**settings)
        L = oracle.lib
        L.orc_parallel_create.restype = C.c_void_p
        L.orc_parallel_create.argtypes = [C.c_int, C.POINTER(AlgoSettings), C.c_uint64,
                                          C.c_uint64]
        L.orc_parallel_destroy.argtypes = [C.c_void_p]
        L.orc_parallel_execute.argtypes = [C.c_void_p, C.POINTER(SetDesc), f32p, f32p, f32p,
                                           C.c_double, C.c_void_p, C.POINTER(ParallelResult),
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        self.h = L.orc_parallel_create(kind, C.byref(self.settings), grid_w, grid_h)
        self.n_sub = grid_w * grid_h
        L.orc_parallel_set_snapshot.argtypes = [C.c_void_p, C.c_int]

    def set_snapshot(self, snapshot):
        """True: every subimage of a pass trims the residual as it was at the
        start of the pass (the product's concurrent pool, max_threads > 1)."""
        self.o.lib.orc_parallel_set_snapshot(self.h, 1 if snapshot else 0)

    def set_rms(self, factor):
        """ParallelDeconvolution::SetRmsFactorImage (None clears it)."""
        L = self.o.lib
        L.orc_parallel_set_rms.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_parallel_set_rms.restype = None
        if factor is None:
            L.orc_parallel_set_rms(self.h, None, 0)
        else:
            f = np.ascontiguousarray(factor, np.float32)
            L.orc_parallel_set_rms(self.h, f.ctypes.data, f.size)

    def set_automask(self, track, use):
        L = self.o.lib
        L.orc_parallel_set_automask.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.orc_parallel_set_automask(self.h, int(track), int(use))

    def update(self, **settings):
        self.settings = algo_settings(**settings)
        L = self.o.lib
        L.orc_parallel_update.argtypes = [C.c_void_p, C.POINTER(AlgoSettings)]
        L.orc_parallel_update(self.h, C.byref(self.settings))

    def execute(self, residual, model, psfs, major_loop_gain, user_mask=None,
                trace_cap=1 << 22):
        n, h, w = residual.shape
        d = Oracle.set_desc(w, h, psfs.shape[0], n // psfs.shape[0], None,
                            spectral=getattr(self, "spectral", None))
        r = ParallelResult()
        boxes = np.zeros((self.n_sub, 4), np.uint32)
        labels = np.zeros((h, w), np.uint16)
        trace = np.zeros((trace_cap, 4), np.uint32)
        um = None if user_mask is None else np.ascontiguousarray(user_mask, np.uint8)
        rc = self.o.lib.orc_parallel_execute(
            self.h, C.byref(d), residual, model, np.ascontiguousarray(psfs, np.float32),
            major_loop_gain, None if um is None else um.ctypes.data, C.byref(r),
            boxes.ctypes.data, labels.ctypes.data, trace.ctypes.data, trace_cap)
        if rc != 0:
            raise RuntimeError(self.o.lib.orc_last_error().decode())
        return r, boxes, labels, trace[: min(r.n_trace, trace_cap)].copy()

    def margins(self):
        """Decision margins of the last execute: (margins, values) of the
        trace entries in trace order, then one end margin per subimage
        (values 0 there)."""
        L = self.o.lib
        L.orc_parallel_margins.restype = C.c_uint64
        L.orc_parallel_margins.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        n = L.orc_parallel_margins(self.h, None, None, 0)
        m, v = np.zeros(n, np.float32), np.zeros(n, np.float32)
        L.orc_parallel_margins(self.h, m.ctypes.data, v.ctypes.data, n)
        return m, v

    def __del__(self):
        try:
            self.o.lib.orc_parallel_destroy(self.h)
        except Exception:
            pass


_ORACLE = None


def get_oracle():
    global _ORACLE
    if _ORACLE is None:
        _ORACLE = Oracle()
    return _ORACLE


def get_ref():
    """The reference's own simple_clean.cc / fft_size_calculations.h, compiled
    from /root/reference by oracle/Makefile (None if it was not built)."""
    if not os.path.exists(REF_SO):
        return None
    L = C.CDLL(REF_SO)
    L.ref_partial_subtract.argtypes = [f32p, f32p, C.c_uint64, C.c_uint64, C.c_uint64,
                                       C.c_uint64, C.c_float, C.c_uint64, C.c_uint64]
    L.ref_good_fft_size.argtypes = [C.c_uint64]
    L.ref_good_fft_size.restype = C.c_uint64
    L.ref_convolution_size.argtypes = [C.c_double, C.c_uint64, C.c_double]
    L.ref_convolution_size.restype = C.c_uint64
    return L
