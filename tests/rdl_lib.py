"""ctypes binding of the product C-ABI (include/rdl_hip.h -> librdl_hip.so).

GPU parity tests call through this boundary; the CPU suite only checks that
the library loads and exports every declared symbol.
"""
import atexit
import ctypes as C
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ska-sdp-func-radler_amd")
HIP_SO = os.path.join(PKG, "lib", "librdl_hip.so")
HEADER = os.path.join(ROOT, "include", "rdl_hip.h")
MAX_IMAGES = 64


def declared_symbols(header=HEADER):
    text = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\*?(rdl_[a-z_0-9]+)\(",
                                 text, re.M)))


class Integration(C.Structure):
    _fields_ = [("n_images", C.c_uint32), ("n_pol", C.c_uint32),
                ("n_channels", C.c_uint32), ("mode", C.c_uint32),
                ("copy_fast_path", C.c_uint32), ("pol_mask", C.c_uint32),
                ("weights", C.c_float * MAX_IMAGES), ("factor", C.c_float)]


def integration(n_channels=1, n_pol=1, weights=None, pol_factor=1.0, mode=0):
    """Host-side factor computation of cpp/image_set.cc:309-462 (see header)."""
    g = Integration()
    n = n_channels * n_pol
    g.n_images, g.n_pol, g.n_channels, g.mode = n, n_pol, n_channels, mode
    w = np.ones(n_channels, np.float32) if weights is None else np.asarray(weights, np.float32)
    g.copy_fast_path = int(n_channels == 1 and n_pol == 1 and mode != 2)
    g.pol_mask = (1 << n_pol) - 1
    for i in range(n):
        g.weights[i] = float(w[i // n_pol])
    wsum = float(sum(float(x) for x in w if x != 0.0))
    if mode == 0:
        g.factor = np.float32(pol_factor / wsum) if wsum > 0 else 0.0
    elif mode == 1:
        if n_channels == 1:
            g.factor = np.sqrt(np.float32(pol_factor))
        else:
            g.factor = np.float32(np.float64(np.sqrt(np.float32(pol_factor))) / wsum)
    else:
        g.factor = np.float32(np.sqrt(pol_factor / wsum)) if wsum > 0 else 0.0
    return g


class Peak(C.Structure):
    _fields_ = [("value", C.c_float), ("x", C.c_uint32), ("y", C.c_uint32),
                ("found", C.c_int32)]


class HogbomParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("n_images", C.c_uint32),
                ("n_pol", C.c_uint32), ("integ", Integration), ("gain", C.c_float),
                ("threshold", C.c_float), ("initial_max", C.c_float),
                ("divergence_limit", C.c_float), ("iteration_start", C.c_uint64),
                ("max_iterations", C.c_uint64), ("allow_negative", C.c_int32),
                ("stop_on_negative", C.c_int32), ("h_border", C.c_uint32),
                ("v_border", C.c_uint32), ("d_mask", C.c_void_p),
                ("start_x", C.c_uint32), ("start_y", C.c_uint32),
                ("start_value", C.c_float), ("start_found", C.c_int32),
                ("d_spectral", C.c_void_p), ("d_rms", C.c_void_p),
                ("logpoly", C.c_void_p)]


class HogbomResult(C.Structure):
    _fields_ = [("iteration", C.c_uint64), ("peak", C.c_float), ("x", C.c_uint32),
                ("y", C.c_uint32), ("found", C.c_int32), ("diverging", C.c_int32)]


class SubminorParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("n_images", C.c_uint32),
                ("n_pol", C.c_uint32), ("integ", Integration), ("h_border", C.c_uint32),
                ("v_border", C.c_uint32), ("allow_negative", C.c_int32),
                ("stop_on_negative", C.c_int32), ("threshold", C.c_float),
                ("gain", C.c_float), ("divergence_limit", C.c_float),
                ("iteration_start", C.c_uint64), ("max_iterations", C.c_uint64),
                ("d_mask", C.c_void_p), ("d_spectral", C.c_void_p),
                ("d_rms", C.c_void_p), ("logpoly", C.c_void_p)]


class SubminorResult(C.Structure):
    _fields_ = [("n_selected", C.c_uint64), ("iteration", C.c_uint64),
                ("has_peak", C.c_int32), ("peak", C.c_float), ("diverging", C.c_int32),
                ("flux_cleaned", C.c_float)]


class LogPoly(C.Structure):
    """rdl_logpoly: the log-polynomial fitter's description."""
    _fields_ = [("n_channels", C.c_uint32), ("n_terms", C.c_uint32),
                ("fit_mask", C.c_uint32), ("reserved", C.c_uint32),
                ("lg", C.c_double * 16)]


def logpoly(frequencies, weights, n_terms):
    """The rdl_logpoly of a fitter (reference = weighted mean frequency)."""
    f = np.asarray(frequencies, np.float64)
    w = np.asarray(weights, np.float32)
    ref = np.sum(f * w) / np.sum(w) if np.sum(w) > 0 else np.mean(f)
    lp = LogPoly()
    lp.n_channels, lp.n_terms = len(f), n_terms
    lp.fit_mask = sum(1 << c for c in range(len(f)) if w[c] > 0)
    for c in range(len(f)):
        lp.lg[c] = np.log10(f[c] / ref)
    return lp


class RdlError(RuntimeError):
    pass


class Rdl:
    """Loads librdl_hip.so. Functions are called as self.<name>(...) and
    raise RdlError on a non-zero status."""

    def __init__(self, path=HIP_SO):
        if not os.path.exists(path):
            raise RdlError(f"librdl_hip.so not built: {path}")
        self.lib = C.CDLL(path)
        self.lib.rdl_last_error.restype = C.c_char_p
        self.lib.rdl_version.restype = C.c_char_p
        self.lib.rdl_session_stream.restype = C.c_void_p
        self.lib.rdl_session_stream.argtypes = [C.c_void_p]
        self.lib.rdl_fft_spectrum_bytes.restype = C.c_size_t
        self.lib.rdl_fft_spectrum_bytes.argtypes = [C.c_void_p]
        self.lib.rdl_conv_spectrum_bytes.restype = C.c_size_t
        self.lib.rdl_conv_spectrum_bytes.argtypes = [C.c_void_p]
        # release the library's device state at interpreter exit, before the
        # runtime's C-level exit handlers (as the radler module does)
        if os.environ.get("RDL_EXIT_SHUTDOWN") != "0":
            atexit.register(self.lib.rdl_shutdown)

    def __getattr__(self, name):
        fn = getattr(self.lib, name)

        def call(*args):
            rc = fn(*args)
            if rc != 0:
                raise RdlError(f"{name}: rc={rc}: {self.lib.rdl_last_error().decode()}")
            return rc
        return call


class DeviceArray:
    """A device buffer holding a numpy array's bytes."""

    def __init__(self, sess, arr=None, shape=None, dtype=np.float32):
        self.sess = sess
        if arr is not None:
            arr = np.ascontiguousarray(arr)
            self.shape, self.dtype = arr.shape, arr.dtype
        else:
            self.shape, self.dtype = tuple(shape), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * np.dtype(self.dtype).itemsize
        p = C.c_void_p()
        sess.rdl.rdl_malloc(sess.h, C.c_size_t(max(self.nbytes, 16)), C.byref(p))
        self.ptr = p.value
        if arr is not None:
            self.upload(arr)
        else:
            sess.rdl.rdl_memset_zero(sess.h, C.c_void_p(self.ptr), C.c_size_t(self.nbytes))

    def upload(self, arr):
        arr = np.ascontiguousarray(arr, dtype=self.dtype)
        assert arr.nbytes == self.nbytes
        self.sess.rdl.rdl_memcpy_h2d(self.sess.h, C.c_void_p(self.ptr),
                                     arr.ctypes.data_as(C.c_void_p), C.c_size_t(self.nbytes))

    def get(self):
        out = np.empty(self.shape, self.dtype)
        self.sess.rdl.rdl_memcpy_d2h(self.sess.h, out.ctypes.data_as(C.c_void_p),
                                     C.c_void_p(self.ptr), C.c_size_t(self.nbytes))
        return out

    @property
    def vp(self):
        return C.c_void_p(self.ptr)

    def offset(self, nbytes):
        return C.c_void_p(self.ptr + nbytes)

    def free(self):
        if self.ptr:
            self.sess.rdl.rdl_free(self.sess.h, C.c_void_p(self.ptr))
            self.ptr = 0


class Session:
    def __init__(self, device=0, rdl=None):
        self.rdl = rdl or Rdl()
        h = C.c_void_p()
        self.rdl.rdl_session_create(device, C.byref(h))
        self.h = h

    def array(self, arr=None, shape=None, dtype=np.float32):
        return DeviceArray(self, arr, shape, dtype)

    def sync(self):
        self.rdl.rdl_session_sync(self.h)

    def find_peak(self, dimg, w, h, allow_negative=True, start_y=0, end_y=None, hb=0, vb=0,
                  dmask=None, avx=True):
        p = Peak()
        self.rdl.rdl_find_peak(self.h, dimg.vp, w, h, start_y, h if end_y is None else end_y,
                               hb, vb, int(allow_negative),
                               None if dmask is None else dmask.vp, int(avx), C.byref(p))
        return bool(p.found), p.x, p.y, p.value

    def close(self):
        if self.h:
            self.rdl.rdl_session_destroy(self.h)
            self.h = None
