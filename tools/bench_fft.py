"""Micro-benchmark: rocFFT (rdl_fft_*) vs the LDS engine (rdl_conv_*) for the
two convolution shapes of the multiscale hot path. Times from the C-ABI's
HIP-event families. Usage: python tools/bench_fft.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rdl_lib import Session  # noqa: E402

FAMS = ["fft", "fft64", "spectrum_multiply", "spectrum_multiply64", "trim_subtract",
        "conv_rows", "conv_cols", "conv64_rows", "conv64_cols"]


def timings(s):
    out = {}
    for f in FAMS:
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        s.rdl.lib.rdl_timing_get(s.h, f.encode(), C.byref(ms), C.byref(n), C.byref(b))
        if n.value:
            out[f] = (ms.value / n.value, n.value, b.value / n.value)
    s.rdl.lib.rdl_timing_reset(s.h)
    return out


def report(tag, t, reps):
    tot = sum(v[0] * v[1] for v in t.values()) / reps
    parts = ", ".join(f"{k} {v[0]*1e3:.0f}us ({v[2]/v[0]/1e6:.0f} GB/s)" for k, v in t.items())
    print(f"{tag:34s} {tot*1e3:8.1f} us/op | {parts}", flush=True)


def main():
    s = Session(0)
    s.rdl.lib.rdl_timing_get.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double),
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    s.rdl.lib.rdl_conv_spectrum_bytes.restype = C.c_size_t
    reps = 10
    cases = ((8192, 8192, False), (9216, 9216, True), (9072, 9072, True), (4096, 4096, False))
    if len(sys.argv) > 1:  # e.g. "9072,9072,1"
        w, h, f = (int(v) for v in sys.argv[1].split(","))
        cases = ((w, h, bool(f)),)
        reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for (w, h, f64) in cases:
        img = np.random.default_rng(1).standard_normal((h, w)).astype(np.float32)
        di = s.array(img)
        cdt = np.complex128 if f64 else np.complex64
        spec = s.array(shape=(h, w // 2 + 1), dtype=cdt)
        kspec = s.array(shape=(h, w // 2 + 1), dtype=cdt)
        work = s.array(shape=(h, w // 2 + 1), dtype=cdt)
        out = s.array(shape=(h, w))
        # rocFFT
        f = C.c_void_p()
        (s.rdl.rdl_fft_create_f64 if f64 else s.rdl.rdl_fft_create)(s.h, w, h, C.byref(f))
        if f64:
            dpl = s.array(shape=(h, w), dtype=np.float64)
            s.rdl.rdl_fft64_forward(f, dpl.vp, kspec.vp)
        else:
            s.rdl.rdl_fft_forward(f, di.vp, kspec.vp)
        s.rdl.rdl_session_sync(s.h)
        s.rdl.lib.rdl_timing_enable(s.h, 1)
        timings(s)
        for _ in range(reps):
            if f64:
                s.rdl.rdl_fft64_convolve(f, dpl.vp, kspec.vp, work.vp)
                s.rdl.rdl_trim_subtract_f64(s.h, out.vp, w - 880, h - 880, dpl.vp, w, h)
            else:
                s.rdl.rdl_fft_convolve(f, di.vp, kspec.vp, work.vp)
        s.rdl.rdl_session_sync(s.h)
        report(f"rocFFT {w}x{h} {'f64' if f64 else 'f32'} convolve", timings(s), reps)
        s.rdl.rdl_fft_destroy(f)
        for columns, cname in ((1, "single"), (2, "split")):
            lds_engine(s, w, h, f64, columns, cname, di, spec, kspec, work, out, reps)
        for x in (di, spec, kspec, work, out):
            x.free()
        if f64:
            dpl.free()


def lds_engine(s, w, h, f64, columns, cname, di, spec, kspec, work, out, reps):
    if True:
        c = C.c_void_p()
        rc = s.rdl.lib.rdl_conv_create_ex(s.h, w, h, int(f64), columns, C.byref(c))
        if rc != 0:
            print("LDS engine unsupported", w, h, cname)
            return
        # spectra of this plan (the tiled float layout pads the last tile)
        nbytes = s.rdl.lib.rdl_conv_spectrum_bytes(c)
        cdt = np.complex128 if f64 else np.complex64
        spec, kspec, work = (s.array(shape=(nbytes // np.dtype(cdt).itemsize,), dtype=cdt)
                             for _ in range(3))
        s.rdl.lib.rdl_timing_enable(s.h, 1)
        s.rdl.rdl_conv_forward(c, di.vp, kspec.vp)
        s.rdl.rdl_session_sync(s.h)
        timings(s)
        for _ in range(reps):
            if f64:
                s.rdl.rdl_conv_rows_forward(c, di.vp, w - 880, h - 880, 440, 440, work.vp)
                s.rdl.rdl_conv_columns(c, work.vp, work.vp, kspec.vp, 1, C.c_double(1.0 / (w * h)))
                s.rdl.rdl_conv_rows_inverse(c, work.vp, out.vp, w - 880, h - 880, 440, 440, 1)
            else:
                s.rdl.rdl_conv_rows_forward(c, di.vp, w, h, 0, 0, work.vp)
                s.rdl.rdl_conv_columns(c, work.vp, work.vp, kspec.vp, 1, C.c_double(1.0 / (w * h)))
                s.rdl.rdl_conv_rows_inverse(c, work.vp, di.vp, w, h, 0, 0, 0)
        s.rdl.rdl_session_sync(s.h)
        report(f"LDS[{cname}] {w}x{h} {'f64' if f64 else 'f32'} convolve", timings(s), reps)
        if not f64:
            s.rdl.rdl_conv_forward(c, di.vp, spec.vp)
            timings(s)
            for _ in range(reps):
                s.rdl.rdl_conv_columns(c, spec.vp, work.vp, kspec.vp, 2, C.c_double(1.0 / (w * h)))
                s.rdl.rdl_conv_rows_inverse(c, work.vp, out.vp, w, h, 0, 0, 0)
            s.rdl.rdl_session_sync(s.h)
            report(f"LDS[{cname}] {w}x{h} f32 spectrum->image", timings(s), reps)
        s.rdl.lib.rdl_timing_enable(s.h, 0)
        s.rdl.rdl_conv_destroy(c)
        for x in (spec, kspec, work):
            x.free()


if __name__ == "__main__":
    main()
