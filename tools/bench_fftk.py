"""Micro-benchmark of the FFT kernel families as the multiscale path runs
them (HIP-event times from the C-ABI's timing families):

  f32  8192^2 scale convolution: rdl_conv_forward (rows forward + four-step
       columns), then per scale rdl_conv_columns mode 2 + rdl_conv_rows_inverse
  f64  9072^2 residual correction of an 8192^2 image: rows forward of a
       sparse model (ROWS non-zero rows), columns with the column-major PSF
       spectrum, rows inverse subtracting into the window

    python tools/bench_fftk.py [reps] [case ...]
    cases: f32 f32_4096 f64 f64_window f64_colout f64_dense f64_4096

Prints one line per family: average us per launch and the algorithmic GB/s
(bytes as the C-ABI counts them).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rdl_lib import Session  # noqa: E402

FAMS = ["conv_rows", "conv_cols", "conv64_rows", "conv64_cols", "conv_rows_sparse",
        "conv_cols_sparse", "conv64_rows_sparse", "conv64_cols_sparse"]
ROW_MAJOR, COL_MAJOR = 0, 1


def timings(s):
    out = {}
    for f in FAMS:
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        s.rdl.lib.rdl_timing_get(s.h, f.encode(), C.byref(ms), C.byref(n), C.byref(b))
        if n.value:
            out[f] = (ms.value / n.value, n.value, b.value / n.value)
    s.rdl.lib.rdl_timing_reset(s.h)
    return out


def report(tag, t):
    for k, (ms, n, b) in t.items():
        print(f"{tag:28s} {k:20s} {ms * 1e3:8.1f} us x{n:<4d} {b / (ms * 1e-3) / 1e9:8.1f} GB/s",
              flush=True)


def f32_case(s, n, reps):
    rng = np.random.default_rng(1)
    img = rng.standard_normal((n, n)).astype(np.float32)
    c = C.c_void_p()
    s.rdl.rdl_conv_create_ex(s.h, n, n, 0, 1, C.byref(c))
    nb = s.rdl.lib.rdl_conv_spectrum_bytes(c)
    di, out = s.array(img), s.array(shape=(n, n))
    spec, kspec, work = (s.array(shape=(nb // 8,), dtype=np.complex64) for _ in range(3))
    s.rdl.rdl_conv_forward(c, di.vp, kspec.vp)
    s.sync()
    timings(s)
    for _ in range(reps):
        s.rdl.rdl_conv_forward(c, di.vp, spec.vp)
    s.sync()
    report(f"f32 {n} forward", timings(s))
    for _ in range(reps):
        s.rdl.rdl_conv_columns(c, spec.vp, work.vp, kspec.vp, 2, C.c_double(1.0 / (n * n)))
        s.rdl.rdl_conv_rows_inverse(c, work.vp, out.vp, n, n, 0, 0, 0)
    s.sync()
    report(f"f32 {n} spectrum->image", timings(s))
    s.rdl.rdl_conv_destroy(c)
    for x in (di, out, spec, kspec, work):
        x.free()


def f64_case(s, pn, n, reps, n_rows=300, out_layout=ROW_MAJOR, dense=False, window=False):
    rng = np.random.default_rng(2)
    ox = oy = (pn - n) // 2
    psf = np.zeros((n, n), np.float32)
    psf[n // 2 - 40:n // 2 + 41, n // 2 - 40:n // 2 + 41] = rng.standard_normal((81, 81))
    model = np.zeros((n, n), np.float32)
    rows = rng.choice(n, n_rows, replace=False)
    for y in rows:
        model[y, rng.choice(n, 3, replace=False)] = rng.standard_normal(3)
    mask = np.zeros(pn, np.uint8)
    mask[rows + oy] = 1
    residual = rng.standard_normal((n, n)).astype(np.float32)
    c = C.c_void_p()
    s.rdl.rdl_conv_create_ex(s.h, pn, pn, 1, 1, C.byref(c))
    nb = s.rdl.lib.rdl_conv_spectrum_bytes(c)
    dpsf, dmod, dres = s.array(psf), s.array(model), s.array(residual)
    dmask = s.array(mask)
    kspec, work, out2 = (s.array(shape=(nb // 16,), dtype=np.complex128) for _ in range(3))
    # the column-major PSF spectrum (as MakePaddedPsfSpectrum)
    s.rdl.rdl_conv_rows_forward(c, dpsf.vp, n, n, ox, oy, work.vp)
    s.rdl.rdl_conv_columns_ex(c, work.vp, kspec.vp, None, 0, C.c_double(1.0), None,
                              ROW_MAJOR, COL_MAJOR)
    s.sync()
    timings(s)
    for _ in range(reps):
        s.rdl.rdl_conv_rows_forward_masked(c, dmod.vp, n, n, ox, oy, work.vp, dmask.vp)
        if window:  # only the window's rows stored (rdl_conv_columns_window)
            s.rdl.rdl_conv_columns_window(c, work.vp, work.vp, kspec.vp,
                                          C.c_double(1.0 / (pn * pn)), dmask.vp, COL_MAJOR,
                                          oy, n)
        else:
            s.rdl.rdl_conv_columns_ex(c, work.vp,
                                      work.vp if out_layout == ROW_MAJOR else out2.vp,
                                      kspec.vp, 1, C.c_double(1.0 / (pn * pn)),
                                      None if dense else dmask.vp, COL_MAJOR, out_layout)
        if out_layout == ROW_MAJOR:
            s.rdl.rdl_conv_rows_inverse(c, work.vp, dres.vp, n, n, ox, oy, 1)
    s.sync()
    tag = ("col-major out" if out_layout != ROW_MAJOR else "dense" if dense else
           "window" if window else "correction")
    report(f"f64 {pn} {tag}", timings(s))
    s.rdl.rdl_conv_destroy(c)
    for x in (dpsf, dmod, dres, dmask, kspec, work, out2):
        x.free()


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cases = sys.argv[2:] or ["f32", "f64"]
    s = Session(0)
    s.rdl.lib.rdl_timing_get.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double),
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    s.rdl.lib.rdl_conv_spectrum_bytes.restype = C.c_size_t
    s.rdl.lib.rdl_timing_enable(s.h, 1)
    for case in cases:
        if case == "f32":
            f32_case(s, 8192, reps)
        elif case == "f32_4096":
            f32_case(s, 4096, reps)
        elif case == "f64":
            f64_case(s, 9072, 8192, reps)
        elif case == "f64_window":
            f64_case(s, 9072, 8192, reps, window=True)
        elif case == "f64_colout":
            f64_case(s, 9072, 8192, reps, out_layout=COL_MAJOR)
        elif case == "f64_dense":
            f64_case(s, 9072, 8192, reps, dense=True)
        elif case == "f64_4096":
            f64_case(s, 4536, 4096, reps)
    s.close()


if __name__ == "__main__":
    main()
