"""Micro-benchmark of CorrectResidualDirty's padded float64 convolution as
the product runs it (rdl_conv_convolve_subtract on a 9072^2 plane, the tiled
float64 layout, an 8192^2 window, a sparse model of ROWS occupied rows):
HIP-event time per family (rows forward sparse, columns, rows inverse with
the subtraction) and the algorithmic GB/s the C-ABI counts.

    python tools/bench_corr.py [reps] [rows] [kernel_f32]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rdl_lib import Session  # noqa: E402

FAMS = ["conv64_rows_sparse", "conv64_cols_sparse", "conv64_rows", "conv64_cols"]
ROW_MAJOR, COL_MAJOR = 0, 1


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n_rows = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    kf = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    pn, n = 9072, 8192
    s = Session(0)
    lib = s.rdl.lib
    lib.rdl_timing_get.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double),
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    lib.rdl_conv_spectrum_bytes.restype = C.c_size_t
    lib.rdl_conv_convolve_subtract_bytes.restype = C.c_size_t
    lib.rdl_conv_convolve_subtract_bytes.argtypes = [C.c_void_p]
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
    s.rdl.rdl_conv_create_ex(s.h, pn, pn, 1, 0, C.byref(c))
    nb = lib.rdl_conv_spectrum_bytes(c)
    dpsf, dmod, dres, dmask = s.array(psf), s.array(model), s.array(residual), s.array(mask)
    kspec = s.array(shape=(nb // 16,), dtype=np.complex128)
    kspec32 = s.array(shape=(nb // 16,), dtype=np.complex64)
    tmp = s.array(shape=(nb // 16,), dtype=np.complex128)
    work = s.array(shape=(lib.rdl_conv_convolve_subtract_bytes(c),), dtype=np.uint8)
    # the column-major PSF spectrum (MakePaddedPsfSpectrum's ForwardColumnMajor)
    s.rdl.rdl_conv_rows_forward(c, dpsf.vp, n, n, ox, oy, tmp.vp)
    s.rdl.rdl_conv_columns_ex(c, tmp.vp, kspec.vp, None, 0, C.c_double(1.0), None,
                              ROW_MAJOR, COL_MAJOR)
    s.rdl.rdl_complex_narrow(s.h, kspec32.vp, kspec.vp, C.c_size_t(nb // 16))
    s.sync()
    s.rdl.rdl_timing_enable(s.h, 1)
    k = kspec32 if kf else kspec
    for _ in range(3):
        s.rdl.rdl_conv_convolve_subtract(c, dmod.vp, n, n, ox, oy, k.vp, COL_MAJOR, kf,
                                         C.c_double(1.0 / (pn * pn)), dmask.vp, work.vp, dres.vp)
    s.sync()
    lib.rdl_timing_reset(s.h)
    for _ in range(reps):
        s.rdl.rdl_conv_convolve_subtract(c, dmod.vp, n, n, ox, oy, k.vp, COL_MAJOR, kf,
                                         C.c_double(1.0 / (pn * pn)), dmask.vp, work.vp, dres.vp)
    s.sync()
    total = 0.0
    for f in FAMS:
        ms, cnt, b = C.c_double(), C.c_uint64(), C.c_double()
        lib.rdl_timing_get(s.h, f.encode(), C.byref(ms), C.byref(cnt), C.byref(b))
        if cnt.value:
            us = 1e3 * ms.value / cnt.value
            total += us
            print(f"{f:22s} {us:8.1f} us x{cnt.value:<4d} "
                  f"{b.value / cnt.value / (us * 1e-6) / 1e9:8.1f} GB/s", flush=True)
    print(f"{'correction':22s} {total:8.1f} us per call ({n_rows} model rows, "
          f"kernel {'f32' if kf else 'f64'})")


if __name__ == "__main__":
    main()
