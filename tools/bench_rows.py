"""Micro-benchmark of the float row passes of the 8192^2 scale convolutions
(the headline's largest kernel family): rdl_conv_rows_inverse_peak (the
inverse rows with the fused peak search, RowsInverseDma), rdl_conv_rows_inverse
and rdl_conv_rows_forward on a tiled four-step plan. HIP-event times per
call from the C-ABI's timing families; prints GB/s of the algorithmic bytes
(spectrum read + image write / image read + spectrum write).

    python tools/bench_rows.py [size] [reps]
"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rdl_lib import Peak, Session  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    s = Session(0)
    lib = s.rdl.lib
    lib.rdl_conv_spectrum_bytes.restype = C.c_size_t
    lib.rdl_timing_get.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double),
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    c = C.c_void_p()
    s.rdl.rdl_conv_create_ex(s.h, n, n, 0, 0, C.byref(c))
    nb = lib.rdl_conv_spectrum_bytes(c)
    img = np.random.default_rng(1).standard_normal((n, n)).astype(np.float32)
    di = s.array(img)
    spec = s.array(shape=(nb,), dtype=np.uint8)
    out = s.array(shape=(n, n))
    s.rdl.rdl_conv_rows_forward(c, di.vp, n, n, 0, 0, spec.vp)
    s.sync()
    s.rdl.rdl_timing_enable(s.h, 1)

    def run(tag, fn, bytes_per):
        for _ in range(3):
            fn()
        s.sync()
        lib.rdl_timing_reset(s.h)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        s.sync()
        wall = (time.perf_counter() - t0) / reps
        ms, k, b = C.c_double(), C.c_uint64(), C.c_double()
        lib.rdl_timing_get(s.h, b"conv_rows", C.byref(ms), C.byref(k), C.byref(b))
        us = 1e3 * ms.value / max(k.value, 1)
        print(f"{tag:28s} {us:8.1f} us/call (events), {1e6 * wall:8.1f} us wall, "
              f"{bytes_per / us / 1e3:7.0f} GB/s", flush=True)

    peak = Peak()
    img_b = 4.0 * n * n
    run("rows_inverse_peak", lambda: (s.rdl.rdl_conv_rows_inverse_peak(
        c, spec.vp, out.vp, n, n, 0, 0, 0, 0, 1, None, 0)), nb + img_b)
    s.rdl.rdl_find_peak_collect(s.h, 1, C.byref(peak))
    run("rows_inverse", lambda: s.rdl.rdl_conv_rows_inverse(c, spec.vp, out.vp, n, n, 0, 0, 0),
        nb + img_b)
    run("rows_forward", lambda: s.rdl.rdl_conv_rows_forward(c, di.vp, n, n, 0, 0, spec.vp),
        nb + img_b)
    print(f"peak {peak.value:.6g} at ({peak.x}, {peak.y})")


if __name__ == "__main__":
    main()
