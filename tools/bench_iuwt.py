#!/usr/bin/env python3
"""IUWT benchmarks (SURVEY.md §8(d) config C4, 4096^2):

1. component: IuwtDecomposition(6).Decompose + Recompose on the device,
   HIP-event time, algorithmic bytes 12 B/px per decomposition scale and
   8 B/px per recomposition scale, against the 8 TB/s HBM peak;
2. algorithm: DeviceRun(algorithm_type=iuwt) for K outer iterations
   (steps/s), beside the oracle (C++ restatement) on the same inputs for a
   bounded number of iterations.

  python tools/bench_iuwt.py [size] [iterations] [oracle_iterations]
"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-radler_amd"))

from rdl_lib import Session  # noqa: E402
from synthetic import problem  # noqa: E402

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def component(size, n_scales=6, reps=5):
    s = Session(0)
    L = s.rdl.lib
    L.rdl_timing_get.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double),
                                 C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    img = np.random.default_rng(1).standard_normal((size, size)).astype(np.float32)
    d_in = s.array(img)
    d_scratch = s.array(shape=(size, size))
    d_coeffs = s.array(shape=(n_scales + 1, size, size))
    d_out = s.array(shape=(size, size))
    s.rdl.rdl_iuwt_decompose(s.h, d_in.vp, d_scratch.vp, size, size, n_scales, d_coeffs.vp, 1)
    s.sync()
    for name, fn in (("decompose", lambda: s.rdl.rdl_iuwt_decompose(
                         s.h, d_in.vp, d_scratch.vp, size, size, n_scales, d_coeffs.vp, 1)),
                     ("recompose", lambda: s.rdl.rdl_iuwt_recompose(
                         s.h, d_coeffs.vp, size, size, n_scales, 1, d_out.vp))):
        L.rdl_timing_reset(s.h)
        L.rdl_timing_enable(s.h, 1)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        s.sync()
        wall = (time.perf_counter() - t0) / reps
        L.rdl_timing_enable(s.h, 0)
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        L.rdl_timing_get(s.h, b"iuwt", C.byref(ms), C.byref(n), C.byref(b))
        px = size * size
        alg = (12.0 if name == "decompose" else 8.0) * px * n_scales
        dev = ms.value / reps * 1e-3
        print(f"IUWT {name} {size}^2 x {n_scales} scales: {dev * 1e3:.2f} ms device "
              f"({wall * 1e3:.2f} ms wall), {alg / dev / 1e9:.0f} GB/s algorithmic "
              f"({alg / dev / 8e12:.3f} of 8 TB/s)", flush=True)


def algorithm(size, iterations, oracle_iterations):
    import radler as rd
    from oracle_lib import OracleAlgorithm, get_oracle
    psf, dirty = problem(size, size, 200, 20, seed=2025)
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.iuwt
    s.trimmed_image_width = s.trimmed_image_height = size
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = iterations
    s.absolute_threshold = 1e-3
    s.border_ratio = 0.0
    s.major_loop_gain = 0.8
    run = rd.gpu.DeviceRun(s, psf, dirty, [], 0.0)
    run.execute()  # warm-up: FFT plans for the box sizes met
    run.restore()
    run.sync()
    t0 = time.perf_counter()
    r = run.execute()
    run.sync()
    dt = time.perf_counter() - t0
    steps = run.iuwt_steps()
    print(f"IUWT algorithm {size}^2 GPU: {r['iterations']} iterations in {dt:.2f} s "
          f"({r['iterations'] / dt:.2f} it/s), {sum(1 for x in steps if x[0])} successful",
          flush=True)
    if oracle_iterations:
        orc = get_oracle()
        orc.set_threads(16)
        alg = OracleAlgorithm(orc, 2, threshold=1e-3, max_iterations=oracle_iterations,
                              border_ratio=0.0, minor_loop_gain=0.1, major_loop_gain=0.8)
        res, mod = dirty[None].copy(), np.zeros((1, size, size), np.float32)
        t0 = time.perf_counter()
        ro, _ = alg.execute(res, mod, psf[None])
        dto = time.perf_counter() - t0
        print(f"IUWT algorithm {size}^2 oracle (CPU, 16 threads for the FFTs): "
              f"{ro.iteration_number} iterations in {dto:.2f} s "
              f"({ro.iteration_number / dto:.3f} it/s)", flush=True)


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    iterations = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    oracle_iterations = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    component(size)
    algorithm(size, iterations, oracle_iterations)


if __name__ == "__main__":
    main()
