"""Micro-benchmark of rdl_subminor_run (the sub-minor loop kernels) on an
8192^2 PSF with a controlled selection size: us per iteration by kernel
variant and workgroup target. Usage: python tools/bench_subminor.py [size]"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rdl_lib import Session, SubminorParams, SubminorResult, integration  # noqa: E402
from synthetic import make_psf_uv  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    s = Session(0)
    psf = make_psf_uv(size, size)
    dpsf = s.array(psf)
    rng = np.random.default_rng(1)
    sm = C.c_void_p()
    s.rdl.rdl_subminor_create(s.h, C.byref(sm))
    # mode -1: the generic kernels (auto policy with the table loop off)
    os.environ["RDL_SUBMINOR_TAB"] = "0"
    sm_old = C.c_void_p()
    s.rdl.rdl_subminor_create(s.h, C.byref(sm_old))
    del os.environ["RDL_SUBMINOR_TAB"]
    sizes = (256, 1024, 4096, 16384, 65536, 262144)
    variants = ((1, 0), (2, 512), (2, 1024), (2, 2048), (2, 4096))
    if os.environ.get("RDL_BENCH_WAVE"):  # single-wave vs eight-wave kernel
        sizes = (64, 128, 256, 400, 512, 768, 1024)
        variants = ((2, 0), (3, 0))
    if os.environ.get("RDL_BENCH_BIGGRID"):  # grids of 1024- vs 512-thread workgroups
        sizes = (4096, 6144, 8192, 12288, 16384, 32768)
        variants = ((0, 1024), (5, 2048), (5, 3072), (5, 4096))
    if os.environ.get("RDL_BENCH_TAB"):  # the table kernel (pixels per participant)
        sizes = (200, 400, 800, 1024, 1500, 2048, 3000, 4096, 6000, 8192, 11000, 16000)
        variants = ((-1, 0), (6, 512), (6, 1024), (6, 2048), (6, 8192), (6, 1 << 20))
        threads = os.environ.get("RDL_SUBMINOR_TAB_THREADS", "")
    if os.environ.get("RDL_BENCH_BIG"):  # one 1024-thread workgroup vs the grid
        sizes = (1536, 2048, 3072, 4096, 6144, 8192)
        variants = ((0, 1024), (4, 0))
    for n_sel in sizes:
        img = np.zeros((size, size), np.float32)
        n_cl = 24
        cx = rng.uniform(500, size - 500, n_cl)
        cy = rng.uniform(500, size - 500, n_cl)
        k = rng.integers(0, n_cl, 4 * n_sel)
        xs = np.clip((cx[k] + rng.normal(0, 60, k.size)).astype(int), 0, size - 1)
        ys = np.clip((cy[k] + rng.normal(0, 60, k.size)).astype(int), 0, size - 1)
        flat = np.unique(ys * size + xs)[:n_sel]
        img.flat[flat] = rng.uniform(1.0, 2.0, flat.size).astype(np.float32)
        dres = s.array(img)
        for mode, target in variants:
            h = sm_old if mode < 0 else sm
            s.rdl.rdl_subminor_set_tuning(h, max(mode, 0), target)
            p = SubminorParams()
            p.width = p.height = size
            p.n_images, p.n_pol = 1, 1
            p.integ = integration(1, 1, mode=0)
            p.allow_negative, p.stop_on_negative = 1, 0
            p.threshold, p.gain, p.divergence_limit = 0.5, 0.1, 0.0
            p.iteration_start, p.max_iterations = 0, 3000
            out = SubminorResult()
            dres.upload(img)
            s.rdl.rdl_session_sync(s.h)
            t = time.perf_counter()
            try:
                # warm (buffers sized), then timed
                s.rdl.rdl_subminor_run(h, dres.vp, dpsf.vp, C.byref(p), C.byref(out), None,
                                       C.c_uint64(0))
                dres.upload(img)
                s.rdl.rdl_session_sync(s.h)
                t = time.perf_counter()
                s.rdl.rdl_subminor_run(h, dres.vp, dpsf.vp, C.byref(p), C.byref(out), None,
                                       C.c_uint64(0))
            except Exception as e:  # noqa: BLE001
                print(f"n_sel={flat.size} mode={mode} target={target}: {e}", flush=True)
                continue
            dt = time.perf_counter() - t
            print(f"n_sel={flat.size:7d} mode={mode} target={target:5d} iters={out.iteration:5d} "
                  f"us/iter={1e6 * dt / max(out.iteration, 1):7.2f}", flush=True)
        dres.free()
    s.rdl.rdl_subminor_destroy(sm)
    s.rdl.rdl_subminor_destroy(sm_old)


if __name__ == "__main__":
    main()
