"""Diagnose the intermittent test_divergence_kat failure (r04 verdict item 1).

The KAT's 5 x 5 split of a 160^2 image has subimages of 40, 34, 32 and 26
pixels; GenericClean pads by 1.1 to 44, 38, 36 and 30. 44 = 4 * 11 and
38 = 2 * 19 are not 2/3/5/7-smooth, so those corrections run on rocFFT
(float64) from 16 concurrent worker threads; 36 and 30 run on the LDS engine.

A: fresh rocFFT f64 plans of non-smooth sizes, executed once right after
   creation on a new non-blocking stream, against numpy.
B: 16 threads, one session each, rocFFT f64 forward transforms of the KAT's
   padded sizes, repeated, against numpy.
C: the KAT itself, repeated in this process, with the failing boxes listed.
"""
import ctypes as C
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rdl_lib import Rdl, Session  # noqa: E402


def fft_forward(sess, w, h, img, plan=None):
    rdl = sess.rdl
    f = plan
    if f is None:
        f = C.c_void_p()
        rdl.rdl_fft_create_f64(sess.h, w, h, C.byref(f))
    d_in = sess.array(img.astype(np.float64))
    d_out = sess.array(shape=(h, w // 2 + 1, 2), dtype=np.float64)
    rdl.rdl_fft64_forward(f, d_in.vp, d_out.vp)
    sess.sync()
    out = d_out.get()
    d_in.free()
    d_out.free()
    return f, out[..., 0] + 1j * out[..., 1]


def part_a(rdl):
    sizes = [22, 26, 34, 38, 44, 46, 52, 58, 62, 66, 74, 76, 78, 82, 86, 88, 92, 94,
             104, 106, 116, 118, 122, 134, 142, 146, 158, 166, 178, 194, 202, 214, 218,
             226, 244, 254, 262, 274, 278, 298, 302, 314, 326, 334, 346, 358, 362, 382]
    rng = np.random.default_rng(1)
    bad = 0
    for k, n in enumerate(sizes):
        w, h = n, sizes[(k + 3) % len(sizes)]
        sess = Session(0, rdl)
        img = rng.standard_normal((h, w))
        f, got = fft_forward(sess, w, h, img)
        ref = np.fft.rfft2(img)
        err = np.abs(got - ref).max() / np.abs(ref).max()
        f2, got2 = fft_forward(sess, w, h, img, f)
        err2 = np.abs(got2 - ref).max() / np.abs(ref).max()
        flag = "BAD" if err > 1e-10 or err2 > 1e-10 else "ok"
        bad += flag == "BAD"
        print(f"A {w}x{h}: first {err:.2e} second {err2:.2e} {flag}", flush=True)
        rdl.rdl_fft_destroy(f)
        sess.close()
    print(f"A: {bad} bad of {len(sizes)}", flush=True)
    return bad


def part_b(rdl, n_threads=16, reps=40):
    shapes = [(44, 44), (38, 44), (44, 38), (30, 44), (44, 30)]
    rng = np.random.default_rng(2)
    imgs = {s: rng.standard_normal((s[1], s[0])) for s in shapes}
    refs = {s: np.fft.rfft2(imgs[s]) for s in shapes}
    errors = []
    lock = threading.Lock()

    def work(t):
        sess = Session(0, rdl)
        plans = {}
        for r in range(reps):
            s = shapes[(t + r) % len(shapes)]
            f, got = fft_forward(sess, s[0], s[1], imgs[s], plans.get(s))
            plans[s] = f
            err = np.abs(got - refs[s]).max() / np.abs(refs[s]).max()
            if err > 1e-10:
                with lock:
                    errors.append((t, r, s, err))

    threads = [threading.Thread(target=work, args=(t,)) for t in range(n_threads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    print(f"B: {len(errors)} bad of {n_threads * reps}", flush=True)
    for e in errors[:20]:
        print("B bad", e, flush=True)
    return len(errors)


def kat(rd):
    grid, sub = 5, 32
    width = height = sub * grid
    pixel_scale = 1.0 / 60.0 / 60.0 * (np.pi / 180.0)
    s = rd.Settings()
    s.trimmed_image_width, s.trimmed_image_height = width, height
    s.pixel_scale.x = s.pixel_scale.y = pixel_scale
    s.minor_iteration_count = 1000000
    s.absolute_threshold = 1.0e-6
    s.parallel.grid_width = s.parallel.grid_height = grid
    s.divergence_limit = 4.0
    s.algorithm_type = rd.AlgorithmType.generic_clean
    s.save_source_list = True
    center = (height // 2) * width + width // 2
    good = np.zeros((height, width), np.float32)
    good.flat[center] = 1.0
    bad = np.zeros((height, width), np.float32)
    bad.flat[center - 2] = 2.0
    bad.flat[center + 2] = 2.0
    residual = np.zeros((height, width), np.float32)
    offsets = []
    for y in range(grid):
        for x in range(grid):
            ix, iy = x * sub + sub // 2, y * sub + sub // 2
            offsets.append((ix, iy))
            residual[iy, ix] = 5.0
            residual[iy, ix + 2] = 3.0
    model = np.zeros_like(residual)
    table = rd.WorkTable(np.array(offsets, np.uint64), 1, 1)
    e = rd.WorkTableEntry()
    e.polarization = rd.Polarization.stokes_i
    e.image_weight = 1.0
    for i in range(25):
        e.psfs.append(bad if i == 19 else good)
    e.residual = residual
    e.model = model
    table.add_entry(e)
    radler = rd.Radler(s, table, pixel_scale)
    radler.perform(1)
    fails = []
    for y in range(grid):
        for x in range(grid):
            i = y * grid + x
            bx, by = x * sub, y * sub
            r = residual[by:by + sub, bx:bx + sub].copy()
            if i == 19:
                r[sub // 2, sub // 2] = r[sub // 2, sub // 2 + 2] = 0
            if not (r < 1e-5).all() or not np.isfinite(r).all():
                k = int(np.nanargmax(np.where(np.isfinite(r), r, np.inf)))
                fails.append((i, k % sub + bx, k // sub + by, float(r.flat[k])))
    return fails, radler.component_list.component_count(0)


def part_c(reps):
    sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-radler_amd"))
    import radler as rd
    n_bad = 0
    for r in range(reps):
        t0 = time.time()
        fails, n = kat(rd)
        n_bad += bool(fails) or n != 48
        print(f"C rep {r}: components {n}, failing boxes {fails[:6]} "
              f"({time.time() - t0:.2f} s)", flush=True)
    print(f"C: {n_bad} bad of {reps}", flush=True)
    return n_bad


if __name__ == "__main__":
    parts = sys.argv[1] if len(sys.argv) > 1 else "ABC"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rdl = Rdl()
    if "C0" in parts:  # the KAT first, in a fresh process
        part_c(reps)
    if "A" in parts:
        part_a(rdl)
    if "B" in parts:
        part_b(rdl)
    if "C" in parts.replace("C0", ""):
        part_c(reps)
