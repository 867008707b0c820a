"""Regression tests for the r04 intermittent test_divergence_kat failure.

Cause: the runtime-plan row transform (lds_fft.hip RowsForward) packs two
plane rows into one complex FFT. With a row mask (CorrectResidualDirty's
model plane, subminor.cc CorrectResidualDirtyWithSpectrum) only the marked
rows of the session's grow-only model scratch are zeroed before the
components are stored; an unmarked row next to a marked one still held
whatever the cached block held before, and that row's values leaked into its
partner's spectrum through the shared transform's rounding (NaN or 1e30-sized
bit patterns gave garbage up to ~1e3 in the corrected residual). Fresh
hipMalloc memory is zero, so the KAT passed alone and failed only after
earlier tests had recycled the block. RDL_POISON=1 (every fresh or reused
allocation filled with 0xff bytes, NaN as float) makes it deterministic.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sess():
    from rdl_lib import Session
    s = Session(0)
    yield s
    s.close()


@pytest.mark.parametrize("w,h,img_w,img_h", [(36, 36, 32, 32), (30, 36, 26, 32),
                                             (36, 30, 32, 26), (64, 48, 58, 44)])
@pytest.mark.parametrize("f64", [1, 0])
@pytest.mark.parametrize("garbage", [np.nan, 1e30])
def test_masked_convolve_subtract_ignores_unmarked_rows(sess, w, h, img_w, img_h, f64, garbage):
    """rdl_conv_convolve_subtract with a row mask: unmarked rows are zero
    whatever the image plane holds there (rdl_hip.h contract). Runtime plans
    (sizes without compile-time kernels), where the forward rows transform
    pairs rows. Bit-identical to the same call with those rows zeroed."""
    lib = sess.rdl.lib
    lib.rdl_conv_convolve_subtract_bytes.restype = C.c_size_t
    lib.rdl_conv_convolve_subtract_bytes.argtypes = [C.c_void_p]
    c = C.c_void_p()
    sess.rdl.rdl_conv_create_ex(sess.h, w, h, f64, 0, C.byref(c))
    assert lib.rdl_conv_fast(c) == 0, "expected a runtime-plan size"
    rng = np.random.default_rng(w * 7 + h + f64)
    nc = w // 2 + 1
    ctype = np.complex128 if f64 else np.complex64
    kern = (rng.standard_normal((h, nc)) + 1j * rng.standard_normal((h, nc))).astype(ctype)
    dk = sess.array(kern)
    work = sess.array(shape=(lib.rdl_conv_convolve_subtract_bytes(c),), dtype=np.uint8)
    ox, oy = (w - img_w) // 2, (h - img_h) // 2
    # components on every third image row: each marked row's pair partner
    # is unmarked
    marked = np.arange(1, img_h, 3)
    clean = np.zeros((img_h, img_w), np.float32)
    clean[marked, rng.integers(0, img_w, marked.size)] = rng.standard_normal(
        marked.size).astype(np.float32)
    stale = clean.copy()
    unmarked = np.setdiff1d(np.arange(img_h), marked)
    stale[unmarked] = np.float32(garbage)
    mask = np.zeros(h, np.uint8)
    mask[marked + oy] = 1
    dmask = sess.array(mask)
    residual = rng.standard_normal((img_h, img_w)).astype(np.float32)
    out = []
    for model in (clean, stale):
        dm, dr = sess.array(model), sess.array(residual)
        sess.rdl.rdl_conv_convolve_subtract(c, dm.vp, img_w, img_h, ox, oy, dk.vp, 0, 0,
                                            C.c_double(1.0 / (w * h)), dmask.vp, work.vp,
                                            dr.vp)
        out.append(dr.get())
        dm.free()
        dr.free()
    assert np.isfinite(out[1]).all()
    assert np.array_equal(out[0], out[1])
    for a in (dk, work, dmask):
        a.free()
    sess.rdl.rdl_conv_destroy(c)


CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
from test_kat_radler_gpu import divergence_kat_failures
fails = divergence_kat_failures()
print("failures:", fails)
sys.exit(1 if fails else 0)
"""


def test_divergence_kat_with_poisoned_allocations():
    """The reference's test_divergence.cc KAT in a process whose every
    device allocation starts as NaN bytes (RDL_POISON=1): a read of memory
    nothing wrote shows in the result. Failed 10 of 10 before the fix."""
    env = dict(os.environ, RDL_POISON="1")
    r = subprocess.run([sys.executable, "-c", CHILD, HERE], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
