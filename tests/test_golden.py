"""Committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle reproduces the REFERENCE-generated vectors (PartialSubtractImage
from cpp/algorithms/simple_clean.cc, FFT sizes from cpp/utils/
fft_size_calculations.h, both compiled from /root/reference into oracle/_ref)
bit-exactly, and its own whole-run fixtures (regression pin).
GPU: the HIP path reproduces the reference vectors bit-exactly and the run
fixtures' component traces exactly (residual within 2e-5 * max|dirty|: FFT
rounding, see test_multiscale_gpu.py).
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)

from make_golden import RUNS, SUBTRACT_CASES, subtract_inputs  # noqa: E402
from oracle_lib import OracleAlgorithm, get_oracle  # noqa: E402
from synthetic import problem  # noqa: E402

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def load(name):
    return np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("w,h,seed", SUBTRACT_CASES)
def test_oracle_subtract_matches_reference_vectors(w, h, seed):
    orc = get_oracle()
    ref = load("ref_subtract")[f"ref_subtract_{w}x{h}_s{seed}"]
    img, psf, steps, factors = subtract_inputs(w, h, seed)
    for (x, y), f in zip(steps, factors):
        orc.subtract(img, psf, x, y, f)
    assert np.array_equal(bits(img), bits(ref))


def test_oracle_fft_sizes_match_reference_vectors():
    orc = get_oracle()
    with open(os.path.join(HERE, "ref_fft_sizes.json")) as fh:
        sizes = json.load(fh)
    for n, good in sizes["good_fft_size"].items():
        assert orc.good_fft_size(int(n)) == good, n
    for s, n, p, size in sizes["convolution_size"]:
        assert orc.convolution_size(s, n, p) == size, (s, n, p)


def run_oracle(name):
    kind, w, n_points, n_blobs, seed, st = RUNS[name]
    psf, dirty = problem(w, w, n_points, n_blobs, seed=seed)
    orc = get_oracle()
    orc.set_threads(4)
    res, mod = dirty[None].copy(), np.zeros((1, w, w), np.float32)
    r, trace = OracleAlgorithm(orc, kind, **st).execute(res, mod, psf[None])
    return r, trace, res[0], mod[0]


@pytest.mark.parametrize("name", sorted(RUNS))
def test_oracle_reproduces_run_fixtures(name):
    g = load(name)
    r, trace, res, mod = run_oracle(name)
    assert r.iteration_number == int(g["iterations"])
    assert np.array_equal(trace, g["trace"])
    assert np.array_equal(bits(res), bits(g["residual"]))
    assert np.array_equal(bits(mod), bits(g["model"]))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("w,h,seed", SUBTRACT_CASES)
def test_gpu_subtract_matches_reference_vectors(w, h, seed):
    from rdl_lib import Session
    s = Session(0)
    ref = load("ref_subtract")[f"ref_subtract_{w}x{h}_s{seed}"]
    img, psf, steps, factors = subtract_inputs(w, h, seed)
    d, dp = s.array(img), s.array(psf)
    for (x, y), f in zip(steps, factors):
        s.rdl.rdl_subtract_psf(s.h, d.vp, dp.vp, w, h, x, y, C.c_float(f))
    assert np.array_equal(bits(d.get()), bits(ref))
    d.free()
    dp.free()
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(RUNS))
def test_gpu_reproduces_run_fixtures(name):
    from radler_import import radler as rd
    g = load(name)
    kind, w, n_points, n_blobs, seed, st = RUNS[name]
    psf, dirty = problem(w, w, n_points, n_blobs, seed=seed)
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale if kind == 1 else rd.AlgorithmType.generic_clean
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = st["max_iterations"]
    s.absolute_threshold = st["threshold"]
    s.border_ratio = st["border_ratio"]
    s.major_loop_gain = st.get("major_loop_gain", 1.0)
    s.generic.use_sub_minor_optimization = bool(st.get("use_sub_minor", 1))
    if kind == 1:
        s.multiscale.max_scales = st["max_scales"]
    beam = st.get("beam_size_in_pixels", 0.0) * PIXEL_SCALE
    run = rd.gpu.DeviceRun(s, psf, dirty, [], beam)
    r = run.execute()
    assert r["iterations"] == int(g["iterations"])
    trace = run.trace()
    assert np.array_equal(trace[:, :2], g["trace"][:, :2])
    if kind == 1:
        assert np.array_equal(trace[:, 2], g["trace"][:, 2])
    tol = 2e-5 * np.abs(dirty).max()
    assert np.abs(run.residual().reshape(w, w) - g["residual"]).max() <= tol
    assert np.abs(run.model().reshape(w, w) - g["model"]).max() <= tol
