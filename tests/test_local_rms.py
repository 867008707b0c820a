"""Local-RMS thresholding: radler::math::rms_image
(cpp/math/rms_image.cc:16-125) and the RMS factor image every peak search
multiplies in (generic_clean.cc:126-128, 255-264; subminor_loop.cc:13-36,
134-149; multiscale_algorithm.cc:401-402, 700-748;
threaded_deconvolution_tools.cc:84-104; parallel_deconvolution.cc:244-250,
332-337, 421-423), driven by Radler::Perform (cpp/radler.cc:172-216).

CPU: the oracle's sliding minimum against a literal numpy restatement of the
reference loops, its RMS image against properties (a constant image has a
constant RMS equal to its magnitude; the factor image is lowest/rms).
GPU: the device sliding minimum (van Herk / Gil-Werman) bit-exact against
the oracle; the device RMS and factor images within 1e-5 relative (float32
FFT vs the oracle's float64 one); CLEAN with a given factor image (Clark,
Högbom, multiscale fast and non-fast, 1x1 and a 2x2 grid) with the same
component trace as the oracle and residual/model within 2e-5 x max|dirty|;
Radler.perform with local RMS over major iterations against the oracle's
Perform restatement.
The RestoreImage window kernel comes from the un-vendored schaapcommon
(restated in oracle/rms_image.cc): the RMS values' parity with the reference
itself is unpinned; their consumption is pinned by the tests above.
"""
import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, OracleParallel, get_oracle
from radler_oracle import OraclePerform
from synthetic import problem

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def sliding_min_reference(img, window):
    """rms_image.cc:35-68, literally."""
    h, w = img.shape
    half = window // 2
    tmp = np.empty_like(img)
    for y in range(h):
        for x in range(w):
            left = max(x, half) - half
            right = min(x, w - half) + half
            tmp[y, x] = img[y, left:right].min()
    out = np.empty_like(img)
    for x in range(w):
        for y in range(h):
            top = max(y, half) - half
            bottom = min(y, h - half) + half
            out[y, x] = tmp[top:bottom, x].min()
    return out


@pytest.mark.parametrize("w,h,window", [(17, 13, 4), (32, 32, 7), (20, 31, 2), (24, 24, 24)])
def test_oracle_sliding_minimum(w, h, window):
    rng = np.random.default_rng(w + window)
    img = rng.standard_normal((h, w)).astype(np.float32)
    np.testing.assert_array_equal(get_oracle().sliding_minimum(img, window),
                                  sliding_min_reference(img, window))


def test_oracle_rms_of_constant_image():
    w = h = 96
    img = np.full((h, w), -0.25, np.float32)
    beam = 2.0 * PIXEL_SCALE
    rms, factor, lowest = get_oracle().local_rms(img, 1, 3.0, beam, PIXEL_SCALE,
                                                 PIXEL_SCALE)
    np.testing.assert_allclose(rms, 0.25, rtol=1e-4)
    np.testing.assert_allclose(factor, np.float32(lowest) / rms, rtol=1e-6)
    # rms_and_minimum_window: max(rms, 0.3 |min|) = rms here
    rms2, _, _ = get_oracle().local_rms(img, 2, 3.0, beam, PIXEL_SCALE, PIXEL_SCALE)
    np.testing.assert_allclose(rms2, rms)


def test_oracle_factor_strengths():
    rng = np.random.default_rng(3)
    img = rng.standard_normal((64, 64)).astype(np.float32)
    beam = 2.0 * PIXEL_SCALE
    rms, f1, low = get_oracle().local_rms(img, 1, 4.0, beam, PIXEL_SCALE, PIXEL_SCALE, 1.0)
    assert abs(low - rms.min()) <= 1e-7 * abs(low)
    np.testing.assert_allclose(f1, (low / rms.astype(np.float64)).astype(np.float32),
                               rtol=1e-6)
    _, f0, _ = get_oracle().local_rms(img, 1, 4.0, beam, PIXEL_SCALE, PIXEL_SCALE, 0.0)
    assert np.all(f0 == 1.0)
    _, f2, _ = get_oracle().local_rms(img, 1, 4.0, beam, PIXEL_SCALE, PIXEL_SCALE, 0.5)
    np.testing.assert_allclose(f2, np.sqrt(low / rms.astype(np.float64)), rtol=1e-6)


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("w,h,window", [(17, 13, 4), (300, 200, 25), (257, 129, 2),
                                        (128, 128, 128), (64, 90, 9)])
def test_sliding_minimum_matches_oracle(w, h, window):
    from radler_import import radler as rd
    rng = np.random.default_rng(w * 3 + window)
    img = rng.standard_normal((h, w)).astype(np.float32)
    np.testing.assert_array_equal(rd.gpu.sliding_minimum(img, window),
                                  get_oracle().sliding_minimum(img, window))


@pytest.mark.gpu
@pytest.mark.parametrize("w,method,window,beam_px,strength", [
    (128, 1, 25.0, 2.0, 1.0), (256, 2, 5.0, 3.0, 1.0), (200, 2, 8.0, 2.5, 0.5),
    (512, 1, 3.0, 4.0, 2.0)])
def test_local_rms_image_matches_oracle(w, method, window, beam_px, strength):
    from radler_import import radler as rd
    psf, dirty = problem(w, w, 30, 3, seed=w, noise=1e-3)
    beam = beam_px * PIXEL_SCALE
    rms_g, f_g, low_g = rd.gpu.local_rms(dirty, method, window, beam, PIXEL_SCALE,
                                         PIXEL_SCALE, strength)
    rms_o, f_o, low_o = get_oracle().local_rms(dirty, method, window, beam, PIXEL_SCALE,
                                               PIXEL_SCALE, strength)
    np.testing.assert_allclose(rms_g, rms_o, rtol=1e-5, atol=1e-6 * rms_o.max())
    assert abs(low_g - low_o) <= 1e-5 * low_o
    np.testing.assert_allclose(f_g, f_o, rtol=2e-5)


def _settings(rd, kind, w, thr, max_iter, variant, grid=(1, 1)):
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale if kind == 1 else \
        rd.AlgorithmType.generic_clean
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = max_iter
    s.absolute_threshold = thr
    s.border_ratio = 0.0
    s.parallel.grid_width, s.parallel.grid_height = grid
    s.parallel.max_threads = 1
    if kind == 1:
        s.multiscale.max_scales = 4
        s.multiscale.fast_sub_minor_loop = variant == "fast"
    else:
        s.generic.use_sub_minor_optimization = variant == "clark"
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("kind,variant,grid", [(0, "clark", (1, 1)), (0, "hogbom", (1, 1)),
                                               (1, "fast", (1, 1)), (1, "slow", (1, 1)),
                                               (1, "fast", (2, 2)), (0, "clark", (2, 2))])
def test_clean_with_rms_factor_matches_oracle(kind, variant, grid):
    """The same factor image on both sides: identical traces."""
    from radler_import import radler as rd
    w = 192
    psf, dirty = problem(w, w, 40, 4, seed=11 + kind, noise=1e-3)
    _, factor, _ = get_oracle().local_rms(dirty, 2, 6.0, 3.0 * PIXEL_SCALE, PIXEL_SCALE,
                                          PIXEL_SCALE)
    thr, max_iter = 3e-3, 1200
    st = dict(threshold=thr, max_iterations=max_iter, border_ratio=0.0)
    if kind == 1:
        st.update(max_scales=4, beam_size_in_pixels=2.0, fast_sub_minor_loop=int(variant == "fast"))
    else:
        st.update(use_sub_minor=int(variant == "clark"))
    orc = get_oracle()
    orc.set_threads(8)
    res_o, mod_o = dirty[None].copy(), np.zeros((1, w, w), np.float32)
    run = rd.gpu.DeviceRun(_settings(rd, kind, w, thr, max_iter, variant, grid), psf, dirty,
                           [], 2.0 * PIXEL_SCALE if kind == 1 else 0.0)
    run.set_rms_factor(factor.ravel())
    r_g = run.execute()
    if grid == (1, 1):
        alg = OracleAlgorithm(orc, kind, **st)
        alg.set_rms(factor)
        r_o, trace_o = alg.execute(res_o, mod_o, psf[None])
        assert r_g["iterations"] == r_o.iteration_number > 20
        t_g = run.trace()
        assert np.array_equal(t_g if kind == 1 else t_g[:, :2],
                              trace_o if kind == 1 else trace_o[:, :2])
    else:
        par = OracleParallel(orc, kind, grid[0], grid[1], major_loop_gain=1.0, **st)
        par.set_rms(factor)
        r_o, _, _, trace_o = par.execute(res_o, mod_o, psf[None], 1.0)
        assert r_g["iterations"] == r_o.total_iterations > 20
        for i in range(grid[0] * grid[1]):
            t_o = trace_o[trace_o[:, 0] == i][:, 1:]
            t_g = run.trace(i)
            assert np.array_equal(t_g if kind == 1 else t_g[:, :2],
                                  t_o if kind == 1 else t_o[:, :2]), i
    tol = 2e-5 * np.abs(dirty).max()
    np.testing.assert_allclose(run.residual().reshape(w, w), res_o[0], atol=tol)
    np.testing.assert_allclose(run.model().reshape(w, w), mod_o[0], atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,method,auto_mask", [(1, 2, None), (0, 1, None), (1, 1, 5.0)])
def test_perform_local_rms_matches_oracle(kind, method, auto_mask):
    """Radler.perform with local RMS (and auto-masking, whose second phase
    drops the RMS image): per major iteration the same continue flag and
    residual/model within 2e-5 x max|dirty| as the oracle's Perform."""
    from radler_import import radler as rd
    w = 256
    psf, dirty = problem(w, w, 40, 4, seed=23 + kind, noise=1e-3)
    gain, minor = 0.1, 3000
    s = _settings(rd, kind, w, 0.0, minor, "fast" if kind == 1 else "clark")
    s.minor_loop_gain = gain
    s.auto_threshold_sigma = 3.0
    s.local_rms.method = rd.LocalRmsMethod.rms_window if method == 1 else \
        rd.LocalRmsMethod.rms_and_minimum_window
    s.local_rms.window = 6.0
    if auto_mask is not None:
        s.auto_mask_sigma = auto_mask
    beam = 3.0 * PIXEL_SCALE
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = rd.Radler(s, psf, residual, model, beam)
    st = dict(border_ratio=0.0)
    if kind == 1:
        st.update(max_scales=4, beam_size_in_pixels=3.0)
    o = OraclePerform(get_oracle(), kind, psf, dirty, minor_loop_gain=gain,
                      auto_threshold_sigma=3.0, auto_mask_sigma=auto_mask,
                      minor_iteration_count=minor, major_iteration_count=20,
                      local_rms=dict(method=method, window=6.0, beam=beam,
                                     pixel_scale=PIXEL_SCALE), **st)
    tol = 2e-5 * np.abs(dirty).max()
    for major in range(1, 6):
        another = r.perform(major)
        another_o = o.perform(major)
        assert another == another_o, major
        assert np.abs(residual - o.residual[0]).max() <= tol, major
        assert np.abs(model - o.model[0]).max() <= tol, major
        if not another:
            break
