"""Multiscale CLEAN on the MI355X (radler.gpu.DeviceRun -> the same
ParallelDeconvolution/MultiScaleAlgorithm path as Radler.perform) against the
CPU restatement (oracle MultiScale, float64 FFT).

Parity: component positions and scales bit-exact (the full trace); residual
and model within atol = 2e-5 * max|dirty| (FFT convolutions differ in
rounding: rocFFT float vs float64). Iteration counts equal.
"""
import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, get_oracle
from radler_import import radler as rd
from synthetic import problem

pytestmark = pytest.mark.gpu

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def gpu_settings(w, h, threshold, max_iter, max_scales, fast=True, shape=0,
                 gain=0.1, mgain=1.0):
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale
    s.trimmed_image_width, s.trimmed_image_height = w, h
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = max_iter
    s.absolute_threshold = threshold
    s.minor_loop_gain = gain
    s.major_loop_gain = mgain
    s.multiscale.max_scales = max_scales
    s.multiscale.fast_sub_minor_loop = fast
    s.multiscale.shape = [rd.MultiscaleShape.tapered_quadratic,
                          rd.MultiscaleShape.gaussian][shape]
    return s


CASES = [
    # w, n_points, n_blobs, threshold, max_iter, max_scales, beam_px, fast, shape
    (128, 10, 2, 5e-3, 500, 4, 2.0, True, 0),
    (256, 40, 4, 5e-3, 2000, 5, 2.0, True, 0),
    (256, 40, 4, 5e-3, 800, 4, 2.0, True, 1),
    (96, 6, 2, 2e-2, 150, 3, 2.0, False, 0),
]


@pytest.mark.parametrize("w,n_points,n_blobs,thr,max_iter,max_scales,beam_px,fast,shape", CASES)
def test_multiscale_parity(w, n_points, n_blobs, thr, max_iter, max_scales, beam_px, fast, shape):
    h = w
    psf, dirty = problem(w, h, n_points, n_blobs, seed=w + n_points)
    orc = get_oracle()
    orc.set_threads(8)
    res_o, mod_o = dirty[None].copy(), np.zeros((1, h, w), np.float32)
    alg = OracleAlgorithm(orc, 1, threshold=thr, max_iterations=max_iter, border_ratio=0.0,
                          max_scales=max_scales, beam_size_in_pixels=beam_px,
                          fast_sub_minor_loop=int(fast), shape=shape)
    r_o, trace_o = alg.execute(res_o, mod_o, psf[None])

    s = gpu_settings(w, h, thr, max_iter, max_scales, fast, shape)
    run = rd.gpu.DeviceRun(s, psf, dirty, [], beam_px * PIXEL_SCALE)
    r_g = run.execute()
    trace_g = run.trace()
    assert r_g["iterations"] == r_o.iteration_number
    assert trace_g.shape == trace_o.shape
    if not np.array_equal(trace_g, trace_o):
        first = int(np.argmax(np.any(trace_g != trace_o, axis=1)))
        pytest.fail(f"component trace differs first at {first}: gpu {trace_g[first]} "
                    f"oracle {trace_o[first]}")
    tol = 2e-5 * np.abs(dirty).max()
    np.testing.assert_allclose(run.residual().reshape(h, w), res_o[0], atol=tol)
    np.testing.assert_allclose(run.model().reshape(h, w), mod_o[0], atol=tol)
    assert r_g["another_iteration_required"] == bool(r_o.another_iteration_required)
    assert abs(r_g["end_peak"] - r_o.final_peak) <= tol


def test_multiscale_restore_is_repeatable():
    """Restore() + Execute() twice gives identical results (determinism)."""
    w = h = 128
    psf, dirty = problem(w, h, 10, 2, seed=5)
    s = gpu_settings(w, h, 5e-3, 300, 4)
    run = rd.gpu.DeviceRun(s, psf, dirty, [], 2.0 * PIXEL_SCALE)
    run.execute()
    a = (run.residual(), run.model(), run.trace())
    run.restore()
    run.execute()
    b = (run.residual(), run.model(), run.trace())
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("w,max_iter", [(256, 1500), (4096, 3000)])
def test_multiscale_scale_lanes_identical(w, max_iter, monkeypatch):
    """The scales' inverse transforms + fused peak searches on two session
    lanes (rdl_session_fork/_lane/_join, per-lane four-step scratch at 4096^2,
    per-slot peak partials) give bit-identical traces and images to one lane
    (RDL_SCALE_LANES=1)."""
    h = w
    psf, dirty = problem(w, h, 40, 4, seed=w + 1)
    out = []
    for lanes in ("1", "2"):
        monkeypatch.setenv("RDL_SCALE_LANES", lanes)
        s = gpu_settings(w, h, 1e-3, max_iter, 6)
        run = rd.gpu.DeviceRun(s, psf, dirty, [], 2.0 * PIXEL_SCALE)
        r = run.execute()
        out.append((r["iterations"], run.trace(), run.residual(), run.model()))
    (i1, t1, r1, m1), (i2, t2, r2, m2) = out
    assert i1 == i2 and i1 > 100
    assert np.array_equal(t1, t2)
    assert np.array_equal(r1, r2)
    assert np.array_equal(m1, m2)


JOINED_CASES = [
    # w, n_channels, weights, max_scales, fast
    (128, 2, None, 4, True),
    (160, 3, [1.0, 0.5, 2.0], 4, True),
    (128, 4, [1.0, 1.0, 0.0, 1.0], 3, True),   # zero-weight channel is skipped
    (96, 2, None, 3, False),
]


@pytest.mark.parametrize("w,n_ch,weights,max_scales,fast", JOINED_CASES)
def test_multiscale_joined_channels_parity(w, n_ch, weights, max_scales, fast):
    """Joined-channel multiscale (ImageSet with n channels, linear
    integration with weights, per-channel PSFs): exact component trace,
    per-channel residual/model within 2e-5 * max|dirty|."""
    h = w
    psf, dirty = problem(w, h, 12, 3, seed=w + n_ch)
    rng = np.random.default_rng(n_ch)
    dirties = np.stack([dirty * np.float32(1.0 + 0.2 * k) +
                        np.float32(1e-3) * rng.standard_normal((h, w)).astype(np.float32)
                        for k in range(n_ch)]).astype(np.float32)
    psfs = np.stack([psf] * n_ch)
    wts = np.ones(n_ch) if weights is None else np.asarray(weights, np.float64)
    thr, max_iter = 8e-3, 600
    orc = get_oracle()
    orc.set_threads(8)
    res_o, mod_o = dirties.copy(), np.zeros_like(dirties)
    psfs_o = psfs.copy()
    # ImageSet::LoadAndAverage / LoadAndAveragePsfs (cpp/image_set.cc:105-207):
    # a channel whose weights sum to zero loads as 0 * (1/0) = NaN and its PSF
    # as zero
    for k in np.nonzero(wts == 0.0)[0]:
        res_o[k] = np.nan
        psfs_o[k] = 0.0
    alg = OracleAlgorithm(orc, 1, threshold=thr, max_iterations=max_iter, border_ratio=0.0,
                          max_scales=max_scales, beam_size_in_pixels=2.0,
                          fast_sub_minor_loop=int(fast))
    r_o, trace_o = alg.execute(res_o, mod_o, psfs_o, weights=wts.astype(np.float32))
    s = gpu_settings(w, h, thr, max_iter, max_scales, fast)
    run = rd.gpu.DeviceRun(s, psfs, dirties, list(wts), 2.0 * PIXEL_SCALE)
    r_g = run.execute()
    assert r_g["iterations"] == r_o.iteration_number
    trace_g = run.trace()
    assert np.array_equal(trace_g, trace_o)
    tol = 2e-5 * np.abs(dirties).max()
    np.testing.assert_allclose(run.residual().reshape(n_ch, h, w), res_o, atol=tol)  # NaN == NaN
    np.testing.assert_allclose(run.model().reshape(n_ch, h, w), mod_o, atol=tol)


def test_multiscale_more_than_eight_scales_on_tiled_plan():
    """A ladder of 10 non-zero scales on a four-step (tiled) plan: 1280^2 with
    a 0.25-pixel beam gives scales 0, 1, 2, 4, ..., 512
    (multiscale_algorithm.cc:97-113). The fused scale convolutions take at most
    8 scales per launch (rdl_conv_scales), so the ladder runs in two chunks of
    one forward half; the trace must equal the oracle's."""
    w = h = 1280
    beam_px, thr, max_iter = 0.25, 2e-2, 60
    psf, dirty = problem(w, h, 30, 6, seed=1280)
    orc = get_oracle()
    orc.set_threads(8)
    res_o, mod_o = dirty[None].copy(), np.zeros((1, h, w), np.float32)
    alg = OracleAlgorithm(orc, 1, threshold=thr, max_iterations=max_iter, border_ratio=0.0,
                          max_scales=0, beam_size_in_pixels=beam_px)
    r_o, trace_o = alg.execute(res_o, mod_o, psf[None])
    s = gpu_settings(w, h, thr, max_iter, 0)
    run = rd.gpu.DeviceRun(s, psf, dirty, [], beam_px * PIXEL_SCALE)
    r_g = run.execute()
    trace_g = run.trace()
    # (every scale is active in the first search: 10 convolutions in one call)
    assert r_g["iterations"] == r_o.iteration_number
    if not np.array_equal(trace_g, trace_o):
        first = int(np.argmax(np.any(trace_g != trace_o, axis=1)))
        pytest.fail(f"component trace differs first at {first}: gpu {trace_g[first]} "
                    f"oracle {trace_o[first]}")
    tol = 2e-5 * np.abs(dirty).max()
    np.testing.assert_allclose(run.residual().reshape(h, w), res_o[0], atol=tol)
