"""Auto-masking: Radler::Perform's auto-mask state
machine (cpp/radler.cc:162-316) with per-scale masks in the multiscale
algorithm (cpp/algorithms/multiscale_algorithm.cc:214-226, 403-404, 444-445,
586-610, 695-696, 716-720; SubMinorLoop::UpdateAutoMask,
subminor_loop.cc:220-228) and the model's non-zero mask for generic clean.

CPU: the oracle's mask bookkeeping (masks hold exactly the tracked
components' pixels; the use phase only cleans inside them).
GPU: Radler.perform() over successive major iterations against the oracle
driven by the same state machine (tests/radler_oracle.py): same number of
major iterations and minor iterations, residual/model within the multiscale
parity tolerance 2e-5 * max|dirty|; and the reference's auto-mask test
(cpp/test/test_radler.cc:172-230: minor gain 0.8, 300 iterations, sigma 4)
restated on a synthetic field (its MWA data set is not in the container).
"""
import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, get_oracle
from radler_oracle import OraclePerform
from synthetic import problem

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def test_oracle_scale_masks_track_components():
    w = h = 128
    psf, dirty = problem(w, h, 20, 3, seed=5, noise=1e-3)
    orc = get_oracle()
    alg = OracleAlgorithm(orc, 1, threshold=2e-2, max_iterations=400, border_ratio=0.0,
                          max_scales=4, beam_size_in_pixels=2.0)
    alg.set_automask(True, False)
    res, mod = dirty[None].copy(), np.zeros((1, h, w), np.float32)
    r, trace = alg.execute(res, mod, psf[None])
    masks = alg.scale_masks(w, h)
    assert masks.shape[0] >= 3 and r.iteration_number > 20
    for s in range(masks.shape[0]):
        t = trace[trace[:, 2] == s]
        # every component's pixel is in its scale's mask, and nothing else
        # (model values of a pixel never return to exactly zero here)
        assert np.all(masks[s][t[:, 1], t[:, 0]] == 1)
        assert masks[s].sum() == len({(int(x), int(y)) for x, y, _ in t})
    # use phase: every new component lies inside its scale's mask
    alg.set_automask(False, True)
    alg.update(threshold=5e-3, max_iterations=800, border_ratio=0.0, max_scales=4,
               beam_size_in_pixels=2.0)
    r2, trace2 = alg.execute(res, mod, psf[None])
    assert len(trace2) > 0
    for x, y, s in trace2:
        assert masks[s][y, x] == 1


def _radler(rd, kind, psf, residual, model, w, *, gain, minor, sigma, thr=0.0,
            major_count=20, auto_threshold=None, max_scales=4, grid=None, threads=1, mgain=1.0):
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale if kind == 1 else \
        rd.AlgorithmType.generic_clean
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = minor
    s.minor_loop_gain = gain
    s.major_loop_gain = mgain
    s.absolute_threshold = thr
    s.auto_mask_sigma = sigma
    s.major_iteration_count = major_count
    s.border_ratio = 0.0
    if auto_threshold is not None:
        s.auto_threshold_sigma = auto_threshold
    if grid is not None:
        s.parallel.grid_width, s.parallel.grid_height = grid
        s.parallel.max_threads = threads
    if kind == 1:
        s.multiscale.max_scales = max_scales
    return rd.Radler(s, psf, residual, model, 2.0 * PIXEL_SCALE if kind == 1 else 0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,auto_threshold", [(1, None), (1, 1.5), (0, 1.0)])
def test_perform_automask_matches_oracle(kind, auto_threshold):
    from radler_import import radler as rd
    w = h = 256
    psf, dirty = problem(w, h, 40, 4, seed=77, noise=1e-3)
    gain, minor, sigma = 0.1, 3000, 6.0
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = _radler(rd, kind, psf, residual, model, w, gain=gain, minor=minor, sigma=sigma,
                auto_threshold=auto_threshold)
    st = dict(border_ratio=0.0)
    if kind == 1:
        st.update(max_scales=4, beam_size_in_pixels=2.0)
    o = OraclePerform(get_oracle(), kind, psf, dirty, minor_loop_gain=gain,
                      auto_mask_sigma=sigma, auto_threshold_sigma=auto_threshold,
                      minor_iteration_count=minor, major_iteration_count=20, **st)
    tol = 2e-5 * np.abs(dirty).max()
    majors = 0
    for major in range(1, 8):
        another = r.perform(major)
        another_o = o.perform(major)
        majors = major
        assert another == another_o, major
        assert r.iteration_number == o.iteration_number, major
        assert np.abs(residual - o.residual[0]).max() <= tol, major
        assert np.abs(model - o.model[0]).max() <= tol, major
        if not another:
            break
    assert o.finished and majors >= 2  # the auto-mask phase was left


@pytest.mark.gpu
@pytest.mark.parametrize("kind,grid,threads", [(1, (2, 2), 1), (1, (3, 2), 4), (0, (2, 2), 1)])
def test_perform_automask_tiled_matches_oracle(kind, grid, threads):
    """Auto-masking through ParallelDeconvolution: per-subimage scale masks
    cut from / merged into the full-image masks
    (parallel_deconvolution.cc:359-462), the model mask handed to the
    subimage split for generic clean; one worker (subimages in index order)
    and the concurrent pool (snapshot semantics)."""
    from radler_import import radler as rd
    w = h = 256
    psf, dirty = problem(w, h, 40, 4, seed=91, noise=1e-3)
    gain, minor, sigma, mgain = 0.1, 3000, 6.0, 0.8
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = _radler(rd, kind, psf, residual, model, w, gain=gain, minor=minor, sigma=sigma,
                grid=grid, threads=threads, mgain=mgain)
    st = dict(border_ratio=0.0)
    if kind == 1:
        st.update(max_scales=4, beam_size_in_pixels=2.0)
    orc = get_oracle()
    orc.set_threads(8)
    o = OraclePerform(orc, kind, psf, dirty, minor_loop_gain=gain, major_loop_gain=mgain,
                      auto_mask_sigma=sigma, minor_iteration_count=minor,
                      major_iteration_count=20, grid=grid, snapshot=threads > 1, **st)
    tol = 2e-5 * np.abs(dirty).max()
    majors = 0
    for major in range(1, 8):
        another = r.perform(major)
        another_o = o.perform(major)
        majors = major
        assert another == another_o, major
        assert r.iteration_number == o.iteration_number, major
        assert np.abs(residual - o.residual[0]).max() <= tol, major
        assert np.abs(model - o.model[0]).max() <= tol, major
        if not another:
            break
    assert o.finished and majors >= 2


@pytest.mark.gpu
def test_reference_automask_case_synthetic():
    """cpp/test/test_radler.cc:172-230 on a synthetic field: multiscale,
    minor gain 0.8, 300 minor iterations, auto-mask sigma 4, threshold 1e-8:
    100 <= iterations <= 300, residual RMS < 0.75 x dirty RMS, max < 0.1 x
    dirty max."""
    from radler_import import radler as rd
    w = h = 512
    # many extended blobs: a diffuse field like the test's Vela image
    psf, dirty = problem(w, h, 20, 60, seed=3, noise=1e-3)
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = _radler(rd, 1, psf, residual, model, w, gain=0.8, minor=300, sigma=4.0, thr=1e-8,
                major_count=30, max_scales=0)
    r.perform(0)
    assert 100 <= r.iteration_number <= 300
    rms = lambda a: float(np.sqrt(np.mean(a.astype(np.float64) ** 2)))  # noqa: E731
    assert rms(residual) < 0.75 * rms(dirty)
    assert residual.max() < 0.1 * dirty.max()
