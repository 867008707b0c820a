"""ParallelDeconvolution tiling.

CPU: the product's host splitter (radler.tiling.make_subimages ->
libradler_amd.so MakeSubImages / DijkstraSplitter) produces exactly the
oracle's subimage geometry (boxes and boundary masks), the masks partition the
image, boxes are even-sized on even images.
GPU: Radler's tiled major iteration (device box transfers + per-subimage
algorithms) matches the oracle's tiled run: same tiles, same per-subimage
component traces, residual/model within 2e-5 * max|dirty|.
"""
import numpy as np
import pytest

from oracle_lib import OracleParallel, get_oracle, make_subimages
from radler_import import radler as rd
from synthetic import problem

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0

GEOMETRY_CASES = [(256, 256, 3, 2, 1), (200, 160, 2, 2, 2), (301, 257, 4, 3, 3),
                  (128, 512, 2, 4, 4), (512, 512, 8, 8, 5), (2048, 1536, 4, 3, 6)]


@pytest.mark.parametrize("w,h,gw,gh,seed", GEOMETRY_CASES)
def test_splitter_matches_oracle(w, h, gw, gh, seed):
    _, dirty = problem(w, h, 30, 3, seed=seed)
    boxes_o, labels_o = make_subimages(get_oracle(), dirty, gw, gh)
    boxes, labels = rd.tiling.make_subimages(dirty, gw, gh)
    assert np.array_equal(boxes, boxes_o)
    assert np.array_equal(labels, labels_o)
    # every pixel belongs to exactly one subimage (boundary masks partition)
    assert labels.min() >= 1 and set(np.unique(labels)) == set(range(1, gw * gh + 1))
    for i, (x, y, bw, bh) in enumerate(boxes):
        ys, xs = np.nonzero(labels == i + 1)
        assert xs.min() >= x and xs.max() < x + bw and ys.min() >= y and ys.max() < y + bh
        if w % 2 == 0:
            assert bw % 2 == 0
        if h % 2 == 0:
            assert bh % 2 == 0


def test_splitter_flat_image_is_deterministic():
    """Equal costs everywhere: tie-breaking follows the heap order exactly."""
    img = np.ones((96, 128), np.float32)
    assert all(np.array_equal(a, b) for a, b in
               zip(rd.tiling.make_subimages(img, 3, 3), make_subimages(get_oracle(), img, 3, 3)))


def _divide_counts():
    return np.array(rd.tiling.divide_stats(), np.int64)


@pytest.mark.parametrize("kind", ["noise", "quantized", "fine_quantized", "zeros", "nan",
                                  "blocked"])
def test_splitter_key_order_search_matches_oracle(kind):
    """The dividers come from the key-order search (radix heap) when no tie
    decides the path, from the key-order path completed by a prefix of the
    reference's heap order when ties decide it only below some key, else from
    the reference's heap order; either way the geometry is the oracle's (whose
    search is the reference's heap). Noisy images take the key-order search;
    tie-heavy ones fall back."""
    rng = np.random.default_rng(11)
    _, img = problem(768, 640, 60, 6, seed=12)
    if kind == "quantized":  # few distinct values: equal path costs everywhere
        img = np.round(img / (np.abs(img).max() * 0.05)).astype(np.float32)
    elif kind == "zeros":
        img = img.copy()
        img[:, ::3] = 0.0
        img[100:300] = 0.0
    elif kind == "nan":
        img = img.copy()
        img[rng.integers(0, 640, 50), rng.integers(0, 768, 50)] = np.nan
    elif kind == "fine_quantized":  # a few equal path costs inside the bands
        img = img + rng.normal(0, np.abs(img).max() * 0.01, img.shape).astype(np.float32)
        step = np.abs(img).max() * 1e-4
        img = (np.round(img / step) * step).astype(np.float32)
    elif kind == "blocked":  # no divider can cross: every search drains its queue
        img = img.copy()
        img[200, :] = np.nan
        img[:, 500] = np.inf
    before = _divide_counts()
    boxes, labels = rd.tiling.make_subimages(img, 4, 3)
    used = _divide_counts() - before
    assert used.sum() == (4 - 1) + (3 - 1)
    boxes_o, labels_o = make_subimages(get_oracle(), img, 4, 3)
    assert np.array_equal(boxes, boxes_o)
    assert np.array_equal(labels, labels_o)
    if kind in ("noise", "nan"):
        assert used[0] == used.sum()  # no tie on any divider
    if kind == "quantized":
        assert used[1] > 0
    if kind == "fine_quantized":  # key-order paths completed from an exact prefix
        assert used[2] > 0


def _settings(kind, w, thr, max_iter, mgain, gw, gh, threads):
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale if kind == 1 else rd.AlgorithmType.generic_clean
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = max_iter
    s.absolute_threshold = thr
    s.border_ratio = 0.0
    s.major_loop_gain = mgain
    s.parallel.grid_width, s.parallel.grid_height = gw, gh
    s.parallel.max_threads = threads
    if kind == 1:
        s.multiscale.max_scales = 4
    return s


def _check_tiled(kind, w, gw, gh, threads, majors=1, staging=False, monkeypatch=None):
    h = w
    psf, dirty = problem(w, h, 40, 4, seed=w + gw)
    thr, max_iter, mgain = 4e-3, 1500, 0.9 if majors == 1 else 0.5
    orc = get_oracle()
    orc.set_threads(8)
    st = dict(threshold=thr, max_iterations=max_iter, border_ratio=0.0,
              major_loop_gain=mgain)
    if kind == 1:
        st.update(max_scales=4, beam_size_in_pixels=2.0)
    par = OracleParallel(orc, kind, gw, gh, **st)
    par.set_snapshot(threads > 1)
    res_o, mod_o = dirty[None].copy(), np.zeros((1, h, w), np.float32)

    if staging:
        monkeypatch.setenv("RADLER_POOL_STAGING", "1")
    s = _settings(kind, w, thr, max_iter, mgain, gw, gh, threads)
    run = rd.gpu.DeviceRun(s, psf, dirty, [], 2.0 * PIXEL_SCALE if kind == 1 else 0.0)
    iterations = 0
    for major in range(majors):
        r_o, boxes_o, labels_o, trace_o = par.execute(res_o, mod_o, psf[None], mgain)
        r = run.execute()
        boxes, labels = run.subimages(w, h)
        assert np.array_equal(boxes, boxes_o)
        assert np.array_equal(labels, labels_o)
        for i in range(gw * gh):
            t_o = trace_o[trace_o[:, 0] == i][:, 1:]
            t_g = run.trace(i)
            assert np.array_equal(t_g if kind == 1 else t_g[:, :2],
                                  t_o if kind == 1 else t_o[:, :2]), (major, i)
        iterations = r_o.total_iterations
        assert r["iterations"] == iterations - (0 if major == 0 else prev)
        prev = iterations
        assert r["another_iteration_required"] == bool(r_o.another_iteration_required)
        tol = 2e-5 * np.abs(dirty).max()
        assert np.abs(run.residual().reshape(h, w) - res_o[0]).max() <= tol
        assert np.abs(run.model().reshape(h, w) - mod_o[0]).max() <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("kind,w,gw,gh", [(1, 256, 3, 2), (0, 192, 2, 2), (1, 320, 2, 3)])
def test_tiled_run_matches_oracle(kind, w, gw, gh):
    """One worker: subimages in index order (the reference with one thread)."""
    _check_tiled(kind, w, gw, gh, threads=1)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,w,gw,gh,threads", [(1, 256, 3, 2, 6), (0, 192, 2, 2, 2),
                                                  (1, 320, 3, 3, 4), (1, 256, 2, 2, 64)])
def test_concurrent_pool_matches_oracle_snapshot(kind, w, gw, gh, threads):
    """max_threads > 1: subimages run concurrently on worker streams; every
    subimage trims the pass-start residual (oracle snapshot mode)."""
    _check_tiled(kind, w, gw, gh, threads=threads)


@pytest.mark.gpu
def test_concurrent_pool_staging_path(monkeypatch):
    """The staging + peer-copy path of workers on another GPU, forced on one
    device (RADLER_POOL_STAGING=1)."""
    _check_tiled(1, 256, 3, 2, threads=3, staging=True, monkeypatch=monkeypatch)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,w,gw,gh,threads", [(1, 320, 3, 3, 4), (0, 192, 2, 2, 3)])
def test_concurrent_pool_queue(kind, w, gw, gh, threads, monkeypatch):
    """RADLER_POOL_QUEUE=1: workers take subimages from a cost-ordered queue
    instead of the round-robin assignment; the snapshot schedule makes the
    result independent of which worker runs which subimage."""
    monkeypatch.setenv("RADLER_POOL_QUEUE", "1")
    _check_tiled(kind, w, gw, gh, threads=threads, majors=2)


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 4])
def test_tiled_two_major_iterations(threads):
    """The worker pool and per-subimage algorithms persist across major
    iterations (iteration counts and scale state carry over)."""
    _check_tiled(1, 256, 2, 2, threads=threads, majors=2)


@pytest.mark.gpu
def test_joined_pool_assignment_modes_identical(monkeypatch):
    """A joined 4-channel set split 3 x 3 on a 4-worker pool: the subimage
    assignment (RADLER_POOL_QUEUE 0 round robin, 1 cost-ordered queue — the
    default for image sets of several images — and 2 index-order queue) does
    not change the result (snapshot schedule): residual, model and
    iteration count bit-identical over two major iterations."""
    from radler_import import radler as rd
    from config_problems import joined_channels
    pixel = 1.0 / 3600.0 * np.pi / 180.0
    w = 288
    freqs = [100e6 + 10e6 * i for i in range(4)]
    psf, dirty = joined_channels(w, 40, 4, seed=33, frequencies=freqs)
    outs = []
    for mode in ("0", None, "2"):
        if mode is None:
            monkeypatch.delenv("RADLER_POOL_QUEUE", raising=False)
        else:
            monkeypatch.setenv("RADLER_POOL_QUEUE", mode)
        s = rd.Settings()
        s.algorithm_type = rd.AlgorithmType.multiscale
        s.pixel_scale.x = s.pixel_scale.y = pixel
        s.trimmed_image_width = s.trimmed_image_height = w
        s.minor_iteration_count = 3000
        s.absolute_threshold = 2e-3
        s.major_loop_gain = 0.5
        s.border_ratio = 0.0
        s.multiscale.max_scales = 4
        s.parallel.grid_width = s.parallel.grid_height = 3
        s.parallel.max_threads = 4
        res, mod = dirty.copy(), np.zeros_like(dirty)
        r = rd.Radler(s, psf, res, mod, 2.0 * pixel, n_deconvolution_groups=4,
                      frequencies=np.array([[f, f] for f in freqs], np.float64),
                      weights=np.ones(4, np.float64))
        for major in range(2):
            r.perform(major)
        outs.append((res.copy(), mod.copy(), r.iteration_number))
    for o in outs[1:]:
        assert np.array_equal(o[0], outs[0][0])
        assert np.array_equal(o[1], outs[0][1])
        assert o[2] == outs[0][2]
    assert outs[0][2] > 0
