"""Component optimisation: math::GradientDescent
(cpp/math/component_optimization.cc:20-177, 265-321) as GenericClean runs it
once the auto-mask is complete (generic_clean.cc:26-48, 89-95;
cpp/radler.cc:180-185): the model's non-zero pixels are re-fitted to the
residual with four line-searched gradient steps through padded (2W x 2H)
FFT convolutions.

CPU: the oracle's PaddedConvolution against numpy's padded FFT convolution,
and the gradient-descent step lowering the residual it fits.
GPU: the device gradient descent against the oracle (the line-search sums
are double on the device, float in pixel order in the reference: values
within 1e-4 x max|model|), Radler.perform with auto-masking and
gradient-descent optimisation against the oracle's Perform, and the
multiscale / linear-solver modes rejected.
"""
import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, get_oracle
from radler_oracle import OraclePerform
from synthetic import problem

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def _padded_conv_numpy(img, psf, pw, ph):
    h, w = img.shape
    a = np.zeros((ph, pw))
    b = np.zeros((ph, pw))
    oy, ox = (ph - h) // 2, (pw - w) // 2
    a[oy:oy + h, ox:ox + w] = img
    b[oy:oy + h, ox:ox + w] = psf
    b = np.roll(b, (-(ph // 2), -(pw // 2)), axis=(0, 1))
    c = np.real(np.fft.ifft2(np.fft.fft2(a) * np.fft.fft2(b)))
    return c[oy:oy + h, ox:ox + w]


def test_oracle_padded_convolution():
    rng = np.random.default_rng(1)
    psf, _ = problem(48, 40, 3, 1, seed=2)
    img = rng.standard_normal((40, 48)).astype(np.float32)
    got = get_oracle().padded_convolution(img, psf, 96, 80)
    np.testing.assert_allclose(got, _padded_conv_numpy(img, psf, 96, 80), atol=1e-5)


def _clean_model(w, seed):
    psf, dirty = problem(w, w, 25, 0, seed=seed, noise=1e-3)
    alg = OracleAlgorithm(get_oracle(), 0, threshold=2e-2, max_iterations=300,
                          border_ratio=0.0)
    res, mod = dirty[None].copy(), np.zeros((1, w, w), np.float32)
    alg.execute(res, mod, psf[None])
    return psf, dirty, res[0], mod[0]


def test_oracle_gradient_descent_lowers_the_residual():
    w = 64
    psf, dirty, res, mod = _clean_model(w, 4)
    assert np.count_nonzero(mod) > 5
    new = get_oracle().gradient_descent(mod, res, psf)
    assert np.array_equal(new != 0, mod != 0) or np.count_nonzero(new) <= np.count_nonzero(mod)
    delta = (new - mod).astype(np.float32)
    after = res - get_oracle().padded_convolution(delta, psf, 2 * w, 2 * w)
    assert np.sqrt(np.mean(after ** 2)) < np.sqrt(np.mean(res ** 2))


@pytest.mark.gpu
@pytest.mark.parametrize("w,seed", [(64, 4), (128, 9), (100, 3)])
def test_gradient_descent_matches_oracle(w, seed):
    from radler_import import radler as rd
    psf, dirty, res, mod = _clean_model(w, seed)
    got = rd.gpu.gradient_descent(mod, res, psf)
    exp = get_oracle().gradient_descent(mod, res, psf)
    assert np.array_equal(got != 0, exp != 0)
    np.testing.assert_allclose(got, exp, atol=1e-4 * np.abs(exp).max())


@pytest.mark.gpu
def test_perform_with_gradient_descent_matches_oracle():
    from radler_import import radler as rd
    w = 128
    psf, dirty = problem(w, w, 30, 0, seed=17, noise=1e-3)
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.generic_clean
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = 3000
    s.minor_loop_gain = 0.1
    s.border_ratio = 0.0
    s.auto_mask_sigma = 6.0
    rd.gpu.set_component_optimization(s, rd.OptimizationAlgorithm.gradient_descent)
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = rd.Radler(s, psf, residual, model, 0.0)
    o = OraclePerform(get_oracle(), 0, psf, dirty, minor_loop_gain=0.1, auto_mask_sigma=6.0,
                      minor_iteration_count=3000, major_iteration_count=20,
                      component_optimization=2, border_ratio=0.0)
    tol = 2e-5 * np.abs(dirty).max()
    for major in range(1, 5):
        another = r.perform(major)
        another_o = o.perform(major)
        assert another == another_o, major
        assert np.abs(residual - o.residual[0]).max() <= tol, major
        assert np.abs(model - o.model[0]).max() <= 1e-4 * np.abs(o.model[0]).max(), major
        if not another:
            break
    assert o.finished


@pytest.mark.gpu
def test_unavailable_optimisations_are_rejected():
    from radler_import import radler as rd
    w = 64
    psf, dirty = problem(w, w, 5, 0, seed=1, noise=1e-3)
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = 100
    s.absolute_threshold = 1e-3
    rd.gpu.set_component_optimization(s, rd.OptimizationAlgorithm.gradient_descent)
    run = rd.gpu.DeviceRun(s, psf, dirty, [], 2.0 * PIXEL_SCALE)
    # multiscale gradient descent fits the component list (save_source_list)
    with pytest.raises(RuntimeError, match="save_source_list"):
        run.execute()


@pytest.mark.gpu
@pytest.mark.parametrize("w,scales", [(96, [0.0, 8.0, 16.0]), (128, [0.0, 8.0])])
def test_ms_full_component_fitter_matches_oracle(w, scales):
    """MultiScaleAlgorithm::RunFullComponentFitter
    (multiscale_algorithm.cc:837-914) with GradientDescentWithVariablePsf
    (component_optimization.cc:323-402): residual and model within 1e-4 x
    their maxima of the oracle's restatement, residual RMS lowered."""
    from radler_import import radler as rd
    psf, dirty = problem(w, w, 20, 3, seed=w, noise=1e-3)
    rng = np.random.default_rng(w)
    lists = []
    model = np.zeros_like(dirty)
    for sc in scales:
        pts = {(int(x), int(y)) for x, y in rng.integers(8, w - 8, (12, 2))}
        lists.append(sorted(pts))
        for x, y in pts:
            model[y, x] += 0.01
    res_g, mod_g = rd.gpu.ms_full_component_fitter(dirty, model, psf, scales, lists)
    res_o, mod_o = get_oracle().ms_full_component_fitter(dirty, model, psf, scales, lists)
    np.testing.assert_allclose(res_g, res_o, atol=1e-4 * np.abs(res_o).max())
    np.testing.assert_allclose(mod_g, mod_o, atol=1e-4 * np.abs(mod_o).max())
    assert np.sqrt(np.mean(res_o ** 2)) < np.sqrt(np.mean(dirty ** 2))
