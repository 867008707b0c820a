"""End-to-end Radler.perform() on the MI355X, restated from the reference's
python/test/test_radler.py and cpp/test/test_radler.cc: a point source (x2.5)
convolved with a 5-pixel PSF must leave |residual| < 2e-6 and the model 2.5 at
the source (atol 2e-6), for generic clean (Clark sub-minor and Högbom) and
multiscale."""
import numpy as np
import pytest

from radler_fixtures import (BEAM_SIZE, HEIGHT, MINOR_ITERATION_COUNT, WIDTH, expected_model,
                             get_psf, get_residual, make_settings)
from radler_import import radler as rd

pytestmark = pytest.mark.gpu

ALGORITHMS = [rd.AlgorithmType.generic_clean, rd.AlgorithmType.multiscale]


@pytest.fixture
def settings():
    return make_settings()


def perform(r, minor_iteration_count=MINOR_ITERATION_COUNT):
    reached = r.perform(0)
    assert reached is False
    assert r.iteration_number <= minor_iteration_count


@pytest.mark.parametrize("algorithm", ALGORITHMS)
@pytest.mark.parametrize("shift", [(0, 0), (-9, 15), (7, -11)])
def test_point_source(settings, algorithm, shift):
    settings.algorithm_type = algorithm
    psf, residual = get_psf(), get_residual(2.5, *shift)
    model = np.zeros_like(residual)
    r = rd.Radler(settings, psf, residual, model, BEAM_SIZE, rd.Polarization.stokes_i)
    perform(r)
    np.testing.assert_allclose(residual, 0.0, atol=2e-6)
    np.testing.assert_allclose(model, expected_model(2.5, *shift), atol=2e-6)


@pytest.mark.parametrize("shift", [(0, 0), (-9, 15)])
def test_point_source_hogbom(settings, shift):
    settings.generic.use_sub_minor_optimization = False
    psf, residual = get_psf(), get_residual(2.5, *shift)
    model = np.zeros_like(residual)
    r = rd.Radler(settings, psf, residual, model, BEAM_SIZE)
    perform(r)
    np.testing.assert_allclose(residual, 0.0, atol=2e-6)
    np.testing.assert_allclose(model, expected_model(2.5, *shift), atol=2e-6)


@pytest.mark.parametrize("algorithm", ALGORITHMS)
def test_one_entry_worktable(settings, algorithm):
    settings.algorithm_type = algorithm
    psf, residual = get_psf(), get_residual(2.5, -9, 15)
    model = np.zeros_like(residual)
    e = rd.WorkTableEntry()
    e.psfs.append(psf)
    e.residual = residual
    e.model = model
    e.original_channel_index = 0
    e.image_weight = 1.0
    t = rd.WorkTable([], 1, 1)
    t.add_entry(e)
    r = rd.Radler(settings, t, BEAM_SIZE)
    perform(r)
    np.testing.assert_allclose(residual, 0.0, atol=2e-6)
    np.testing.assert_allclose(model, expected_model(2.5, -9, 15), atol=2e-6)


@pytest.mark.parametrize("algorithm", ALGORITHMS)
def test_ndeconvolution_is_noriginal(settings, algorithm):
    settings.algorithm_type = algorithm
    scales, shifts = [2.5, 4.0], [(0, 0), (-9, 23)]
    psf = get_psf()
    residuals = [get_residual(scales[i], *shifts[i]) for i in range(2)]
    models = [np.zeros_like(residuals[0]) for _ in range(2)]
    t = rd.WorkTable([], 2, 2)
    for i in range(2):
        e = rd.WorkTableEntry()
        e.psfs.append(psf)
        e.residual = residuals[i]
        e.model = models[i]
        e.original_channel_index = i
        e.index = i
        e.image_weight = 1.0
        t.add_entry(e)
    r = rd.Radler(settings, t, BEAM_SIZE)
    perform(r)
    for i in range(2):
        np.testing.assert_allclose(residuals[i], 0.0, atol=2e-6)
        np.testing.assert_allclose(models[i], expected_model(scales[i], *shifts[i]), atol=2e-6)


@pytest.mark.parametrize("algorithm", ALGORITHMS)
def test_image_cube_non_joined(settings, algorithm):
    settings.algorithm_type = algorithm
    scales, shifts = [2.5, 4.0], [(0, 0), (-9, 23)]
    psfs = np.resize(get_psf(), (2, HEIGHT, WIDTH))
    residuals = np.array([get_residual(scales[i], *shifts[i]) for i in range(2)])
    models = np.zeros_like(residuals)
    r = rd.Radler(settings, psfs, residuals, models, BEAM_SIZE)
    perform(r)
    for i in range(2):
        np.testing.assert_allclose(residuals[i], 0.0, atol=2e-6)
        np.testing.assert_allclose(models[i], expected_model(scales[i], *shifts[i]), atol=2e-6)


def test_component_count_generic(settings):
    """python/test/test_radler.py:286-305 (component list part): a flat residual
    takes the maximum number of iterations, each on a distinct pixel."""
    settings.minor_iteration_count = 42
    psf = get_psf()
    residual = np.ones((HEIGHT, WIDTH), np.float32)
    model = np.zeros_like(residual)
    r = rd.Radler(settings, psf, residual, model, BEAM_SIZE)
    perform(r, 42)
    cl = r.component_list
    assert cl.n_scales == 1
    assert cl.component_count(0) == 42
