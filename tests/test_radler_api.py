"""Constructor contract of radler.Radler (python/pyradler.cc:23-208 checks,
cpp/radler.cc:52-112). No device is opened until perform(), so these run on
the CPU suite. Cases restated from the reference's python/test/test_radler.py."""
import numpy as np
import pytest

from radler_fixtures import BEAM_SIZE, HEIGHT, WIDTH, get_psf, get_residual, make_settings
from radler_import import radler as rd


@pytest.fixture
def settings():
    return make_settings()


def test_num_threads(settings):
    psf, residual = get_psf(), get_residual(1.0, 0, 0)
    model = np.zeros_like(residual)
    settings.thread_count = 0
    with pytest.raises(RuntimeError):
        rd.Radler(settings, psf, residual, model, BEAM_SIZE)
    settings.thread_count = 1
    rd.Radler(settings, psf, residual, model, BEAM_SIZE)


def test_input_dtype(settings):
    psf, residual = get_psf(), get_residual(1.0, 0, 0)
    model = np.zeros_like(residual)
    with pytest.raises(TypeError):
        rd.Radler(settings, psf.astype(np.float64), residual, model, BEAM_SIZE)
    with pytest.raises(TypeError):
        rd.Radler(settings, psf, residual.astype(np.float16), model, BEAM_SIZE)
    with pytest.raises(TypeError):
        rd.Radler(settings, psf, residual, model.astype(int), BEAM_SIZE)
    rd.Radler(settings, psf, residual, model, BEAM_SIZE)


def test_matching_arrays(settings):
    valid = np.zeros((3, HEIGHT, WIDTH), np.float32)
    rd.Radler(settings, valid, valid, valid, BEAM_SIZE,
              frequencies=np.zeros((3, 2)), weights=np.zeros(3))
    one_d = np.zeros(42, np.float32)
    with pytest.raises(RuntimeError):
        rd.Radler(settings, one_d, one_d, one_d, BEAM_SIZE)
    with pytest.raises(RuntimeError):
        rd.Radler(settings, valid, valid, valid, BEAM_SIZE, frequencies=np.zeros(5))
    with pytest.raises(RuntimeError):
        rd.Radler(settings, valid, valid, valid, BEAM_SIZE, weights=np.zeros((3, 3)))
    bad = np.zeros((3, WIDTH + 42, HEIGHT + 42), np.float32)
    for args in ((valid, valid, bad), (valid, bad, valid), (bad, valid, valid)):
        with pytest.raises(RuntimeError):
            rd.Radler(settings, *args, BEAM_SIZE)
    with pytest.raises(RuntimeError):
        rd.Radler(settings, bad, valid, valid, BEAM_SIZE, frequencies=np.zeros((42, 2)))
    with pytest.raises(RuntimeError):
        rd.Radler(settings, bad, valid, valid, BEAM_SIZE, weights=np.zeros(42))


def test_require_frequencies(settings):
    image = np.zeros((HEIGHT, WIDTH), np.float32)
    settings.spectral_fitting.mode = rd.SpectralFittingMode.polynomial
    with pytest.raises(RuntimeError):
        rd.Radler(settings, image, image, image, BEAM_SIZE)


def test_default_args(settings):
    psf, residual = get_psf(), get_residual(1.0, 0, 0)
    rd.Radler(settings, psf, residual, np.zeros_like(residual), BEAM_SIZE)


def test_grid_must_be_positive(settings):
    """cpp/radler.cc:102-112"""
    psf, residual = get_psf(), get_residual(1.0, 0, 0)
    for attr in ("grid_width", "grid_height", "max_threads"):
        s = make_settings()
        setattr(s.parallel, attr, 0)
        with pytest.raises(RuntimeError):
            rd.Radler(s, psf, residual, np.zeros_like(residual), BEAM_SIZE)


def test_work_table_without_entries_is_nothing_to_clean(settings):
    """cpp/radler.cc:339-341: a table whose groups are empty cannot be cleaned
    (the reference throws on OriginalGroups().empty(); WorkTable always has one
    group, so Perform() is what reports it here)."""
    t = rd.WorkTable([], 1, 1)
    r = rd.Radler(settings, t, BEAM_SIZE)
    assert r is not None
