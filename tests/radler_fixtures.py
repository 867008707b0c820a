"""Synthetic inputs restated from the reference's python/test/test_radler.py
(point source convolved with a 5-pixel PSF) and cpp/test/test_radler.cc."""
import numpy as np

from radler_import import radler as rd

WIDTH = 64
HEIGHT = 64
BEAM_SIZE = 0.0
PIXEL_SCALE = 1.0 / 60.0 * (np.pi / 180.0)
MINOR_ITERATION_COUNT = 1000


def make_settings():
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.generic_clean
    s.trimmed_image_width = WIDTH
    s.trimmed_image_height = HEIGHT
    s.pixel_scale.x = PIXEL_SCALE
    s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = MINOR_ITERATION_COUNT
    s.absolute_threshold = 1e-8
    return s


def point_source():
    return np.array([[0.0, 0.4, 0.0], [0.25, 1.0, 0.5], [0.0, 0.6, 0.0]], np.float32)


def get_psf():
    p = point_source()
    psf = np.zeros((HEIGHT, WIDTH), np.float32)
    oy, ox = HEIGHT // 2 - 1, WIDTH // 2 - 1
    psf[oy:oy + 3, ox:ox + 3] = p
    return psf


def get_residual(scale, shift_x, shift_y):
    p = scale * point_source()
    r = np.zeros((HEIGHT, WIDTH), np.float32)
    oy, ox = HEIGHT // 2 + shift_y - 1, WIDTH // 2 + shift_x - 1
    r[oy:oy + 3, ox:ox + 3] = p
    return r


def expected_model(scale, shift_x, shift_y):
    m = np.zeros((HEIGHT, WIDTH), np.float32)
    m[HEIGHT // 2 + shift_y, WIDTH // 2 + shift_x] = scale
    return m
