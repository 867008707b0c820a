"""radler.Settings layout and defaults, restated from the reference's
python/test/test_settings.py (cpp/settings.h:132-534 defaults)."""
import multiprocessing
import re

from radler_import import radler as rd


def test_layout():
    settings = rd.Settings()
    nested = set(filter(lambda x: re.match("^[A-Z]{1}", x), dir(settings)))
    assert nested == {"Generic", "LocalRms", "MoreSane", "Multiscale", "Parallel",
                      "PixelScale", "Python", "SpectralFitting"}
    properties = set(filter(lambda x: re.match("^[a-z]+", x), dir(settings)))
    assert len(properties) == 35


def test_default():
    s = rd.Settings()
    assert s.trimmed_image_width == 0 and s.trimmed_image_height == 0
    assert s.channels_out == 1
    assert s.pixel_scale.x == 0 and s.pixel_scale.y == 0.0
    assert s.prefix_name == "wsclean"
    assert s.thread_count == multiprocessing.cpu_count()
    assert s.linked_polarizations == set()
    assert s.parallel.grid_width == 1 and s.parallel.grid_height == 1
    assert s.parallel.max_threads > 0
    assert s.absolute_threshold == 0.0
    assert s.minor_loop_gain == 0.1
    assert s.major_loop_gain == 1.0
    assert s.auto_threshold_sigma is None and s.auto_mask_sigma is None
    assert s.save_source_list is False
    assert s.minor_iteration_count == 0
    assert s.major_iteration_count == 12
    assert s.divergence_limit == 4.0
    assert s.allow_negative_components is True
    assert s.stop_on_negative_components is False
    assert s.squared_joins is False
    assert s.spectral_correction_frequency == 0.0
    assert s.spectral_correction == []
    assert s.border_ratio == 0.0
    assert s.fits_mask == "" and s.casa_mask == ""
    assert s.horizon_mask_distance is None and s.horizon_mask_filename == ""
    assert s.local_rms.method == rd.LocalRmsMethod.none
    assert s.local_rms.window == 25.0 and s.local_rms.image == ""
    assert s.spectral_fitting.mode == rd.SpectralFittingMode.no_fitting
    assert s.spectral_fitting.terms == 0 and s.spectral_fitting.forced_filename == ""
    assert s.algorithm_type == rd.AlgorithmType.generic_clean
    assert s.python.filename == ""
    assert s.more_sane.location == "" and s.more_sane.arguments == ""
    assert s.more_sane.sigma_levels == []
    assert s.multiscale.fast_sub_minor_loop is True
    assert s.multiscale.sub_minor_loop_gain == 0.2
    assert s.multiscale.scale_bias == 0.6
    assert s.multiscale.max_scales == 0
    assert s.multiscale.convolution_padding == 1.1
    assert s.multiscale.scale_list == []
    assert s.multiscale.shape == rd.MultiscaleShape.tapered_quadratic
    assert s.generic.use_sub_minor_optimization is True


def test_readwrite():
    s = rd.Settings()
    s.trimmed_image_width, s.trimmed_image_height = 200, 300
    assert (s.trimmed_image_width, s.trimmed_image_height) == (200, 300)
    s.algorithm_type = rd.AlgorithmType.multiscale
    assert s.algorithm_type == rd.AlgorithmType.multiscale
    linked = {rd.Polarization.stokes_i, rd.Polarization.stokes_q, rd.Polarization.xy}
    s.linked_polarizations = linked
    assert s.linked_polarizations == linked
    s.spectral_correction.append(20.0)   # value semantics: a copy is changed
    assert s.spectral_correction == []
    s.spectral_correction = [20.0]
    assert s.spectral_correction == [20.0]
    s.multiscale.sub_minor_loop_gain = 20.0
    assert s.multiscale.sub_minor_loop_gain == 20.0
