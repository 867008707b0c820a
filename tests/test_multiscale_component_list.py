"""The multiscale component list (save_source_list,
cpp/algorithms/multiscale_algorithm.cc:228-236, 447-448, 502-504;
SubMinorLoop::UpdateComponentList, subminor_loop.cc:230-246;
ParallelDeconvolution::GetComponentList, parallel_deconvolution.cc:184-196,
464-479): per scale, the component positions with their summed values.
Against the oracle's component trace: the same positions per scale; with a
scale-0-only run the values are exactly the model image at those pixels;
gridded runs gather the subimage lists at their offsets.
"""
import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, get_oracle
from synthetic import problem

PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0


def _radler(rd, w, psf, residual, model, fast, scale_list=None, grid=(1, 1)):
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale
    s.trimmed_image_width = s.trimmed_image_height = w
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = 800
    s.absolute_threshold = 5e-3
    s.border_ratio = 0.0
    s.save_source_list = True
    s.parallel.grid_width, s.parallel.grid_height = grid
    s.parallel.max_threads = 1
    s.multiscale.max_scales = 4
    s.multiscale.fast_sub_minor_loop = fast
    if scale_list is not None:
        s.multiscale.scale_list = scale_list
    return rd.Radler(s, psf, residual, model, 2.0 * PIXEL_SCALE)


def _positions(cl):
    out = {}
    for sc in range(cl.n_scales):
        for i in range(cl.component_count(sc)):
            x, y, v = cl.get_component(sc, i)
            out.setdefault(sc, {})[(x, y)] = v
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("fast", [True, False])
def test_component_list_positions_match_oracle_trace(fast):
    from radler_import import radler as rd
    w = 128
    psf, dirty = problem(w, w, 25, 3, seed=8, noise=1e-3)
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = _radler(rd, w, psf, residual, model, fast)
    r.perform(0)
    comps = _positions(r.component_list)
    alg = OracleAlgorithm(get_oracle(), 1, threshold=5e-3, max_iterations=800,
                          border_ratio=0.0, max_scales=4, beam_size_in_pixels=2.0,
                          fast_sub_minor_loop=int(fast))
    res_o, mod_o = dirty[None].copy(), np.zeros((1, w, w), np.float32)
    _, trace = alg.execute(res_o, mod_o, psf[None])
    expected = {}
    for x, y, sc in trace:
        expected.setdefault(int(sc), set()).add((int(x), int(y)))
    assert set(comps) == set(expected)
    for sc in expected:
        # the fast loop lists every selected pixel whose model is non-zero:
        # those are exactly the component positions
        assert set(comps[sc]) == expected[sc], sc
        assert all(np.isfinite(v[0]) and v[0] != 0.0 for v in comps[sc].values())


@pytest.mark.gpu
def test_scale0_component_values_are_the_model():
    from radler_import import radler as rd
    w = 96
    psf, dirty = problem(w, w, 15, 0, seed=2, noise=1e-3)
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = _radler(rd, w, psf, residual, model, True, scale_list=[0.0])
    r.perform(0)
    comps = _positions(r.component_list)
    assert list(comps) == [0]
    m = np.zeros_like(model)
    for (x, y), v in comps[0].items():
        m[y, x] = v[0]
    np.testing.assert_allclose(m, model, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_gridded_component_list_gathers_subimages():
    from radler_import import radler as rd
    w = 128
    psf, dirty = problem(w, w, 25, 0, seed=5, noise=1e-3)
    residual, model = dirty.copy(), np.zeros_like(dirty)
    r = _radler(rd, w, psf, residual, model, True, scale_list=[0.0], grid=(2, 2))
    r.perform(0)
    comps = _positions(r.component_list)
    m = np.zeros_like(model)
    for (x, y), v in comps.get(0, {}).items():
        m[y, x] = v[0]
    assert np.count_nonzero(m) > 10
    np.testing.assert_allclose(m, model, rtol=1e-6, atol=1e-9)
