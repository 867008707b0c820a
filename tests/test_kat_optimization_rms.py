"""The reference's known-answer tests for component optimisation
(cpp/math/test/test_component_optimization.cc:12-318), the RMS factor image
(cpp/math/test/test_rms_image.cc:13-53) and the FFT sizes
(tests/golden/ref_fft_sizes.json, made by the reference's own
fft_size_calculations.h compiled in oracle/_ref), restated:

* on the CPU against the oracle (oracle/component_optimization.cc,
  oracle/rms_image.cc) and, for the sizes, against the product's
  csrc/host/fft_sizes.h (radler.utils, host code);
* on the GPU against the product (radler.gpu: the device GradientDescent /
  GradientDescentWithVariablePsf with padded FFT convolutions, the host
  LinearComponentSolve, the device MakeRmsFactorImage).

The reference runs each gradient-descent case with and without FFT
convolution; the product and the oracle implement the FFT form (the one
GenericClean and MultiScaleAlgorithm call, generic_clean.cc:38-39,
multiscale_algorithm.cc:877-879), so the FFT cases are restated.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

KX = [3, 4, 5, 3, 9]
KY = [7, 7, 7, 8, 9]
FITTED = [3.0, 1.0, -1.0, 9.0, 21.0]
START = [1.0, 2.0, 3.0, 4.0, 5.0]


def gd_problem(complex_psf):
    data = np.zeros((10, 10), np.float32)
    model = np.zeros_like(data)
    for x, y, f, s in zip(KX, KY, FITTED, START):
        data[y, x] = f
        model[y, x] = s
    psf = np.zeros_like(data)
    psf[5, 5] = 2.0
    if complex_psf:
        psf[5, 6] = 0.5
    return model, data, psf


# TestGradientDescentSimple / TestGradientDescentComplex (:12-90)
GD_RANGES = {False: [(1.49, 1.51), (0.49, 0.51), (-0.51, -0.49), (4.49, 4.51), (10.49, 10.51)],
             True: [(1.4, 1.65), (0.0, 1.0), (-1.0, 0.0), (4.0, 4.7), (10.3, 10.7)]}


def check_gradient_descent(result, complex_psf):
    for y in range(10):
        for x in range(10):
            hit = [i for i in range(5) if (KX[i], KY[i]) == (x, y)]
            if hit:
                lo, hi = GD_RANGES[complex_psf][hit[0]]
                assert lo + START[hit[0]] < result[y, x] < hi + START[hit[0]], (x, y)
            else:
                assert abs(result[y, x]) < 1e-6


def variable_psf_single():
    """TestVariablePsfWithSinglePsf (:92-130)."""
    data = np.zeros((10, 10), np.float32)
    for x, y, f in zip(KX, KY, FITTED):
        data[y, x] = f
    psf = np.zeros_like(data)
    psf[5, 5] = 2.0
    psf[5, 6] = 0.5
    components = [[], list(zip(KX, KY))]
    return components, data, [psf * 10.0, psf]


def check_variable_psf_single(deltas):
    assert len(deltas) == 2
    for i in range(5):
        lo, hi = GD_RANGES[True][i]
        assert lo < deltas[1][KY[i], KX[i]] < hi


MX = [3, 4, 7, 3, 9]
MY = [2, 7, 7, 8, 9]
MPSF = [0, 1, 0, 1, 0]


def variable_psf_multi():
    """TestVariablePsfWithMultiPsf (:132-183)."""
    def draw1(img, x, y, v):
        img[y, x] += 2.0 * v

    def draw2(img, x, y, v):
        img[y, x] += v
        if x + 1 < img.shape[1]:
            img[y, x + 1] += v
        if x > 0:
            img[y, x - 1] += v
        if y + 1 < img.shape[0]:
            img[y + 1, x] += v
        if y > 0:
            img[y - 1, x] += v

    data = np.zeros((10, 10), np.float32)
    psf1 = np.zeros_like(data)
    draw1(psf1, 5, 5, 1.0)
    psf2 = np.zeros_like(data)
    draw2(psf2, 5, 5, 1.0)
    components = [[], []]
    for x, y, p, f in zip(MX, MY, MPSF, FITTED):
        components[p].append((x, y))
        (draw1 if p == 0 else draw2)(data, x, y, f)
    return components, data, [psf1, psf2]


def check_variable_psf_multi(deltas):
    assert len(deltas) == 2
    for y in range(10):
        for x in range(10):
            for p in range(2):
                hit = [i for i in range(5) if (MX[i], MY[i], MPSF[i]) == (x, y, p)]
                if hit:
                    assert deltas[p][y, x] == pytest.approx(FITTED[hit[0]], rel=1e-3)
                else:
                    assert abs(deltas[p][y, x]) < 1e-6


# single_fit_simple / multi_fit_simple / multi_fit_with_overlap (:189-284)
def linear_cases():
    cases = []
    data = np.zeros((10, 10), np.float32)
    model = np.zeros_like(data)
    psf = np.zeros_like(data)
    data[7, 3] = 3.0
    model[7, 3] = 1.0
    psf[5, 5] = 1.0
    cases.append(("single_fit_simple", model, data, psf, {(3, 7): 4.0}))
    xs, ys, fit, start = [3, 4, 3, 9], [7, 7, 8, 9], [3.0, 0.0, 9.0, 21.0], [1.0, 2.0, 3.0, 4.0]
    data = np.zeros((10, 10), np.float32)
    model = np.zeros_like(data)
    for x, y, f, s in zip(xs, ys, fit, start):
        data[y, x], model[y, x] = f, s
    psf = np.zeros_like(data)
    psf[5, 5] = 1.0
    cases.append(("multi_fit_simple", model, data, psf,
                  {(x, y): s + f for x, y, f, s in zip(xs, ys, fit, start)}))
    model, data, psf = gd_problem(True)
    expected = [1.5, 0.125, -0.53125, 4.5, 10.5]
    cases.append(("multi_fit_with_overlap", model, data, psf,
                  {(x, y): e + s for x, y, e, s in zip(KX, KY, expected, START)}))
    return cases


def check_linear(result, expected):
    for y in range(10):
        for x in range(10):
            if (x, y) in expected:
                assert result[y, x] == pytest.approx(expected[(x, y)], rel=1e-6)
            else:
                assert abs(result[y, x]) < 1e-6


# make_rms_factor_image (test_rms_image.cc:14-53)
RMS_CASES = [([4.0, 16.0, 9.0], 0.0, [1.0, 1.0, 1.0]),
             ([4.0, 16.0, 9.0], 1.0, [1.0, 0.25, 4.0 / 9.0]),
             ([4.0, 16.0, 9.0], 0.5, [1.0, 0.5, 2.0 / 3.0]),
             ([0.0, 1.0, 16.0], 0.0, [1.0, 1.0, 1.0]),
             ([0.0, 1.0, 16.0], 1.0, [0.0, 0.0, 0.0])]


def check_rms(out, expect):
    for v, e in zip(out, expect):
        assert v == pytest.approx(e, rel=1e-6, abs=0 if e else 1e-12)


# ---- oracle / host (CPU) ---------------------------------------------------

@pytest.mark.parametrize("complex_psf", [False, True])
def test_oracle_gradient_descent_kat(complex_psf):
    from oracle_lib import get_oracle
    model, data, psf = gd_problem(complex_psf)
    check_gradient_descent(get_oracle().gradient_descent(model, data, psf), complex_psf)


def test_oracle_variable_psf_single_kat():
    from oracle_lib import get_oracle
    components, data, psfs = variable_psf_single()
    check_variable_psf_single(get_oracle().gradient_descent_variable_psf(components, data, psfs))


def test_oracle_variable_psf_multi_kat():
    from oracle_lib import get_oracle
    components, data, psfs = variable_psf_multi()
    check_variable_psf_multi(get_oracle().gradient_descent_variable_psf(components, data, psfs))


@pytest.mark.parametrize("case", linear_cases(), ids=lambda c: c[0])
def test_oracle_linear_component_solve_kat(case):
    from oracle_lib import get_oracle
    _name, model, data, psf, expected = case
    check_linear(get_oracle().linear_component_solve(model, data, psf), expected)


@pytest.mark.parametrize("values,strength,expect", RMS_CASES)
def test_oracle_rms_factor_kat(values, strength, expect):
    from oracle_lib import get_oracle
    out, _lowest = get_oracle().make_rms_factor_image(np.float32(values), strength)
    check_rms(out, expect)


def test_product_fft_sizes_match_reference_vectors():
    """csrc/host/fft_sizes.h (the product's) against the sizes the reference's
    own fft_size_calculations.h produced (tests/golden/make_golden.py)."""
    from radler_import import radler as rd
    with open(os.path.join(HERE, "golden", "ref_fft_sizes.json")) as fh:
        sizes = json.load(fh)
    for n, good in sizes["good_fft_size"].items():
        assert rd.utils.calculate_good_fft_size(int(n)) == good, n
    for s, n, p, size in sizes["convolution_size"]:
        assert rd.utils.get_convolution_size(s, n, p) == size, (s, n, p)


# ---- product (GPU) ---------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("complex_psf", [False, True])
def test_gradient_descent_kat(complex_psf):
    from radler_import import radler as rd
    model, data, psf = gd_problem(complex_psf)
    check_gradient_descent(rd.gpu.gradient_descent(model, data, psf), complex_psf)


@pytest.mark.gpu
def test_variable_psf_single_kat():
    from radler_import import radler as rd
    components, data, psfs = variable_psf_single()
    check_variable_psf_single(rd.gpu.gradient_descent_with_variable_psf(components, data, psfs))


@pytest.mark.gpu
def test_variable_psf_multi_kat():
    from radler_import import radler as rd
    components, data, psfs = variable_psf_multi()
    check_variable_psf_multi(rd.gpu.gradient_descent_with_variable_psf(components, data, psfs))


@pytest.mark.gpu
@pytest.mark.parametrize("case", linear_cases(), ids=lambda c: c[0])
def test_linear_component_solve_kat(case):
    from radler_import import radler as rd
    _name, model, data, psf, expected = case
    check_linear(rd.gpu.linear_component_solve(model, data, psf), expected)


@pytest.mark.gpu
@pytest.mark.parametrize("values,strength,expect", RMS_CASES)
def test_rms_factor_kat(values, strength, expect):
    from radler_import import radler as rd
    out, _lowest = rd.gpu.make_rms_factor_image(np.float32(values), strength)
    check_rms(out, expect)
