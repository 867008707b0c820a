"""Pin the CPU restatement (oracle/) before trusting it.

* peak finder: the 13 known-answer cases of cpp/math/test/test_peak_finder.cc:48-185
* PSF subtract: bit-exact against the reference's own cpp/algorithms/simple_clean.cc
  compiled where it lies (oracle/_ref, built by oracle/Makefile)
* FFT sizes: cpp/utils/test/test_fft_size_calculations.cc KATs + the compiled header
* convolution: against numpy float64 FFT (schaapcommon::math::Convolve is absent:
  its contract is restated from call sites, see oracle/fft.h)
* end-to-end: cpp/test/test_radler.cc:106-172 point-source cases at algorithm level
"""
import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, get_oracle, get_ref


@pytest.fixture(scope="module")
def orc():
    return get_oracle()


# ---------------------------------------------------------------- peak finder
# (pixel values, width, height, expected x, y) from test_peak_finder.cc
PEAK_KATS = [
    ({0: 1}, 4, 2, 0, 0),
    ({0: 1, 1: 2}, 4, 2, 1, 0),
    ({0: 1, 1: 2, 4: 3}, 4, 2, 0, 1),
    ({0: 1, 1: 2, 4: 3, 7: 4}, 4, 2, 3, 1),
    ({0: 1, 1: 2, 4: 3, 7: 4, 15: 6}, 4, 4, 3, 3),
    ({0: 1, 1: 2, 4: 3, 7: 4, 15: 6, 14: 5}, 3, 5, 2, 4),
    ({0: 1}, 6, 6, 0, 0),
    ({0: 1, 1: 2}, 6, 6, 1, 0),
    ({0: 1, 1: 2, 6: 3}, 6, 6, 0, 1),
    ({0: 1, 1: 2, 6: 3, 9: 4}, 6, 6, 3, 1),
    ({0: 1, 1: 2, 6: 3, 9: 4, 35: 6}, 6, 6, 5, 5),
    ({0: 1, 1: 2, 6: 3, 9: 4, 35: 6}, 2, 18, 1, 17),
    ({0: 1, 1: 2, 6: 3, 9: 4, 35: 6, 37: 7}, 6, 6, 5, 5),
]


@pytest.mark.parametrize("vals,w,h,ex,ey", PEAK_KATS)
def test_peak_finder_kat(orc, vals, w, h, ex, ey):
    buf = np.zeros(max(w * h, 38), np.float32)
    for k, v in vals.items():
        buf[k] = v
    img = buf[: w * h].reshape(h, w)
    has, x, y, _ = orc.find_peak(img, True, 0, h)
    assert has and (x, y) == (ex, ey)


def test_peak_finder_semantics(orc):
    img = np.zeros((8, 8), np.float32)
    # nothing above FLT_MIN: AVX variant returns (0,0)/image[0], Simple returns none
    has, x, y, v = orc.find_peak(img)
    assert has and (x, y, v) == (0, 0, 0.0)
    has, *_ = orc.find_peak(img, simple=True)
    assert not has
    # ties -> first row-major index; sign kept; NaN never wins
    img[2, 5] = -3.0
    img[4, 1] = 3.0
    img[1, 1] = np.nan
    has, x, y, v = orc.find_peak(img, allow_negative=True)
    assert (x, y, v) == (5, 2, -3.0)
    has, x, y, v = orc.find_peak(img, allow_negative=False)
    assert (x, y, v) == (1, 4, 3.0)
    # border and mask
    has, x, y, v = orc.find_peak(img, hb=2, vb=3)
    assert (x, y) == (2, 4) or v == 0.0
    mask = np.zeros((8, 8), bool)
    mask[4, 1] = True
    has, x, y, v = orc.find_peak(img, mask=mask)
    assert has and (x, y, v) == (1, 4, 3.0)
    has, *_ = orc.find_peak(np.zeros((8, 8), np.float32), mask=mask)
    assert not has


# ---------------------------------------------------------------- subtract
@pytest.mark.parametrize("w,h", [(64, 64), (63, 65), (128, 96), (17, 31)])
def test_subtract_matches_reference_build(orc, w, h):
    ref = get_ref()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(42)
    for trial in range(20):
        img = rng.standard_normal((h, w)).astype(np.float32)
        psf = rng.standard_normal((h, w)).astype(np.float32)
        x, y = int(rng.integers(0, w)), int(rng.integers(0, h))
        f = np.float32(rng.standard_normal())
        a, b = img.copy(), img.copy()
        s0 = int(rng.integers(0, h))
        s1 = int(rng.integers(s0, h + 1))
        ref.ref_partial_subtract(a, psf, w, h, x, y, f, s0, s1)
        orc.partial_subtract(b, psf, x, y, f, s0, s1)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (trial, x, y)


def test_subtract_fma_contraction_is_what_reference_does(orc):
    """With FMA the result differs from the two-rounding numpy expression on some
    pixels; the reference build (GCC -O3 AVX2/FMA) agrees with the fma oracle."""
    ref = get_ref()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(7)
    w = h = 256
    img = rng.standard_normal((h, w)).astype(np.float32)
    psf = rng.standard_normal((h, w)).astype(np.float32)
    f = np.float32(0.3719)
    a = img.copy()
    ref.ref_partial_subtract(a, psf, w, h, 128, 128, f, 0, h)
    two_round = (img - psf * f).astype(np.float32)
    assert not np.array_equal(a, two_round)


# ---------------------------------------------------------------- fft sizes
def test_fft_size_kats(orc):
    assert orc.good_fft_size(1) == 2
    for i in range(2, 10, 2):
        assert orc.good_fft_size(i) == i
    assert orc.good_fft_size(11) == 12
    assert orc.good_fft_size(15) == 16
    assert orc.good_fft_size(17) == 18
    assert orc.good_fft_size(1000) == 1000
    assert orc.good_fft_size(1152) == 1152
    for i in range(1154, 1177):
        assert orc.good_fft_size(i) == 1176
    assert orc.convolution_size(0.0, 1024, 1.0) == 1024
    assert orc.convolution_size(0.0, 1150, 1.0) == 1152
    assert orc.convolution_size(0.0, 1154, 1.0) == 1176
    assert orc.convolution_size(0.0, 1010, 1.1) == 1120
    assert orc.convolution_size(10.0, 1010, 1.1) == 1134
    # SURVEY.md §8(a) a6 sizes
    assert [orc.convolution_size(s, 4096, 1.1) for s in (0, 16, 32, 64, 128, 256)] == [
        4536, 4536, 4608, 4704, 4800, 5000]


def test_fft_size_matches_reference_build(orc):
    ref = get_ref()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    for n in list(range(1, 3000, 7)) + [4096, 8192, 16384, 4506]:
        assert ref.ref_good_fft_size(n) == orc.good_fft_size(n)
    for s in (0.0, 4.0, 16.0, 100.0, 256.0):
        for n in (64, 1000, 2048, 4096, 8192):
            assert ref.ref_convolution_size(s, n, 1.1) == orc.convolution_size(s, n, 1.1)


# ---------------------------------------------------------------- convolution
@pytest.mark.parametrize("w,h", [(64, 64), (48, 30), (94, 94), (1128 // 8, 47)])
def test_convolution_matches_numpy(orc, w, h):
    rng = np.random.default_rng(3)
    img = rng.standard_normal((h, w)).astype(np.float32)
    ker = rng.standard_normal((h, w)).astype(np.float32)
    expect = np.real(np.fft.ifft2(np.fft.fft2(img.astype(np.float64)) *
                                  np.fft.fft2(ker.astype(np.float64))))
    out = img.copy()
    orc.convolve(out, ker)
    np.testing.assert_allclose(out, expect, rtol=0, atol=1e-5 * np.abs(expect).max())


def test_shape_functions(orc):
    for s in (4.0, 16.0, 33.0, 256.0):
        k = orc.shape_function(s, 1024, 0)
        assert k.shape[0] == 2 * int(np.ceil(s / 2)) + 1
        assert abs(k.sum() - 1.0) < 1e-5
        assert np.argmax(k) == k.size // 2
    k = orc.shape_function(16.0, 1024, 1)  # gaussian: 12 sigma box, sigma=3s/16
    assert k.shape[0] == int(np.ceil(3.0 * 12 / 2)) * 2 + 1
    assert abs(k.sum() - 1.0) < 1e-5
    assert orc.shape_function(0.0, 64, 0).shape == (1, 1)


# ---------------------------------------------------------------- point sources
W = H = 64


def fill_psf_residual(factor, sx=0, sy=0):
    """cpp/test/test_radler.cc:54-82"""
    psf = np.zeros((H, W), np.float32)
    res = np.zeros((H, W), np.float32)
    c = (H // 2, W // 2)
    for img, (cy, cx), f in ((psf, c, 1.0), (res, (c[0] + sy, c[1] + sx), factor)):
        img[cy, cx] = 1.0 * f
        img[cy, cx - 1] = 0.25 * f
        img[cy, cx + 1] = 0.5 * f
        img[cy - 1, cx] = 0.4 * f
        img[cy + 1, cx] = 0.6 * f
    return psf, res


@pytest.mark.parametrize("kind,use_sub_minor", [(0, False), (0, True), (1, True)])
@pytest.mark.parametrize("shift", [(0, 0), (7, -11)])
def test_point_source(orc, kind, use_sub_minor, shift):
    psf, res = fill_psf_residual(2.5, *shift)
    residual = res[None].copy()
    model = np.zeros_like(residual)
    alg = OracleAlgorithm(orc, kind, threshold=1e-8, max_iterations=1000,
                          border_ratio=0.0, use_sub_minor=int(use_sub_minor),
                          beam_size_in_pixels=1.0)
    r, trace = alg.execute(residual, model, psf[None])
    assert np.abs(residual).max() < 2e-6
    cy, cx = H // 2 + shift[1], W // 2 + shift[0]
    assert abs(model[0, cy, cx] - 2.5) < 2.5e-6 * 2.5
    m = model[0].copy()
    m[cy, cx] = 0
    assert np.abs(m).max() < 2e-6
    assert tuple(trace[0, :2]) == (cx, cy)
