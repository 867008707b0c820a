"""GPU parity of the C-ABI kernels against the CPU restatement (oracle/).

Bit-exact for peak positions/values, PSF subtraction, integration, the
Högbom loop and the sub-minor loop's component trace and model values; FFT
convolutions within a float tolerance (rocFFT vs the oracle's float64 FFT):
|err| <= 2e-6 * max|x| per convolution (tolerance written in each test).
"""
import ctypes as C

import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, get_oracle
from rdl_lib import (HogbomParams, HogbomResult, RdlError, Session, SubminorParams, SubminorResult,
                     integration)

pytestmark = pytest.mark.gpu

RDL_CONV_ROW_MAJOR, RDL_CONV_COL_MAJOR = 0, 1  # rdl_hip.h


@pytest.fixture(scope="module")
def sess():
    s = Session(0)
    yield s
    s.close()


@pytest.fixture(scope="module")
def orc():
    return get_oracle()


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


# ------------------------------------------------------------------ peak
PEAK_CASES = [
    (64, 64, 0, 0), (63, 65, 3, 2), (1024, 1024, 51, 51), (4096, 17, 0, 1),
    (17, 4096, 2, 100), (2, 18, 0, 0), (1000, 999, 0, 0),
]


@pytest.mark.parametrize("w,h,hb,vb", PEAK_CASES)
@pytest.mark.parametrize("allow_negative", [True, False])
def test_find_peak_random(sess, orc, w, h, hb, vb, allow_negative):
    rng = np.random.default_rng(w * 7 + h)
    img = rng.standard_normal((h, w)).astype(np.float32)
    d = sess.array(img)
    for start_y, end_y in ((0, h), (h // 3, h - h // 4)):
        g = sess.find_peak(d, w, h, allow_negative, start_y, end_y, hb, vb)
        o = orc.find_peak(img, allow_negative, start_y, end_y, hb, vb)
        assert g[:3] == o[:3] and bits(g[3]) == bits(o[3])
    d.free()


def test_find_peak_ties_nan_mask(sess, orc):
    rng = np.random.default_rng(1)
    w, h = 300, 200
    img = rng.integers(-3, 4, (h, w)).astype(np.float32)   # many exact ties
    img[5, 7] = np.nan
    d = sess.array(img)
    mask = (rng.random((h, w)) < 0.3)
    dm = sess.array(mask.astype(np.uint8))
    for an in (True, False):
        assert sess.find_peak(d, w, h, an)[:3] == orc.find_peak(img, an)[:3]
        g = sess.find_peak(d, w, h, an, dmask=dm)
        o = orc.find_peak(img, an, mask=mask)
        assert g[:3] == o[:3]
    # nothing qualifies: Avx returns (0,0)/image[0]; mask/simple return none
    z = np.zeros((h, w), np.float32)
    z[0, 0] = -1e-39   # denormal, <= FLT_MIN: never a peak
    dz = sess.array(z)
    assert sess.find_peak(dz, w, h)[:3] == (True, 0, 0)
    assert sess.find_peak(dz, w, h, avx=False)[0] is False
    assert sess.find_peak(dz, w, h, dmask=dm)[0] is False
    # box degenerates when the border swallows the image
    assert sess.find_peak(d, w, h, True, 0, h, 200, 0)[:3] == orc.find_peak(img, True, 0, h, 200, 0)[:3]
    for x in (d, dm, dz):
        x.free()


# ------------------------------------------------------------------ subtract
@pytest.mark.parametrize("w,h", [(64, 64), (63, 65), (257, 130)])
def test_subtract_bit_exact(sess, orc, w, h):
    rng = np.random.default_rng(5)
    img = rng.standard_normal((h, w)).astype(np.float32)
    psf = rng.standard_normal((h, w)).astype(np.float32)
    d, dp = sess.array(img), sess.array(psf)
    ref = img.copy()
    for x, y in [(0, 0), (w - 1, h - 1), (w // 2, h // 2), (3, h - 2), (w - 5, 1)]:
        f = np.float32(rng.standard_normal())
        sess.rdl.rdl_subtract_psf(sess.h, d.vp, dp.vp, w, h, x, y, C.c_float(f))
        orc.subtract(ref, psf, x, y, f)
    assert np.array_equal(bits(d.get()), bits(ref))
    d.free()
    dp.free()


# ------------------------------------------------------------------ integrate
@pytest.mark.parametrize("n_ch,n_pol,weights,mode", [
    (1, 1, None, 0), (3, 1, [0.5, 0.0, 4.2], 0), (4, 1, [1, 2, 3, 4], 1),
    (2, 2, [0.7, 1.3], 0), (1, 4, None, 1), (3, 2, [1.0, 0.0, 2.0], 1)])
def test_integrate_bit_exact(sess, orc, n_ch, n_pol, weights, mode):
    rng = np.random.default_rng(9)
    n, h, w = n_ch * n_pol, 37, 53
    imgs = rng.standard_normal((n, h, w)).astype(np.float32)
    if weights is not None and 0.0 in weights:
        imgs[weights.index(0.0) * n_pol] = np.nan  # zero-weight channel may be NaN
    pf = 0.5 if n_pol == 2 else 1.0
    g = integration(n_ch, n_pol, weights, pf, mode)
    di, dd = sess.array(imgs), sess.array(shape=(h, w))
    sess.rdl.rdl_integrate(sess.h, C.byref(g), di.vp, C.c_size_t(h * w), dd.vp)
    expect = orc.integrate(imgs, weights, n_pol, pf, square=(mode == 1))
    assert np.array_equal(bits(dd.get()), bits(expect))
    di.free()
    dd.free()


# ------------------------------------------------------------------ FFT
def fft_convolve(sess, img, kernel):
    h, w = img.shape
    f = C.c_void_p()
    sess.rdl.rdl_fft_create(sess.h, w, h, C.byref(f))
    nb = sess.rdl.lib.rdl_fft_spectrum_bytes(f)
    di, dk = sess.array(img), sess.array(kernel)
    spec_k = sess.array(shape=(nb // 4,))
    work = sess.array(shape=(nb // 4,))
    sess.rdl.rdl_fft_forward(f, dk.vp, spec_k.vp)
    sess.rdl.rdl_fft_convolve(f, di.vp, spec_k.vp, work.vp)
    out = di.get()
    for x in (di, dk, spec_k, work):
        x.free()
    sess.rdl.rdl_fft_destroy(f)
    return out


@pytest.mark.parametrize("w,h", [(64, 64), (1128, 96), (94, 47), (512, 512)])
def test_fft_convolve(sess, orc, w, h):
    rng = np.random.default_rng(11)
    img = rng.standard_normal((h, w)).astype(np.float32)
    ker = rng.standard_normal((h, w)).astype(np.float32)
    g = fft_convolve(sess, img, ker)
    o = img.copy()
    orc.convolve(o, ker)
    tol = 2e-6 * np.abs(o).max() * np.sqrt(np.log2(w * h))
    assert np.abs(g - o).max() <= tol


@pytest.mark.parametrize("w,h", [(64, 64), (94, 47), (1128, 96)])
def test_fft64_residual_correction(sess, orc, w, h):
    """rdl_fft64_convolve + rdl_trim_subtract_f64: residual -= float(model (*) psf)
    on a padded plane; against the oracle (float64 FFT, rounded to float), the
    result agrees to float rounding (|err| <= 2 ulp of max(|conv|, |residual|))."""
    rng = np.random.default_rng(21)
    pw, ph = w + 10, h + 6
    psf = rng.standard_normal((h, w)).astype(np.float32)
    model = np.zeros((h, w), np.float32)
    idx = rng.choice(w * h, 40, replace=False)
    model.flat[idx] = rng.standard_normal(40).astype(np.float32)
    residual = rng.standard_normal((h, w)).astype(np.float32)
    f = C.c_void_p()
    sess.rdl.rdl_fft_create_f64(sess.h, pw, ph, C.byref(f))
    nb = sess.rdl.lib.rdl_fft_spectrum_bytes(f)
    assert nb == (pw // 2 + 1) * ph * 16
    dpsf, dres = sess.array(psf), sess.array(residual)
    kern = sess.array(shape=(ph, pw), dtype=np.float64)
    spec, work = sess.array(shape=(nb // 8,), dtype=np.float64), sess.array(shape=(nb // 8,), dtype=np.float64)
    sess.rdl.rdl_prepare_psf_kernel_f64(sess.h, kern.vp, pw, ph, dpsf.vp, w, h)
    sess.rdl.rdl_fft64_forward(f, kern.vp, spec.vp)
    unt = np.zeros((ph, pw), np.float64)
    unt[(ph - h) // 2:(ph - h) // 2 + h, (pw - w) // 2:(pw - w) // 2 + w] = model
    dm = sess.array(unt)
    sess.rdl.rdl_fft64_convolve(f, dm.vp, spec.vp, work.vp)
    sess.rdl.rdl_trim_subtract_f64(sess.h, dres.vp, w, h, dm.vp, pw, ph)
    # oracle: Untrim, PrepareConvolutionKernel, Convolve, Trim, subtract
    k = np.zeros((ph, pw), np.float32)
    k[(ph - h) // 2:(ph - h) // 2 + h, (pw - w) // 2:(pw - w) // 2 + w] = psf
    k = np.roll(k, (-(ph // 2), -(pw // 2)), axis=(0, 1)).copy()
    o = unt.astype(np.float32)
    orc.convolve(o, k)
    trimmed = o[(ph - h) // 2:(ph - h) // 2 + h, (pw - w) // 2:(pw - w) // 2 + w]
    expect = residual - trimmed
    err = np.abs(dres.get() - expect).max()
    assert err <= 2.4e-7 * max(np.abs(trimmed).max(), np.abs(residual).max())
    for x in (dpsf, dres, kern, spec, work, dm):
        x.free()
    sess.rdl.rdl_fft_destroy(f)


CONV_SIZES = [(64, 64), (128, 200), (210, 150), (96, 7), (2, 48), (1134, 96), (8, 1536),
              (2016, 10)]


RDL_CONV_COLUMNS_AUTO, RDL_CONV_COLUMNS_SINGLE, RDL_CONV_COLUMNS_SPLIT = 0, 1, 2


def conv_create(sess, w, h, f64, columns=None):
    c = C.c_void_p()
    if columns is None:
        rc = sess.rdl.lib.rdl_conv_create(sess.h, w, h, int(f64), C.byref(c))
    else:
        rc = sess.rdl.lib.rdl_conv_create_ex(sess.h, w, h, int(f64), columns, C.byref(c))
    return c if rc == 0 else None


def split_ok(h):
    """Column lengths the split passes accept (largest divisor <= sqrt >= 4)."""
    n1 = max(d for d in range(1, int(h ** 0.5) + 1) if h % d == 0)
    return n1 >= 4 and h // n1 >= 4


@pytest.mark.parametrize("w,h", CONV_SIZES)
@pytest.mark.parametrize("f64", [False, True])
@pytest.mark.parametrize("columns", ["single", "split"])
def test_lds_fft_forward(sess, w, h, f64, columns):
    """Full 2-D forward transform vs numpy's float64 rfft2 (same layout and
    normalisation): |err| <= eps_T * 8 * sqrt(log2 N) * sum|x|^(1/2)-scale.
    Both column strategies (one strided pass / split four-step passes)."""
    if columns == "split" and not split_ok(h):
        assert conv_create(sess, w, h, f64, RDL_CONV_COLUMNS_SPLIT) is None
        return
    strategy = RDL_CONV_COLUMNS_SPLIT if columns == "split" else RDL_CONV_COLUMNS_SINGLE
    c = conv_create(sess, w, h, f64, strategy)
    assert c is not None
    assert sess.rdl.lib.rdl_conv_columns_split(c) == (columns == "split")
    rng = np.random.default_rng(w * 31 + h)
    img = rng.standard_normal((h, w)).astype(np.float32)
    nb = sess.rdl.lib.rdl_conv_spectrum_bytes(c)
    assert nb == (w // 2 + 1) * h * (16 if f64 else 8)
    di = sess.array(img)
    spec = sess.array(shape=(h, w // 2 + 1), dtype=np.complex128 if f64 else np.complex64)
    sess.rdl.rdl_conv_forward(c, di.vp, spec.vp)
    got = spec.get()
    ref = np.fft.rfft2(img.astype(np.float64))
    eps = 2.3e-16 if f64 else 1.2e-7
    tol = eps * 8 * np.sqrt(np.log2(w * h)) * np.sqrt(w * h)
    assert np.abs(got - ref).max() <= tol
    di.free()
    spec.free()
    sess.rdl.rdl_conv_destroy(c)


def test_lds_fft_unsupported(sess):
    for w, h in [(94, 47), (11, 64), (64, 22)]:
        assert conv_create(sess, w, h, False) is None
    assert conv_create(sess, 20480 * 2, 8, False) is None
    assert conv_create(sess, 8, 10240 * 2, True) is None


@pytest.mark.parametrize("w,h", [(64, 64), (210, 150), (96, 7), (1134, 96), (40, 2048)])
@pytest.mark.parametrize("f64", [False, True])
@pytest.mark.parametrize("columns", ["single", "split"])
def test_lds_fft_convolutions(sess, orc, w, h, f64, columns):
    """In-place convolution (rows, columns mode 1, rows) and the shared-spectrum
    form (columns mode 2) against the oracle's float64 circular convolution."""
    if columns == "split" and not split_ok(h):
        return
    c = conv_create(sess, w, h, f64,
                    RDL_CONV_COLUMNS_SPLIT if columns == "split" else RDL_CONV_COLUMNS_SINGLE)
    rng = np.random.default_rng(5 + w)
    img = rng.standard_normal((h, w)).astype(np.float32)
    ker = rng.standard_normal((h, w)).astype(np.float32)
    o = img.copy()
    orc.convolve(o, ker)
    cdt = np.complex128 if f64 else np.complex64
    dk, di = sess.array(ker), sess.array(img)
    kspec = sess.array(shape=(h, w // 2 + 1), dtype=cdt)
    work = sess.array(shape=(h, w // 2 + 1), dtype=cdt)
    sspec = sess.array(shape=(h, w // 2 + 1), dtype=cdt)
    out = sess.array(shape=(h, w))
    sess.rdl.rdl_conv_forward(c, dk.vp, kspec.vp)
    norm = 1.0 / (w * h) if f64 else float(np.float32(1.0 / (w * h)))
    sess.rdl.rdl_conv_rows_forward(c, di.vp, w, h, 0, 0, work.vp)
    sess.rdl.rdl_conv_columns(c, work.vp, work.vp, kspec.vp, 1, C.c_double(norm))
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, di.vp, w, h, 0, 0, 0)
    tol = (1e-12 if f64 else 2e-6) * np.abs(o).max() * np.sqrt(np.log2(w * h))
    assert np.abs(di.get() - o).max() <= max(tol, 1.2e-7 * np.abs(o).max())
    di.upload(img)
    sess.rdl.rdl_conv_forward(c, di.vp, sspec.vp)
    sess.rdl.rdl_conv_columns(c, sspec.vp, work.vp, kspec.vp, 2, C.c_double(norm))
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, out.vp, w, h, 0, 0, 0)
    assert np.abs(out.get() - o).max() <= max(tol, 1.2e-7 * np.abs(o).max())
    for x in (dk, di, kspec, work, sspec, out):
        x.free()
    sess.rdl.rdl_conv_destroy(c)


@pytest.mark.parametrize("w,h,pw,ph", [(64, 64, 72, 72), (200, 150, 224, 168), (90, 60, 98, 64)])
@pytest.mark.parametrize("columns", [RDL_CONV_COLUMNS_SINGLE, RDL_CONV_COLUMNS_SPLIT])
def test_lds_fft_correction(sess, orc, w, h, pw, ph, columns):
    """SubMinorLoop::CorrectResidualDirty in one call sequence: model placed at
    the centred offset of the padded plane, x padded PSF spectrum, trimmed and
    subtracted from the residual (float64 transforms): agrees with the oracle
    to float rounding."""
    c = conv_create(sess, pw, ph, True, columns)
    rng = np.random.default_rng(pw)
    psf = rng.standard_normal((h, w)).astype(np.float32)
    model = np.zeros((h, w), np.float32)
    model.flat[rng.choice(w * h, 50, replace=False)] = rng.standard_normal(50).astype(np.float32)
    residual = rng.standard_normal((h, w)).astype(np.float32)
    dpsf, dmod, dres = sess.array(psf), sess.array(model), sess.array(residual)
    kplane = sess.array(shape=(ph, pw))
    kspec = sess.array(shape=(ph, pw // 2 + 1), dtype=np.complex128)
    work = sess.array(shape=(ph, pw // 2 + 1), dtype=np.complex128)
    sess.rdl.rdl_prepare_psf_kernel(sess.h, kplane.vp, pw, ph, dpsf.vp, w, h)
    sess.rdl.rdl_conv_forward(c, kplane.vp, kspec.vp)
    ox, oy = (pw - w) // 2, (ph - h) // 2
    sess.rdl.rdl_conv_rows_forward(c, dmod.vp, w, h, ox, oy, work.vp)
    sess.rdl.rdl_conv_columns(c, work.vp, work.vp, kspec.vp, 1, C.c_double(1.0 / (pw * ph)))
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, dres.vp, w, h, ox, oy, 1)
    k = np.zeros((ph, pw), np.float32)
    k[oy:oy + h, ox:ox + w] = psf
    k = np.roll(k, (-(ph // 2), -(pw // 2)), axis=(0, 1)).copy()
    o = np.zeros((ph, pw), np.float32)
    o[oy:oy + h, ox:ox + w] = model
    orc.convolve(o, k)
    expect = residual - o[oy:oy + h, ox:ox + w]
    err = np.abs(dres.get() - expect).max()
    assert err <= 2.4e-7 * max(np.abs(o).max(), np.abs(residual).max())
    for x in (dpsf, dmod, dres, kplane, kspec, work):
        x.free()
    sess.rdl.rdl_conv_destroy(c)


def test_prepare_kernels(sess, orc):
    w, h, pw, ph = 40, 30, 48, 36
    rng = np.random.default_rng(2)
    psf = rng.standard_normal((h, w)).astype(np.float32)
    dp, dk = sess.array(psf), sess.array(shape=(ph, pw))
    sess.rdl.rdl_prepare_psf_kernel(sess.h, dk.vp, pw, ph, dp.vp, w, h)
    unt = np.zeros((ph, pw), np.float32)
    unt[(ph - h) // 2:(ph - h) // 2 + h, (pw - w) // 2:(pw - w) // 2 + w] = psf
    expect = np.roll(unt, (-(ph // 2), -(pw // 2)), axis=(0, 1))
    assert np.array_equal(dk.get(), expect)
    k = orc.shape_function(8.0, 64, 0)
    n = k.shape[0]
    sess.rdl.rdl_prepare_small_kernel(sess.h, dk.vp, pw, ph, k.ctypes.data_as(C.c_void_p), n)
    full = np.zeros((ph, pw), np.float32)
    full[:n, :n] = k
    assert np.array_equal(dk.get(), np.roll(full, (-(n // 2), -(n // 2)), axis=(0, 1)))
    dp.free()
    dk.free()


@pytest.mark.parametrize("w,h", [(128, 128), (200, 150), (520, 300)])
@pytest.mark.parametrize("scale", [8.0, 16.0, 32.0, 64.0, 128.0])
@pytest.mark.parametrize("shape", [0, 1])
def test_small_kernel_and_shape_component(sess, orc, w, h, scale, shape):
    """Kernels of every multiscale size (n up to 257 -> 264 KiB uploads):
    placement is exact, AddShapeComponent bit-exact vs the oracle."""
    k = orc.shape_function(scale, min(w, h), shape)
    n = k.shape[0]
    if n > min(w, h):
        pytest.skip("kernel larger than image")
    d = sess.array(shape=(h, w))
    sess.rdl.rdl_prepare_small_kernel(sess.h, d.vp, w, h, k.ctypes.data_as(C.c_void_p), n)
    full = np.zeros((h, w), np.float32)
    full[:n, :n] = k
    assert np.array_equal(d.get(), np.roll(full, (-(n // 2), -(n // 2)), axis=(0, 1)))
    rng = np.random.default_rng(n)
    img = rng.standard_normal((h, w)).astype(np.float32)
    d.upload(img)
    expect = img.copy()
    for (x, y, g) in ((w // 2, h // 2, 0.25), (1, h - 2, -0.5), (w - 1, 0, 1.5)):
        sess.rdl.rdl_add_shape_component(sess.h, d.vp, w, h, k.ctypes.data_as(C.c_void_p), n,
                                         x, y, C.c_float(g))
        orc.add_shape_component(expect, scale, x, y, g, shape)
    assert np.array_equal(bits(d.get()), bits(expect))
    d.free()


def test_median(sess):
    rng = np.random.default_rng(4)
    for n in (1, 2, 1001, 4096):
        v = rng.standard_normal(n).astype(np.float32)
        d = sess.array(v)
        out = C.c_float()
        sess.rdl.rdl_median(sess.h, d.vp, C.c_size_t(n), 0, C.c_float(0), C.byref(out))
        s = np.sort(v)
        med = s[n // 2] if n % 2 else np.float32(0.5) * (s[n // 2 - 1] + s[n // 2])
        assert out.value == med
        d.free()


# ------------------------------------------------------------------ loops
def synthetic(w, h, n_src, seed, psf_fwhm=3.0):
    """Small deterministic sky ⊛ analytic PSF (peak exactly 1.0 at (w/2, h/2))."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    s = psf_fwhm / 2.355
    r2 = ((xx - w // 2) ** 2 + (yy - h // 2) ** 2)
    psf = np.exp(-r2 / (2 * s * s)) + 0.05 * np.cos(2 * np.pi * np.sqrt(r2) / 9.0) * np.exp(-np.sqrt(r2) / 20.0)
    psf = (psf / psf[h // 2, w // 2]).astype(np.float32)
    sky = np.zeros((h, w))
    xs = rng.integers(8, w - 8, n_src)
    ys = rng.integers(8, h - 8, n_src)
    fl = np.exp(rng.uniform(np.log(0.01), np.log(1.0), n_src))
    for x, y, f in zip(xs, ys, fl):
        sky[y, x] += f
    P = np.fft.fft2(np.fft.ifftshift(psf.astype(np.float64)))
    dirty = np.real(np.fft.ifft2(np.fft.fft2(sky) * P))
    dirty += 1e-3 * rng.standard_normal((h, w))
    return psf, dirty.astype(np.float32)


def test_hogbom_bit_exact(sess, orc):
    w = h = 256
    psf, dirty = synthetic(w, h, 40, 3)
    niter, gain = 400, 0.1
    # oracle
    res_o, mod_o = dirty[None].copy(), np.zeros((1, h, w), np.float32)
    alg = OracleAlgorithm(orc, 0, threshold=0.0, max_iterations=niter, border_ratio=0.0,
                          use_sub_minor=0)
    r, trace_o = alg.execute(res_o, mod_o, psf[None])
    # GPU: initial FindPeak on the (linear) integrated image, then the loop
    dres, dmod, dpsf = sess.array(dirty), sess.array(shape=(h, w)), sess.array(psf)
    found, x, y, v = sess.find_peak(dres, w, h)
    p = HogbomParams()
    p.width, p.height, p.n_images, p.n_pol = w, h, 1, 1
    p.integ = integration(1, 1, mode=1)
    p.gain, p.threshold, p.initial_max = gain, 0.0, abs(v)
    p.divergence_limit = 4.0
    p.iteration_start, p.max_iterations = 0, niter
    p.allow_negative, p.stop_on_negative = 1, 0
    p.start_x, p.start_y, p.start_value, p.start_found = x, y, v, int(found)
    res = HogbomResult()
    trace = np.zeros((niter, 2), np.uint32)
    sess.rdl.rdl_hogbom_run(sess.h, dres.vp, dmod.vp, dpsf.vp, C.byref(p), C.byref(res),
                            trace.ctypes.data_as(C.c_void_p), C.c_uint64(niter))
    assert res.iteration == r.iteration_number == niter
    assert np.array_equal(trace, trace_o[:, :2])
    assert np.array_equal(bits(dres.get()), bits(res_o[0]))
    assert np.array_equal(bits(dmod.get()), bits(mod_o[0]))
    assert bits(res.peak) == bits(r.final_peak)
    for a in (dres, dmod, dpsf):
        a.free()


SUBMINOR_CASES = [
    # w, n_src, threshold_frac, mgain, max_iter, n_ch, mode, target
    (128, 10, 0.0, 0.8, 300, 1, 0, 0),        # small set: one workgroup
    (512, 200, 0.002, 1.0, 2000, 1, 0, 0),    # noise-level selection: multi-workgroup
    (128, 10, 0.0, 0.8, 300, 1, 1, 0),        # LDS-resident kernel forced
    (512, 200, 0.002, 1.0, 2000, 1, 1, 0),
    (256, 60, 0.001, 1.0, 1500, 1, 2, 512),   # register kernel spread over many blocks
    (256, 60, 0.001, 1.0, 1500, 1, 2, 4096),
    (200, 30, 0.002, 0.9, 800, 2, 0, 0),      # joined channels
    (200, 30, 0.002, 0.9, 800, 3, 2, 700),
    (160, 20, 0.003, 0.9, 600, 5, 0, 0),
    (160, 20, 0.003, 0.9, 600, 8, 2, 600),
    (160, 20, 0.003, 0.9, 600, 5, 1, 0),
    (128, 10, 0.0, 0.8, 300, 1, 3, 0),        # single-wave kernel forced
    (128, 10, 0.0, 0.8, 300, 1, 4, 0),        # one 1024-thread workgroup forced
    (512, 200, 0.002, 1.0, 2000, 1, 5, 2048),  # grid of 1024-thread workgroups
    (200, 30, 0.002, 0.9, 800, 3, 5, 1024),
    (128, 10, 0.0, 0.8, 300, 1, 6, 512),     # table kernel forced (pixels per participant)
]


@pytest.mark.parametrize("w,n_src,threshold_frac,mgain,max_iter,n_ch,mode,target",
                         SUBMINOR_CASES)
def test_subminor_loop_bit_exact(sess, orc, w, n_src, threshold_frac, mgain, max_iter,
                                 n_ch, mode, target):
    """GenericClean's Clark path: the sub-minor loop's component trace and
    model values are bit-exact (every kernel variant, 1..8 joined channels);
    the residual after CorrectResidualDirty is FFT-based (rocFFT vs float64),
    |err| <= 5e-6 * max|dirty|."""
    h = w
    psf, dirty = synthetic(w, h, n_src, 7)
    dirties = np.stack([dirty * np.float32(1.0 + 0.15 * k) + np.float32(1e-3 * k) *
                        np.roll(dirty, 3 * k, axis=1) for k in range(n_ch)]).astype(np.float32)
    psfs = np.stack([psf] * n_ch)
    res_o, mod_o = dirties.copy(), np.zeros((n_ch, h, w), np.float32)
    integ = orc.integrate(dirties) if n_ch > 1 else dirties[0]
    pk = float(np.abs(integ).max())
    thr = threshold_frac * pk
    alg = OracleAlgorithm(orc, 0, threshold=thr, max_iterations=max_iter, border_ratio=0.0,
                          use_sub_minor=1, major_loop_gain=mgain)
    r, trace_o = alg.execute(res_o, mod_o, psfs)
    # GPU, as GenericClean::ExecuteMajorIteration with sub-minor optimisation
    dres, dpsf = sess.array(dirties), sess.array(psfs)
    _, _, _, v = orc.find_peak(integ, True)
    # generic_clean.cc:99-112 in float arithmetic
    first = max(np.float32(thr),
                np.float32(abs(v)) * (np.float32(1.0) - np.float32(mgain)))
    sm = C.c_void_p()
    sess.rdl.rdl_subminor_create(sess.h, C.byref(sm))
    sess.rdl.rdl_subminor_set_tuning(sm, mode, target)
    p = SubminorParams()
    p.width, p.height, p.n_images, p.n_pol = w, h, n_ch, 1
    p.integ = integration(n_ch, 1, mode=0)
    p.allow_negative, p.stop_on_negative = 1, 0
    p.threshold, p.gain, p.divergence_limit = np.float32(first), 0.1, 4.0
    p.iteration_start, p.max_iterations = 0, max_iter
    out = SubminorResult()
    trace = np.zeros((max_iter, 2), np.uint32)
    sess.rdl.rdl_subminor_run(sm, dres.vp, dpsf.vp, C.byref(p), C.byref(out),
                              trace.ctypes.data_as(C.c_void_p), C.c_uint64(max_iter))
    n_it = out.iteration
    assert n_it == r.iteration_number
    assert np.array_equal(trace[:n_it], trace_o[:n_it, :2])
    if n_ch > 1:
        dmod = sess.array(shape=(h, w))
        for k in range(n_ch):
            sess.rdl.rdl_subminor_model(sm, k, dmod.vp, w, h, 0, 0, 0)
            assert np.array_equal(bits(dmod.get()), bits(mod_o[k]))
        sess.rdl.rdl_subminor_destroy(sm)
        for a in (dres, dpsf, dmod):
            a.free()
        return
    # model via the scatter path; CorrectResidualDirty on the padded grid
    dmod = sess.array(shape=(h, w))
    sess.rdl.rdl_subminor_model(sm, 0, dmod.vp, w, h, 0, 0, 1)
    assert np.array_equal(bits(dmod.get()), bits(mod_o[0]))
    pw = ph = int(np.ceil(np.float32(1.1) * np.float32(w)))
    pw += pw % 2
    ph = pw
    f = C.c_void_p()
    sess.rdl.rdl_fft_create(sess.h, pw, ph, C.byref(f))
    nb = sess.rdl.lib.rdl_fft_spectrum_bytes(f)
    kern, spec_k = sess.array(shape=(ph, pw)), sess.array(shape=(nb // 4,))
    padded, work = sess.array(shape=(ph, pw)), sess.array(shape=(nb // 4,))
    sess.rdl.rdl_prepare_psf_kernel(sess.h, kern.vp, pw, ph, dpsf.vp, w, h)
    sess.rdl.rdl_fft_forward(f, kern.vp, spec_k.vp)
    sess.rdl.rdl_subminor_model(sm, 0, padded.vp, pw, ph, (pw - w) // 2, (ph - h) // 2, 0)
    sess.rdl.rdl_fft_convolve(f, padded.vp, spec_k.vp, work.vp)
    sess.rdl.rdl_trim_subtract(sess.h, dres.vp, w, h, padded.vp, pw, ph)
    g = dres.get()
    assert np.abs(g - res_o[0]).max() <= 5e-6 * np.abs(dirty).max()
    sess.rdl.rdl_fft_destroy(f)
    sess.rdl.rdl_subminor_destroy(sm)
    for a in (dres, dpsf, dmod, kern, spec_k, padded, work):
        a.free()


@pytest.mark.parametrize("n_target,per_participant,neg,quantum", [
    (300, 1 << 20, 1, 0), (1500, 512, 1, 0), (1500, 1 << 20, 1, 0), (5000, 256, 1, 0),
    (5000, 1024, 1, 0), (5000, 1 << 20, 1, 0), (11000, 512, 1, 0), (11000, 4096, 1, 0),
    # one 1024-thread workgroup of 16 pixels per thread, and two of 8
    (16000, 1 << 20, 1, 0), (16000, 8192, 1, 0),
    # positive components only (the single-key argmax)
    (1500, 1 << 20, 0, 0), (5000, 1024, 0, 0),
    # exact |value| ties (values on a 2^-12 grid, both signs): the lowest
    # selection index wins, inside a thread, a wave, a workgroup and a grid
    (3000, 1 << 20, 1, 2.0 ** -12), (3000, 512, 1, 2.0 ** -12)])
def test_subminor_table_kernel_bit_exact(sess, orc, n_target, per_participant, neg, quantum):
    """The pairwise-table loop (rdl_subminor_set_tuning mode 6) on one
    workgroup and on grids of 2..22 participants: the threshold is set so
    that about n_target pixels are selected; trace and model values bit-exact
    against the oracle's sub-minor loop (GenericClean's Clark path)."""
    _table_kernel_case(sess, orc, n_target, per_participant, neg, quantum)


@pytest.mark.gpu
@pytest.mark.parametrize("exchange,sharing", [("agent", 0), (None, 16), ("agent", 16)])
@pytest.mark.parametrize("quantum", [0, 2.0 ** -12])
def test_subminor_table_grid_exchange_forms(sess, orc, exchange, sharing, quantum, monkeypatch):
    """The grid table loop's participant exchange in its other forms, against
    the oracle like the default (fast: workgroup-scope stores, every
    participant on one XCD): agent-scope stores (RDL_SUBMINOR_EXCHANGE=agent),
    and a pooled session's share of the GPU (rdl_session_set_concurrency 16:
    16 blocks for ~10 participants, so one launched block per participant,
    spread over the XCDs, which makes the kernel pick agent-scope stores)."""
    if exchange:
        monkeypatch.setenv("RDL_SUBMINOR_EXCHANGE", exchange)
    if sharing:
        sess.rdl.rdl_session_set_concurrency(sess.h, sharing)
    try:
        _table_kernel_case(sess, orc, 5000, 512, 1, quantum)
    finally:
        sess.rdl.rdl_session_set_concurrency(sess.h, 1)


def _table_kernel_case(sess, orc, n_target, per_participant, neg, quantum):
    w = h = 512
    psf, dirty = synthetic(w, h, 200, 7)
    if quantum:
        dirty = (np.round(dirty / quantum) * quantum).astype(np.float32)
        psf = (np.round(psf / quantum) * quantum).astype(np.float32)
    thr = float(np.sort(np.abs(dirty if neg else np.maximum(dirty, 0)).ravel())[-n_target])
    max_iter = 1500
    res_o, mod_o = dirty[None].copy(), np.zeros((1, h, w), np.float32)
    alg = OracleAlgorithm(orc, 0, threshold=thr, max_iterations=max_iter, border_ratio=0.0,
                          use_sub_minor=1, major_loop_gain=1.0, allow_negative=neg)
    r, trace_o = alg.execute(res_o, mod_o, psf[None])
    dres, dpsf = sess.array(dirty[None]), sess.array(psf[None])
    sm = C.c_void_p()
    sess.rdl.rdl_subminor_create(sess.h, C.byref(sm))
    sess.rdl.rdl_subminor_set_tuning(sm, 6, per_participant)
    p = SubminorParams()
    p.width, p.height, p.n_images, p.n_pol = w, h, 1, 1
    p.integ = integration(1, 1, mode=0)
    p.allow_negative, p.stop_on_negative = neg, 0
    p.threshold, p.gain, p.divergence_limit = np.float32(thr), 0.1, 4.0
    p.iteration_start, p.max_iterations = 0, max_iter
    out = SubminorResult()
    trace = np.zeros((max_iter, 2), np.uint32)
    sess.rdl.rdl_subminor_run(sm, dres.vp, dpsf.vp, C.byref(p), C.byref(out),
                              trace.ctypes.data_as(C.c_void_p), C.c_uint64(max_iter))
    n_it = out.iteration
    print(f"n_sel {out.n_selected}, {n_it} iterations")
    if not quantum:
        assert abs(int(out.n_selected) - n_target) <= n_target // 10 + 5
    assert n_it == r.iteration_number
    assert np.array_equal(trace[:n_it], trace_o[:n_it, :2])
    dmod = sess.array(shape=(h, w))
    sess.rdl.rdl_subminor_model(sm, 0, dmod.vp, w, h, 0, 0, 1)
    assert np.array_equal(bits(dmod.get()), bits(mod_o[0]))
    sess.rdl.rdl_subminor_destroy(sm)
    for a in (dres, dpsf, dmod):
        a.free()


@pytest.mark.parametrize("w,h,pw,ph,rows", [(64, 64, 72, 72, (3, 40)), (200, 150, 224, 168, (0, 1, 77, 149)),
                                            (90, 60, 98, 64, ()), (90, 60, 98, 64, (59,))])
@pytest.mark.parametrize("columns", [RDL_CONV_COLUMNS_SINGLE, RDL_CONV_COLUMNS_SPLIT])
def test_lds_fft_correction_sparse_rows(sess, w, h, pw, ph, rows, columns):
    """The correction with a row mask (empty model rows neither read nor
    transformed) and (single-pass columns) a column-major PSF spectrum is
    bit-identical to the dense row-major sequence: the skipped rows are exact
    zeros either way."""
    c = conv_create(sess, pw, ph, True, columns)
    split = columns == RDL_CONV_COLUMNS_SPLIT
    rng = np.random.default_rng(pw + len(rows))
    psf = rng.standard_normal((h, w)).astype(np.float32)
    model = np.zeros((h, w), np.float32)
    for y in rows:
        xs = rng.choice(w, 5, replace=False)
        model[y, xs] = rng.standard_normal(5).astype(np.float32)
    residual = rng.standard_normal((h, w)).astype(np.float32)
    ox, oy = (pw - w) // 2, (ph - h) // 2
    mask = np.zeros(ph, np.uint8)
    for y in rows:
        mask[y + oy] = 1
    dpsf, dmod = sess.array(psf), sess.array(model)
    dres_a, dres_b = sess.array(residual), sess.array(residual)
    dmask = sess.array(mask, dtype=np.uint8)
    kplane = sess.array(shape=(ph, pw))
    kspec = sess.array(shape=(ph, pw // 2 + 1), dtype=np.complex128)
    kspec_cm = sess.array(shape=(pw // 2 + 1, ph), dtype=np.complex128)
    work = sess.array(shape=(ph, pw // 2 + 1), dtype=np.complex128)
    sess.rdl.rdl_prepare_psf_kernel(sess.h, kplane.vp, pw, ph, dpsf.vp, w, h)
    sess.rdl.rdl_conv_forward(c, kplane.vp, kspec.vp)
    # column-major forward spectrum == the row-major one transposed
    if not split:
        sess.rdl.rdl_conv_rows_forward(c, kplane.vp, pw, ph, 0, 0, work.vp)
        sess.rdl.rdl_conv_columns_ex(c, work.vp, kspec_cm.vp, None, 0, C.c_double(1.0), None,
                                     RDL_CONV_ROW_MAJOR, RDL_CONV_COL_MAJOR)
        assert np.array_equal(kspec_cm.get(), kspec.get().T)
    norm = C.c_double(1.0 / (pw * ph))
    sess.rdl.rdl_conv_rows_forward(c, dmod.vp, w, h, ox, oy, work.vp)
    sess.rdl.rdl_conv_columns(c, work.vp, work.vp, kspec.vp, 1, norm)
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, dres_a.vp, w, h, ox, oy, 1)
    work.upload(np.full((ph, pw // 2 + 1), np.nan, np.complex128))  # skipped rows stay unread
    sess.rdl.rdl_conv_rows_forward_masked(c, dmod.vp, w, h, ox, oy, work.vp, dmask.vp)
    sess.rdl.rdl_conv_columns_ex(c, work.vp, work.vp, kspec.vp if split else kspec_cm.vp, 1,
                                 norm, dmask.vp,
                                 RDL_CONV_ROW_MAJOR if split else RDL_CONV_COL_MAJOR,
                                 RDL_CONV_ROW_MAJOR)
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, dres_b.vp, w, h, ox, oy, 1)
    a, b = dres_a.get(), dres_b.get()
    assert np.array_equal(a, b)
    if not rows:
        assert np.array_equal(b, residual)
    for x in (dpsf, dmod, dres_a, dres_b, dmask, kplane, kspec, kspec_cm, work):
        x.free()
    sess.rdl.rdl_conv_destroy(c)


@pytest.mark.parametrize("w,h", [(256, 256), (301, 257), (262, 222), (498, 350),
                                 (1100, 1000), (2100, 1900)])
@pytest.mark.parametrize("shape", [0, 1])
def test_ms_transform_any_size(orc, w, h, shape):
    """MultiScaleTransforms::Transform (circular at W x H): sizes that are not
    even 7-smooth run in a periodically extended plane of a friendly size
    (rdl_periodic_extend + crop); the result is the oracle's float64
    circular convolution within float32 FFT rounding."""
    from radler_import import radler as rd
    rng = np.random.default_rng(w * h)
    img = rng.standard_normal((h, w)).astype(np.float32)
    scales = [8.0, 16.0, 32.0, 64.0]
    out, pw, ph = rd.gpu.ms_transform(img, scales, max(scales), shape)
    friendly = orc.good_fft_size(w) == w and orc.good_fft_size(h) == h
    assert (pw, ph) == (w, h) if friendly else (pw > w and ph > h)
    for i, sc in enumerate(scales):
        expect = orc.ms_transform(img.copy(), sc, shape)
        err = np.abs(out[i] - expect).max()
        assert err <= 2e-6 * np.abs(img).max() * np.sqrt(np.log2(pw * ph)), (sc, err)


@pytest.mark.parametrize("w,h,n,k", [(300, 200, 33, 400), (256, 256, 129, 400),
                                     (1000, 130, 65, 400), (130, 97, 97, 400),
                                     (2048, 1024, 9, 4000), (1536, 1536, 31, 6000)])
def test_subminor_shape_model_stamp(sess, w, h, n, k):
    """rdl_subminor_add_shape_model (the scale > 0 model update): every
    selected component's n x n stamp added circularly, each pixel summing the
    components in selection order — against the same sums in numpy float32
    (partial edge tiles, stamps wrapping both edges, tiles no stamp reaches;
    k selected pixels: many 256-component chunks, most of which a tile skips
    by their stamps' bounding box)."""
    rng = np.random.default_rng(w + n)
    psf, dirty = synthetic(w, h, 40, 3)
    dirty = dirty.astype(np.float32)
    dres, dpsf = sess.array(dirty[None]), sess.array(psf[None])
    sm = C.c_void_p()
    sess.rdl.rdl_subminor_create(sess.h, C.byref(sm))
    p = SubminorParams()
    p.width, p.height, p.n_images, p.n_pol = w, h, 1, 1
    p.integ = integration(1, 1, mode=0)
    p.allow_negative, p.stop_on_negative = 1, 0
    p.threshold = float(np.sort(np.abs(dirty).ravel())[-k])
    p.gain, p.divergence_limit = 0.1, 0.0
    p.iteration_start, p.max_iterations = 0, 300
    out = SubminorResult()
    sess.rdl.rdl_subminor_run(sm, dres.vp, dpsf.vp, C.byref(p), C.byref(out), None,
                              C.c_uint64(0))
    n_sel = int(out.n_selected)
    pos = np.zeros(n_sel, np.uint32)
    mod = np.zeros(n_sel, np.float32)
    sess.rdl.rdl_subminor_get(sm, pos.ctypes.data_as(C.c_void_p),
                              mod.ctypes.data_as(C.c_void_p), C.c_uint64(n_sel))
    kern = rng.random((n, n)).astype(np.float32)
    dk = sess.array(kern)
    dmodel = sess.array(np.zeros((h, w), np.float32))
    sess.rdl.rdl_subminor_add_shape_model(sm, 0, dk.vp, n, dmodel.vp, w, h)
    acc = np.zeros((h, w), np.float32)
    hh = n // 2
    for p_, v in zip(pos, mod):
        if v == 0.0:
            continue
        xc, yc = int(p_ & 0xffff), int(p_ >> 16)
        ys = (np.arange(-hh, hh + 1) + yc) % h
        xs = (np.arange(-hh, hh + 1) + xc) % w
        acc[np.ix_(ys, xs)] += np.float32(v) * kern
    assert (mod != 0).sum() > 10
    assert np.array_equal(dmodel.get(), acc)
    sess.rdl.rdl_subminor_destroy(sm)
    for a in (dres, dpsf, dk, dmodel):
        a.free()


@pytest.mark.parametrize("n_ch,n_target,neg", [
    (2, 300, 1), (2, 2500, 1), (4, 1500, 1), (8, 600, 1), (8, 3000, 1), (8, 5000, 1),
    (3, 1500, 0), (8, 2000, 0)])
def test_subminor_joined_table_kernel_bit_exact(sess, orc, n_ch, n_target, neg):
    """The joined-image table loop (SubminorLoopTabN: 2..8 images, linear
    integration, one workgroup up to 1024 pixels, then XCD-local participants
    of <= 1024): trace and model values bit-exact against the oracle's Clark
    sub-minor loop over the same joined image set."""
    w = h = 512
    psf, dirty = synthetic(w, h, 200, 7)
    dirties = np.stack([dirty * np.float32(1.0 + 0.15 * k) + np.float32(1e-3 * k) *
                        np.roll(dirty, 3 * k, axis=1) for k in range(n_ch)]).astype(np.float32)
    psfs = np.stack([np.roll(psf, k, axis=0) * np.float32(1.0 - 0.02 * k)
                     for k in range(n_ch)]).astype(np.float32)
    integ = orc.integrate(dirties)
    val = np.abs(integ) if neg else np.maximum(integ, 0)
    thr = float(np.sort(val.ravel())[-n_target])
    max_iter = 1200
    res_o, mod_o = dirties.copy(), np.zeros((n_ch, h, w), np.float32)
    alg = OracleAlgorithm(orc, 0, threshold=thr, max_iterations=max_iter, border_ratio=0.0,
                          use_sub_minor=1, major_loop_gain=1.0, allow_negative=neg)
    r, trace_o = alg.execute(res_o, mod_o, psfs)
    dres, dpsf = sess.array(dirties), sess.array(psfs)
    sm = C.c_void_p()
    sess.rdl.rdl_subminor_create(sess.h, C.byref(sm))
    p = SubminorParams()
    p.width, p.height, p.n_images, p.n_pol = w, h, n_ch, 1
    p.integ = integration(n_ch, 1, mode=0)
    p.allow_negative, p.stop_on_negative = neg, 0
    p.threshold, p.gain, p.divergence_limit = np.float32(thr), 0.1, 4.0
    p.iteration_start, p.max_iterations = 0, max_iter
    out = SubminorResult()
    trace = np.zeros((max_iter, 2), np.uint32)
    sess.rdl.rdl_subminor_run(sm, dres.vp, dpsf.vp, C.byref(p), C.byref(out),
                              trace.ctypes.data_as(C.c_void_p), C.c_uint64(max_iter))
    n_it = out.iteration
    print(f"n_sel {out.n_selected}, {n_it} iterations")
    assert n_it == r.iteration_number
    assert np.array_equal(trace[:n_it], trace_o[:n_it, :2])
    for k in range(n_ch):
        dmod = sess.array(shape=(h, w))
        sess.rdl.rdl_subminor_model(sm, k, dmod.vp, w, h, 0, 0, 0)
        assert np.array_equal(bits(dmod.get()), bits(mod_o[k])), k
        dmod.free()
    sess.rdl.rdl_subminor_destroy(sm)
    for a in (dres, dpsf):
        a.free()


@pytest.mark.parametrize("w,h,border,frac,masked", [
    (4096, 4096, 0, 0.001, 0), (1000, 700, 13, 0.05, 0), (300, 200, 0, 1.0, 0),
    (8192, 1024, 100, 0.0002, 0), (1000, 700, 13, 0.05, 1), (998, 301, 7, 0.3, 1),
    (20000, 40, 3, 0.01, 0), (40000, 24, 3, 0.01, 0)])
def test_subminor_selection_modes_agree(sess, w, h, border, frac, masked):
    """The sparse two-phase selection (default; 16-byte loads where the width
    is a multiple of 4, RDL_SUBMINOR_SELECT=4 forces its scalar loads), the
    single-pass look-back (=1) and count + scan + scatter (=3) select the same
    pixels in the same (box) order: sparse selections, a clean border, a clean
    mask, every pixel of the box (frac 1), rows too wide for the vector path."""
    import os
    rng = np.random.default_rng(w + h)
    img = rng.standard_normal((h, w)).astype(np.float32)
    box = img[border:h - border, border:w - border]
    thr = 0.0 if frac >= 1.0 else float(np.quantile(np.abs(box), 1.0 - frac))
    psf = np.zeros((h, w), np.float32)
    psf[h // 2, w // 2] = 1.0
    dres, dpsf = sess.array(img), sess.array(psf)
    mask = (rng.random((h, w)) < 0.7).astype(np.uint8) if masked else None
    dmask = sess.array(mask, dtype=np.uint8) if masked else None
    got = []
    for mode in ("0", "4", "1", "3"):
        os.environ["RDL_SUBMINOR_SELECT"] = mode
        sm = C.c_void_p()
        try:
            sess.rdl.rdl_subminor_create(sess.h, C.byref(sm))
        finally:
            del os.environ["RDL_SUBMINOR_SELECT"]
        p = SubminorParams()
        p.width, p.height, p.n_images, p.n_pol = w, h, 1, 1
        p.integ = integration(1, 1, mode=0)
        p.h_border = p.v_border = border
        if masked:
            p.d_mask = dmask.vp
        p.allow_negative, p.stop_on_negative = 1, 0
        p.threshold, p.gain, p.divergence_limit = thr, 0.1, 0.0
        p.iteration_start, p.max_iterations = 0, 0
        out = SubminorResult()
        sess.rdl.rdl_subminor_run(sm, dres.vp, dpsf.vp, C.byref(p), C.byref(out), None,
                                  C.c_uint64(0))
        n = int(out.n_selected)
        pos = np.zeros(max(n, 1), np.uint32)
        mod = np.zeros(max(n, 1), np.float32)
        sess.rdl.rdl_subminor_get(sm, pos.ctypes.data_as(C.c_void_p),
                                  mod.ctypes.data_as(C.c_void_p), C.c_uint64(n))
        got.append(pos[:n])
        sess.rdl.rdl_subminor_destroy(sm)
    keep = np.abs(box) >= np.float32(thr)
    if masked:
        keep &= mask[border:h - border, border:w - border] != 0
    ys, xs = np.nonzero(keep)
    expect = ((ys + border).astype(np.uint32) << 16) | (xs + border).astype(np.uint32)
    for g in got:
        assert np.array_equal(g, expect)
    for a in (dres, dpsf) + ((dmask,) if masked else ()):
        a.free()


def test_subminor_selection_lookback_timeout_is_reported(sess):
    """The single-pass selection's decoupled look-back gives up after a spin
    limit (never reached in practice). With the limit forced to 0
    (RDL_SELECT_SPIN_LIMIT, read by rdl_subminor_create) any chunk that has
    to wait for a predecessor gives up: the run must then fail with an error,
    never return a wrong selection (every pixel of a 4096^2 box is selected
    at threshold 0, so a correct run selects exactly 4096^2)."""
    import os
    w = h = 4096
    rng = np.random.default_rng(11)
    img = rng.standard_normal((h, w)).astype(np.float32) + np.float32(2.0)
    psf = np.zeros((h, w), np.float32)
    psf[h // 2, w // 2] = 1.0
    dres, dpsf = sess.array(img), sess.array(psf)
    failed = ok = 0
    for _ in range(8):
        os.environ["RDL_SELECT_SPIN_LIMIT"] = "0"
        os.environ["RDL_SUBMINOR_SELECT"] = "1"  # the single pass (not the default)
        sm = C.c_void_p()
        try:
            sess.rdl.rdl_subminor_create(sess.h, C.byref(sm))
        finally:
            del os.environ["RDL_SELECT_SPIN_LIMIT"]
            del os.environ["RDL_SUBMINOR_SELECT"]
        p = SubminorParams()
        p.width, p.height, p.n_images, p.n_pol = w, h, 1, 1
        p.integ = integration(1, 1, mode=0)
        p.allow_negative, p.stop_on_negative = 1, 0
        p.threshold, p.gain, p.divergence_limit = 0.0, 0.1, 4.0
        p.iteration_start, p.max_iterations = 0, 1
        out = SubminorResult()
        trace = np.zeros((1, 2), np.uint32)
        try:
            sess.rdl.rdl_subminor_run(sm, dres.vp, dpsf.vp, C.byref(p), C.byref(out),
                                      trace.ctypes.data_as(C.c_void_p), C.c_uint64(1))
            assert out.n_selected == w * h, out.n_selected
            ok += 1
        except RdlError as e:
            assert "timed out" in str(e), e
            failed += 1
        sess.sync()
        sess.rdl.rdl_subminor_destroy(sm)
    print(f"look-back with spin limit 0: {failed} runs reported a timeout, {ok} exact")
    assert failed >= 1
    for a in (dres, dpsf):
        a.free()


def test_out_of_memory_flushes_every_session_cache():
    """rdl_malloc keeps freed blocks in its session's cache. A block cached by
    one session (a pool worker's, which live for the process) must not make
    another session's allocation fail: on out-of-memory every cache on the
    device is handed back before the retry."""
    hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
    a, b = Session(0), Session(0)
    try:
        f, t = C.c_size_t(), C.c_size_t()
        assert hip.hipSetDevice(0) == 0 and hip.hipMemGetInfo(C.byref(f), C.byref(t)) == 0
        free0, total = f.value, t.value
        block = int(0.2 * total)
        x = a.array(shape=(block // 4,))
        x.free()  # cached by session a (within its cap of total / 4)
        # more than what is free while a's block is cached, less than what is
        # free without it
        want = free0 - block // 2
        p = C.c_void_p()
        b.rdl.rdl_malloc(b.h, C.c_size_t(want), C.byref(p))
        b.rdl.rdl_free(b.h, p)
    finally:
        a.close()
        b.close()
