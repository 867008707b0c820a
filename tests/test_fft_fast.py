"""The compile-time-planned FFT kernels (csrc/hip/fft_fast.hip) at the sizes
they cover: the float64 padded residual-correction planes of 4096^2 / 8192^2
images (utils::GetConvolutionSize(scale, W, 1.1), cpp/utils/
fft_size_calculations.h:45-50) and the float32 scale-convolution planes.

Reference: numpy's float64 FFT (an independent algorithm). Tolerances:
float64 |err| <= 1e-12 * scale, float32 |err| <= 2e-6 * scale (written per
check). Also: the masked (sparse-row) correction sequence equals the dense
one, rows outside the output window are left untouched, and the fast and the
runtime-plan kernels (RDL_FFT_FAST=0 in a subprocess) agree.
"""
import ctypes as C

import numpy as np
import pytest

from rdl_lib import Session

pytestmark = pytest.mark.gpu

RDL_CONV_ROW_MAJOR, RDL_CONV_COL_MAJOR = 0, 1
RDL_CONV_COLUMNS_SINGLE = 1


@pytest.fixture(scope="module")
def sess():
    s = Session(0)
    yield s
    s.close()


def conv(sess, w, h, f64):
    c = C.c_void_p()
    sess.rdl.rdl_conv_create_ex(sess.h, w, h, int(f64), RDL_CONV_COLUMNS_SINGLE, C.byref(c))
    return c


RDL_CONV_FAST_TILED = 4  # rdl_hip.h


def tiled(sess, c):
    return bool(sess.rdl.lib.rdl_conv_fast(c) & RDL_CONV_FAST_TILED)


def spectrum_array(sess, c, w, h, cdt):
    n = sess.rdl.lib.rdl_conv_spectrum_bytes(c) // np.dtype(cdt).itemsize
    return sess.array(shape=(n,), dtype=cdt)


def natural(sess, c, flat, w, h):
    """A spectrum buffer's contents as [row][column] (h x w/2+1)."""
    if not tiled(sess, c):
        return flat.reshape(h, w // 2 + 1)
    nt = (w // 2 + 1 + 15) // 16
    t = flat.reshape(nt, h, 16).transpose(1, 0, 2).reshape(h, nt * 16)
    return t[:, :w // 2 + 1]


# (width, height, f64): rows use the half-length plan of `width`, columns the
# plan of `height`
CASES = [(4536, 4608, True), (4800, 5000, True), (4704, 4536, True), (9072, 9216, True),
         (9450, 9408, True), (8192, 4096, False), (4096, 8192, False),
         # 9072-point float64 columns: the 8192^2 correction's (ColumnsConvPair)
         (9216, 9072, True),
         # the subimage planes of tiled runs (CanonicalFftSize ladder)
         (2560, 3072, False), (3584, 1280, False), (1536, 2048, False), (2048, 1792, False),
         # the float64 corrections of gridded runs' subimages
         (1440, 1344, True), (1250, 1176, True), (1890, 1512, True), (1050, 1620, True),
         (2646, 3430, True), (3500, 2160, True), (2048, 2916, True)]


@pytest.mark.parametrize("w,h,f64", CASES)
def test_fast_forward_matches_numpy(sess, w, h, f64):
    rng = np.random.default_rng(w + h)
    img = rng.standard_normal((h, w)).astype(np.float32)
    c = conv(sess, w, h, f64)
    cdt = np.complex128 if f64 else np.complex64
    di = sess.array(img)
    spec = spectrum_array(sess, c, w, h, cdt)
    sess.rdl.rdl_conv_forward(c, di.vp, spec.vp)
    ref = np.fft.rfft2(img.astype(np.float64))
    assert tiled(sess, c) == (not f64)
    err = np.abs(natural(sess, c, spec.get(), w, h) - ref).max()
    scale = np.sqrt(w * h) * np.sqrt(np.log2(w * h))
    assert err <= (1e-13 if f64 else 2e-6) * scale, err
    for x in (di, spec):
        x.free()
    sess.rdl.rdl_conv_destroy(c)


@pytest.mark.parametrize("w,h,f64", CASES[:3] + CASES[5:])
def test_fast_convolutions_match_numpy(sess, w, h, f64):
    """In-place (columns mode 1) and shared-spectrum (mode 2) circular
    convolution with a kernel spectrum in both layouts."""
    rng = np.random.default_rng(3 * w + h)
    img = rng.standard_normal((h, w)).astype(np.float32)
    ker = np.zeros((h, w), np.float32)
    ker[:7, :9] = rng.standard_normal((7, 9))
    ker = np.roll(ker, (-3, -4), axis=(0, 1)).copy()
    ref = np.fft.irfft2(np.fft.rfft2(img.astype(np.float64)) *
                        np.fft.rfft2(ker.astype(np.float64)), s=(h, w))
    c = conv(sess, w, h, f64)
    cdt = np.complex128 if f64 else np.complex64
    dk, di = sess.array(ker), sess.array(img)
    kspec, kspec_cm, work, sspec = (spectrum_array(sess, c, w, h, cdt) for _ in range(4))
    out = sess.array(shape=(h, w))
    sess.rdl.rdl_conv_forward(c, dk.vp, kspec.vp)
    sess.rdl.rdl_conv_rows_forward(c, dk.vp, w, h, 0, 0, work.vp)
    sess.rdl.rdl_conv_columns_ex(c, work.vp, kspec_cm.vp, None, 0, C.c_double(1.0), None,
                                 RDL_CONV_ROW_MAJOR, RDL_CONV_COL_MAJOR)
    if tiled(sess, c):  # one layout for every spectrum
        assert np.array_equal(kspec_cm.get(), kspec.get())
    else:
        cm = kspec_cm.get()[:(w // 2 + 1) * h].reshape(w // 2 + 1, h)
        assert np.abs(cm.T - natural(sess, c, kspec.get(), w, h)).max() == 0.0
    norm = 1.0 / (w * h) if f64 else float(np.float32(1.0 / (w * h)))

    def close(got):
        # float64: the float output is the exact result rounded (half an ulp
        # of float32, + 1e-12 * scale for the transform); float32: 2e-6 * scale
        scale = np.abs(ref).max() * np.sqrt(np.log2(w * h))
        if f64:
            half_ulp = 0.5 * np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
            return np.all(np.abs(got - ref) <= half_ulp + 1e-12 * scale)
        return np.abs(got - ref).max() <= 2e-6 * scale
    for kern, layout in ((kspec, RDL_CONV_ROW_MAJOR), (kspec_cm, RDL_CONV_COL_MAJOR)):
        di.upload(img)
        sess.rdl.rdl_conv_rows_forward(c, di.vp, w, h, 0, 0, work.vp)
        sess.rdl.rdl_conv_columns_ex(c, work.vp, work.vp, kern.vp, 1, C.c_double(norm), None,
                                     layout, RDL_CONV_ROW_MAJOR)
        sess.rdl.rdl_conv_rows_inverse(c, work.vp, di.vp, w, h, 0, 0, 0)
        assert close(di.get())
    di.upload(img)
    sess.rdl.rdl_conv_forward(c, di.vp, sspec.vp)
    sess.rdl.rdl_conv_columns(c, sspec.vp, work.vp, kspec.vp, 2, C.c_double(norm))
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, out.vp, w, h, 0, 0, 0)
    assert close(out.get())
    for x in (dk, di, kspec, kspec_cm, work, sspec, out):
        x.free()
    sess.rdl.rdl_conv_destroy(c)


@pytest.mark.parametrize("pw,ph,w,h", [(4536, 4536, 4096, 4096), (9216, 9216, 8192, 8192),
                                       (4800, 4800, 4096, 4096), (9072, 9072, 8192, 8192)])
def test_fast_masked_correction(sess, pw, ph, w, h):
    """CorrectResidualDirty's sequence: sparse model rows (row mask) placed at
    the centred offset, x column-major PSF spectrum, trimmed subtraction from
    the residual window; equals numpy float64 and leaves nothing outside the
    window touched."""
    rng = np.random.default_rng(pw)
    psf = np.zeros((h, w), np.float32)
    psf[h // 2 - 20:h // 2 + 21, w // 2 - 20:w // 2 + 21] = rng.standard_normal((41, 41))
    model = np.zeros((h, w), np.float32)
    idx = rng.choice(w * h, 300, replace=False)
    model.flat[idx] = rng.standard_normal(300).astype(np.float32)
    residual = rng.standard_normal((h, w)).astype(np.float32)
    ox, oy = (pw - w) // 2, (ph - h) // 2
    # numpy: circular convolution at the padded size
    kp = np.zeros((ph, pw))
    kp[oy:oy + h, ox:ox + w] = psf
    kp = np.roll(kp, (-(ph // 2), -(pw // 2)), axis=(0, 1))
    mp = np.zeros((ph, pw))
    mp[oy:oy + h, ox:ox + w] = model
    conv_ref = np.fft.irfft2(np.fft.rfft2(mp) * np.fft.rfft2(kp), s=(ph, pw))
    expect = residual - conv_ref[oy:oy + h, ox:ox + w].astype(np.float32)

    c = conv(sess, pw, ph, True)
    dpsf, dmod = sess.array(psf), sess.array(model)
    dres = sess.array(shape=(h + 2, w))  # a guard row after the window
    guard = np.full((h + 2, w), 7.0, np.float32)
    guard[:h] = residual
    dres.upload(guard)
    kplane = sess.array(shape=(ph, pw))
    kspec = sess.array(shape=(pw // 2 + 1, ph), dtype=np.complex128)
    work = sess.array(shape=(ph, pw // 2 + 1), dtype=np.complex128)
    mask = np.zeros(ph, np.uint8)
    mask[oy + np.unique(idx // w)] = 1
    dmask = sess.array(mask, dtype=np.uint8)
    sess.rdl.rdl_prepare_psf_kernel(sess.h, kplane.vp, pw, ph, dpsf.vp, w, h)
    sess.rdl.rdl_conv_rows_forward(c, kplane.vp, pw, ph, 0, 0, work.vp)
    sess.rdl.rdl_conv_columns_ex(c, work.vp, kspec.vp, None, 0, C.c_double(1.0), None,
                                 RDL_CONV_ROW_MAJOR, RDL_CONV_COL_MAJOR)
    sess.rdl.rdl_conv_rows_forward_masked(c, dmod.vp, w, h, ox, oy, work.vp, dmask.vp)
    sess.rdl.rdl_conv_columns_ex(c, work.vp, work.vp, kspec.vp, 1,
                                 C.c_double(1.0 / (pw * ph)), dmask.vp, RDL_CONV_COL_MAJOR,
                                 RDL_CONV_ROW_MAJOR)
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, dres.vp, w, h, ox, oy, 1)
    got = dres.get()
    assert np.all(got[h:] == 7.0)
    err = np.abs(got[:h] - expect).max()
    assert err <= 2.4e-7 * max(np.abs(conv_ref).max(), np.abs(residual).max()), err
    for x in (dpsf, dmod, dres, kplane, kspec, work, dmask):
        x.free()
    sess.rdl.rdl_conv_destroy(c)


_PIPELINE = r"""
import sys, numpy as np
sys.path.insert(0, {tests!r})
from radler_import import radler as rd
import config_problems as cp
from test_configs_gpu import settings
psfs, dirty = cp.problem("c2")
run = rd.gpu.DeviceRun(settings(rd, "c2"), psfs[0], dirty[0], [],
                       cp.BEAM_PX * cp.PIXEL_SCALE)
r = run.execute()
np.savez({out!r}, trace=run.trace(), residual=run.residual(), model=run.model(),
         iterations=r["iterations"])
"""


def test_pipeline_fast_vs_runtime_plan_kernels(tmp_path):
    """The C2 configuration (4096^2, 6 scales: float64 corrections at
    4536..5000, i.e. the compile-time-planned kernels) with the fast kernels
    and with the runtime-plan kernels (RDL_FFT_FAST=0). The two float64
    engines round differently in the last bits, so each is compared with the
    oracle fixture tie-aware (tests/trace_compare.py): identical up to its
    first divergence, which may only fall on a decision whose oracle margin
    is below the float tolerance."""
    import os
    import subprocess
    import sys
    from test_configs_gpu import RTOL, fixture
    from trace_compare import assert_tie_aware
    fx = fixture("c2")
    tests = os.path.dirname(os.path.abspath(__file__))
    for fast in ("1", "0"):
        out = str(tmp_path / f"fast{fast}.npz")
        env = dict(os.environ, RDL_FFT_FAST=fast)
        subprocess.run([sys.executable, "-c", _PIPELINE.format(tests=tests, out=out)],
                       env=env, check=True, timeout=300)
        a = np.load(out)
        c = assert_tie_aware(a["trace"], fx["trace"], fx["margins"], fx["values"], RTOL)
        print(f"RDL_FFT_FAST={fast}: {c}")
        assert c.matched > 1000


class _Peak(C.Structure):
    _fields_ = [("value", C.c_float), ("x", C.c_uint32), ("y", C.c_uint32),
                ("found", C.c_int32)]


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,hb,vb,neg,masked,win", [
    (4096, 4096, 204, 204, 1, False, None), (4096, 4096, 0, 0, 0, False, None),
    (2048, 1536, 17, 40, 1, True, None), (8192, 4096, 410, 205, 0, True, None),
    (1280, 1280, 700, 0, 1, False, None),
    # windows of periodically extended planes (tiled subimages), even and odd
    (1536, 1536, 10, 12, 1, True, (1400, 1300, 68, 118)),
    (2560, 3072, 0, 5, 0, False, (2301, 2999, 33, 41))])
def test_rows_inverse_fused_peak_matches_find_peak(sess, w, h, hb, vb, neg, masked, win):
    """rdl_conv_rows_inverse_peak (the per-scale peak search fused into the
    inverse row pass) writes the same image (window) as rdl_conv_rows_inverse
    and returns exactly rdl_find_peak's result on it (box, mask, sign rules,
    first index on ties)."""
    ww, wh, ox, oy = win if win else (w, h, 0, 0)
    c = conv(sess, w, h, False)
    rng = np.random.default_rng(w + h + hb)
    img = rng.standard_normal((h, w)).astype(np.float32)
    img[h // 3, w // 5] = 40.0
    img[h // 2, w // 2] = -55.0  # wins only with allow_negative
    di = sess.array(img)
    spec = spectrum_array(sess, c, w, h, np.complex64)
    work = spectrum_array(sess, c, w, h, np.complex64)
    kspec = spectrum_array(sess, c, w, h, np.complex64)
    delta = np.zeros((h, w), np.float32)
    delta[0, 0] = 1.0
    dk = sess.array(delta)
    sess.rdl.rdl_conv_forward(c, dk.vp, kspec.vp)
    sess.rdl.rdl_conv_forward(c, di.vp, spec.vp)
    mask = (rng.random((wh, ww)) < 0.7).astype(np.uint8)
    dmask = sess.array(mask) if masked else None
    mptr = dmask.vp if masked else None
    out_a = sess.array(shape=(wh, ww))
    out_b = sess.array(shape=(wh, ww))
    norm = C.c_double(1.0 / (w * h))
    sess.rdl.rdl_conv_columns(c, spec.vp, work.vp, kspec.vp, 2, norm)
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, out_a.vp, ww, wh, ox, oy, 0)
    ref = _Peak()
    sess.rdl.rdl_find_peak(sess.h, out_a.vp, ww, wh, 0, wh, hb, vb, neg, mptr, 1, C.byref(ref))
    sess.rdl.rdl_conv_columns(c, spec.vp, work.vp, kspec.vp, 2, norm)
    sess.rdl.rdl_conv_rows_inverse_peak(c, work.vp, out_b.vp, ww, wh, ox, oy, hb, vb, neg, mptr,
                                        3)
    got = (_Peak * 4)()
    sess.rdl.rdl_find_peak_collect(sess.h, 4, got)
    a, b = out_a.get(), out_b.get()
    assert np.array_equal(a, b)
    g = got[3]
    assert (g.value, g.x, g.y, g.found) == (ref.value, ref.x, ref.y, ref.found)
    for x in (di, spec, work, kspec, dk, out_a, out_b) + ((dmask,) if masked else ()):
        x.free()
    sess.rdl.rdl_conv_destroy(c)
