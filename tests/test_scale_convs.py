"""The fused multi-scale convolution path of the four-step (tiled) float
plans (rdl_conv_forward_half / rdl_conv_real_kernel / rdl_conv_scales /
rdl_conv_scale_finish, csrc/hip/fft_fast.hip ColStepBScales + ColStepAInv):
FindMultiScalePeak's per-scale MultiScaleTransforms::Transform of one image
(cpp/algorithms/multiscale/multiscale_transforms.cc:9-21,
threaded_deconvolution_tools.cc:52-107) against numpy float64.

* the real kernel spectrum against numpy's rfft2 of the placed kernel
  (PrepareSmallConvolutionKernel) in float64: within float rounding of the
  spectrum's peak, and numpy's imaginary part is rounding noise (the kernel is
  even in x and y);
* several scales through one launch against numpy float64 convolutions,
  within the same bound as the two-pass path (tests/test_configs_gpu.py RTOL:
  a third of 1e-6 x the convolved image's peak), on the headline 8192^2
  plane, C2's 4096^2 and tiled runs' subimage planes (non-square included).
"""
import ctypes as C

import numpy as np
import pytest

RTOL = 1e-6  # tests/test_configs_gpu.py


def placed_kernel(k, w, h):
    n = k.shape[0]
    ker = np.zeros((h, w), np.float64)
    ker[:n, :n] = k
    return np.roll(ker, (-(n // 2), -(n // 2)), axis=(0, 1))


def untile(flat, w, h, dtype):
    nu = w // 2 + 1
    nt = (nu + 15) // 16
    t = np.asarray(flat).view(dtype).reshape(nt, h, 16)
    return t.transpose(1, 0, 2).reshape(h, nt * 16)[:, :nu]


@pytest.fixture(scope="module")
def sess():
    from rdl_lib import Session
    s = Session(0)
    yield s
    s.close()


@pytest.fixture(scope="module")
def orc():
    from oracle_lib import get_oracle
    return get_oracle()


def make_conv(sess, w, h):
    c = C.c_void_p()
    sess.rdl.rdl_conv_create_ex(sess.h, w, h, 0, 1, C.byref(c))
    assert sess.rdl.lib.rdl_conv_fast(c) & 4, "expected a four-step (tiled) plan"
    return c


def real_kernel(sess, c, k):
    sess.rdl.lib.rdl_conv_real_kernel_bytes.restype = C.c_size_t
    sess.rdl.lib.rdl_conv_real_kernel_bytes.argtypes = [C.c_void_p]
    nb = sess.rdl.lib.rdl_conv_real_kernel_bytes(c)
    dk = sess.array(shape=(nb // 4,), dtype=np.float32)
    k = np.ascontiguousarray(k, np.float32)
    sess.rdl.rdl_conv_real_kernel(c, k.ctypes.data_as(C.c_void_p), k.shape[0], dk.vp)
    return dk


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,scale", [(8192, 8192, 256.0), (4096, 4096, 16.0),
                                       (2048, 2048, 64.0), (1536, 1280, 32.0)])
def test_real_kernel_spectrum(sess, orc, w, h, scale):
    k = orc.shape_function(scale, min(w, h))
    c = make_conv(sess, w, h)
    dk = real_kernel(sess, c, k)
    got = untile(dk.get(), w, h, np.float32)
    ref = np.fft.rfft2(placed_kernel(k.astype(np.float64), w, h))
    peak = np.abs(ref).max()
    print(f"{w}x{h} scale {scale:g}: |Im| {np.abs(ref.imag).max() / peak:.3g}, "
          f"|K - Re| {np.abs(got - ref.real).max() / peak:.3g} x peak")
    assert np.abs(ref.imag).max() <= 1e-12 * peak
    assert np.abs(got - ref.real).max() <= 1.2e-7 * peak
    dk.free()
    sess.rdl.rdl_conv_destroy(c)


def fused(sess, c, img, kernels):
    """The fused path: every kernel's convolution of img (list of arrays)."""
    h, w = img.shape
    nb = sess.rdl.lib.rdl_conv_spectrum_bytes(c)
    di = sess.array(img)
    half, work = (sess.array(shape=(nb // 8,), dtype=np.complex64) for _ in range(2))
    outs = [sess.array(shape=(nb // 8,), dtype=np.complex64) for _ in kernels]
    dks = [real_kernel(sess, c, k) for k in kernels]
    sess.rdl.rdl_conv_forward_half(c, di.vp, w, h, 0, 0, half.vp)
    kp = (C.c_void_p * len(kernels))(*[d.ptr for d in dks])
    op = (C.c_void_p * len(kernels))(*[o.ptr for o in outs])
    sess.rdl.rdl_conv_scales(c, half.vp, len(kernels), kp, op,
                             C.c_double(float(np.float32(1.0 / (w * h)))))
    dout = sess.array(shape=(h, w))
    res = []
    for o in outs:
        sess.rdl.rdl_conv_scale_finish(c, o.vp, work.vp)
        sess.rdl.rdl_conv_rows_inverse(c, work.vp, dout.vp, w, h, 0, 0, 0)
        res.append(dout.get())
    for a in [di, half, work, dout] + outs + dks:
        a.free()
    return res


def two_pass(sess, c, img, k):
    """The two-pass path (forward spectrum, complex float kernel spectrum,
    rdl_conv_columns mode 2), as the multiscale loop ran it before."""
    h, w = img.shape
    nb = sess.rdl.lib.rdl_conv_spectrum_bytes(c)
    di = sess.array(img)
    ker = sess.array(placed_kernel(k, w, h).astype(np.float32))
    kspec, spec, work = (sess.array(shape=(nb // 8,), dtype=np.complex64) for _ in range(3))
    sess.rdl.rdl_conv_forward(c, ker.vp, kspec.vp)
    sess.rdl.rdl_conv_forward(c, di.vp, spec.vp)
    sess.rdl.rdl_conv_columns(c, spec.vp, work.vp, kspec.vp, 2,
                              C.c_double(float(np.float32(1.0 / (w * h)))))
    dout = sess.array(shape=(h, w))
    sess.rdl.rdl_conv_rows_inverse(c, work.vp, dout.vp, w, h, 0, 0, 0)
    out = dout.get()
    for a in (di, ker, kspec, spec, work, dout):
        a.free()
    return out


def float64_conv(img, k):
    h, w = img.shape
    return np.fft.irfft2(np.fft.rfft2(img.astype(np.float64)) *
                         np.fft.rfft2(placed_kernel(k.astype(np.float64), w, h)), s=(h, w))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,scales", [(8192, 8192, (16.0, 64.0, 256.0)),
                                        (4096, 4096, (16.0, 32.0, 64.0, 128.0, 256.0)),
                                        (2048, 2048, (16.0, 64.0)),
                                        (1536, 1280, (32.0,))])
def test_scales_against_float64(sess, orc, w, h, scales):
    """Noise plus a bright point: every scale within float rounding of the
    float64 convolution, and no further from it than the two-pass path is
    (at most 1.25x its error, the two paths round differently)."""
    rng = np.random.default_rng(7)
    img = rng.standard_normal((h, w)).astype(np.float32)
    img[h // 3, w // 5] = 50.0
    c = make_conv(sess, w, h)
    kernels = [orc.shape_function(s, min(w, h)) for s in scales]
    got = fused(sess, c, img, kernels)
    for s, k, g in zip(scales, kernels, got):
        ref = float64_conv(img, k)
        peak = np.abs(ref).max()
        err = float(np.abs(g - ref).max() / peak)
        err2 = float(np.abs(two_pass(sess, c, img, k) - ref).max() / peak)
        print(f"{w}x{h} scale {s:g}: max |float32 - float64| fused {err:.3g}, "
              f"two-pass {err2:.3g} x peak")
        assert err <= RTOL / 2, err
        assert err <= 1.25 * err2 + 2e-8, (err, err2)
    sess.rdl.rdl_conv_destroy(c)


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [16.0, 64.0, 256.0])
def test_scales_c2_image_bound(sess, orc, scale):
    """RTOL's measurement on the fused path: the C2 dirty image (as
    tests/test_configs_gpu.py test_scale_convolution_error_4096 measures the
    two-pass path) within a third of RTOL x the convolved image's peak."""
    import config_problems as cp
    _, dirty = cp.problem("c2")
    img = dirty[0]
    k = orc.shape_function(scale, img.shape[1])
    c = make_conv(sess, img.shape[1], img.shape[0])
    g = fused(sess, c, img, [k])[0]
    ref = float64_conv(img, k)
    err = float(np.abs(g - ref).max() / np.abs(ref).max())
    print(f"C2 scale {scale:g}: fused max |float32 - float64| = {err:.3g} x peak")
    assert err <= RTOL / 3, err
    sess.rdl.rdl_conv_destroy(c)
