"""IUWT à-trous decomposition.

CPU: the oracle's decomposition/recomposition round trip reproduces the
input within float rounding; the aliased form (input used as scratch, as the
reference's IUWT deconvolution calls it) differs from the plain one and
overwrites the input.
GPU: rdl_iuwt_decompose / rdl_iuwt_recompose are bit-exact with the oracle
(tap order per boundary region and FMA contraction of the reference build),
aliased and not, with and without the approximation plane.
"""
import os
import ctypes as C

import numpy as np
import pytest

from oracle_lib import get_oracle, iuwt_decompose, iuwt_recompose

CASES = [(64, 64, 3), (100, 80, 3), (256, 256, 6), (300, 260, 5), (1024, 512, 6)]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def image(w, h, seed):
    rng = np.random.default_rng(seed)
    img = rng.standard_normal((h, w)).astype(np.float32) * np.float32(1e-2)
    yy, xx = np.mgrid[0:h, 0:w]
    img += np.exp(-((xx - w / 3) ** 2 + (yy - h / 2) ** 2) / (2 * 6.0 ** 2)).astype(np.float32)
    return img


@pytest.mark.parametrize("w,h,n", CASES[:4])
def test_oracle_round_trip(w, h, n):
    orc = get_oracle()
    img = image(w, h, w)
    coeffs, after = iuwt_decompose(orc, img, n)
    assert np.array_equal(after, img)  # not aliased: input untouched
    back = iuwt_recompose(orc, coeffs, n)
    assert np.abs(back - img).max() <= 1e-5 * np.abs(img).max()
    # without the approximation the recomposition is the detail sum only
    no_approx = iuwt_recompose(orc, coeffs, n, include_largest=False)
    assert np.abs(no_approx - back).max() > 0
    aliased, clobbered = iuwt_decompose(orc, img, n, aliased=True)
    assert not np.array_equal(aliased[0], coeffs[0])
    assert not np.array_equal(clobbered, img)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n", CASES)
@pytest.mark.parametrize("aliased", [False, True])
@pytest.mark.parametrize("include_largest", [True, False])
def test_gpu_iuwt_bit_exact(w, h, n, aliased, include_largest):
    from rdl_lib import Session
    orc = get_oracle()
    img = image(w, h, w + n)
    coeffs_o, after_o = iuwt_decompose(orc, img, n, aliased, include_largest)
    s = Session(0)
    d_in = s.array(img)
    d_scratch = d_in if aliased else s.array(shape=(h, w))
    d_coeffs = s.array(shape=(n + 1, h, w))
    s.rdl.rdl_iuwt_decompose(s.h, d_in.vp, d_scratch.vp, w, h, n, d_coeffs.vp,
                             int(include_largest))
    got = d_coeffs.get()
    for k in range(n + 1):
        assert np.array_equal(bits(got[k]), bits(coeffs_o[k])), k
    if aliased:
        assert np.array_equal(bits(d_in.get()), bits(after_o))
    d_out = s.array(shape=(h, w))
    s.rdl.rdl_iuwt_recompose(s.h, d_coeffs.vp, w, h, n, int(include_largest), d_out.vp)
    expect = iuwt_recompose(orc, coeffs_o, n, include_largest)
    assert np.array_equal(bits(d_out.get()), bits(expect))
    for x in {id(a): a for a in (d_in, d_scratch, d_coeffs, d_out)}.values():
        x.free()
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n", [(4096, 4096, 6), (1000, 37, 6), (8192, 64, 6),
                                   (260, 300, 7), (2048, 1500, 8)])
@pytest.mark.parametrize("include_largest", [True, False])
@pytest.mark.parametrize("mode", ["2", "3", "1"])
def test_gpu_iuwt_fused_equal_four_pass(w, h, n, include_largest, mode):
    """The fused kernels against the four-pass kernels (RDL_IUWT_FUSED=0),
    bit for bit: mode 2 (the default) the fused row decomposition
    (IuwtDecomposeRows, the intermediate row in LDS) and the row-chain
    recomposition (IuwtRecomposeChain: one launch per scale, five filtered
    rows per chain in LDS), mode 3 the row chains for the decomposition too
    (IuwtDecomposeChain), mode 1 the fused rows with the four-pass
    recomposition; at the C4 size, at
    heights and widths below the larger spacings (d = 63, 127, 255 against 37,
    64, 260 and 300 rows) and with partial column strips."""
    from rdl_lib import Session
    img = image(w, h, 77)
    s = Session(0)
    outs = []
    for fused in (mode, "0"):
        os.environ["RDL_IUWT_FUSED"] = fused
        try:
            d_in, d_scratch = s.array(img), s.array(shape=(h, w))
            d_coeffs = s.array(shape=(n + 1, h, w))
            d_out = s.array(shape=(h, w))
            s.rdl.rdl_iuwt_decompose(s.h, d_in.vp, d_scratch.vp, w, h, n, d_coeffs.vp,
                                     int(include_largest))
            s.rdl.rdl_iuwt_recompose(s.h, d_coeffs.vp, w, h, n, int(include_largest),
                                     d_out.vp)
            outs.append((d_coeffs.get(), d_out.get(), d_in.get()))
            for x in (d_in, d_scratch, d_coeffs, d_out):
                x.free()
        finally:
            del os.environ["RDL_IUWT_FUSED"]
    s.close()
    for k in range(n + 1):
        assert np.array_equal(bits(outs[0][0][k]), bits(outs[1][0][k])), k
    assert np.array_equal(bits(outs[0][1]), bits(outs[1][1]))
    assert np.array_equal(bits(outs[0][2]), bits(img))  # the input is not written


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n", [(4096, 512, 6), (1000, 37, 6), (260, 300, 7), (64, 64, 3)])
def test_gpu_iuwt_aliased_recurrences_equal_row_kernel(w, h, n):
    """The aliased decomposition (input as its own scratch, as the IUWT
    deconvolution calls it): its first horizontal pass is a recursive
    in-place filter. The recurrence kernel (IuwtHorizontalInPlaceChains, one
    thread per row and residue, taps in registers) against the
    one-thread-per-row kernel (RDL_IUWT_FUSED=0), bit for bit, including the
    overwritten input."""
    from rdl_lib import Session
    img = image(w, h, 91)
    s = Session(0)
    outs = []
    for fused in ("2", "0"):
        os.environ["RDL_IUWT_FUSED"] = fused
        try:
            d_in = s.array(img)
            d_coeffs = s.array(shape=(n + 1, h, w))
            s.rdl.rdl_iuwt_decompose(s.h, d_in.vp, d_in.vp, w, h, n, d_coeffs.vp, 0)
            outs.append((d_coeffs.get(), d_in.get()))
            for x in (d_in, d_coeffs):
                x.free()
        finally:
            del os.environ["RDL_IUWT_FUSED"]
    s.close()
    for k in range(n + 1):
        assert np.array_equal(bits(outs[0][0][k]), bits(outs[1][0][k])), k
    assert np.array_equal(bits(outs[0][1]), bits(outs[1][1]))
