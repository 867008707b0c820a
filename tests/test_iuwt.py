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
@pytest.mark.parametrize("w,h", [(4096, 4096), (1000, 37), (8192, 64)])
@pytest.mark.parametrize("include_largest", [True, False])
def test_gpu_iuwt_fused_rows_equal_four_pass(w, h, include_largest):
    """The fused decomposition (r06: IuwtDecomposeRows, the intermediate row
    in LDS, approximation planes alternating instead of copied, float4 tap
    rows) against the four-pass kernels (RDL_IUWT_FUSED=0), bit for bit, at
    the C4 size and at widths / heights below the larger spacings; the
    recomposition is the same kernels either way."""
    from rdl_lib import Session
    n = 6
    img = image(w, h, 77)
    s = Session(0)
    outs = []
    for fused in ("1", "0"):
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
    assert np.array_equal(bits(outs[0][0]), bits(outs[1][0]))
    assert np.array_equal(bits(outs[0][1]), bits(outs[1][1]))
    assert np.array_equal(bits(outs[0][2]), bits(img))  # the input is not written
