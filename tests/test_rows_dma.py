"""The LDS-DMA row kernels (ff::RowsInverseDma / RowsForwardDma: the next
row fetched by global_load_lds while this row is transformed) against the
persistent row kernels they replace (RDL_ROWS_DMA=0): the same arithmetic,
so the spectra and images are bit-identical and the fused peak searches
return the same peaks. The switch is read once per process, so each side
runs in its own process (one at a time)."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = r"""
import ctypes as C, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from rdl_lib import Session
out_path, w, h = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])

class Peak(C.Structure):
    _fields_ = [("value", C.c_float), ("x", C.c_uint32), ("y", C.c_uint32), ("found", C.c_int32)]

s = Session(0)
c = C.c_void_p()
s.rdl.rdl_conv_create_ex(s.h, w, h, 0, 1, C.byref(c))
assert s.rdl.lib.rdl_conv_fast(c) & 4
nb = s.rdl.lib.rdl_conv_spectrum_bytes(c)
rng = np.random.default_rng(w + 3 * h)
img = rng.standard_normal((h, w)).astype(np.float32)
img[h // 3, w // 5] = 40.0
img[h // 2, w // 2] = -55.0
di = s.array(img)
spec = s.array(shape=(nb // 8,), dtype=np.complex64)
work = s.array(shape=(nb // 8,), dtype=np.complex64)
s.rdl.rdl_conv_rows_forward(c, di.vp, w, h, 0, 0, spec.vp)
res = {"rows_spectrum": spec.get()}
s.rdl.rdl_conv_forward(c, di.vp, spec.vp)
for neg in (0, 1):
    out = s.array(shape=(h, w))
    s.rdl.rdl_memcpy_d2d(s.h, work.vp, spec.vp, C.c_size_t(nb))
    s.rdl.rdl_conv_rows_inverse_peak(c, work.vp, out.vp, w, h, 0, 0, 17, 9, neg, None, 0)
    p = (Peak * 1)()
    s.rdl.rdl_find_peak_collect(s.h, 1, p)
    res[f"img{neg}"] = out.get()
    res[f"peak{neg}"] = np.array([p[0].value, p[0].x, p[0].y, p[0].found], np.float64)
    out.free()
np.savez(out_path, **res)
"""


def run_side(tmp_path, w, h, dma):
    path = str(tmp_path / f"rows_{w}_{h}_{dma}.npz")
    env = dict(os.environ, RDL_ROWS_DMA="1" if dma else "0")
    r = subprocess.run([sys.executable, "-c", CHILD, HERE, path, str(w), str(h)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(path)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(8192, 8192), (4096, 4096)])
def test_rows_dma_bit_identical(tmp_path, w, h):
    a = run_side(tmp_path, w, h, True)
    b = run_side(tmp_path, w, h, False)
    # the forward rows (RowsForwardDma) of the whole plane
    assert np.array_equal(a["rows_spectrum"].view(np.uint32), b["rows_spectrum"].view(np.uint32))
    for neg in (0, 1):
        ia, ib = a[f"img{neg}"], b[f"img{neg}"]
        assert np.array_equal(ia.view(np.uint32), ib.view(np.uint32)), neg
        assert np.array_equal(a[f"peak{neg}"], b[f"peak{neg}"]), (a[f"peak{neg}"], b[f"peak{neg}"])
