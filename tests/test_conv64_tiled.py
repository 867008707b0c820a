"""CorrectResidualDirty's padded float64 convolve-and-subtract
(rdl_conv_convolve_subtract; subminor_loop.cc:199-216) with its spectrum in
the tiled layout (the default on float64 convolution-column plans) against
the row-major passes it replaces (RDL_CONV64_TILED=0): the same kernels and
arithmetic with other addresses, so the residuals are bit-identical. Masked
(sparse model rows) and unmasked, float64 and float kernel spectra, a
1 024-thread (9072) and a 512-thread (4536) column plan. The layout switch is
read once per process, so each side runs in its own process."""
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
out_path, n, img = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
s = Session(0)
lib = s.rdl.lib
lib.rdl_conv_convolve_subtract_bytes.restype = C.c_size_t
lib.rdl_conv_convolve_subtract_bytes.argtypes = [C.c_void_p]
c = C.c_void_p()
s.rdl.rdl_conv_create_ex(s.h, n, n, 1, 0, C.byref(c))
assert lib.rdl_conv_fast(c) & 8, "no float64 convolution-column plan"
nc = n // 2 + 1
work = s.array(shape=(lib.rdl_conv_convolve_subtract_bytes(c),), dtype=np.uint8)
rng = np.random.default_rng(n + img)
# a column-major kernel spectrum (column k at k * n), float64 and narrowed
kern = (rng.standard_normal((nc, n)) + 1j * rng.standard_normal((nc, n))).astype(np.complex128)
dk = s.array(kern)
dk32 = s.array(shape=(nc, n), dtype=np.complex64)
s.rdl.rdl_complex_narrow(s.h, dk32.vp, dk.vp, C.c_size_t(nc * n))
ox = oy = (n - img) // 2
model = np.zeros((img, img), np.float32)
rows = rng.choice(img, 300, replace=False)
model[rows, rng.integers(0, img, 300)] = rng.standard_normal(300).astype(np.float32)
mask = np.zeros(n, np.uint8)
mask[rows + oy] = 1
dm, dmask = s.array(model), s.array(mask)
res = {}
for masked in (0, 1):
    for kf in (0, 1):
        r = rng.standard_normal((img, img)).astype(np.float32)
        dr = s.array(r)
        s.rdl.rdl_conv_convolve_subtract(c, dm.vp, img, img, ox, oy, dk32.vp if kf else dk.vp,
                                         1, kf, C.c_double(1.0 / (n * n)),
                                         dmask.vp if masked else None, work.vp, dr.vp)
        res[f"r{masked}{kf}"] = dr.get()
        dr.free()
np.savez(out_path, **res)
"""


def run_side(tmp_path, n, img, tiled):
    path = str(tmp_path / f"cs_{n}_{tiled}.npz")
    env = dict(os.environ, RDL_CONV64_TILED="1" if tiled else "0")
    r = subprocess.run([sys.executable, "-c", CHILD, HERE, path, str(n), str(img)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(path)


@pytest.mark.gpu
@pytest.mark.parametrize("n,img", [(9072, 8192), (4536, 4096)])
def test_convolve_subtract_tiled_bit_identical(tmp_path, n, img):
    a = run_side(tmp_path, n, img, True)
    b = run_side(tmp_path, n, img, False)
    for k in a.files:
        assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k
        assert np.isfinite(a[k]).all()
