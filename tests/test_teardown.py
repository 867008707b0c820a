"""Process teardown and the session's single sub-minor result slot.

* rdl_shutdown (include/rdl_hip.h) runs from an atexit handler registered by
  the first rdl_session_create, i.e. before the HIP runtime's own exit
  handlers: every process-lifetime session (the per-GPU session, the subimage
  pool's workers), block cache, plan and mapped host buffer is released while
  the runtime is whole. Checked in child processes that exit with live
  sessions, buffers and worker pools.
* A session keeps ONE mapped loop-result slot: while one rdl_subminor handle
  has a launched, uncollected loop, another handle of the same session may
  not launch (it would overwrite the pending result); the first handle's
  collect still returns its own result.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

CHILD_RAW = r"""
import ctypes as C, sys
sys.path.insert(0, {here!r})
import numpy as np
from rdl_lib import Session
s = Session(0)
a = s.array(np.arange(1 << 20, dtype=np.float32))
s.find_peak(a, 1024, 1024)
# exit with the session, its buffer and its caches alive
print("child done", flush=True)
"""

CHILD_POOL = r"""
import sys
sys.path.insert(0, {here!r})
import numpy as np
from radler_import import radler as rd
from synthetic import problem
psf, dirty = problem(256, 256, 12, 2, seed=5)
s = rd.Settings()
s.algorithm_type = rd.AlgorithmType.multiscale
s.trimmed_image_width = s.trimmed_image_height = 256
s.pixel_scale.x = s.pixel_scale.y = 1.0 / 3600.0 * np.pi / 180.0
s.minor_iteration_count = 200
s.absolute_threshold = 1e-3
s.parallel.grid_width = s.parallel.grid_height = 2
s.parallel.max_threads = 4
res, mod = dirty.copy(), np.zeros_like(dirty)
r = rd.Radler(s, psf, res, mod, 2.0 * s.pixel_scale.x)
r.perform(0)
print("child done", r.iteration_number, flush=True)
# the Radler object, the process-wide session and 4 worker sessions stay
# alive until exit
"""


def _run_child(code, extra_env=None):
    env = dict(os.environ, RDL_SHUTDOWN_LOG="1")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "-c", code.format(here=HERE)], env=env,
                          capture_output=True, text=True, timeout=300)


@pytest.mark.gpu
@pytest.mark.parametrize("child", ["raw", "pool"])
def test_exit_releases_everything(child):
    p = _run_child(CHILD_RAW if child == "raw" else CHILD_POOL)
    print(p.stdout, p.stderr[-2000:])
    assert p.returncode == 0, p.stderr[-4000:]
    assert "child done" in p.stdout
    line = [ln for ln in p.stderr.splitlines() if "[rdl] shutdown:" in ln]
    assert len(line) == 1, p.stderr[-4000:]
    n_sessions = int(line[0].split("shutdown:")[1].split("sessions")[0])
    n_blocks = int(line[0].split(",")[1].split("blocks")[0])
    assert n_sessions >= (1 if child == "raw" else 5)
    assert n_blocks > 0


@pytest.mark.gpu
def test_exit_without_shutdown_still_supported():
    """RDL_EXIT_SHUTDOWN=0 leaves teardown to the runtime (the r05 behaviour)."""
    p = _run_child(CHILD_RAW, {"RDL_EXIT_SHUTDOWN": "0"})
    assert p.returncode == 0, p.stderr[-4000:]
    assert "[rdl] shutdown:" not in p.stderr


@pytest.mark.gpu
def test_interleaved_handles_keep_their_results():
    from rdl_lib import RdlError, Session, SubminorParams, SubminorResult, integration
    from synthetic import problem
    w = h = 256
    psf, dirty = problem(w, h, 20, 2, seed=11)
    sess = Session(0)
    dpsf = sess.array(psf)

    def params(max_iter):
        p = SubminorParams()
        p.width, p.height, p.n_images, p.n_pol = w, h, 1, 1
        p.integ = integration(1, 1, mode=0)
        p.allow_negative, p.stop_on_negative = 1, 0
        p.threshold = np.float32(0.2 * np.abs(dirty).max())
        p.gain, p.divergence_limit = 0.1, 4.0
        p.iteration_start, p.max_iterations = 0, max_iter
        return p

    # the reference result of each loop, run alone
    ref = []
    for max_iter in (37, 91):
        sm = C.c_void_p()
        sess.rdl.rdl_subminor_create(sess.h, C.byref(sm))
        dres = sess.array(dirty)
        out = SubminorResult()
        p = params(max_iter)
        sess.rdl.rdl_subminor_run(sm, dres.vp, dpsf.vp, C.byref(p), C.byref(out), None,
                                  C.c_uint64(0))
        ref.append((out.iteration, out.peak, out.flux_cleaned))
        sess.rdl.rdl_subminor_destroy(sm)
        dres.free()
    assert ref[0][0] == 37 and 37 < ref[1][0] <= 91  # (91: capped or at the threshold)

    a, b = C.c_void_p(), C.c_void_p()
    sess.rdl.rdl_subminor_create(sess.h, C.byref(a))
    sess.rdl.rdl_subminor_create(sess.h, C.byref(b))
    ra, rb = sess.array(dirty), sess.array(dirty)
    pa, pb = params(37), params(91)
    oa, ob = SubminorResult(), SubminorResult()
    sess.rdl.rdl_subminor_launch(a, ra.vp, dpsf.vp, C.byref(pa), C.byref(oa))
    with pytest.raises(RdlError, match="not collected"):
        sess.rdl.rdl_subminor_launch(b, rb.vp, dpsf.vp, C.byref(pb), C.byref(ob))
    with pytest.raises(RdlError, match="not collected"):
        sess.rdl.rdl_subminor_run(b, rb.vp, dpsf.vp, C.byref(pb), C.byref(ob), None,
                                  C.c_uint64(0))
    sess.rdl.rdl_subminor_collect(a, C.byref(oa))
    assert (oa.iteration, oa.peak, oa.flux_cleaned) == ref[0]
    # once A is collected, B launches and gets its own result
    sess.rdl.rdl_subminor_launch(b, rb.vp, dpsf.vp, C.byref(pb), C.byref(ob))
    sess.rdl.rdl_subminor_collect(b, C.byref(ob))
    assert (ob.iteration, ob.peak, ob.flux_cleaned) == ref[1]
    for hnd in (a, b):
        sess.rdl.rdl_subminor_destroy(hnd)
    for x in (ra, rb, dpsf):
        x.free()
    sess.close()
