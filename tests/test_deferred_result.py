"""The multiscale outer loop reads each sub-minor loop's result only after
queuing the work that does not depend on it (the residual correction, the
model update, the next peak searches; rdl_subminor_launch / _collect,
multiscale_algorithm.cc:436-462, 521-524) whenever no component trace is
recorded — the Radler.perform path. With a trace it reads the result first.
Same operations in the same stream order: the two must give bit-identical
residuals, models and component counts (C2 problem, 4096^2, 6 scales)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_deferred_loop_result_matches_synchronous():
    from radler_import import radler as rd
    import config_problems as cp
    from test_configs_gpu import settings
    psfs, dirty = cp.problem("c2")
    out = []
    for trace in (True, False):  # synchronous (trace), then deferred
        run = rd.gpu.DeviceRun(settings(rd, "c2"), psfs[0], dirty[0], [],
                               cp.BEAM_PX * cp.PIXEL_SCALE, trace=trace)
        r = run.execute()
        out.append((r["iterations"], r["another_iteration_required"], run.residual(),
                    run.model()))
        del run
    assert out[0][0] == out[1][0] > 0
    assert out[0][1] == out[1][1]
    assert np.array_equal(out[0][2], out[1][2])
    assert np.array_equal(out[0][3], out[1][3])


CHILD = r"""
import sys
sys.path.insert(0, {here!r})
import numpy as np
from radler_import import radler as rd
from config_problems import joined_channels
from synthetic import problem
case = {case!r}
pixel = 1.0 / 3600.0 * np.pi / 180.0
s = rd.Settings()
s.algorithm_type = rd.AlgorithmType.multiscale
s.pixel_scale.x = s.pixel_scale.y = pixel
s.minor_iteration_count = 3000
s.absolute_threshold = 2e-3
s.border_ratio = 0.0
s.multiscale.max_scales = 4
s.auto_mask_sigma = 4.0          # tracked per-scale masks (multiscale_algorithm.cc:214-226)
if case == "joined":
    w = 256
    freqs = [100e6 + 10e6 * i for i in range(4)]
    psf, dirty = joined_channels(w, 40, 4, seed=31, frequencies=freqs)
    extra = dict(n_deconvolution_groups=4,
                 frequencies=np.array([[f, f] for f in freqs], np.float64),
                 weights=np.ones(4, np.float64))
else:  # the concurrent subimage pool
    w = 512
    psf, dirty = problem(w, w, 60, 6, seed=32)
    s.parallel.grid_width = s.parallel.grid_height = 3
    s.parallel.max_threads = 4
    extra = {{}}
s.trimmed_image_width = s.trimmed_image_height = w
res, mod = dirty.copy(), np.zeros_like(dirty)
r = rd.Radler(s, psf, res, mod, 2.0 * pixel, **extra)
flags = []
for major in range(4):
    flags.append(r.perform(major))
np.savez({out!r}, residual=res, model=mod, flags=np.array(flags),
         iterations=np.int64(r.iteration_number))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["joined", "pool"])
def test_deferred_result_joined_and_pool_with_masks(tmp_path, case):
    """the deferred loop result (the Radler.perform path) against
    the synchronous one (RDL_SUBMINOR_DEFER=0, read once per process: child
    processes) on a joined 4-channel set and on the concurrent subimage pool,
    both with auto-masking's tracked per-scale masks, over four major
    iterations (the mask phases of radler.cc:162-316): bit-identical images,
    flags and iteration counts."""
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    outs = []
    for defer in ("1", "0"):
        out = str(tmp_path / f"{case}_{defer}.npz")
        env = dict(os.environ, RDL_SUBMINOR_DEFER=defer)
        p = subprocess.run([sys.executable, "-c", CHILD.format(here=here, case=case, out=out)],
                           env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-4000:]
        outs.append(dict(np.load(out)))
    for key in ("residual", "model", "flags", "iterations"):
        assert np.array_equal(outs[0][key], outs[1][key]), key
    assert outs[0]["iterations"] > 0
