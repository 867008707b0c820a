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
