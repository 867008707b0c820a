"""pytest plugin: after every GPU test, run the divergence KAT (tools/
diag_divergence.kat) a few times in the same process and log any failing
boxes with the test that ran just before, to find which process state makes
test_divergence_kat fail.  Use: PYTHONPATH=tools pytest -p kat_probe_plugin ...
"""
import os
import sys

import pytest

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _HERE)
LOG = os.environ.get("KAT_PROBE_LOG", "gpurun_out/kat_probe.log")
REPS = int(os.environ.get("KAT_PROBE_REPS", "3"))


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_teardown(item, nextitem):
    yield
    if item.get_closest_marker("gpu") is None:
        return
    import diag_divergence as dd
    sys.path.insert(0, os.path.join(dd.ROOT, "ska-sdp-func-radler_amd"))
    import radler as rd
    lines = []
    for r in range(REPS):
        try:
            fails, n = dd.kat(rd)
        except Exception as e:  # noqa: BLE001
            fails, n = [("error", repr(e))], -1
        if fails or n != 48:
            lines.append(f"FAIL after {item.nodeid} rep {r}: n={n} boxes={fails[:8]}")
    lines.append(f"probe after {item.nodeid}: {'FAIL' if len(lines) else 'ok'}")
    with open(LOG, "a") as f:
        f.write("\n".join(lines) + "\n")
