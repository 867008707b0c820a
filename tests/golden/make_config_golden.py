"""Oracle fixtures for the five BASELINE.json configurations at their stated
sizes (tests/config_problems.py), for tests/test_configs_gpu.py:

    make -C oracle && python tests/golden/make_config_golden.py [c1 c2 ...]

Each tests/golden/config_<name>.npz holds the SHA-256 of the regenerated
inputs, the oracle's component trace (or IUWT step records) with the
decision margins of every component (tests/trace_compare.py), and checksums
plus a fixed random sample of the oracle's residual and model. The inputs
themselves are not stored: both machines regenerate them from seeds.
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import config_problems as cp  # noqa: E402
from oracle_lib import OracleAlgorithm, OracleParallel, get_oracle  # noqa: E402

SAMPLE = 65536
THREADS = int(os.environ.get("ORACLE_THREADS", os.cpu_count() or 8))


def sample_index(n_pixels, seed=1):
    return np.sort(np.random.default_rng(seed).choice(n_pixels, SAMPLE, replace=False))


def image_summary(prefix, planes):
    planes = np.ascontiguousarray(planes, np.float32)
    n = planes.shape[-1] * planes.shape[-2]
    idx = sample_index(n)
    flat = planes.reshape(-1, n)
    return {f"{prefix}_sha256": cp.sha256(planes),
            f"{prefix}_sample": flat[:, idx],
            f"{prefix}_absmax": np.abs(flat).max(axis=1),
            f"{prefix}_rms": np.sqrt(np.mean(flat.astype(np.float64) ** 2, axis=1)),
            f"{prefix}_sum": flat.astype(np.float64).sum(axis=1)}


def settings(c):
    st = dict(threshold=c["threshold"], border_ratio=0.0, minor_loop_gain=0.1,
              major_loop_gain=1.0, allow_negative=1)
    if c["kind"] == "hogbom":
        st.update(max_iterations=c["max_iterations"], use_sub_minor=0)
    elif c["kind"] == "iuwt":
        st.update(max_iterations=c["cap"])
    else:
        st.update(max_iterations=c["cap"], max_scales=c["max_scales"],
                  beam_size_in_pixels=cp.BEAM_PX)
    return st


def make(name):
    c = cp.CONFIGS[name]
    t0 = time.time()
    psfs, dirty = cp.problem(name)
    out = {"psf_sha256": cp.sha256(psfs), "dirty_sha256": cp.sha256(dirty),
           "dirty_absmax": np.float32(np.abs(dirty).max())}
    print(f"{name}: inputs {dirty.shape} in {time.time() - t0:.1f} s", flush=True)
    orc = get_oracle()
    orc.set_threads(THREADS)
    res, mod = dirty.copy(), np.zeros_like(dirty)
    t0 = time.time()
    if c["kind"] == "tiled":
        par = OracleParallel(orc, 1, c["grid"], c["grid"], **settings(c))
        par.set_snapshot(bool(c.get("snapshot", False)))
        r, boxes, labels, trace = par.execute(res, mod, psfs, 1.0)
        m, v = par.margins()
        out.update(boxes=boxes, labels_sha256=cp.sha256(labels), trace=trace,
                   margins=m, values=v, start_peak=r.start_peak, end_peak=r.end_peak,
                   total_iterations=r.total_iterations,
                   first_iteration_number=r.first_iteration_number,
                   another_iteration_required=r.another_iteration_required)
    else:
        kind = {"hogbom": 0, "multiscale": 1, "joined": 1, "iuwt": 2}[c["kind"]]
        alg = OracleAlgorithm(orc, kind, **settings(c))
        r, trace = alg.execute(res, mod, psfs)
        out.update(trace=trace, iteration_number=r.iteration_number,
                   final_peak=r.final_peak,
                   another_iteration_required=r.another_iteration_required)
        if kind == 1:
            m, v = alg.margins()
            out.update(margins=m, values=v)
        if kind == 2:
            steps = alg.iuwt_steps()
            out.update(steps=steps.view(np.uint8).reshape(len(steps), -1),
                       n_steps=len(steps))
    print(f"{name}: oracle {time.time() - t0:.1f} s, trace {len(out['trace'])}",
          flush=True)
    out.update(image_summary("residual", res))
    out.update(image_summary("model", mod))
    if c["kind"] == "hogbom":  # sparse model, exact
        nz = np.flatnonzero(mod.reshape(-1))
        out.update(model_index=nz.astype(np.int64), model_value=mod.reshape(-1)[nz])
    out["oracle_seconds"] = np.float64(time.time() - t0)
    path = os.path.join(HERE, f"config_{name}.npz")
    np.savez_compressed(path, **out)
    if "image_cap" in c:
        checkpoint(name)
    if "image_cap2" in c:
        checkpoint(name, "image_cap2", "ck2_")


RTOL = 1e-6  # tests/test_configs_gpu.py


def first_near_tie(fx, rtol=RTOL):
    """Index of the fixture's first component whose oracle decision margin is
    below rtol x |peak| (tests/test_configs_gpu.py min_prefix): the GPU trace
    is required to be identical up to there, so an image checkpoint at this
    count is comparable pixel for pixel whatever the GPU's rounding."""
    r = fx["margins"] / np.maximum(np.abs(fx["values"]), 1e-30)
    near = np.flatnonzero(r < rtol)
    return int(near[0]) if len(near) else len(fx["trace"])


def checkpoint(name, key="image_cap", prefix="ck_"):
    """Add the image checkpoint (`ck_*` keys; `ck2_*` for image_cap2) to an
    existing fixture: the oracle rerun with max_iterations = image_cap from
    the same inputs; its trace is the full run's prefix (checked here).
    image_cap "near_tie" puts the checkpoint at the fixture's first
    near-tie."""
    c = cp.CONFIGS[name]
    path = os.path.join(HERE, f"config_{name}.npz")
    out = dict(np.load(path))
    psfs, dirty = cp.problem(name)
    assert cp.sha256(dirty) == str(out["dirty_sha256"])
    orc = get_oracle()
    orc.set_threads(THREADS)
    res, mod = dirty.copy(), np.zeros_like(dirty)
    st = settings(c)
    cap = c[key]
    if cap == "near_tie":
        cap = first_near_tie(out)
    st["max_iterations"] = cap
    t0 = time.time()
    alg = OracleAlgorithm(orc, 1, **st)
    r, trace = alg.execute(res, mod, psfs)
    n = len(trace)
    assert n == r.iteration_number == cap, (n, r.iteration_number)
    assert np.array_equal(trace, out["trace"][:n]), "checkpoint trace is not the full prefix"
    print(f"{name}: checkpoint at {n} components, oracle {time.time() - t0:.1f} s", flush=True)
    out[f"{prefix}iterations"] = np.int64(n)
    out.update({f"{prefix}{k}": v for k, v in image_summary("residual", res).items()})
    out.update({f"{prefix}{k}": v for k, v in image_summary("model", mod).items()})
    np.savez_compressed(path, **out)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args[:1] == ["--checkpoint"]:
        for name in args[1:]:
            checkpoint(name)
    elif args[:1] == ["--checkpoint2"]:
        for name in args[1:]:
            checkpoint(name, "image_cap2", "ck2_")
    else:
        # (t2k is bench.py's live to-threshold problem: no fixture)
        for name in args or [n for n, c in cp.CONFIGS.items()
                             if "cap" in c or "max_iterations" in c]:
            make(name)
