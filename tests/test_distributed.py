"""Process-per-GPU split of ParallelDeconvolution.

Subimage i runs on rank i mod N from the pass-start residual; the start peak
is the max-allreduce of the ranks' local maxima; every finished subimage's
residual/model boxes are broadcast by their owner and merged by all ranks in
subimage order (cpp/algorithms/parallel_deconvolution.cc:556-654). The result
must not depend on N: it equals the one-process run in snapshot order (the
oracle's `set_snapshot(True)` mode, and the concurrent subimage pool).

CPU (gloo, world 2): the host communicator plumbing (broadcast of a host
buffer, max) and the static ownership.
GPU (gloo, world 2 and 3, all ranks on cuda:0): distributed tiled runs vs the
oracle (same tiles, per-subimage traces identical, residual/model within
2e-5 * max|dirty|) and vs each other (bit-identical on every rank), for one
field and for joined channels (4 and 8 channels, the C3 image set split by
subimage).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle_lib import OracleAlgorithm, OracleParallel, get_oracle
from synthetic import problem

# the residual/model agreement of tests/test_configs_gpu.py (x max|dirty|)
IMG_TOL = 1e-6

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(tmp_path, world, case, extra=(), timeout=240):
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"),
                               "--rank", str(r), "--world", str(world), "--port", str(port),
                               "--out", str(tmp_path), "--case", case, *extra],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            logs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-4000:]
    return [dict(np.load(os.path.join(tmp_path, f"rank{r}.npz"))) for r in range(world)]


def test_subimage_owner_round_robin():
    from radler_import import radler as rd
    owner = rd.distributed.subimage_owner
    assert [owner(i, 1) for i in range(5)] == [0] * 5
    assert [owner(i, 3) for i in range(7)] == [0, 1, 2, 0, 1, 2, 0]


def test_lpt_owners():
    """Cost-ordered ownership of the cleaning pass: deterministic, balanced,
    lower index / lower rank first on ties."""
    from radler_import import radler as rd
    lpt = rd.distributed.lpt_owners
    assert lpt([5.0, 1.0, 1.0], 1) == [0, 0, 0]
    assert lpt([1.0, 1.0, 1.0, 1.0], 2) == [0, 1, 0, 1]
    # 8 on rank 0; 5 and 3 share rank 1 (8 = 5 + 3); 2 goes to rank 0
    assert lpt([3.0, 8.0, 5.0, 2.0], 2) == [1, 0, 1, 0]
    rng = np.random.default_rng(5)
    costs = list(rng.uniform(1, 100, 64))
    owners = lpt(costs, 8)
    assert owners == lpt(costs, 8)
    loads = np.zeros(8)
    for c, o in zip(costs, owners):
        loads[o] += c
    # LPT is within 4/3 of optimal; the mean is a lower bound for the optimum
    assert loads.max() <= 4.0 / 3.0 * max(loads.mean(), max(costs))


def test_host_communicator_gloo_world2(tmp_path):
    outs = _launch(tmp_path, 2, "host")
    expect = ((np.arange(1 << 16) * 7 + 3) % 251).astype(np.uint8)
    for o in outs:
        assert np.array_equal(o["bcast"], expect)
        assert o["max"] == np.float32(1.5 - 7.0)
        assert list(o["owners"]) == [0, 1] * 5


@pytest.mark.gpu
@pytest.mark.parametrize("world,kind,w,gw,gh,channels", [
    (2, 1, 256, 2, 2, 1), (3, 1, 320, 3, 2, 1), (2, 0, 192, 2, 2, 1),
    # joined channels split by subimage over the ranks
    (2, 1, 256, 2, 2, 4), (3, 1, 256, 3, 2, 8),
    (1, 1, 256, 3, 2, 8), (2, 1, 256, 3, 2, 8), (3, 1, 256, 3, 2, 4), (3, 1, 256, 3, 2, 1)])
def test_distributed_tiled_matches_oracle_snapshot(tmp_path, world, kind, w, gw, gh, channels):
    from dist_worker import tiled_problem
    majors = 2
    outs = _launch(tmp_path, world, "tiled",
                   ["--kind", str(kind), "--size", str(w), "--grid", str(gw), str(gh),
                    "--majors", str(majors), "--channels", str(channels)])
    h = w
    psf, dirty = tiled_problem(w, gw, channels)
    if channels == 1:
        psf, dirty = psf[None], dirty[None]
    thr, max_iter, mgain = 4e-3, 1500, 0.5
    orc = get_oracle()
    orc.set_threads(8)
    st = dict(threshold=thr, max_iterations=max_iter, border_ratio=0.0,
              major_loop_gain=mgain)
    if kind == 1:
        st.update(max_scales=4, beam_size_in_pixels=2.0)
    par = OracleParallel(orc, kind, gw, gh, **st)
    par.set_snapshot(True)
    res_o, mod_o = dirty.copy(), np.zeros((channels, h, w), np.float32)
    prev = 0
    tol = IMG_TOL * np.abs(dirty).max()
    for major in range(majors):
        r_o, _, _, trace_o = par.execute(res_o, mod_o, psf, mgain)
        # every rank holds the same merged images and counters
        for o in outs[1:]:
            assert np.array_equal(o[f"residual{major}"], outs[0][f"residual{major}"])
            assert np.array_equal(o[f"model{major}"], outs[0][f"model{major}"])
            assert o[f"iterations{major}"] == outs[0][f"iterations{major}"]
            assert o[f"another{major}"] == outs[0][f"another{major}"]
        owners = outs[0][f"owners{major}"]
        for o in outs[1:]:  # every rank computed the same LPT ownership
            assert np.array_equal(o[f"owners{major}"], owners)
        for i in range(gw * gh):
            t_o = trace_o[trace_o[:, 0] == i][:, 1:]
            t_g = outs[int(owners[i])][f"trace{major}_{i}"]
            assert np.array_equal(t_g if kind == 1 else t_g[:, :2],
                                  t_o if kind == 1 else t_o[:, :2]), (major, i)
        assert int(outs[0][f"iterations{major}"]) == r_o.total_iterations - prev
        prev = r_o.total_iterations
        assert bool(outs[0][f"another{major}"]) == bool(r_o.another_iteration_required)
        dr = np.abs(outs[0][f"residual{major}"].reshape(res_o.shape) - res_o).max()
        dm = np.abs(outs[0][f"model{major}"].reshape(mod_o.shape) - mod_o).max()
        print(f"major {major}: residual {dr:.3g}, model {dm:.3g} (tolerance {tol:.3g})")
        assert dr <= tol and dm <= tol, (dr, dm, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("world,channels", [(2, 8), (3, 8), (2, 4)])
def test_channel_sharded_joined_equals_one_process(tmp_path, world, channels):
    """SURVEY.md 8(e) C3 as the reference computes it: ONE joined image set
    (grid 1 x 1), its per-channel residual corrections and model updates
    shared by the ranks (image i on rank i % world), the integrated-image
    work on every rank, corrected planes broadcast from their owners. Every
    rank ends with the same images, bit-identical to the one-process run, and
    the component traces are the oracle's unsplit joined run's
    (image_set.cc:423-462 integration, multiscale_algorithm.cc:323-543)."""
    majors = 2
    extra = ["--size", "256", "--majors", str(majors), "--channels", str(channels)]
    (tmp_path / "one").mkdir()
    (tmp_path / "many").mkdir()
    one = _launch(tmp_path / "one", 1, "channels", extra)[0]
    outs = _launch(tmp_path / "many", world, "channels", extra)
    from dist_worker import tiled_problem
    psf, dirty = tiled_problem(256, 1, channels)
    orc = get_oracle()
    orc.set_threads(8)
    alg = OracleAlgorithm(orc, 1, threshold=4e-3, max_iterations=1500, border_ratio=0.0,
                          major_loop_gain=0.5, max_scales=4, beam_size_in_pixels=2.0)
    res_o, mod_o = dirty.copy(), np.zeros_like(dirty)
    tol = IMG_TOL * np.abs(dirty).max()
    for major in range(majors):
        r_o, trace_o = alg.execute(res_o, mod_o, psf)
        for o in outs:
            for key in ("residual", "model", "trace", "iterations", "another"):
                assert np.array_equal(o[f"{key}{major}"], one[f"{key}{major}"]), (major, key)
        assert np.array_equal(one[f"trace{major}"], trace_o), major
        assert bool(one[f"another{major}"]) == bool(r_o.another_iteration_required)
        dr = np.abs(one[f"residual{major}"].reshape(res_o.shape) - res_o).max()
        dm = np.abs(one[f"model{major}"].reshape(mod_o.shape) - mod_o).max()
        print(f"world {world}, {channels} channels, major {major}: "
              f"{len(trace_o)} components identical to the oracle; residual {dr:.3g}, "
              f"model {dm:.3g} (tolerance {tol:.3g})")
        assert dr <= tol and dm <= tol, (dr, dm, tol)


@pytest.mark.gpu
def test_rccl_communicator_single_rank():
    """The RCCL transport (rdl_comm_init/allreduce/broadcast) on one rank: the
    distributed path with itself as the only owner equals the oracle's
    snapshot run."""
    from radler_import import radler as rd
    from dist_worker import PIXEL_SCALE, tiled_settings
    w, gw, gh, kind = 256, 2, 2, 1
    psf, dirty = problem(w, w, 40, 4, seed=w + gw)
    thr, max_iter, mgain = 4e-3, 1500, 0.9
    comm = rd.distributed.RcclCommunicator(0, 1, 0, rd.distributed.rccl_unique_id())
    assert (comm.rank, comm.size) == (0, 1)
    s = tiled_settings(rd, kind, w, thr, max_iter, mgain, gw, gh)
    run = rd.gpu.DeviceRun(s, psf, dirty, [], 2.0 * PIXEL_SCALE)
    run.set_communicator(comm)
    r = run.execute()
    par = OracleParallel(get_oracle(), kind, gw, gh, threshold=thr, max_iterations=max_iter,
                         border_ratio=0.0, major_loop_gain=mgain, max_scales=4,
                         beam_size_in_pixels=2.0)
    par.set_snapshot(True)
    res_o, mod_o = dirty[None].copy(), np.zeros((1, w, w), np.float32)
    r_o, _, _, trace_o = par.execute(res_o, mod_o, psf[None], mgain)
    assert r["iterations"] == r_o.total_iterations
    for i in range(gw * gh):
        assert np.array_equal(run.trace(i), trace_o[trace_o[:, 0] == i][:, 1:])
    tol = IMG_TOL * np.abs(dirty).max()
    assert np.abs(run.residual().reshape(w, w) - res_o[0]).max() <= tol
    assert np.abs(run.model().reshape(w, w) - mod_o[0]).max() <= tol
    del run
