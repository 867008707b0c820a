#!/usr/bin/env python3
"""Benchmark: CLEAN components/sec and wall-clock-to-threshold of Radler's
multiscale CLEAN on an 8192^2 synthetic sky (BASELINE.json metric), on the
MI355X-native engine.

`value` / `ms_per_step`: one step = one major iteration of
ParallelDeconvolution -> MultiScaleAlgorithm to the 5-sigma threshold
(major_loop_gain 1) on an image set resident in HBM when the timed region
starts (radler.gpu.DeviceRun: restore the dirty image from its HBM copy +
execute; `device_resident` holds the same numbers). `perform_host_buffers`
times the drop-in API over host buffers: one
`Radler.perform` = load and average the residual/model/PSF through the
work-table accessors (host -> HBM over PCIe), the same major iteration, and
the residual/model stores (HBM -> host); every step gets its own Radler over
its own copy of the dirty image, built before the timed region. The split
workloads (tiled, joined at N > 1) have no resident leg: their `value` is
the Radler.perform rate (config.step names which).

Workloads (--workload):
  fields  one independent 8192^2 field per GPU (weak scaling; N = 1 default)
  tiled   ONE image split into grid x grid subimages (ParallelDeconvolution,
          SURVEY.md C5) shared by the ranks: find-peak pass, one RCCL
          allreduce(max) of the start peak, owner broadcasts of the subimage
          results (strong scaling; N > 1 default, 8192^2 8 x 8)
  joined  the C3 image set (8 channels x 4096^2); at N > 1 one image set
          whose per-channel work (residual corrections, model updates) the
          ranks share by channel, the integrated-image work on every rank
          (--joined-split channels, the default), or the set split into
          subimages shared by the ranks like `tiled` (--joined-split subimages)

At N = 1 the line also carries: tiled_n1 / joined_n1 (the split workloads
and the unsplit C3 run on this GPU), c2_to_threshold, and cpu_baseline with a
live to-threshold run of a smaller problem on the CPU and the GPU
(`--to-threshold-live`, default t2k: 2048^2).

Multi-GPU: one process per GPU. `--gpus N` without a launcher re-launches
itself under torch.distributed.run (before anything touches the GPU); under a
launcher WORLD_SIZE must equal N. Barrier + device sync bracket the timed
region and the slowest rank's time is used; value = components of all ranks /
that time.

Also reported: `roofline` of the dominant kernel family (HIP events on the
stream of every session of the process, algorithmic bytes per SURVEY.md
§8(d)) and `cpu_baseline` = the oracle (C++ restatement, std::thread, float64
FFT) on a bounded sample of the same workload: its cleaning rate after setup,
with all affinity cores and with one, and the setup time separately.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-radler_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PIXEL_SCALE = 1.0 / 3600.0 * np.pi / 180.0  # 1 arcsec
BEAM_PX = 4.0
NOISE = 1e-4
SEED = 20251015


def make_problem(size, seed, n_points, n_blobs, fwhm=4.0):
    from synthetic import make_dirty, make_psf_uv, make_sky
    psf = make_psf_uv(size, size, fwhm=fwhm)
    sky = make_sky(size, size, n_points, n_blobs, seed, flux_range=(1e-3, 1.0),
                   blob_sigma=(2.0, 40.0))
    dirty = make_dirty(psf, sky, NOISE, seed)
    return psf, dirty


def settings_for(rd, size, max_iter, max_scales, threshold, grid, threads):
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.multiscale
    s.trimmed_image_width = s.trimmed_image_height = size
    s.pixel_scale.x = s.pixel_scale.y = PIXEL_SCALE
    s.minor_iteration_count = max_iter
    s.absolute_threshold = threshold
    s.minor_loop_gain = 0.1
    s.major_loop_gain = 1.0
    s.allow_negative_components = True
    s.border_ratio = 0.0
    s.multiscale.max_scales = max_scales
    s.parallel.grid_width = s.parallel.grid_height = grid
    s.parallel.max_threads = threads
    return s


# algorithmic bytes per launch are accumulated by the C-ABI per family
FAMILIES = ["conv_rows", "conv_cols", "conv64_rows", "conv64_cols", "conv_rows_sparse",
            "conv_cols_sparse", "conv64_rows_sparse", "conv64_cols_sparse", "fft", "fft64",
            "spectrum_multiply", "spectrum_multiply64", "find_peak", "subminor_loop",
            "subminor_select", "subminor_table", "trim_subtract", "add", "integrate", "rms", "axpy",
            "radix_select", "iuwt", "box", "stamp_model"]


class Timing:
    """Kernel-family timing over every session of the process
    (rdl_timing_*_all: the main session and a subimage pool's workers)."""

    def __init__(self):
        self.lib = C.CDLL(os.path.join(ROOT, "ska-sdp-func-radler_amd", "lib", "librdl_hip.so"))
        self.lib.rdl_timing_get_all.argtypes = [C.c_char_p, C.POINTER(C.c_double),
                                                C.POINTER(C.c_uint64), C.POINTER(C.c_double)]

    def enable(self, on):
        # RDL_BENCH_EVENTS=0: no HIP event pairs at all (a profiler run of the
        # pooled legs, whose interception of thousands of event records from
        # 16 worker threads faults inside the profiler); no roofline then
        if os.environ.get("RDL_BENCH_EVENTS") == "0":
            return
        self.lib.rdl_timing_enable_all(int(on))

    def only(self, family):
        """Record events for this family only (None: every family)."""
        self.lib.rdl_timing_filter_all(family.encode() if family else None)

    def reset(self):
        self.lib.rdl_timing_reset_all()

    def get(self):
        out = {}
        for fam in FAMILIES:
            ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
            self.lib.rdl_timing_get_all(fam.encode(), C.byref(ms), C.byref(n), C.byref(b))
            if n.value:
                out[fam] = {"ms": ms.value, "launches": n.value, "bytes": b.value}
        return out


def measured_traffic(family, bytes_per_launch):
    """HBM bytes per launch of `family` from the committed PMC summary
    (profiles/r*_traffic.json, made by tools/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this benchmark): the
    measured traffic/algorithmic ratio applied to this run's launch size."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return None, None
    try:
        fam = json.load(open(files[-1]))["families"].get(family)
    except (OSError, ValueError, KeyError):
        return None, None
    if not fam or not fam.get("traffic_over_algorithmic"):
        return None, None
    return (round(fam["traffic_over_algorithmic"] * bytes_per_launch),
            os.path.relpath(files[-1], ROOT))


def affinity_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_share():
    """Threads for the CPU baseline: the job's CPU share (OMP_NUM_THREADS, 16
    per GPU on the pool's boxes, where the affinity mask shows the whole
    machine), else the affinity core count."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return min(n, affinity_cores()) if n > 0 else affinity_cores()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(psf, dirty, max_scales, threshold, threads, outer_all, outer_single):
    """The oracle (tests/oracle_lib -> oracle/build/liboracle.so, float64
    FFT where the reference uses FFTW float) on the same workload (same
    inputs, settings and threshold), in ONE run: the setup (scale-convolved
    PSFs, first peak search) and the first `outer_all` multiscale outer
    iterations on `threads` threads, then `outer_single` more on one thread.
    Each leg's rate is its components over its cleaning time; the setup is
    reported on its own. A heartbeat on stderr covers the silent native
    call."""
    import threading
    from oracle_lib import OracleAlgorithm, get_oracle
    orc = get_oracle()
    size = dirty.shape[0]
    orc.set_threads(threads)
    res, mod = dirty[None].copy(), np.zeros_like(dirty)[None]
    alg = OracleAlgorithm(orc, 1, threshold=threshold, max_iterations=10 ** 9,
                          border_ratio=0.0, max_scales=max_scales,
                          beam_size_in_pixels=BEAM_PX, minor_loop_gain=0.1,
                          major_loop_gain=1.0)
    alg.set_clean_threads(1 if outer_single else 0, outer_all, outer_all + outer_single)
    print(f"[cpu_baseline] oracle: setup + {outer_all} outer iterations on {threads} threads, "
          f"{outer_single} on 1 thread ...", file=sys.stderr, flush=True)
    done = threading.Event()

    def heartbeat():
        t = time.perf_counter()
        while not done.wait(30.0):
            print(f"[cpu_baseline] running {time.perf_counter() - t:.0f} s", file=sys.stderr,
                  flush=True)

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    t0 = time.perf_counter()
    try:
        r, _ = alg.execute(res, mod, psf[None], trace_cap=1)
    finally:
        done.set()
        hb.join()
    total = time.perf_counter() - t0
    orc.set_threads(threads)
    setup = alg.setup_seconds()
    clean = total - setup
    n = int(r.iteration_number)
    if outer_single:
        t_switch, n_switch = alg.switch_info()
    else:
        t_switch, n_switch = clean, n
    runs = [{"threads": threads, "outer_iterations": outer_all, "components": n_switch,
             "clean_s": round(t_switch, 2), "value": round(n_switch / max(t_switch, 1e-9), 2)}]
    if outer_single and n > n_switch:
        runs.append({"threads": 1, "outer_iterations": outer_single,
                     "components": n - n_switch, "clean_s": round(clean - t_switch, 2),
                     "value": round((n - n_switch) / max(clean - t_switch, 1e-9), 2)})
    best = runs[0]
    return {"value": best["value"], "unit": "components/s", "cores": threads,
            "kind": "port", "cpu_model": cpu_model(), "affinity_cores": affinity_cores(),
            "setup_s": round(setup, 2), "runs": runs,
            "sample": (f"oracle MultiScale (C++ restatement of the reference, std::thread, "
                       f"float64 FFT; the reference uses FFTW float) on the same "
                       f"{size}x{size} {max_scales}-scale sky and threshold: setup "
                       f"({round(setup, 1)} s on {threads} threads, not in the rate), then "
                       f"the first {outer_all} outer iterations ({best['components']} "
                       f"components) on {threads} threads"
                       + (f"; runs[1]: the next {outer_single} on 1 thread "
                          f"({runs[1]['components']} components)" if len(runs) > 1 else ""))}


def cpu_to_threshold(name, threads):
    """The CPU baseline to the threshold (north_star's wall-clock-to-threshold
    beside the CPU): the oracle's MultiScale major iteration on the
    configuration `name` of tests/config_problems.py (c2: 4096^2, 1000 points
    + 100 blobs; t2k: 2048^2, 250 points + 25 blobs; 6 scales, threshold
    5 sigma, no component cap), setup (scale-convolved PSFs, first peak
    search) included and also reported alone. Host only (no GPU call); a
    heartbeat on stderr covers the silent native call."""
    import threading
    import config_problems as cp
    from oracle_lib import OracleAlgorithm, get_oracle
    psfs, dirty = cp.problem(name)
    c = cp.CONFIGS[name]
    orc = get_oracle()
    orc.set_threads(threads)
    res, mod = dirty.copy(), np.zeros_like(dirty)
    alg = OracleAlgorithm(orc, 1, threshold=c["threshold"], max_iterations=10 ** 9,
                          border_ratio=0.0, max_scales=c["max_scales"],
                          beam_size_in_pixels=cp.BEAM_PX, minor_loop_gain=0.1,
                          major_loop_gain=1.0, allow_negative=1)
    done = threading.Event()

    def heartbeat():
        t = time.perf_counter()
        while not done.wait(30.0):
            print(f"[cpu_to_threshold] {name}: running {time.perf_counter() - t:.0f} s",
                  file=sys.stderr, flush=True)

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    t0 = time.perf_counter()
    try:
        r, _ = alg.execute(res, mod, psfs, trace_cap=1)
    finally:
        done.set()
        hb.join()
    total = time.perf_counter() - t0
    setup = alg.setup_seconds()
    n = int(r.iteration_number)
    size = c["size"]
    return {"workload": (f"{name}: multiscale {size}x{size}, {c['max_scales']} scales, "
                         f"{c['points']} points + {c['blobs']} blobs, threshold 5 sigma "
                         f"(tests/config_problems.py)"),
            "kind": "port", "threads": threads, "cpu_model": cpu_model(),
            "affinity_cores": affinity_cores(),
            "wall_clock_to_threshold_s": round(total, 3), "setup_s": round(setup, 3),
            "clean_s": round(total - setup, 3), "components": n,
            "final_peak": float(r.final_peak),
            "stop": "the multiscale loop's threshold countdown (multiscale_algorithm.cc:"
                    "323-328, 378-384): it ends max(8, 1.5 x scales) sub-minor loops after "
                    "the sub-loop threshold reaches the final threshold; final_peak is the "
                    "last selected scale's peak, as the reference reports it",
            "components_per_s_with_setup": round(n / total, 2),
            "components_per_s_after_setup": round(n / max(total - setup, 1e-9), 2),
            "note": "oracle MultiScale (C++ restatement of the reference, std::thread, "
                    "float64 FFT; the reference uses FFTW float), one major iteration "
                    "(major_loop_gain 1) to the threshold"}


def gpu_to_threshold(rd, name):
    """The same problem to the threshold through Radler.perform on this GPU
    (accessor load + major iteration + store; warm-up + one timed run).
    Returns (components, seconds)."""
    import config_problems as cp
    c = cp.CONFIGS[name]
    psfs, dirty = cp.problem(name)
    st = settings_for(rd, c["size"], 10 ** 9, c["max_scales"], c["threshold"], 1, 1)

    def once():
        arrays = (psfs[0], dirty[0].copy(), np.zeros_like(dirty[0]))
        r = rd.Radler(st, *arrays, cp.BEAM_PX * cp.PIXEL_SCALE)
        t = time.perf_counter()
        r.perform(0)
        return rd.gpu.total_iteration_number(r), time.perf_counter() - t

    once()
    return once()


def with_amdahl(rd, once):
    """Run `once()` with the host profile's pass sections on: the wall clock
    of the find-peak and cleaning passes over the subimages (the part that
    N ranks split) against the whole Perform (load, split, passes, model
    merge, store). serial_fraction f bounds the N-rank speedup at
    1 / (f + (1 - f) / N), before load imbalance between ranks."""
    rd.gpu.host_profile_reset()
    rd.gpu.host_profile_enable(True)
    try:
        out = once()
    finally:
        rd.gpu.host_profile_enable(False)
    prof = rd.gpu.host_profile()
    total = prof.get("perform.total", (0, 0.0))[1]
    passes = sum(prof.get(k, (0, 0.0))[1] for k in ("par.findpeak_pass", "par.clean_pass"))
    if total <= 0.0:
        return out, None
    f = max(0.0, total - passes) / total
    serial = {k: round(prof[k][1], 4) for k in ("par.split", "split.divide", "split.masks",
                                                "perform.load", "perform.load_psfs",
                                                "perform.store") if k in prof}
    return out, {"perform_s": round(total, 4), "subimage_passes_s": round(passes, 4),
                 "serial_fraction": round(f, 4), "serial_sections_s": serial,
                 "speedup_bound": {str(n): round(1.0 / (f + (1.0 - f) / n), 2)
                                   for n in (2, 4, 8)},
                 "note": "passes: find-peak + cleaning over the subimages (split over "
                         "ranks); serial: accessor load, split, model copy, store. The "
                         "subimage merges run inside the passes (on N ranks every rank "
                         "merges all of them), so f is a lower bound"}


def iuwt_leg(rd, reps=10):
    """SURVEY.md C4 (IUWT, 4096^2) on this GPU: (1) the component the config
    names, IuwtDecomposition(6 scales).Decompose + Recompose on one 4096^2
    plane (rdl_iuwt_decompose / _recompose, include_largest), HIP-event device
    time per call against the algorithmic bytes of SURVEY.md 8(d) (12 B/px
    per decomposition scale, 8 B/px per recomposition scale); (2) the IUWT
    deconvolution algorithm on the C4 problem (tests/config_problems.py: 1000
    points + 100 blobs, 5 sigma, the fixture's 24 steps) to its stop, with
    every kernel family's device time."""
    import config_problems as cp
    from rdl_lib import Session
    size, n_scales = 4096, 6
    sess = Session(0)
    lib = sess.rdl.lib
    lib.rdl_timing_get.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double),
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    img = np.random.default_rng(1).standard_normal((size, size)).astype(np.float32)
    d_in, d_scratch = sess.array(img), sess.array(shape=(size, size))
    d_coeffs = sess.array(shape=(n_scales + 1, size, size))
    d_out = sess.array(shape=(size, size))
    px = size * size
    calls = {"decompose": (lambda: sess.rdl.rdl_iuwt_decompose(
                 sess.h, d_in.vp, d_scratch.vp, size, size, n_scales, d_coeffs.vp, 1),
                 12.0 * px * n_scales),
             "recompose": (lambda: sess.rdl.rdl_iuwt_recompose(
                 sess.h, d_coeffs.vp, size, size, n_scales, 1, d_out.vp),
                 8.0 * px * n_scales)}
    comp = {}
    for name, (fn, alg_bytes) in calls.items():
        fn()
        sess.sync()
        lib.rdl_timing_reset(sess.h)
        lib.rdl_timing_enable(sess.h, 1)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        sess.sync()
        wall = (time.perf_counter() - t0) / reps
        lib.rdl_timing_enable(sess.h, 0)
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        lib.rdl_timing_get(sess.h, b"iuwt", C.byref(ms), C.byref(n), C.byref(b))
        dev_s = ms.value / reps * 1e-3
        comp[name] = {"device_ms": round(dev_s * 1e3, 4), "wall_ms": round(wall * 1e3, 4),
                      "launches_per_call": n.value // reps,
                      "algorithmic_bytes": alg_bytes,
                      "achieved": round(alg_bytes / dev_s / 1e9, 1), "unit": "GB/s",
                      "frac": round(alg_bytes / dev_s / 1e9 / HBM_PEAK_GBS, 4)}
    for x in (d_in, d_scratch, d_coeffs, d_out):
        x.free()
    sess.close()
    # the algorithm on C4
    psfs, dirty = cp.problem("c4")
    c = cp.CONFIGS["c4"]
    st = rd.Settings()
    st.algorithm_type = rd.AlgorithmType.iuwt
    st.trimmed_image_width = st.trimmed_image_height = size
    st.pixel_scale.x = st.pixel_scale.y = cp.PIXEL_SCALE
    st.absolute_threshold = c["threshold"]
    st.minor_loop_gain = 0.1
    st.major_loop_gain = 1.0
    st.allow_negative_components = True
    st.border_ratio = 0.0
    st.minor_iteration_count = c["cap"]
    run = rd.gpu.DeviceRun(st, psfs[0], dirty[0], [], 0.0)
    run.execute()  # warm-up (plans for the box sizes met)
    timing = Timing()
    run.restore()
    run.sync()
    timing.reset()
    timing.only(None)
    timing.enable(True)
    t0 = time.perf_counter()
    r = run.execute()
    run.sync()
    el = time.perf_counter() - t0
    timing.enable(False)
    fams = timing.get()
    timing.reset()
    steps = run.iuwt_steps()
    del run
    dev = sum(v["ms"] for v in fams.values())
    top = []
    for k, v in sorted(fams.items(), key=lambda kv: -kv[1]["ms"])[:6]:
        gbs = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0.0
        top.append({"kernel": k, "share_of_device_time": round(v["ms"] / dev, 3) if dev else None,
                    "avg_launch_us": round(1e3 * v["ms"] / v["launches"], 2),
                    "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)})
    return {"workload": "c4: IUWT 4096x4096 (SURVEY.md C4, tests/config_problems.py)",
            "decomposition_6_scales": comp,
            "algorithm": {"seconds": round(el, 4), "iterations": int(r["iterations"]),
                          "steps": len(steps),
                          "successful_steps": int(sum(1 for x in steps if x[0])),
                          "another_iteration_required": bool(r["another_iteration_required"]),
                          "device_ms": round(dev, 2), "families": top,
                          "note": "one DeviceRun.execute to the algorithm's stop (the "
                                  "fixture's 24-step cap), HIP events on every family"}}


def committed_cpu_to_threshold(pattern="r*_cpu_c2_to_threshold.json"):
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
    except (OSError, ValueError):
        return None
    d["source"] = os.path.relpath(files[-1], ROOT)
    return d


def relaunch(args):
    """--gpus N without a launcher: run this script under
    torch.distributed.run as a child (nothing here has touched the GPU) and
    exit with its status."""
    with socket.socket() as sock:
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["fields", "tiled", "joined"], default=None,
                    help="default: fields at N = 1, tiled at N > 1")
    ap.add_argument("--size", type=int, default=None,
                    help="image side (default 8192; joined: 4096, SURVEY.md C3)")
    ap.add_argument("--channels", type=int, default=8, help="joined: channels")
    ap.add_argument("--joined-split", choices=["channels", "subimages"], default="channels",
                    help="joined at N > 1: share the per-channel work of ONE image set "
                         "(channels; the C3 computation itself) or split the set into "
                         "subimages (subimages; a different problem)")
    ap.add_argument("--grid", type=int, default=8, help="tiled: subimages per axis")
    ap.add_argument("--pool", type=int, default=16,
                    help="tiled: subimages in flight per GPU (settings.parallel.max_threads)")
    ap.add_argument("--scales", type=int, default=6)
    ap.add_argument("--points", type=int, default=2000)
    ap.add_argument("--blobs", type=int, default=200)
    ap.add_argument("--max-iter", type=int, default=10 ** 9)
    ap.add_argument("--sigma", type=float, default=5.0)
    ap.add_argument("--tiled-reference", type=int, default=1,
                    help="N = 1 fields: also time the tiled N > 1 workload on this GPU")
    ap.add_argument("--joined-reference", type=int, default=1,
                    help="N = 1: also time the joined-channel workload, unsplit (the C3 "
                         "computation) and split by subimage (the N > 1 partitioning)")
    ap.add_argument("--device-resident", type=int, default=1,
                    help="also time the HBM-resident major iteration (0 = skip)")
    ap.add_argument("--cpu-outer", type=int, default=2,
                    help="multiscale outer iterations of the CPU baseline on all threads "
                         "(0 = skip the CPU baseline)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the all-cores CPU run (0: OMP_NUM_THREADS, else the "
                         "affinity core count)")
    ap.add_argument("--cpu-single-thread", type=int, default=1,
                    help="outer iterations of the CPU baseline on one thread after the "
                         "all-threads ones (0 = skip; one 8192^2 outer iteration on one "
                         "thread takes one to two minutes)")
    ap.add_argument("--iuwt-reference", type=int, default=1,
                    help="N = 1 fields: also time SURVEY.md C4 (IUWT 4096^2: the 6-scale "
                         "decomposition component and the algorithm to its stop)")
    ap.add_argument("--c2-reference", type=int, default=1,
                    help="N = 1 fields: also time Radler.perform to the threshold on the C2 "
                         "configuration (4096^2), the workload of the committed CPU "
                         "to-threshold run")
    ap.add_argument("--to-threshold-live", default="t2k",
                    help="N = 1 fields: a tests/config_problems.py problem run to the "
                         "threshold by the GPU and by the CPU oracle in this job "
                         "(cpu_baseline.to_threshold; 'none' = skip)")
    ap.add_argument("--cpu-to-threshold", metavar="OUT_JSON",
                    help="host only: run the CPU oracle to the threshold on C2 (setup "
                         "included), write the JSON and exit")
    ap.add_argument("--cpu-to-threshold-config", default="c2",
                    help="the tests/config_problems.py problem of --cpu-to-threshold (c2, "
                         "h8kt: the headline 8192^2 problem)")
    ap.add_argument("--breakdown", action="store_true", help="per-kernel times to stderr")
    ap.add_argument("--timing-all", action="store_true",
                    help="count every launch of the process (PMC passes, tools/pmc_traffic.py)")
    ap.add_argument("--dump-families", help="write the per-family launch/byte counts here")
    args = ap.parse_args()

    if args.cpu_to_threshold:
        out = cpu_to_threshold(args.cpu_to_threshold_config, args.cpu_threads or cpu_share())
        with open(args.cpu_to_threshold, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out), flush=True)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    workload = args.workload or ("fields" if world == 1 else "tiled")
    tiled = workload == "tiled"
    joined = workload == "joined"
    if args.size is None:
        args.size = 4096 if joined else 8192
    # joined over N > 1 ranks: the image set (all channels) split into
    # grid x grid subimages owned by the ranks, as tiled
    split = tiled or (joined and world > 1 and args.joined_split == "subimages")
    # joined over N > 1 ranks by channel: every rank the whole computation's
    # integrated work, its own channels' corrections (MultiScaleAlgorithm::
    # SetChannelShard); every rank reports the same components
    chan_shard = joined and world > 1 and args.joined_split == "channels"
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist
    os.environ.setdefault("RADLER_DEVICE", str(local_rank))

    import radler as rd

    threshold = args.sigma * NOISE
    extra = {}
    if joined:
        # one sky over 100-170 MHz (spectral index -0.7), one
        # PSF per channel (FWHM ~ 1/nu), weights 1, 8 deconvolution channels
        from config_problems import joined_channels
        freqs = [100e6 + 10e6 * i for i in range(args.channels)]
        psf, dirty = joined_channels(args.size, args.points, args.blobs, SEED, freqs)
        extra = dict(n_deconvolution_groups=args.channels,
                     frequencies=np.array([[f, f] for f in freqs], np.float64),
                     weights=np.ones(args.channels, np.float64))
    else:
        # tiled: every rank holds the same image (one field); fields: one per rank
        psf, dirty = make_problem(args.size, SEED + (0 if tiled else rank), args.points,
                                  args.blobs)
    s = settings_for(rd, args.size, args.max_iter, args.scales, threshold,
                     args.grid if split else 1, args.pool if split else 1)
    comm = None
    if (split or chan_shard) and dist is not None:
        # RCCL communicator of the product (rdl_comm_*), id from rank 0
        import torch
        idl = torch.zeros(rd.distributed.rccl_id_size(), dtype=torch.uint8, device="cuda")
        if rank == 0:
            idl.copy_(torch.frombuffer(bytearray(rd.distributed.rccl_unique_id()),
                                       dtype=torch.uint8))
        dist.broadcast(idl, src=0)
        uid = bytes(idl.cpu().numpy().tobytes())
        comm = rd.distributed.RcclCommunicator(local_rank, world, rank, uid)

    def make_radler():
        # the accessors borrow these arrays (cpp/radler.h:38-40)
        arrays = (psf, dirty.copy(), np.zeros_like(dirty))
        r = rd.Radler(s, *arrays, BEAM_PX * PIXEL_SCALE, **extra)
        if comm is not None:
            r.set_communicator(comm)
        return r, arrays

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    timing = Timing()
    if args.timing_all:
        timing.enable(True)
    print(f"[bench] rank {rank}: {workload} {args.size}^2 inputs ready; {args.warmup} warm-up "
          f"+ {args.steps} timed Perform steps", file=sys.stderr, flush=True)
    # the N > 1 default workload (tiled 8 x 8) on this one GPU, the
    # same-workload reference point of the scaling curve
    tiled_ref = None
    if args.tiled_reference and world == 1 and workload == "fields":
        st = settings_for(rd, args.size, args.max_iter, args.scales, threshold,
                          args.grid, args.pool)

        def tiled_once():
            arrays = (psf, dirty.copy(), np.zeros_like(dirty))
            r = rd.Radler(st, *arrays, BEAM_PX * PIXEL_SCALE)
            t = time.perf_counter()
            r.perform(0)
            return rd.gpu.total_iteration_number(r), time.perf_counter() - t

        print("[bench] tiled reference (warm-up + 1 step) ...", file=sys.stderr, flush=True)
        # measured before the headline: after the fields runs the subimage
        # streams of this process ran 1.3x slower (7.96 vs 6.07 s per step)
        tiled_once()
        (t_comps, t_el), t_amdahl = with_amdahl(rd, tiled_once)
        tiled_ref = {"workload": (f"multiscale-{args.size}x{args.size}-{args.scales}scales"
                                  f"-tiled{args.grid}x{args.grid}"),
                     "value": round(t_comps / t_el, 2), "ms_per_step": round(1e3 * t_el, 2),
                     "wall_clock_to_threshold_s": round(t_el, 4),
                     "components_per_step": t_comps, "pool": args.pool,
                     "amdahl": t_amdahl,
                     "note": "the default N > 1 workload (ParallelDeconvolution subimages) "
                             "on one GPU, for the same-workload scaling curve"}

    # the joined-channel workload (8 channels x 4096^2) split
    # into grid x grid subimages on this one GPU: the N = 1 point of
    # `--workload joined --gpus N` (N > 1 splits the subimages over ranks)
    joined_ref = None
    if args.joined_reference and world == 1 and workload == "fields":
        from config_problems import joined_channels
        jsize, jch = 4096, args.channels
        jfreqs = [100e6 + 10e6 * i for i in range(jch)]
        j_psf, j_dirty = joined_channels(jsize, args.points, args.blobs, SEED, jfreqs)
        sj = settings_for(rd, jsize, args.max_iter, args.scales, threshold, args.grid, args.pool)
        jextra = dict(n_deconvolution_groups=jch,
                      frequencies=np.array([[f, f] for f in jfreqs], np.float64),
                      weights=np.ones(jch, np.float64))

        def joined_once(settings=sj):
            arrays = (j_psf, j_dirty.copy(), np.zeros_like(j_dirty))
            r = rd.Radler(settings, *arrays, BEAM_PX * PIXEL_SCALE, **jextra)
            t = time.perf_counter()
            r.perform(0)
            return rd.gpu.total_iteration_number(r), time.perf_counter() - t

        # split first (kept so the r05-r06 lines compare): before the
        # per-device stream pool (r06), worker sessions made after the
        # 8-channel unsplit runs got streams bound to busier hardware queues
        # and this leg ran 9.4 s instead of 4.6 s (DESIGN.md §5, Round-6 work)
        print("[bench] joined reference, split (warm-up + 1 step) ...", file=sys.stderr,
              flush=True)
        joined_once()
        (j_comps, j_el), j_amdahl = with_amdahl(rd, joined_once)
        # unsplit: the C3 computation itself (one image set, one GPU)
        su = settings_for(rd, jsize, args.max_iter, args.scales, threshold, 1, 1)
        print("[bench] joined reference, unsplit (warm-up + 1 step) ...", file=sys.stderr,
              flush=True)
        joined_once(su)
        u_comps, u_el = joined_once(su)
        # the channel-sharded form of the same run (`--workload joined --gpus
        # N`, MultiScaleAlgorithm::SetChannelShard): its per-image work (the
        # float64 residual corrections and the model stamping) is what N ranks
        # share; one more unsplit run with every family timed prices it
        timing.reset()
        timing.only(None)
        timing.enable(True)
        joined_once(su)
        timing.enable(False)
        jf = timing.get()
        timing.reset()
        dev_ms = sum(v["ms"] for v in jf.values())
        shard_ms = sum(v["ms"] for k, v in jf.items()
                       if k.startswith("conv64") or k == "stamp_model")
        outer = jf.get("subminor_loop", {}).get("launches", 0)
        f_shard = shard_ms / dev_ms if dev_ms else 0.0
        plane_bytes = jsize * jsize * 4
        link_gbs = 153.0  # one xGMI link (MI355X_MICROARCH.md: 7 per GPU)
        chan_bound = {}
        for n in (2, 4, 8):
            # every rank receives the other ranks' corrected planes each outer
            # iteration: (n - 1) / n of the channels' planes
            xbytes = outer * (n - 1) / n * jch * plane_bytes
            chan_bound[str(n)] = {
                "compute_bound_s": round(u_el * ((1.0 - f_shard) + f_shard / n), 4),
                "exchange_gb": round(xbytes / 1e9, 2),
                "exchange_s_ring_one_link": round(xbytes / (link_gbs * 1e9), 4),
                "exchange_s_all_links": round(xbytes / (min(n - 1, 7) * link_gbs * 1e9), 4)}
        channel_shard = {
            "shardable_device_fraction": round(f_shard, 4),
            "device_ms": round(dev_ms, 1), "shardable_ms": round(shard_ms, 1),
            "outer_iterations": outer, "bound": chan_bound,
            "note": "`--workload joined --gpus N` (default --joined-split channels): ONE "
                    "image set, image i's residual correction + model update on rank i % N, "
                    "the integrated-image work (integration, scale convolutions, peak "
                    "searches, selection, sub-minor loop) on every rank, corrected planes "
                    "broadcast from their owners each outer iteration. compute_bound_s = "
                    "the unsplit run with the shardable device time divided by N; the "
                    "exchange adds exchange_s (one link: a ring; all links: a full mesh) "
                    "unless overlapped. Bit-identical to the unsplit run "
                    "(tests/test_distributed.py::test_channel_sharded_joined_equals_one_process)"}
        joined_ref = {"workload": (f"joined{jch}ch-multiscale-{jsize}x{jsize}-{args.scales}"
                                   f"scales-tiled{args.grid}x{args.grid}"),
                      "value": round(j_comps / j_el, 2), "ms_per_step": round(1e3 * j_el, 2),
                      "wall_clock_to_threshold_s": round(j_el, 4),
                      "components_per_step": j_comps, "pool": args.pool,
                      "amdahl": j_amdahl,
                      "unsplit": {"workload": (f"joined{jch}ch-multiscale-{jsize}x{jsize}-"
                                               f"{args.scales}scales"),
                                  "value": round(u_comps / u_el, 2),
                                  "wall_clock_to_threshold_s": round(u_el, 4),
                                  "components_per_step": u_comps,
                                  "channel_shard": channel_shard,
                                  "note": "SURVEY.md C3 as one image set on one GPU: the "
                                          "joined N = 1 point of the C3 computation"},
                      "note": "`--workload joined --gpus N` at N = 1: the channels' image set "
                              "split into grid x grid subimages (the partitioning N > 1 "
                              "shares over ranks, DESIGN.md §6), a different problem from "
                              "the unsplit C3 run in `unsplit`"}
        # the split run's best case on N ranks (its Amdahl bound) against the
        # unsplit C3 run on one GPU: what the subimage split can reach
        bound = {n: round(j_el / f, 4) for n, f in j_amdahl.get("speedup_bound", {}).items()}
        joined_ref["vs_unsplit"] = {
            "unsplit_s": round(u_el, 4), "split_bound_s": bound,
            "note": ("best-case wall clock of the split problem on N ranks (perform_s / "
                     "speedup_bound) beside the unsplit run on one GPU; the channel-sharded "
                     "form of the unsplit run is unsplit.channel_shard")}
        del j_psf, j_dirty

    # C4: the IUWT decomposition component and algorithm on this GPU
    iuwt_ref = None
    if args.iuwt_reference and world == 1 and workload == "fields":
        print("[bench] C4 IUWT 4096^2 (decomposition + algorithm) ...", file=sys.stderr,
              flush=True)
        iuwt_ref = iuwt_leg(rd)

    # C2 (4096^2) to the threshold on this GPU: the same problem as the
    # committed CPU to-threshold run (wall clock against wall clock)
    c2_ref = None
    if args.c2_reference and world == 1 and workload == "fields":
        print("[bench] C2 4096^2 to threshold (warm-up + 1 step) ...", file=sys.stderr,
              flush=True)
        c_comps, c_el = gpu_to_threshold(rd, "c2")
        c2_ref = {"workload": "c2: multiscale 4096x4096, 6 scales (tests/config_problems.py)",
                  "wall_clock_to_threshold_s": round(c_el, 4), "components": c_comps,
                  "value": round(c_comps / c_el, 2),
                  "step": "Radler.perform (accessor load + major iteration + store)"}

    # the live CPU-vs-GPU to-threshold problem, GPU side (the CPU side runs
    # after the timed region, with cpu_baseline)
    live_tt = None
    if (args.to_threshold_live != "none" and args.cpu_outer > 0 and world == 1
            and workload == "fields"):
        print(f"[bench] {args.to_threshold_live} to threshold on the GPU (warm-up + 1) ...",
              file=sys.stderr, flush=True)
        live_tt = gpu_to_threshold(rd, args.to_threshold_live)

    # Per-launch HIP events cost time (in the gridded runs, with 16 streams of
    # small kernels, 15-35 % of a step), so every family is timed on the last
    # warm-up step only; the timed steps record events for the dominant
    # family alone (its roofline stays measured live over the timed region).
    # That profiled step runs the scales' transforms on one lane
    # (RDL_SCALE_LANES=1, read per major iteration): on two lanes the
    # transforms of two scales overlap and each launch's event time includes
    # the other lane's share of HBM, which no per-kernel roofline can use.
    fams_all = None
    for w in range(args.warmup):
        profile = w == args.warmup - 1 and not args.timing_all
        lanes_env = os.environ.get("RDL_SCALE_LANES")
        if profile:
            timing.reset()
            timing.only(None)
            timing.enable(True)
            os.environ["RDL_SCALE_LANES"] = "1"
        r, arrays = make_radler()
        r.perform(0)
        del r, arrays
        if profile:
            timing.enable(False)
            fams_all = timing.get()
            if lanes_env is None:
                del os.environ["RDL_SCALE_LANES"]
            else:
                os.environ["RDL_SCALE_LANES"] = lanes_env
    dominant = (max(fams_all.items(), key=lambda kv: kv[1]["ms"])[0]
                if fams_all else None)
    steps = [make_radler() for _ in range(args.steps)]
    if os.environ.get("RADLER_HOST_PROFILE") == "1":
        rd.gpu.host_profile_reset()  # the printed host profile covers the timed steps

    # the roofline's HIP events are recorded over the leg `value` comes from:
    # the HBM-resident DeviceRun leg when there is one, else these steps
    has_resident = bool(args.device_resident) and not split

    def events_on():
        if not args.timing_all:
            timing.reset()
            timing.only(dominant)
        timing.enable(True)

    def events_off():
        if not args.timing_all:
            timing.enable(False)
            timing.only(None)
        return timing.get()

    if not has_resident:
        events_on()
    barrier()
    t0 = time.perf_counter()
    comps = 0
    for r, _ in steps:
        r.perform(0)  # Perform returns after the residual/model stores (D2H)
        comps += rd.gpu.total_iteration_number(r)
    barrier()
    elapsed = time.perf_counter() - t0
    fams = None
    if not has_resident:
        fams = events_off()
    del steps

    # the same major iteration on an HBM-resident image set (no host transfers)
    resident = None
    if has_resident:
        run = rd.gpu.DeviceRun(s, psf, dirty, [1.0] * args.channels if joined else [],
                               BEAM_PX * PIXEL_SCALE, trace=False)
        if comm is not None:
            run.set_communicator(comm)
        run.restore()
        run.execute()  # warm-up
        run.sync()
        events_on()
        barrier()
        t1 = time.perf_counter()
        rcomps = 0
        for _ in range(args.steps):
            run.restore()
            rcomps += run.execute()["iterations"]
        run.sync()
        barrier()
        relapsed = time.perf_counter() - t1
        fams = events_off()
        resident = {"ms_per_step": round(1e3 * relapsed / args.steps, 2),
                    "components_per_step": rcomps // args.steps, "elapsed": relapsed,
                    "components": rcomps}
        del run
    if args.dump_families and rank == 0:
        with open(args.dump_families, "w") as f:
            json.dump(fams, f, indent=1)

    total_comps, max_elapsed = comps, elapsed
    if dist is not None:
        import torch
        vals = [elapsed, comps] + ([resident["elapsed"], resident["components"]]
                                   if resident else [0.0, 0.0])
        t = torch.tensor([vals[0], vals[2]], dtype=torch.float64, device="cuda")
        c = torch.tensor([vals[1], vals[3]], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if not (split or chan_shard):  # split / by channel: every rank reports the job's
            dist.all_reduce(c, op=dist.ReduceOp.SUM)
        max_elapsed, total_comps = float(t[0].item()), int(c[0].item())
        if resident:
            resident["elapsed"], resident["components"] = float(t[1].item()), int(c[1].item())
    if resident:  # the slowest rank's time (all ranks' components)
        resident["ms_per_step"] = round(1e3 * resident["elapsed"] / args.steps, 2)
        resident["value"] = round(resident.pop("components") / resident.pop("elapsed"), 2)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    ms_per_step = 1e3 * max_elapsed / args.steps
    # device-time shares from the every-family profile of the last warm-up
    # step (the timed steps record the dominant family only)
    prof = fams_all if fams_all else fams
    device_ms = sum(v["ms"] for v in prof.values())
    # dominant kernel family by device time, timed over the timed region
    dom_name, dom = max(fams.items(), key=lambda kv: kv[1]["ms"]) if fams else (None, None)
    roofline = None
    if dom is not None and dom["ms"] > 0:
        avg_ms = dom["ms"] / dom["launches"]
        bytes_per_launch = dom["bytes"] / dom["launches"]
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = measured_traffic(dom_name, bytes_per_launch)
        roofline = {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": traffic_src,
                    "avg_launch_us": round(avg_ms * 1e3, 2),
                    "bytes_per_launch": bytes_per_launch,
                    "share_of_device_time": (round(prof[dom_name]["ms"] / device_ms, 3)
                                             if device_ms and dom_name in prof else None),
                    "timed_over": ("the DeviceRun leg `value` comes from" if has_resident
                                   else "the timed Radler.perform steps")}
    # the other large families against the same HBM roofline (algorithmic
    # bytes per launch / average launch time)
    families = []
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])[:8]:
        if v["ms"] <= 0 or v["bytes"] <= 0:
            continue
        gbs = v["bytes"] / (v["ms"] * 1e-3) / 1e9
        families.append({"kernel": k, "share_of_device_time":
                         round(v["ms"] / device_ms, 3) if device_ms else None,
                         "avg_launch_us": round(1e3 * v["ms"] / v["launches"], 2),
                         "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)})
    if roofline is not None:
        roofline["families"] = families
        roofline["families_source"] = ("last warm-up step, every family timed, "
                                       "scale transforms on one lane"
                                       if fams_all else "timed steps")
    if args.breakdown:
        # per family over the profiled warm-up step (one step)
        for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"]):
            gbs = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0.0
            print(f"[breakdown] {k:18s} {v['ms']:10.2f} ms {v['launches']:8d} launches "
                  f"{gbs:8.1f} GB/s", file=sys.stderr)
        print(f"[breakdown] device {device_ms:.1f} ms (all streams) in "
              f"{'one warm-up step' if fams_all else f'{1e3 * elapsed:.1f} ms wall'}",
              file=sys.stderr)

    cpu = None
    if args.cpu_outer > 0 and world == 1 and workload == "fields":
        threads = args.cpu_threads or cpu_share()
        cpu = cpu_baseline(psf, dirty, args.scales, threshold, threads, args.cpu_outer,
                           args.cpu_single_thread if threads > 1 else 0)
        cpu["cores_note"] = (
            "threads = OMP_NUM_THREADS, the job's CPU share on the pool's one-GPU boxes "
            "(16); the affinity mask lists all of the machine's cores, which other jobs "
            "share, so they are not used")
        if live_tt is not None:
            # measured live, in this job: the oracle on the same problem and
            # threads as above, to the threshold, against the GPU's run of it
            print(f"[cpu_baseline] {args.to_threshold_live} to threshold on {threads} "
                  f"threads ...", file=sys.stderr, flush=True)
            tt = cpu_to_threshold(args.to_threshold_live, threads)
            g_comps, g_el = live_tt
            tt.update({"measured": "live, this job",
                       "gpu_wall_clock_to_threshold_s": round(g_el, 4),
                       "gpu_components": g_comps,
                       "gpu_components_per_s": round(g_comps / g_el, 2),
                       "speedup_wall_clock": round(tt["wall_clock_to_threshold_s"] / g_el, 1),
                       "speedup_wall_clock_after_cpu_setup": round(tt["clean_s"] / g_el, 1)})
            cpu["to_threshold"] = tt
        ref = committed_cpu_to_threshold()
        if ref is not None:
            # the larger C2 (4096^2) CPU run, committed from an earlier job on
            # the same kind of box; the GPU side is this job's c2_to_threshold
            if c2_ref is not None:
                ref["gpu_wall_clock_to_threshold_s"] = c2_ref["wall_clock_to_threshold_s"]
                ref["gpu_components"] = c2_ref["components"]
                ref["speedup_wall_clock"] = round(
                    ref["wall_clock_to_threshold_s"] / c2_ref["wall_clock_to_threshold_s"], 1)
            ref["measured"] = "committed file (not this job)"
            cpu["to_threshold_c2_committed"] = ref
        h8k = committed_cpu_to_threshold("r*_cpu_h8k_to_threshold*.json")
        if h8k is not None:
            # the headline problem itself to the threshold on the CPU (the
            # oracle run behind tests/golden/config_h8kt.npz); the GPU side is
            # this job's DeviceRun leg (`value`)
            if resident is not None:
                h8k["gpu_wall_clock_to_threshold_s"] = round(resident["ms_per_step"] / 1e3, 4)
                h8k["gpu_components"] = resident["components_per_step"]
                h8k["speedup_wall_clock"] = round(
                    h8k["wall_clock_to_threshold_s"] / (resident["ms_per_step"] / 1e3), 1)
            h8k["measured"] = "committed file (not this job)"
            cpu["to_threshold_h8k_committed"] = h8k

    grid = f"-tiled{args.grid}x{args.grid}" if split else ""
    chans = f"joined{args.channels}ch-" if joined else ""
    # `value` is the rate with the inputs resident in HBM when the timed
    # region starts (DeviceRun: restore the dirty image from its HBM copy +
    # the major iteration, K steps between barrier + sync); the drop-in
    # Radler.perform over host buffers (accessor load over PCIe + the same
    # iteration + store) is reported beside it. The split workloads have no
    # resident leg: their line is the Radler.perform rate (config.step says so).
    host = {"ms_per_step": round(ms_per_step, 2),
            "value": round(total_comps / max_elapsed, 2),
            "components_per_step": total_comps // (args.steps * (1 if split or chan_shard
                                                                 else world)),
            "step": "Radler.perform (accessor load over PCIe + major iteration + store)"}
    if resident:
        v_value, v_ms = resident["value"], resident["ms_per_step"]
        v_comps = resident["components_per_step"]
        step_desc = ("DeviceRun (inputs resident in HBM: restore the dirty image from its "
                     "HBM copy + one major iteration)")
    else:
        v_value, v_ms, v_comps = host["value"], host["ms_per_step"], host["components_per_step"]
        step_desc = host["step"]
    line = {
        "metric": "CLEAN components/sec (multiscale, to 5-sigma threshold)",
        "value": v_value,
        "unit": "components/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": v_ms,
        "wall_clock_to_threshold_s": round(v_ms / 1e3, 4),
        "components_per_step": v_comps,
        "higher_is_better": True,
        # r05+: `value` is the HBM-resident rate (DeviceRun) where the
        # workload has one; r01-r04 lines carried the Radler.perform rate over
        # host buffers there, which stays in `perform_host_buffers.value`
        "value_definition": ("v2: HBM-resident DeviceRun (restore + major iteration)"
                             if resident else
                             "v1: Radler.perform over host buffers (accessor load + major "
                             "iteration + store)"),
        "scaling": "strong" if split or chan_shard else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded sky: points + Gaussian blobs, analytic PSF, noise)",
        "config": {"workload": (f"{chans}multiscale-{args.size}x{args.size}-"
                                f"{args.scales}scales{grid}"),
                   "step": step_desc,
                   "image": [args.size, args.size], "scales": args.scales,
                   "points": args.points, "blobs": args.blobs, "noise": NOISE,
                   "threshold": threshold, "minor_loop_gain": 0.1, "major_loop_gain": 1.0,
                   "channels": args.channels if joined else 1,
                   "fields_per_gpu": 0 if split or chan_shard else 1,
                   "parallelism": (f"subimages{args.grid * args.grid}/ranks{world}"
                                   f"/pool{args.pool}" if split else
                                   f"channels{args.channels}/ranks{world}" if chan_shard
                                   else f"fields{world}"),
                   **({"problem": ("the joined image set split into grid x grid subimages "
                                   "shared by the ranks (ParallelDeconvolution over the "
                                   "channels' set): at N > 1 this solves the tiled problem, "
                                   "not the unsplit C3 run (joined_n1.unsplit of the N = 1 "
                                   "line)")} if joined and split else {})},
        "device_resident": resident,
        "perform_host_buffers": host,
        "tiled_n1": tiled_ref,
        "joined_n1": joined_ref,
        "c2_to_threshold": c2_ref,
        "iuwt_c4": iuwt_ref,
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    import gc
    gc.collect()  # release device buffers while the runtime is fully alive
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
