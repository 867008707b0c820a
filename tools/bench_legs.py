#!/usr/bin/env python3
"""Run bench.py's workloads as legs in a chosen order in ONE process and time
each leg's Radler.perform steps, to find process-state dependence (the r05
verdict: the split joined leg took 5.6 s after the tiled leg and 9.8 s
without it).

    python tools/bench_legs.py joined_split,joined_split,tiled,joined_split [--reps 2]

Legs: headline (8192^2 unsplit), tiled (8192^2 8x8, pool 16), tiled1 (the
same with one worker: every kernel dispatched from one thread), joined (8 x
4096^2 unsplit), joined_split (8 x 4096^2 8x8, pool 16). Every leg runs one
warm-up Perform, then `--reps` timed ones; per timed Perform the wall clock,
the components, the host profile's top sections and the device time of every
kernel family (HIP events, every session of the process) are printed as one
JSON line per leg.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-radler_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("legs")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--events", type=int, default=0,
                    help="1: HIP-event device time per family (costs time in pooled legs)")
    args = ap.parse_args()
    import radler as rd
    from config_problems import joined_channels
    thr = 5.0 * bench.NOISE
    cache = {}

    def problem(kind):
        if kind not in cache:
            if kind == "single":
                cache[kind] = bench.make_problem(8192, bench.SEED, 2000, 200)
            else:
                freqs = [100e6 + 10e6 * i for i in range(8)]
                cache[kind] = (joined_channels(4096, 2000, 200, bench.SEED, freqs), freqs)
        return cache[kind]

    def leg_once(name):
        if name in ("headline", "tiled", "tiled1"):
            psf, dirty = problem("single")
            grid = 1 if name == "headline" else 8
            pool = 16 if name == "tiled" else 1  # tiled1: one worker (serial)
            s = bench.settings_for(rd, 8192, 10 ** 9, 6, thr, grid, pool)
            arrays = (psf, dirty.copy(), np.zeros_like(dirty))
            r = rd.Radler(s, *arrays, bench.BEAM_PX * bench.PIXEL_SCALE)
        else:
            (psf, dirty), freqs = problem("joined")
            grid = 8 if name == "joined_split" else 1
            s = bench.settings_for(rd, 4096, 10 ** 9, 6, thr, grid, 16 if grid > 1 else 1)
            arrays = (psf, dirty.copy(), np.zeros_like(dirty))
            r = rd.Radler(s, *arrays, bench.BEAM_PX * bench.PIXEL_SCALE,
                          n_deconvolution_groups=8,
                          frequencies=np.array([[f, f] for f in freqs], np.float64),
                          weights=np.ones(8, np.float64))
        t = time.perf_counter()
        r.perform(0)
        return rd.gpu.total_iteration_number(r), time.perf_counter() - t

    timing = bench.Timing()
    for k, name in enumerate(args.legs.split(",")):
        leg_once(name)  # warm-up
        out = {"leg": name, "position": k, "runs": []}
        for _ in range(args.reps):
            rd.gpu.host_profile_reset()
            rd.gpu.host_profile_enable(True)
            if args.events:
                timing.reset()
                timing.enable(True)
            comps, el = leg_once(name)
            rd.gpu.host_profile_enable(False)
            fams = {}
            if args.events:
                timing.enable(False)
                fams = {f: round(v["ms"], 2) for f, v in timing.get().items()}
            prof = sorted(rd.gpu.host_profile().items(), key=lambda kv: -kv[1][1])[:14]
            out["runs"].append({"s": round(el, 4), "components": comps,
                                "device_ms": round(sum(fams.values()), 1) if fams else None,
                                "families_ms": fams,
                                "host": {kk: [v[0], round(v[1], 4)] for kk, v in prof}})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
