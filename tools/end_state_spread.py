#!/usr/bin/env python3
"""The rounding sensitivity of a multiscale run's END STATE to threshold, on
the GPU: the yardstick for tests/test_configs_gpu.py's end-state tolerances
(c2t, h8kt).

A run to threshold is a long chain of argmax decisions; float rounding flips
near-tied decisions and the trajectory separates from any other arithmetic's
(the float64 oracle's included) after its first near-ties. What can be
compared past that point are quantities the separation hardly changes. How
much each one moves under rounding-level changes is measured here by an
ensemble of GPU runs of the same problem:

  * `base`: the problem as given;
  * `ulp<k>`: the dirty image with a random half of its pixels moved by one
    float ulp (np.nextafter, seed k): an input perturbation at the level of
    one rounding;
  * `twopass`: the scale convolutions through the two-pass column path
    (RDL_FUSED_SCALES=0) instead of the fused multi-scale launch: the same
    mathematics with different float32 rounding.

For every member: component count, another_iteration_required, final peak,
residual RMS / max|.|, model sum / max|.|, and the residual / model at the
fixture's 65 536 sampled pixels (tests/golden/make_config_golden.py). The
spread of each scalar (max |member - base| relative to base) and the
pairwise RMS distance of the samples (relative to the base's sample RMS)
are written as JSON.

    python tools/end_state_spread.py c2t [--ulp 6] > profiles/r06_end_state_spread_c2t.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-radler_amd"))

import config_problems as cp  # noqa: E402


def sample_index(n_pixels, seed=1):
    return np.sort(np.random.default_rng(seed).choice(n_pixels, 65536, replace=False))


LABELS = {}  # tiled configurations: subimage label (+1) of every sampled pixel


def end_state(rd, name, psfs, dirty):
    from test_configs_gpu import settings
    tiled = cp.CONFIGS[name]["kind"] == "tiled"
    run = rd.gpu.DeviceRun(settings(rd, name), psfs[0], dirty[0], [],
                           cp.BEAM_PX * cp.PIXEL_SCALE, trace=tiled)
    t = time.perf_counter()
    r = run.execute()
    run.sync()
    el = time.perf_counter() - t
    res = run.residual().reshape(-1)
    mod = run.model().reshape(-1)
    idx = sample_index(res.size)
    out = {"components": int(r["iterations"]),
           "another_iteration_required": bool(r["another_iteration_required"]),
           "final_peak": float(r["end_peak"]),
           "residual_rms": float(np.sqrt(np.mean(res.astype(np.float64) ** 2))),
           "residual_absmax": float(np.abs(res).max()),
           "model_sum": float(mod.astype(np.float64).sum()),
           "model_absmax": float(np.abs(mod).max()), "seconds": round(el, 3)}
    samples = (res[idx].astype(np.float64), mod[idx].astype(np.float64))
    if tiled and name not in LABELS:
        size = dirty.shape[-1]
        LABELS[name] = run.subimages(size, size)[1].reshape(-1)[idx].astype(np.int64) - 1
    del run
    return out, samples


SCALARS = ["components", "final_peak", "residual_rms", "residual_absmax", "model_sum",
           "model_absmax"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name", help="a tests/config_problems.py multiscale configuration")
    ap.add_argument("--ulp", type=int, default=6, help="ulp-perturbed members")
    ap.add_argument("--twopass", type=int, default=1)
    args = ap.parse_args()
    from radler_import import radler as rd
    psfs, dirty = cp.problem(args.name)
    members = {}
    samples = {}
    print(f"[spread] {args.name}: base", file=sys.stderr, flush=True)
    members["base"], samples["base"] = end_state(rd, args.name, psfs, dirty)
    for k in range(args.ulp):
        rng = np.random.default_rng(1000 + k)
        d = dirty.copy()
        flip = rng.random(d.shape) < 0.5
        up = rng.random(d.shape) < 0.5
        d[flip] = np.where(up[flip], np.nextafter(d[flip], np.float32(np.inf)),
                           np.nextafter(d[flip], np.float32(-np.inf)))
        print(f"[spread] {args.name}: ulp{k}", file=sys.stderr, flush=True)
        members[f"ulp{k}"], samples[f"ulp{k}"] = end_state(rd, args.name, psfs, d)
    if args.twopass:
        os.environ["RDL_FUSED_SCALES"] = "0"
        print(f"[spread] {args.name}: twopass", file=sys.stderr, flush=True)
        members["twopass"], samples["twopass"] = end_state(rd, args.name, psfs, dirty)
        del os.environ["RDL_FUSED_SCALES"]
    base = members["base"]
    spread = {}
    for key in SCALARS + ["abs_final_peak"]:
        if key == "abs_final_peak":  # the last selected scale's signed peak: its size
            devs = [abs(abs(m["final_peak"]) - abs(base["final_peak"])) /
                    max(abs(base["final_peak"]), 1e-30) for n, m in members.items() if n != "base"]
        else:
            devs = [abs(m[key] - base[key]) / max(abs(base[key]), 1e-30)
                    for n, m in members.items() if n != "base"]
        spread[key] = {"max_rel": max(devs, default=0.0),
                       "mean_rel": float(np.mean(devs)) if devs else 0.0}
    names = list(samples)
    pair = {"residual": [], "model": []}
    ref_rms = {"residual": float(np.sqrt(np.mean(samples["base"][0] ** 2))),
               "model": float(np.sqrt(np.mean(samples["base"][1] ** 2)))}
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            for k, key in enumerate(("residual", "model")):
                a, b = samples[names[i]][k], samples[names[j]][k]
                pair[key].append(float(np.sqrt(np.mean((a - b) ** 2))) / ref_rms[key])
    per_sub = None
    if args.name in LABELS:
        # tiled: the same distances per subimage (its own samples, over its
        # own base RMS); tests/test_configs_gpu.py compares the samples of the
        # subimages whose traces separate from the oracle's with the largest
        lab = LABELS[args.name]
        per_sub = {"residual": [], "model": []}
        for sub in range(int(lab.max()) + 1):
            sel = lab == sub
            for k, key in enumerate(("residual", "model")):
                base_rms = float(np.sqrt(np.mean(samples["base"][k][sel] ** 2)))
                worst = 0.0
                for i in range(len(names)):
                    for j in range(i + 1, len(names)):
                        a, b = samples[names[i]][k][sel], samples[names[j]][k][sel]
                        worst = max(worst, float(np.sqrt(np.mean((a - b) ** 2))) /
                                    max(base_rms, 1e-30))
                per_sub[key].append(worst)
    out = {"config": args.name, "members": members, "spread": spread,
           "subimage_sample_rms_distance": per_sub,
           "sample_rms_distance": {k: {"max": max(v, default=0.0),
                                       "mean": float(np.mean(v)) if v else 0.0}
                                   for k, v in pair.items()},
           "sample_rms": ref_rms,
           "note": "spread = max over members of |member - base| / |base|; sample "
                   "distance = RMS over the fixture's 65 536 sampled pixels of the "
                   "difference of two members, over the base's sample RMS (pairs of "
                   "all members)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
