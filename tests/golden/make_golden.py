"""Generate the committed golden fixtures under tests/golden/ (run in the
development container, where /root/reference exists):

    make -C oracle && make -C oracle ref && python tests/golden/make_golden.py

Two kinds of vectors:
  * ref_*      — outputs of the REFERENCE's own code (cpp/algorithms/
                 simple_clean.cc PartialSubtractImage, cpp/utils/
                 fft_size_calculations.h), compiled from /root/reference into
                 oracle/_ref by oracle/Makefile. These let the GPU box (which
                 has no /root/reference) check the HIP path against the
                 reference itself.
  * oracle_*   — outputs of the CPU restatement (oracle/) for whole CLEAN
                 runs (Högbom, Clark sub-minor, multiscale). They pin the
                 oracle against regressions and give the GPU tests a fixed
                 expected trace.
Inputs are regenerated from seeds by the tests (synthetic.py); only expected
outputs and the seeds/settings are stored.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle_lib import OracleAlgorithm, get_oracle, get_ref  # noqa: E402
from synthetic import problem  # noqa: E402

SUBTRACT_CASES = [  # w, h, seed
    (64, 64, 1), (63, 65, 2), (257, 130, 3), (1024, 33, 4)]
FFT_SIZES = list(range(1, 600)) + [1024, 1128, 2048, 2268, 4096, 4506, 8192, 9012, 16384]
CONV_SIZES = [(s, n, p) for s in (0.0, 16.0, 32.0, 64.0, 128.0, 256.0)
              for n in (64, 128, 1000, 2048, 4096, 8192) for p in (1.0, 1.1, 1.5)]

RUNS = {
    # name: (kind, w, n_points, n_blobs, seed, settings)
    "oracle_hogbom_96": (0, 96, 12, 0, 11, dict(threshold=0.0, max_iterations=400,
                                                  border_ratio=0.0, use_sub_minor=0)),
    "oracle_clark_128": (0, 128, 20, 2, 12, dict(threshold=2e-3, max_iterations=1500,
                                                   border_ratio=0.0, use_sub_minor=1,
                                                   major_loop_gain=0.9)),
    "oracle_multiscale_128": (1, 128, 10, 2, 138, dict(threshold=5e-3, max_iterations=500,
                                                         border_ratio=0.0, max_scales=4,
                                                         beam_size_in_pixels=2.0)),
}


def subtract_inputs(w, h, seed):
    rng = np.random.default_rng(seed)
    img = rng.standard_normal((h, w)).astype(np.float32)
    psf = rng.standard_normal((h, w)).astype(np.float32)
    steps = [(0, 0), (w - 1, h - 1), (w // 2, h // 2), (3, h - 2), (w - 5, 1)]
    factors = rng.standard_normal(len(steps)).astype(np.float32)
    return img, psf, steps, factors


def main():
    ref = get_ref()
    if ref is None:
        sys.exit("oracle/_ref not built: make -C oracle ref")
    out = {}
    for w, h, seed in SUBTRACT_CASES:
        img, psf, steps, factors = subtract_inputs(w, h, seed)
        for (x, y), f in zip(steps, factors):
            ref.ref_partial_subtract(img, psf, w, h, x, y, float(f), 0, h)
        out[f"ref_subtract_{w}x{h}_s{seed}"] = img
    np.savez_compressed(os.path.join(HERE, "ref_subtract.npz"), **out)
    sizes = {
        "good_fft_size": {str(n): int(ref.ref_good_fft_size(n)) for n in FFT_SIZES},
        "convolution_size": [[s, n, p, int(ref.ref_convolution_size(s, n, p))]
                             for s, n, p in CONV_SIZES],
    }
    with open(os.path.join(HERE, "ref_fft_sizes.json"), "w") as fh:
        json.dump(sizes, fh, indent=0)

    orc = get_oracle()
    orc.set_threads(8)
    for name, (kind, w, n_points, n_blobs, seed, st) in RUNS.items():
        psf, dirty = problem(w, w, n_points, n_blobs, seed=seed)
        res, mod = dirty[None].copy(), np.zeros((1, w, w), np.float32)
        alg = OracleAlgorithm(orc, kind, **st)
        r, trace = alg.execute(res, mod, psf[None])
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), trace=trace, residual=res[0], model=mod[0],
            iterations=np.uint64(r.iteration_number), final_peak=np.float32(r.final_peak),
            meta=json.dumps(dict(kind=kind, w=w, n_points=n_points, n_blobs=n_blobs,
                                 seed=seed, settings=st)))
        print(name, r.iteration_number, "components")


if __name__ == "__main__":
    main()
