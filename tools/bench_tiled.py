#!/usr/bin/env python3
"""Gridded (ParallelDeconvolution) multiscale major iteration on one field:
subimages one after another (max_threads=1) vs the concurrent worker pool
(max_threads=k, one stream per worker). Same synthetic sky as bench.py.

  python tools/bench_tiled.py [size] [grid] [threads,threads,...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-radler_amd"))

import bench  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    threads = [int(t) for t in (sys.argv[3] if len(sys.argv) > 3 else "1,4,16").split(",")]
    import radler as rd
    psf, dirty = bench.make_problem(size, bench.SEED, 2000, 200)
    threshold = 5.0 * bench.NOISE
    for k in threads:
        s = bench.settings_for(rd, size, 1000000, 6, threshold)
        s.parallel.grid_width = s.parallel.grid_height = grid
        s.parallel.max_threads = k
        run = rd.gpu.DeviceRun(s, psf, dirty, [], bench.BEAM_PX * bench.PIXEL_SCALE)
        run.execute()  # warm-up: plans, scale kernels, worker streams
        times, comps = [], 0
        rd.gpu.host_profile_reset()
        runs = int(os.environ.get("BENCH_TILED_RUNS", "2"))
        for _ in range(runs):
            run.restore()
            run.sync()
            t0 = time.perf_counter()
            r = run.execute()
            run.sync()
            times.append(time.perf_counter() - t0)
            comps = r["iterations"]
        best = min(times)
        print(f"size={size} grid={grid}x{grid} max_threads={k}: {best:.3f} s, "
              f"{comps} components, {comps / best:.0f} components/s", flush=True)
        prof = rd.gpu.host_profile()
        for name, (count, sec) in sorted(prof.items(), key=lambda kv: -kv[1][1]):
            print(f"  [host] {name:30s} {count:9d} {sec / runs:9.3f} s/run "
                  f"{1e6 * sec / max(count, 1):9.1f} us", flush=True)
        del run


if __name__ == "__main__":
    main()
