"""Run tests/dist_worker.py's tiled case with RADLER_VERBOSE=1 on every rank
and keep each rank's log (gpurun_out/<tag>/rank<r>.log) and its npz.
Usage: python tools/debug_dist.py <tag> <world> [worker args...]"""
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
tag, world, extra = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
out = os.path.join("gpurun_out", tag)
os.makedirs(out, exist_ok=True)
with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
env = dict(os.environ, RADLER_VERBOSE="1")
procs = []
for r in range(world):
    log = open(os.path.join(out, f"rank{r}.log"), "w")
    procs.append(subprocess.Popen(
        [sys.executable, os.path.join(HERE, "..", "tests", "dist_worker.py"), "--rank", str(r),
         "--world", str(world), "--port", str(port), "--out", out, "--case", "tiled", *extra],
        stdout=log, stderr=subprocess.STDOUT, env=env))
rc = 0
for p in procs:
    rc |= p.wait(timeout=240)
sys.exit(rc)
