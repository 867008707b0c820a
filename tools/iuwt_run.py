#!/usr/bin/env python3
"""bench.py's C4 leg alone (IuwtDecomposition 4096^2 decompose / recompose
device time, then the IUWT algorithm to its stop), one JSON line; for
strip-width and mode comparisons (RDL_IUWT_FUSED, RDL_IUWT_CHAIN_WS) and for
a kernel trace of the algorithm without the rest of the bench."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-radler_amd"))

import bench  # noqa: E402


def main():
    import radler as rd
    out = bench.iuwt_leg(rd)
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("RDL_IUWT")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
