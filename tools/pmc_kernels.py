"""Per-kernel PMC counters per dispatch from a rocprofv3 database (one
`--pmc` pass): every counter of the pass, averaged over the kernel's
dispatches, for the kernels whose name matches a pattern.

    python tools/pmc_kernels.py <run_results.db> [name regex]
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import load_pmc  # noqa: E402


def main():
    pmc, disp = load_pmc(sys.argv[1])
    rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for name in sorted(pmc, key=lambda k: -sum(pmc[k].values())):
        if not rx.search(name):
            continue
        n = max(1, disp.get(name, 1))
        print(f"{name[:110]}  ({n} dispatches)")
        for cnt, v in sorted(pmc[name].items()):
            print(f"    {cnt:24s} {v / n:16.4g}")


if __name__ == "__main__":
    main()
