#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd database (the default output
of `rocprofv3 --kernel-trace` on ROCm 7.2), and per-kernel PMC sums when the
database holds counter collection (`--pmc`).

  python tools/rocpd_stats.py run_results.db [--csv out.csv] [--top out.txt]
         [--title "command line"]
  python tools/rocpd_stats.py pmc.db --pmc          # per-kernel counter sums

The rocprofv3 process can crash at exit after the database is written (seen
on this image); the dispatch rows are complete by then, so the statistics are
computed here instead of relying on its --stats CSVs.
"""
import argparse
import csv
import sqlite3
import sys
from collections import defaultdict


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0, float("inf"), 0.0])
    for name, dur in rows:
        a = agg[name]
        a[0] += 1
        a[1] += dur
        a[2] = min(a[2], dur)
        a[3] = max(a[3], dur)
    total = sum(a[1] for a in agg.values())
    out = []
    for name, (n, t, lo, hi) in agg.items():
        out.append({"name": name, "calls": n, "total_ns": t, "avg_ns": t / n,
                    "min_ns": lo, "max_ns": hi, "percent": 100.0 * t / total if total else 0.0})
    out.sort(key=lambda r: -r["total_ns"])
    return out, total


def pmc_stats(db):
    """{kernel name: {counter: (sum, dispatches)}} from the counters_collection view."""
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    q = (f"select {name_col}, counter_name, sum(value), count(distinct dispatch_id) "
         f"from counters_collection group by {name_col}, counter_name")
    out = defaultdict(dict)
    for name, counter, total, n in c.execute(q):
        out[name][counter] = (float(total), int(n))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top")
    ap.add_argument("--title", default="")
    ap.add_argument("--pmc", action="store_true")
    ap.add_argument("-n", type=int, default=40)
    a = ap.parse_args()
    if a.pmc:
        for name, counters in sorted(pmc_stats(a.db).items()):
            print(name[:90], {k: v for k, v in counters.items()})
        return
    rows, total = kernel_stats(a.db)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage",
                        "MinNs", "MaxNs"])
            for r in rows:
                w.writerow([r["name"], r["calls"], int(r["total_ns"]), round(r["avg_ns"], 1),
                            round(r["percent"], 4), int(r["min_ns"]), int(r["max_ns"])])
    lines = []
    if a.title:
        lines.append(a.title)
    lines.append(f"total kernel time {total / 1e6:.1f} ms")
    lines.append(f"{'kernel':90s} {'calls':>7s} {'total ms':>9s} {'avg us':>9s} {'%':>6s}")
    for r in rows[: a.n]:
        lines.append(f"{r['name'][:90]:90s} {r['calls']:7d} {r['total_ns'] / 1e6:9.2f} "
                     f"{r['avg_ns'] / 1e3:9.1f} {r['percent']:6.2f}")
    text = "\n".join(lines) + "\n"
    if a.top:
        open(a.top, "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
