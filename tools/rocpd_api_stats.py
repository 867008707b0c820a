#!/usr/bin/env python3
"""HIP API and GPU-idle summary of a rocprofv3 rocpd database made with
--hip-trace (or --runtime-trace) --kernel-trace.

  python tools/rocpd_api_stats.py run_results.db [--out summary.txt]

Prints the database's views/columns (the rocpd schema varies by ROCm
version), per-API call counts and total/avg durations, and the GPU busy
fraction (union of kernel and copy intervals over the traced span).
"""
import argparse
import sqlite3
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--out")
    a = ap.parse_args()
    out = open(a.out, "w") if a.out else sys.stdout
    c = sqlite3.connect(a.db)
    objs = c.execute("select name, type from sqlite_master where type in ('view','table') "
                     "order by type, name").fetchall()
    cols = {}
    for name, typ in objs:
        try:
            cols[name] = [r[1] for r in c.execute(f"pragma table_info('{name}')")]
        except sqlite3.Error:
            cols[name] = []
    print("# schema", file=out)
    for name, typ in objs:
        if not name.startswith("rocpd_") or typ == "view":
            print(f"{typ:5s} {name}: {', '.join(cols[name][:16])}", file=out)
    # API regions
    for view in ("regions", "region"):
        if view in cols and {"name", "start", "end"} <= set(cols[view]):
            rows = c.execute(f"select name, start, end from {view}").fetchall()
            agg = defaultdict(lambda: [0, 0])
            for n, s, e in rows:
                agg[n][0] += 1
                agg[n][1] += e - s
            print(f"\n# {view}: {len(rows)} calls", file=out)
            print(f"{'api':50s} {'calls':>9s} {'total ms':>11s} {'avg us':>9s}", file=out)
            for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
                print(f"{n[:50]:50s} {k:9d} {t * 1e-6:11.2f} {t * 1e-3 / k:9.2f}", file=out)
            break
    # GPU busy fraction
    iv = []
    for view in ("kernels", "memory_copies"):
        if view in cols and {"start", "end"} <= set(cols[view]):
            iv += c.execute(f"select start, end from {view}").fetchall()
    if iv:
        iv.sort()
        busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        span = max(e for _, e in iv) - iv[0][0]
        print(f"\n# GPU busy {busy * 1e-9:.3f} s of {span * 1e-9:.3f} s span "
              f"({100.0 * busy / span:.1f} %), {len(iv)} intervals", file=out)
        # idle gaps and the host API calls overlapping them: what the host was
        # doing while the GPU had nothing to run
        gaps = []
        cur_e = iv[0][1]
        for s_, e_ in iv[1:]:
            if s_ > cur_e:
                gaps.append((cur_e, s_))
            cur_e = max(cur_e, e_)
        total_gap = sum(b - a for a, b in gaps)
        big = [g for g in gaps if g[1] - g[0] > 20000]
        print(f"# idle gaps: {len(gaps)} totalling {total_gap * 1e-9:.3f} s; "
              f"{len(big)} longer than 20 us totalling "
              f"{sum(b - a for a, b in big) * 1e-9:.3f} s", file=out)
        if "regions" in cols:
            regs = sorted(c.execute("select name, start, end from regions").fetchall(),
                          key=lambda r: r[1])
            import bisect
            starts = [r[1] for r in regs]
            blame = defaultdict(int)
            for a_, b_ in big:
                i = max(0, bisect.bisect_left(starts, a_) - 2000)
                while i < len(regs) and regs[i][1] < b_:
                    n, rs, re_ = regs[i]
                    ov = min(re_, b_) - max(rs, a_)
                    if ov > 0:
                        blame[n] += ov
                    i += 1
            print("# host API time overlapping the >20 us idle gaps", file=out)
            for n, t in sorted(blame.items(), key=lambda kv: -kv[1])[:25]:
                print(f"{n[:60]:60s} {t * 1e-6:11.2f} ms", file=out)


if __name__ == "__main__":
    main()
