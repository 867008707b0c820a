"""Per-launch sub-minor loop statistics from RDL_TRACE_SUBMINOR=1/2 stderr
([subminor] lines): launches binned by selection size with us per
iteration and share of the loop time.

    python tools/subminor_stats.py trace.err [--last-iterations N]

--last-iterations N keeps only the trailing launches whose iterations add up
to N (e.g. one Perform of the bench: its components_per_step).
"""
import re
import sys

BINS = [64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 1 << 30]


def main():
    path = sys.argv[1]
    last = None
    if "--last-iterations" in sys.argv:
        last = int(sys.argv[sys.argv.index("--last-iterations") + 1])
    rows = []
    for line in open(path):
        if not line.startswith("[subminor]"):
            continue
        d = dict(re.findall(r"(\w+)=([\d.]+)", line))
        rows.append({k: float(v) for k, v in d.items()})
    if last is not None:
        acc, keep = 0, []
        for r in reversed(rows):
            if acc >= last:
                break
            acc += r["iters"]
            keep.append(r)
        rows = list(reversed(keep))
    tot_us = sum(r["us"] for r in rows)
    tot_it = sum(r["iters"] for r in rows)
    print(f"{len(rows)} launches, {tot_it:.0f} iterations, {tot_us / 1e3:.1f} ms "
          f"({tot_us / max(tot_it, 1):.2f} us/iteration)")
    print(f"{'n_sel <=':>9} {'launches':>8} {'iters':>9} {'ms':>8} {'share':>6} {'us/it':>6} "
          f"{'kinds (kind/threads/g)'}")
    lo = 0
    for hi in BINS:
        sel = [r for r in rows if lo < r["n_sel"] <= hi]
        lo = hi
        if not sel:
            continue
        us = sum(r["us"] for r in sel)
        it = sum(r["iters"] for r in sel)
        kinds = sorted({(int(r["kind"]), int(r["threads"]), int(r["g"])) for r in sel})
        ks = " ".join(f"{k}/{t}/{g}" for k, t, g in kinds[:6])
        print(f"{hi:9d} {len(sel):8d} {it:9.0f} {us / 1e3:8.1f} {us / tot_us:6.1%} "
              f"{us / max(it, 1):6.2f} {ks}")
    ph = ["gather", "integ", "wred", "bar", "xchg", "dec"]
    if any(r.get("gather", 0) for r in rows):
        print("phase cycles per iteration (workgroup 0, wave 0), by bin:")
        lo = 0
        for hi in BINS:
            sel = [r for r in rows if lo < r["n_sel"] <= hi]
            lo = hi
            it = sum(r["iters"] for r in sel)
            if not sel or not it:
                continue
            print(f"{hi:9d} " + " ".join(
                f"{p} {sum(r.get(p, 0) for r in sel) / it:7.0f}" for p in ph))


if __name__ == "__main__":
    main()
