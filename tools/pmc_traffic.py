#!/usr/bin/env python3
"""HBM traffic per launch of bench.py's kernel families, from rocprofv3 PMC
passes (MI355X_MICROARCH.md, "HBM" and "rocprofv3 PMC slots"):

  FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950, so each gets its
  own run of the same command:
    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D1 -o run -- python3 bench.py \
        --warmup 0 --steps 1 --cpu-outer 0 --tiled-reference 0 --device-resident 0 --timing-all --dump-families D1/fams.json
    rocprofv3 --pmc WRITE_SIZE ...  (same, into D2)
  then
    python tools/pmc_traffic.py D1/run_results.db D2/run_results.db D1/fams.json \
        --out profiles/r01_traffic.json

gfx950 corrections: FETCH_SIZE counts half the bytes of wide coalesced
streaming reads, so it is doubled; WRITE_SIZE is taken as is. The unit of
both (rocprofv3 reports KiB) is calibrated here on the streaming element-wise
families whose bytes are exact (integrate, add): the calibration is printed
and stored next to the result.

A family's traffic per launch = the summed bytes of the kernels that only that
family launches / the family's launch count in the same run (--timing-all
counts every launch of the process).
"""
import argparse
import json
import re
import sqlite3
import sys
from collections import defaultdict

# kernels that belong to exactly one bench.py family (regex on the kernel name)
FAMILY_KERNELS = {
    "fft": r"_sp_",  # rocFFT single-precision kernels (only rdl_fft_* launches them)
    "spectrum_multiply": r"^rdl::SpectrumMultiply\(",
    "subminor_loop": r"SubminorLoop",
    "subminor_table": r"BuildPairTable",
    "subminor_select": r"^rdl::Sel(Count|Scan|Scatter|SinglePass|Gather|Local|LocalQuad|Place)\(",
    "find_peak": r"^void rdl::FindPeak|^rdl::FindPeakFinal",
    "integrate": r"^rdl::IntegrateKernel\(",
    "add": r"^rdl::AddKernel\(",
    # the LDS FFT engine: float32 scale convolutions (four-step columns)
    "conv_cols": r"rdl::ff::(ColStepA|ColStepB|ColStepBScales|ColStepAInv|Columns<float)",
    "conv_rows": r"rdl::ff::Rows(Inverse|Forward)(<float|Dma<)",
}
# families whose kernels are shared with a sibling family: measured together,
# over the summed launches and algorithmic bytes of both (the *_sparse
# families count a lower bound: the skipped zero rows are not known on the host)
GROUPS = {
    "conv64_cols+conv64_cols_sparse": (r"rdl::ff::Columns(ConvD)?<(double|512u|1024u)",
                                       ("conv64_cols", "conv64_cols_sparse")),
    "conv64_rows+conv64_rows_sparse": (r"rdl::ff::Rows(Inverse|Forward)<double",
                                       ("conv64_rows", "conv64_rows_sparse")),
}
CALIBRATION = ("integrate", "add")


def load_pmc(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    name_col = next((n for n in ("kernel_name", "name") if n in cols), None)
    val_col = next((n for n in ("value", "counter_value") if n in cols), None)
    cnt_col = next((n for n in ("counter_name", "counter") if n in cols), None)
    if not (name_col and val_col and cnt_col):
        sys.exit(f"unexpected counters_collection columns: {cols}")
    out = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    did = "dispatch_id" if "dispatch_id" in cols else None
    q = f"select {name_col}, {cnt_col}, {val_col}" + (f", {did}" if did else "") + \
        " from counters_collection"
    for row in c.execute(q):
        out[row[0]][row[1]] += float(row[2])
        if did:
            disp[row[0]].add(row[3])
    return out, {k: len(v) for k, v in disp.items()}


def family_sum(pmc, counter, pattern):
    rx = re.compile(pattern)
    return sum(v.get(counter, 0.0) for k, v in pmc.items() if rx.search(k))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_db")
    ap.add_argument("write_db")
    ap.add_argument("families")
    ap.add_argument("--out")
    a = ap.parse_args()
    fetch, _ = load_pmc(a.fetch_db)
    write, _ = load_pmc(a.write_db)
    fams = json.load(open(a.families))

    # unit calibration on exact streaming families: bytes / (2*FETCH + WRITE)
    ratios = []
    for f in CALIBRATION:
        if f not in fams or not fams[f]["launches"]:
            continue
        raw = 2.0 * family_sum(fetch, "FETCH_SIZE", FAMILY_KERNELS[f]) + \
            family_sum(write, "WRITE_SIZE", FAMILY_KERNELS[f])
        if raw > 0:
            ratios.append(fams[f]["bytes"] / raw)
    unit = 1024.0
    if ratios:
        r = sorted(ratios)[len(ratios) // 2]
        unit = 1024.0 if abs(r / 1024.0 - 1.0) < 0.5 else (1.0 if abs(r - 1.0) < 0.5 else r)
    result = {"unit_bytes_per_count": unit, "calibration_ratio": ratios,
              "fetch_doubled": True, "families": {}}
    for f, pattern in FAMILY_KERNELS.items():
        if f not in fams or not fams[f]["launches"]:
            continue
        n = fams[f]["launches"]
        rd = 2.0 * family_sum(fetch, "FETCH_SIZE", pattern) * unit
        wr = family_sum(write, "WRITE_SIZE", pattern) * unit
        alg = fams[f]["bytes"] / n
        result["families"][f] = {
            "launches": n, "read_bytes_per_launch": rd / n, "write_bytes_per_launch": wr / n,
            "traffic_per_launch": (rd + wr) / n, "algorithmic_per_launch": alg,
            "traffic_over_algorithmic": (rd + wr) / n / alg if alg else None}
    for g, (pattern, members) in GROUPS.items():
        n = sum(fams[f]["launches"] for f in members if f in fams)
        alg_total = sum(fams[f]["bytes"] for f in members if f in fams)
        if not n:
            continue
        rd = 2.0 * family_sum(fetch, "FETCH_SIZE", pattern) * unit
        wr = family_sum(write, "WRITE_SIZE", pattern) * unit
        result["families"][g] = {
            "launches": n, "read_bytes_per_launch": rd / n, "write_bytes_per_launch": wr / n,
            "traffic_per_launch": (rd + wr) / n, "algorithmic_per_launch": alg_total / n,
            "traffic_over_algorithmic": (rd + wr) / alg_total if alg_total else None,
            "note": "shared kernels; sparse members count a lower bound of their bytes"}
    text = json.dumps(result, indent=1)
    if a.out:
        open(a.out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
