"""Summarise a tools/profile.sh run: per library kernel, launches, mean duration (kernel trace)
and mean HBM bytes per launch from the PMC passes (FETCH_SIZE x 2 on gfx950 + WRITE_SIZE,
MI355X_MICROARCH.md § HBM).

Usage: python tools/prof_summary.py gpurun_out/prof [profiles/rNN_traffic.json] > profiles/rNN_summary.md
The optional JSON records the dominant gemv kernel's figures for bench.py's roofline.traffic."""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    return name.split("(")[0].replace("void ", "")


def main(d, json_out=None):
    dur = defaultdict(list)
    for r in rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = defaultdict(lambda: defaultdict(list))
    for sub in ("pmc_fetch", "pmc_write"):
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | launches | mean us | FETCH_SIZE x2 MB/launch | WRITE_SIZE MB/launch | HBM MB/launch | GB/s at mean duration |")
    print("|---|---|---|---|---|---|---|")
    best = None
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        if "lk::" not in k:
            continue
        n = len(dur[k])
        us = sum(dur[k]) / n / 1e3
        c = ctr.get(k, {})
        fetch = 2 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) / 1e3 if c.get("FETCH_SIZE") else float("nan")  # KB -> MB
        write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) / 1e3 if c.get("WRITE_SIZE") else float("nan")
        hbm = fetch + write
        print(f"| {k} | {n} | {us:.3f} | {fetch:.3f} | {write:.3f} | {hbm:.3f} | {hbm / us * 1e3:.1f} |")
        if "gemv" in k and best is None:
            best = {"kernel": k, "launches": n, "mean_us": round(us, 3), "hbm_bytes_per_launch": round(hbm * 1e6),
                    "fetch_size_x2_bytes": round(fetch * 1e6), "write_size_bytes": round(write * 1e6)}
    if json_out and best:
        import json
        with open(json_out, "w") as fh:
            json.dump(best, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof", sys.argv[2] if len(sys.argv) > 2 else None)
