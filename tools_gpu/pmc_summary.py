#!/usr/bin/env python3
"""Summarise a profile.sh output directory: per-kernel average duration from
the kernel-trace stats and per-launch averages of every PMC counter.

usage: pmc_summary.py DIR [kernel-substring ...]
HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md: FETCH_SIZE and
WRITE_SIZE are in KiB; gfx950 FETCH_SIZE counts half the lines (x2)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pats = sys.argv[2:] or ["gen_", "pair_plan", "eval_", "sel_"]
    stats = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    if stats:
        print("== kernel-trace stats")
        for r in csv.DictReader(open(stats[0])):
            if any(p in r["Name"] for p in pats):
                print(f'{r["Name"][:90]:90s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"]) / 1e3:9.2f}'
                      f' pct={float(r["Percentage"]):6.2f}')
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not any(p in name for p in pats):
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in acc.items():
        print("==", name[:110])
        vals = {}
        for c, v in sorted(cs.items()):
            vals[c] = sum(v) / len(v)
            print(f"   {c:24s} {vals[c]:16.4g}  (n={len(v)})")
        if "FETCH_SIZE" in vals or "WRITE_SIZE" in vals:
            hbm = 2 * 1024 * vals.get("FETCH_SIZE", 0.0) + 1024 * vals.get("WRITE_SIZE", 0.0)
            print(f"   HBM bytes/launch (FETCH x2 + WRITE) {hbm:.4g}")


if __name__ == "__main__":
    main()
