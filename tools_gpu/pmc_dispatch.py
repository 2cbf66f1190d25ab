#!/usr/bin/env python3
"""Per-dispatch PMC values of one kernel, grouped by launch index mod G (e.g.
the deme of tools_gpu/alloc_probe.py, which launches demes round robin).

usage: pmc_dispatch.py DIR KERNEL_SUBSTRING [G] [SKIP]
DIR holds rocprofv3 --pmc outputs (any depth); SKIP drops the first launches
(warm-up)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d, pat = sys.argv[1], sys.argv[2]
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    per = defaultdict(dict)  # (file, dispatch) -> counter -> value
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            key = (f, int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    byfile = defaultdict(list)
    for (f, did), cs in per.items():
        byfile[f].append((did, cs))
    for f, lst in byfile.items():
        lst.sort()
        lst = lst[skip:]
        print("==", f, len(lst), "dispatches")
        groups = defaultdict(lambda: defaultdict(list))
        for i, (_, cs) in enumerate(lst):
            for c, v in cs.items():
                groups[i % G][c].append(v)
        names = sorted({c for g in groups.values() for c in g})
        print("%-44s" % "counter" + "".join("%16s" % ("group %d" % g) for g in range(G)))
        for c in names:
            print("%-44s" % c + "".join(
                "%16.5g" % (sum(groups[g][c]) / max(1, len(groups[g][c]))) for g in range(G)))


if __name__ == "__main__":
    main()
