#!/usr/bin/env python3
"""Per-selection VALU instructions of C5's front peel from a rocprofv3 --pmc
counter-collection CSV (not a test; run on the GPU box after
``rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -- python
bench.py --config c5 ...``).  Selection boundaries are the count-pass
dispatches (one bd_count_kernel per selNSGA2); the peel_order_kernel dispatches
between two of them belong to one selection.  Writes the median selection's
sums as profiles/c5_peel_pmc.json (bench.py's C5 roofline reads it).

usage: c5_peel_pmc.py PMC_DIR OUT_JSON SOURCE_TAG"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    d, out, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    disp = defaultdict(dict)  # dispatch id -> {name, counters}
    for r in rows:
        k = int(r["Dispatch_Id"])
        disp[k]["name"] = r["Kernel_Name"]
        disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    order = sorted(disp)
    sels, cur = [], None
    for k in order:
        name = disp[k]["name"]
        if "bd_count_kernel" in name:
            cur = defaultdict(float)
            sels.append(cur)
        elif "peel_order_kernel" in name and cur is not None:
            for c, v in disp[k].items():
                if c != "name":
                    cur[c] += v
            cur["launches"] += 1
    sels = [s for s in sels if s.get("launches")]
    med = sorted(sels, key=lambda s: s["SQ_INSTS_VALU"])[len(sels) // 2]
    res = {"kernel": "peel_order_kernel<2>", "selections": len(sels),
           "SQ_INSTS_VALU_per_selection": med["SQ_INSTS_VALU"],
           "SQ_WAVE_CYCLES_per_selection": med.get("SQ_WAVE_CYCLES"),
           "SQ_ACTIVE_INST_VALU_per_selection": med.get("SQ_ACTIVE_INST_VALU"),
           "SQ_ACTIVE_INST_VALU_over_SQ_WAVE_CYCLES":
               (med["SQ_ACTIVE_INST_VALU"] / med["SQ_WAVE_CYCLES"]) if med.get("SQ_WAVE_CYCLES") else None,
           "launches_per_selection": med["launches"],
           "spread_SQ_INSTS_VALU": [min(s["SQ_INSTS_VALU"] for s in sels),
                                    max(s["SQ_INSTS_VALU"] for s in sels)],
           "source": tag}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
