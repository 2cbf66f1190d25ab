"""Per-deme tables from tools_gpu/placement_pmc_probe.py's counter passes
(gpurun_out/<tag>/p1..p4: channel RDREQ / WRREQ / RDREQ_DRAM_CREDIT_STALL and
per-XCC RDREQ / WRREQ).  python tools_gpu/placement_pmc_report.py DIR [WARM]"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 8
vals = {}  # (counter, deme) -> [values]
dur = {}
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    rows = [r for r in csv.DictReader(open(f)) if "gen_pipe" in r["Kernel_Name"]]
    disp = sorted({int(r["Dispatch_Id"]) for r in rows})
    order = {x: i for i, x in enumerate(disp)}
    for r in rows:
        k = order[int(r["Dispatch_Id"])]
        if k < warm:
            continue
        deme = (k - warm) % 4
        vals.setdefault((r["Counter_Name"], deme), []).append(float(r["Counter_Value"]))
        dur.setdefault(deme, {})[(f, k)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
out = {"dispatch_ms": {str(m): round(sum(v.values()) / len(v), 4) for m, v in sorted(dur.items())}}
names = sorted({c for c, _ in vals})
for c in names:
    out[c] = [round(sum(vals[(c, m)]) / len(vals[(c, m)]) / 1e6, 4) for m in range(4)]
print(json.dumps(out, indent=0))
