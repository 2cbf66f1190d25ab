"""Kernels launched after the probe's marker (philox_blocks_kernel) in a
rocprofv3 kernel trace: ``python tools_gpu/trace_names.py TRACE.csv [OUT.json]``.
Prints (and writes) the kernel names with their launch counts and the
at::native ones separately; exit status 1 when any at::native kernel ran
after the marker."""
import csv
import json
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
start = None
for r in rows:
    if "philox_blocks_kernel" in r["Kernel_Name"]:
        start = int(r["End_Timestamp"])
        break
if start is None:
    sys.exit("no marker kernel in the trace")
after = Counter()
for r in rows:
    if int(r["Start_Timestamp"]) > start:
        after[r["Kernel_Name"].split("(")[0]] += 1
native = {k: v for k, v in after.items() if "at::native" in k}
out = {"launches_after_marker": sum(after.values()), "kernels": dict(after.most_common()),
       "at_native": native}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)
sys.exit(1 if native else 0)
