"""One selNSGA2 from a rocprofv3 kernel trace: the launches between the k-th
and (k+1)-th count-pass kernel (argv[2], default the 3rd), kernel time per
name, wall, and the peel / order durations and the gaps between launches."""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[3] if len(sys.argv) > 3 else "bd_count"
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
seq = rows[idx[k] - 12: idx[k + 1] - 12] if k + 1 < len(idx) else rows[idx[k] - 12:]
t0 = int(seq[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in seq)
agg = defaultdict(float)
cnt = defaultdict(int)
for r in seq:
    agg[r["Kernel_Name"][:48]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[r["Kernel_Name"][:48]] += 1
print("launches %d, wall %.1f us, kernels %.1f us" % (len(seq), (end - t0) / 1e3, sum(agg.values())))
for n, v in sorted(agg.items(), key=lambda x: -x[1])[:14]:
    print("  %-48s %4d %8.1f" % (n, cnt[n], v))
pe = [r for r in seq if "peel" in r["Kernel_Name"] or "front_order" in r["Kernel_Name"]]
print("peel/order durations and the gap before each (us):")
line = []
for a, b in zip(pe, pe[1:]):
    gap = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    line.append("%s%.0f+%.0f" % ("P" if "peel" in b["Kernel_Name"] else "o",
                                  (int(b["End_Timestamp"]) - int(b["Start_Timestamp"])) / 1e3, gap))
print(" ".join(line))
