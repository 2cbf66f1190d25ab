"""Print a rocprofv3 kernel_stats.csv compactly: calls, total ms, avg us, %."""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    print("==", path)
    for r in rows[:int(__import__("os").environ.get("TOP", "16"))]:
        name = r["Name"].split("(")[0].replace("void ", "")[:48]
        print("%-48s %6s %9.3f ms %9.1f us %6.2f%%" % (
            name, r["Calls"], int(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3,
            float(r["Percentage"])))
