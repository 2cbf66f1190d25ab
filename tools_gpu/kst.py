"""Print the top kernels of a rocprofv3 kernel_stats.csv (name, calls, total us, avg us)."""
import csv, sys
for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    print(path)
    for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:int(__import__("os").environ.get("TOP", "12"))]:
        print("  %-58s %6s %10.1f us %8.1f avg" % (x["Name"][:58], x["Calls"], float(x["TotalDurationNs"]) / 1e3,
                                                  float(x["AverageNs"]) / 1e3))
