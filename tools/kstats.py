"""Summarise a rocprofv3 kernel_stats.csv (and per-launch trace) of a bench run."""
import csv
import glob
import sys

d = sys.argv[1]
path = sorted(glob.glob(d + "/**/*kernel_stats.csv", recursive=True))[0]
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r["Name"]
    name = name[:name.index("(")] if "(" in name else name
    print("%-62s calls=%5s total=%8.2fms avg=%8.3fms %5.1f%%" % (
        name[:62], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6,
        100 * float(r["TotalDurationNs"]) / tot))
