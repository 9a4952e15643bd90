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
# the build's own work: mtg kernels + device copies (the exchanges of an in-process rank group)
own = sum(float(r["TotalDurationNs"]) for r in rows if "mtg::" in r["Name"] or "copyBuffer" in r["Name"])
print("TOTAL all=%.2fms build=%.2fms" % (tot / 1e6, own / 1e6))
# GPU-busy time of the build (union of its kernel intervals) and of its last third (the timed step
# of dist_sim --steps 1 after 2 warmups)
tr = sorted(glob.glob(d + "/**/*kernel_trace.csv", recursive=True))
if tr:
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(tr[0]))
                if "mtg::" in r["Kernel_Name"] or "copyBuffer" in r["Kernel_Name"])
    busy, cs, ce = 0, None, None
    for a, b in iv:
        if ce is None or a > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if ce is not None:
        busy += ce - cs
    print("BUSY build-union=%.2fms span=%.2fms" % (busy / 1e6, (iv[-1][1] - iv[0][0]) / 1e6 if iv else 0))
