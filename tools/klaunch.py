"""Per-launch kernel durations of the last bench step from a rocprofv3 --kernel-trace run:
the launches from the last `extract_hist_fast_kernel` (the first kernel of a step) up to the
next step, in order, numbered per kernel.  Usage: klaunch.py <rocprof dir> [first-kernel regex]"""
import csv
import glob
import re
import sys

d = sys.argv[1]
first = re.compile(sys.argv[2] if len(sys.argv) > 2 else "extract_hist_fast_kernel")
path = sorted(glob.glob(d + "/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first.search(r["Kernel_Name"])]
if len(starts) < 2:
    sys.exit("fewer than two steps in the trace")
a, b = starts[-2], starts[-1]  # the last complete step (the final one may be followed by host legs)
seen = {}
tot = 0.0
for r in rows[a:b]:
    n = r["Kernel_Name"]
    n = n[:n.index("(")] if "(" in n else n
    seen[n] = seen.get(n, 0) + 1
    ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot += ms
    print("%8.3f ms  %s #%d" % (ms, n[:90], seen[n]))
print("%8.3f ms  total kernel time of the step" % tot)
