"""Overlap of the multi-GPU exchange with the build, from a rocprofv3 --kernel-trace of
tools/dist_sim.py (P ranks as host threads on one GPU).  Per rank thread: every exchange copy
(local_copy_kernel) on the exchange stream, and the time the same rank's build-stream kernels ran
while it was in flight.  Usage: overlap.py <rocprof dir> [step index from the end, default 1]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
path = sorted(glob.glob(d + "/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(path)))
sid = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"


def short(n):
    return n[:n.index("(")] if "(" in n else n


by_thread = defaultdict(list)
for r in rows:
    by_thread[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[sid],
                                      short(r["Kernel_Name"])))
tot_copy = tot_hidden = 0.0
for th, ks in sorted(by_thread.items()):
    ks.sort()
    copies = [k for k in ks if k[3].endswith("local_copy_kernel")]
    if not copies:
        continue
    # the exchange stream runs nothing but copies (the build stream also runs the blocking exchanges' copies)
    other = {k[2] for k in ks if not k[3].endswith("local_copy_kernel")}
    xstreams = {k[2] for k in copies} - other
    copies = [k for k in copies if k[2] in xstreams]
    work = [k for k in ks if k[2] not in xstreams]
    print("rank thread %s: %d kernels, %d exchange copies on stream(s) %s" % (th, len(ks), len(copies),
                                                                              sorted(xstreams)))
    for (a, b, s, n) in copies:
        ov = defaultdict(float)
        for (c0, c1, s2, n2) in work:
            lo, hi = max(a, c0), min(b, c1)
            if hi > lo:
                ov[n2] += (hi - lo) / 1e6
        hid = sum(ov.values())
        tot_copy += (b - a) / 1e6
        tot_hidden += min(hid, (b - a) / 1e6)
        if ov:
            top = ", ".join("%s %.3f" % (k, v) for k, v in sorted(ov.items(), key=lambda x: -x[1])[:4])
            print("  copy %.3f ms at +%.3f ms on stream %s, under: %s" % ((b - a) / 1e6, (a - ks[0][0]) / 1e6, s, top))
print("exchange copies %.3f ms, of which %.3f ms ran beside the same rank's build-stream kernels" %
      (tot_copy, tot_hidden))
