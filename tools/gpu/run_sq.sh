#!/bin/bash
# One PMC pass of SQ counters (wave cycles, stalls, LDS) over selected kernels of one bench step.
# Usage: tools/gpu/run_sq.sh <tag> <kernel regex> <counters...>
R="$GRAFT_REPO_ROOT"; TAG=${1:-sq}; KRE=$2; shift 2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d "$OUT/pmc" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --host-steps 0 > "$OUT/bench.log" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/bench.log"; exit 1; }
python3 - "$OUT/pmc" <<'PY'
import csv, glob, sys, collections
f = sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True))[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]; n = n[:n.index("(")] if "(" in n else n
    acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, d in acc.items():
    print(n[:70]); print("   " + "  ".join("%s=%.3g" % kv for kv in sorted(d.items())))
PY
