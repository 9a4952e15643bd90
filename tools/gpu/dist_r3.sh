#!/bin/bash
# dist_sim at P = 1, 2, 8: concurrent wall ratios, and serial work ratios (one rank on the device at a
# time, each rank's device time measured alone); kernel profile of the serial P = 8 ranks.
# Usage: tools/gpu/dist_r3.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG=${1:-dist}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
for P in 1 2 8; do
  N=10000000; [ $P = 8 ] && N=2500000
  timeout -k 10 300 python3 -u tools/dist_sim.py --ranks $P --reads $N > "$OUT/p$P.json" 2> "$OUT/p$P.err" || { echo "p$P failed"; tail -5 "$OUT/p$P.err"; exit 1; }
  timeout -k 10 300 python3 -u tools/dist_sim.py --ranks $P --reads $N --serial > "$OUT/s$P.json" 2> "$OUT/s$P.err" || { echo "s$P failed"; tail -5 "$OUT/s$P.err"; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys
for p in (1, 2, 8):
    d = json.load(open("%s/p%d.json" % (sys.argv[1], p)))
    s = json.load(open("%s/s%d.json" % (sys.argv[1], p)))
    print(p, "single %.1f ms, concurrent %.1f ms (%.2f), serial wall %.1f ms, work ratio %s, max-rank ratio %s"
          % (d["single_ms"], d["dist_wall_ms"], d["dist_wall_ms"] / d["single_ms"], s["dist_wall_ms"],
             s["work_ratio"], s["max_rank_ratio"]))
    print("   held", s["rank_held_ms"])
    print("   rank0", s["rank_stages"][0])
PY
cd /tmp && export TMPDIR=/tmp
export MTG_LOCAL_SERIAL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof8" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks 8 --reads 2500000 --steps 1 --no-single --serial > "$OUT/prof8.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof8.log"; exit 1; }
unset MTG_LOCAL_SERIAL
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof8s" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks 8 --reads 2500000 --steps 1 --only-single > "$OUT/prof8s.log" 2>&1 || { echo "prof single failed"; tail -5 "$OUT/prof8s.log"; exit 1; }
echo "== P=8 ranks (serial)"; python3 "$R/tools/kstats.py" "$OUT/prof8" 40
echo "== single"; python3 "$R/tools/kstats.py" "$OUT/prof8s" 25
