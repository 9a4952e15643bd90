#!/bin/bash
# Round 4: multi-GPU cost model per collect mode (serial dist_sim: per-rank device time alone, and the
# bytes every rank sends), P = 2 (10 M reads per rank) and P = 8 (2.5 M reads per rank).
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r4d"; mkdir -p "$OUT"; cd "$R"
for P in 2 8; do
  N=10000000; [ $P = 8 ] && N=2500000
  for mode in routed superkmer local; do
    [ $P = 2 ] && [ $mode = local ] && continue
    timeout -k 10 300 python3 -u tools/dist_sim.py --ranks $P --reads $N --serial --collect $mode > "$OUT/s${P}_$mode.json" 2> "$OUT/s${P}_$mode.err" || { echo "s$P $mode failed"; tail -5 "$OUT/s${P}_$mode.err"; exit 1; }
    python3 - "$OUT/s${P}_$mode.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sb = d.get("sent_bytes") or [0]
print("%s: single %.1f ms, work ratio %s, max-rank ratio %s, held %s, sent GB/rank max %.2f" % (
    sys.argv[1].split("/")[-1], d["single_ms"], d["work_ratio"], d["max_rank_ratio"], d["rank_held_ms"], max(sb) / 1e9))
PY
  done
done
