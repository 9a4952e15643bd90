#!/bin/bash
# Round 4: multi-GPU cost model per collect mode (serial dist_sim: per-rank device time alone, and the
# bytes every rank sends), P = 2 (10 M reads per rank) and P = 8 (2.5 M reads per rank); P = 2 also with
# the 9-bit routing digit (MTG_WIDE_B1=0).
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r4d}"; mkdir -p "$OUT"; cd "$R"
run() {  # tag P N collect [env]
  env $5 timeout -k 10 300 python3 -u tools/dist_sim.py --ranks $2 --reads $3 --serial --collect $4 > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "$1 failed"; tail -5 "$OUT/$1.err"; exit 1; }
  python3 - "$OUT/$1.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sb = d.get("sent_bytes") or [0]
print("%s: single %.1f ms, work ratio %s, max-rank ratio %s, held %s, sent GB/rank max %.2f" % (
    sys.argv[1].split("/")[-1], d["single_ms"], d["work_ratio"], d["max_rank_ratio"], d["rank_held_ms"], max(sb) / 1e9))
PY
}
run s2_routed 2 10000000 routed || exit 1
run s2_routed_b9 2 10000000 routed MTG_WIDE_B1=0 || exit 1
run s2_superkmer 2 10000000 superkmer || exit 1
run s8_routed 8 2500000 routed || exit 1
run s8_superkmer 8 2500000 superkmer || exit 1
run s8_local 8 2500000 local || exit 1
