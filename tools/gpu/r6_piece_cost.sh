#!/bin/bash
# Where the exchange pieces' extra rank time goes: kernel stats of P = 2 serial ranks (10 M reads each)
# with 1 and 4 pieces.  Usage: tools/gpu/r6_piece_cost.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG=${1:-r6pc}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for pc in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_p$pc" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks 2 --reads 10000000 --steps 2 --serial --no-single --pieces $pc > "$OUT/sim_p$pc.json" 2> "$OUT/sim_p$pc.err" || { echo "prof rc=$?"; tail -5 "$OUT/sim_p$pc.err"; exit 1; }
  python3 "$R/tools/kstats.py" "$OUT/stats_p$pc" 40 > "$OUT/kernel_stats_p$pc.txt" 2>&1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pieces', sys.argv[2], 'held', d['rank_held_ms'])" "$OUT/sim_p$pc.json" $pc
  head -25 "$OUT/kernel_stats_p$pc.txt"
done
