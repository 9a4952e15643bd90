#!/bin/bash
# The pipelined routed rounds on one GPU: a kernel trace of P = 2 ranks (threads, concurrent) with three
# forced rounds, whose exchange copies should run beside the next round's pass B and the previous round's
# owner sort; and the serial cost model with the rounds pipelined / serial.  Usage: tools/gpu/r6_rounds.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG=${1:-r6rounds}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
MTG_RANGES=3 timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks 2 --reads 5000000 --steps 1 --no-single > "$OUT/trace_sim.json" 2> "$OUT/trace_sim.err" || { echo "trace rc=$?"; tail -5 "$OUT/trace_sim.err"; exit 1; }
python3 "$R/tools/overlap.py" "$OUT/trace" > "$OUT/overlap.txt" 2>&1; tail -8 "$OUT/overlap.txt"
cd "$R"
for pc in 1 4; do
  MTG_RANGES=3 timeout -k 10 300 python3 tools/dist_sim.py --ranks 2 --reads 10000000 --steps 3 --no-single --pieces $pc > "$OUT/c2_r3_p${pc}.json" 2> "$OUT/c2_r3_p${pc}.err" || { echo "conc rc=$?"; tail -5 "$OUT/c2_r3_p${pc}.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'wall', round(d['dist_wall_ms'],2), [ (s['exchange_ms'], s['exchange_hidden_ms']) for s in d['rank_stages']])" "$OUT/c2_r3_p${pc}.json"
  MTG_RANGES=3 timeout -k 10 300 python3 tools/dist_sim.py --ranks 2 --reads 10000000 --steps 3 --serial --pieces $pc > "$OUT/s2_r3_p${pc}.json" 2> "$OUT/s2_r3_p${pc}.err" || { echo "serial rc=$?"; tail -5 "$OUT/s2_r3_p${pc}.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'held', d['rank_held_ms'], 'work', d['work_ratio'])" "$OUT/s2_r3_p${pc}.json"
done
