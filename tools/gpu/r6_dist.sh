#!/bin/bash
# Multi-GPU evidence on one GPU: a kernel trace of P ranks (threads, concurrent) with the exchange
# pieces on their own stream, and the serial cost model at P = 2 and 8 (pieces on / off).
# Usage: tools/gpu/r6_dist.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG=${1:-r6dist}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks 2 --reads 5000000 --steps 1 --no-single > "$OUT/trace_sim.json" 2> "$OUT/trace_sim.err" || { echo "trace rc=$?"; tail -5 "$OUT/trace_sim.err"; exit 1; }
python3 "$R/tools/overlap.py" "$OUT/trace" > "$OUT/overlap.txt" 2>&1; tail -12 "$OUT/overlap.txt"
cd "$R"
for P in 2 8; do
  N=$((20000000 / P))
  for pc in 1 2 4; do
    timeout -k 10 300 python3 tools/dist_sim.py --ranks $P --reads $N --steps 3 --serial --pieces $pc > "$OUT/s${P}_p${pc}.json" 2> "$OUT/s${P}_p${pc}.err" || { echo "sim P=$P rc=$?"; tail -5 "$OUT/s${P}_p${pc}.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'held', d['rank_held_ms'], 'work', d['work_ratio'], 'single', round(d['single_ms'],2), 'sent GB', round(max(d['sent_bytes'])/1e9,3))" "$OUT/s${P}_p${pc}.json"
  done
  timeout -k 10 300 python3 tools/dist_sim.py --ranks $P --reads $N --steps 3 --serial --collect local > "$OUT/s${P}_local.json" 2> "$OUT/s${P}_local.err" || { echo "sim local P=$P rc=$?"; tail -5 "$OUT/s${P}_local.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'held', d['rank_held_ms'], 'work', d['work_ratio'], 'sent GB', round(max(d['sent_bytes'])/1e9,3))" "$OUT/s${P}_local.json"
  timeout -k 10 300 python3 tools/dist_sim.py --ranks $P --reads $N --steps 3 --no-single > "$OUT/c${P}.json" 2> "$OUT/c${P}.err" || { echo "conc P=$P rc=$?"; tail -5 "$OUT/c${P}.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'wall', round(d['dist_wall_ms'],2), [ (s['exchange_ms'], s['exchange_hidden_ms']) for s in d['rank_stages']])" "$OUT/c${P}.json"
done
