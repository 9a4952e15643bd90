#!/bin/bash
# The round's default bench line (full parity, cpu_baseline, host legs) and its profiles (kernel stats +
# launch list, FETCH_SIZE / WRITE_SIZE passes, SQ counters).  Usage: tools/gpu/r6_final.sh <tag>
R="$GRAFT_REPO_ROOT"; TAG=${1:-r6final}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json" | cut -c1-400
bash tools/gpu/round_profiles.sh "$TAG/prof" || exit 1
