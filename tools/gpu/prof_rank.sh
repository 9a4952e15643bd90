#!/bin/bash
# Kernel breakdown of the serial ranks of tools/dist_sim.py (no single build).
# Usage: tools/gpu/prof_rank.sh <tag> <P> <reads per rank> [dist_sim args...]
R="$GRAFT_REPO_ROOT"; TAG=$1; P=$2; N=$3; shift 3; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks $P --reads $N --steps 1 --serial --no-single "$@" > "$OUT/sim.json" 2> "$OUT/sim.err" || { echo "prof rc=$?"; tail -5 "$OUT/sim.err"; exit 1; }
python3 "$R/tools/kstats.py" "$OUT/stats" 60 > "$OUT/kernel_stats.txt" 2>&1
head -40 "$OUT/kernel_stats.txt"
