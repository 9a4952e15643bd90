#!/bin/bash
# Kernel-time breakdown of tools/dist_sim.py (P ranks as threads on one GPU + the single build of
# the same reads): rocprofv3 --kernel-trace --stats.  Usage: tools/gpu/prof_dist.sh <tag> <P> <reads per rank>
R="$GRAFT_REPO_ROOT"; TAG=${1:-pdist}; P=${2:-8}; N=${3:-2500000}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks $P --reads $N --steps 1 $4 > "$OUT/sim.json" 2> "$OUT/sim.err" || { echo "prof rc=$?"; tail -5 "$OUT/sim.err"; exit 1; }
python3 "$R/tools/kstats.py" "$OUT/stats" > "$OUT/kernel_stats.txt" 2>&1; head -40 "$OUT/kernel_stats.txt"
