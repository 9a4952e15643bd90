#!/bin/bash
# Kernel stats + the per-launch listing of the last step of a config preset (two steps traced).
# Usage: tools/gpu/prof_cfg_launches.sh <tag> <config> <first-kernel regex> [extra bench args]
R="$GRAFT_REPO_ROOT"; TAG=${1:-prof}; CFG=${2:-cfg3}; FIRST=${3:-extract_hist}; shift 3
bash "$R/tools/gpu/prof_cfg.sh" "$TAG" "$CFG" --warmup 1 "$@" > /dev/null || exit 1
python3 "$R/tools/klaunch.py" "$R/gpurun_out/$TAG/stats" "$FIRST" > "$R/gpurun_out/$TAG/kernel_launches.txt" 2>&1
head -40 "$R/gpurun_out/$TAG/kernel_stats.txt"
