#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) of one bench step of a config preset.
# Usage: tools/gpu/prof_cfg.sh <tag> <config> [extra bench args]
R="$GRAFT_REPO_ROOT"; TAG=${1:-prof}; CFG=${2:-cfg2}; shift 2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --host-steps 0 "$@" > "$OUT/bench_stats.log" 2>&1 || { echo "stats rc=$?"; tail -20 "$OUT/bench_stats.log"; exit 1; }
python3 "$R/tools/kstats.py" "$OUT/stats" 40 > "$OUT/kernel_stats.txt" 2>&1
cat "$OUT/kernel_stats.txt"
