#!/bin/bash
# Kernel breakdown of the default bench's device path under an environment setting.
# Usage: tools/gpu/kprof_env.sh <tag> "<VAR=v ...>"|-   (outputs under gpurun_out/<tag>)
R="$GRAFT_REPO_ROOT"; TAG=$1; E=$2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
[ "$E" != "-" ] && export $E
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "prof rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
python3 "$R/tools/kstats.py" "$OUT/stats" 60 > "$OUT/kernel_stats.txt" 2>&1
