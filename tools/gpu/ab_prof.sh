#!/bin/bash
# Per-launch kernel durations of one bench step for each prebuilt library variant ab/<v>/libmtg_boss.so
# (rocprofv3 --kernel-trace; tools/klaunch.py).  Usage: tools/gpu/ab_prof.sh <tag> <variant>...
R="$GRAFT_REPO_ROOT"; TAG=$1; shift; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
LIB="$R/projects2014-metagenome_amd/libmtg_boss.so"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  cp "$R/ab/$v/libmtg_boss.so" "$LIB" || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --fasta-reads 0 > "$OUT/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/$v.log"; exit 1; }
  python3 "$R/tools/klaunch.py" "$OUT/$v" > "$OUT/$v.launches.txt" 2>&1
  echo "== $v"; awk '$1 > 0.1' "$OUT/$v.launches.txt"
done
