#!/bin/bash
# Round 4: kernel breakdown of the serial P = 8 and P = 2 routed ranks (no single build), per-launch traces.
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-r4n}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-"8 2500000" "2 10000000"}; do
  set -- $cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/p$1" -o run --output-format csv -- python3 "$R/tools/dist_sim.py" --ranks $1 --reads $2 --steps 1 --serial --no-single $EXTRA > "$OUT/p$1.json" 2> "$OUT/p$1.err" || { echo "prof P=$1 rc=$?"; tail -5 "$OUT/p$1.err"; exit 1; }
  python3 "$R/tools/kstats.py" "$OUT/p$1" 60 > "$OUT/p$1_kernel_stats.txt" 2>&1
  python3 "$R/tools/klaunch.py" "$OUT/p$1" > "$OUT/p$1_launches.txt" 2>&1
  head -45 "$OUT/p$1_kernel_stats.txt"
done
