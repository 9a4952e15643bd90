#!/bin/bash
# rocprofv3 kernel stats of the default bench, then separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# for the dominant kernel.  Usage: run_prof.sh <tag> [bench args...]
R="$GRAFT_REPO_ROOT"; TAG=${1:-r1}; shift
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 $ARGS > "$OUT/bench_stats.log" 2>&1 || { echo "stats rc=$?"; tail -20 "$OUT/bench_stats.log"; exit 1; }
echo stats ok
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex onesweep -d "$OUT/fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 $ARGS > "$OUT/pmc_fetch.log" 2>&1 || { echo "fetch rc=$?"; tail -20 "$OUT/pmc_fetch.log"; exit 1; }
echo fetch ok
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex onesweep -d "$OUT/write" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 $ARGS > "$OUT/pmc_write.log" 2>&1 || { echo "write rc=$?"; tail -20 "$OUT/pmc_write.log"; exit 1; }
echo write ok
find "$OUT" -name "*.csv" | head -20
