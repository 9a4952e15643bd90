#!/bin/bash
# End-of-round profile of the default bench: rocprofv3 kernel stats, then separate FETCH_SIZE /
# WRITE_SIZE passes (counter collection only) over the bench and over an 8-byte-lane copy of known
# size that calibrates the counters.  Needs tools/stage_bench (make -C tools).
# Usage: tools/gpu/prof_round.sh <tag> [stats]   (outputs under gpurun_out/<tag>; `stats` skips the PMC passes)
R="$GRAFT_REPO_ROOT"; TAG=${1:-prof}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 > "$OUT/bench_stats.log" 2>&1 || { echo "stats rc=$?"; tail -20 "$OUT/bench_stats.log"; exit 1; }
echo "stats ok"
python3 "$R/tools/kstats.py" "$OUT/stats" > "$OUT/kernel_stats.txt" 2>&1 || true
[ "$2" = "stats" ] && exit 0
KRE="msd_partition_kernel|msd_hist_kernel|local_unique|extract_partition|extract_hist|merge_kernel|split_emit|dummy_sink|dummy_rank|group_gather|rc_map"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "copy8_kernel" -d "$OUT/calib_$ctr" -o run --output-format csv -- "$R/tools/stage_bench" calib > "$OUT/calib_$ctr.log" 2>&1 || { echo "calib $ctr failed"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex "$KRE" -d "$OUT/bench_$ctr" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --host-steps 0 > "$OUT/bench_$ctr.log" 2>&1 || { echo "bench $ctr failed"; exit 1; }
  echo "$ctr ok"
done
