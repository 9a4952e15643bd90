#!/bin/bash
# HBM traffic of the K2 partition pass: separate FETCH_SIZE / WRITE_SIZE passes (PMC runs with
# nothing but counter collection), over the bench and over an 8-byte-lane copy of known size
# (calibration of the counters at this access width).  Usage: run_pmc.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex "copy8_kernel" -d "$OUT/calib_$ctr" -o run --output-format csv -- "$GRAFT_REPO_ROOT/tools/stage_bench" calib > "$OUT/calib_$ctr.log" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex "msd_partition_kernel|msd_hist_kernel|local_unique|local_merge|group_gather|rc_map|extract_kernel|extract_partition|extract_hist|merge_kernel|emit_fast|split_emit|dummy_sink|dummy_rank|onesweep" -d "$OUT/bench_$ctr" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/bench_$ctr.log" 2>&1 || exit 1
  echo "$ctr done"
done
