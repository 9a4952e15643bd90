#!/bin/bash
# Round 4 final evidence on the committed build: PMC HBM traffic of the default step (calibrated), the
# kernel stats / per-launch trace / SQ counters, then the default bench line exactly as the driver runs it
# (with the new stored partition traffic).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4f; mkdir -p $OUT
make -s -C tools stage_bench -j8 > $OUT/make.txt 2>&1 || { echo "stage_bench build failed"; cat $OUT/make.txt; exit 1; }
bash tools/gpu/prof_round.sh r4f/pmc || exit 1
python3 tools/pmc_summary.py gpurun_out/r4f/pmc gpurun_out/r4f/r4 > $OUT/pmc_summary.txt 2>&1; head -n 30 $OUT/pmc_summary.txt
cp gpurun_out/r4f/r4_partition_traffic.json profiles/r4_partition_traffic.json || exit 1
bash tools/gpu/prof_r3.sh r4f/prof "local_unique|local_merge|dummy_sink|extract_partition_fast" > $OUT/prof.txt 2>&1 || { echo "prof failed"; tail $OUT/prof.txt; exit 1; }
tail -3 $OUT/prof.txt
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-600
