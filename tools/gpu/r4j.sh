#!/bin/bash
# Round 4: kernel stats + per-launch trace of the default step, HBM traffic (FETCH_SIZE / WRITE_SIZE
# passes, calibrated), SQ counters of the local passes.
cd "$GRAFT_REPO_ROOT" || exit 1
make -s -C tools stage_bench -j8 > gpurun_out/r4j_make.txt 2>&1 || { echo "stage_bench build failed"; cat gpurun_out/r4j_make.txt; exit 1; }
bash tools/gpu/prof_r3.sh r4j/prof "local_unique|local_merge|dummy_sink|extract_partition_fast" || exit 1
bash tools/gpu/prof_round.sh r4j/pmc || exit 1
python3 tools/pmc_summary.py gpurun_out/r4j/pmc gpurun_out/r4j/r4 > gpurun_out/r4j/pmc_summary.txt 2>&1; head -n 40 gpurun_out/r4j/pmc_summary.txt
