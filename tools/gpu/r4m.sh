#!/bin/bash
# Round 4: profiles of the default step (kernel stats + launches, SQ counters of the local passes and
# the fused pass B, calibrated HBM traffic), then the multi-GPU cost model (tools/gpu/r4d.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4m
make -s -C tools stage_bench -j8 > gpurun_out/r4m/make.txt 2>&1 || { echo "stage_bench build failed"; cat gpurun_out/r4m/make.txt; exit 1; }
bash tools/gpu/prof_r3.sh r4m/prof "local_unique|local_merge|dummy_sink|extract_partition_fast" || exit 1
bash tools/gpu/prof_round.sh r4m/pmc || exit 1
python3 tools/pmc_summary.py gpurun_out/r4m/pmc gpurun_out/r4m/r4 > gpurun_out/r4m/pmc_summary.txt 2>&1; head -n 30 gpurun_out/r4m/pmc_summary.txt
bash tools/gpu/r4d.sh
