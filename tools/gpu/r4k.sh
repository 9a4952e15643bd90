#!/bin/bash
# Round 4: A/B of local_unique_kernel's FAST probe loop (MTG_LU_FAST), then the whole -m gpu suite
# and the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4k; mkdir -p $OUT
bash tools/gpu/ab_env.sh r4k/ab 3 "MTG_LU_FAST=0" "MTG_LU_FAST=1" || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -n 4 $OUT/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -n 3 $OUT/bench.err; cat $OUT/bench.json; exit $rc
