#!/bin/bash
# Round 4: the dummy-sink ablations (tools/sink_bench), A/B of local_unique's deferred list positions
# (MTG_LU_FAST), and the parity tests of the sort paths.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4l; mkdir -p $OUT
timeout -k 10 180 tools/sink_bench > $OUT/sink_bench.txt 2>&1; rc=$?; cat $OUT/sink_bench.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_env.sh r4l/ab 3 "MTG_LU_FAST=0" "MTG_LU_FAST=1" || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_rounds.py tests/test_gpu_scale.py -m gpu > $OUT/pytest.txt 2>&1
rc=$?; tail -n 4 $OUT/pytest.txt; exit $rc
