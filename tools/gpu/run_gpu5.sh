#!/bin/bash
# stage microbenchmark, then tests + bench + kernel stats.  Usage: run_gpu5.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; mkdir -p gpurun_out/$TAG
timeout -k 10 200 ./tools/stage_bench > gpurun_out/$TAG/stage_bench.log 2>&1
rc=$?; echo "stage_bench rc=$rc"; cat gpurun_out/$TAG/stage_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/run_gpu4.sh $TAG
