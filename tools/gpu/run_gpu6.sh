#!/bin/bash
# sort checker + stage microbenchmark, then tests + bench + kernel stats.  Usage: run_gpu6.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 ./tools/msd_test > gpurun_out/$TAG/msd_test.log 2>&1
rc=$?; echo "msd_test rc=$rc"; tail -3 gpurun_out/$TAG/msd_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/run_gpu5.sh $TAG
