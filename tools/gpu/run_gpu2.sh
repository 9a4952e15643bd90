#!/bin/bash
# parity tests + default bench + kernel stats.  Usage: run_gpu2.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/$TAG/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/run_prof.sh $TAG/prof
