#!/bin/bash
# tests + bench + kernel stats (no PMC).  Usage: run_gpu4.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench.log | cut -c1-1600
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/stats" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log" 2>&1
echo "prof rc=$?"
