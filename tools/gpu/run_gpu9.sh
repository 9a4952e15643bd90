#!/bin/bash
# parity tests (incl. the multi-rank build) then bench + kernel stats.  Usage: run_gpu9.sh <tag> [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; mkdir -p gpurun_out/$TAG
KEXPR=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/$TAG/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench.log | cut -c1-1600
exit $rc
