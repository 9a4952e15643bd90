#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 ./tools/sort_bench 1200000000 > gpurun_out/$TAG/sort_bench.log 2>&1
rc=$?; echo "sort_bench rc=$rc"; grep -E "msd|mtg|copy|rocprim|ok=" gpurun_out/$TAG/sort_bench.log | head -30
if [ $rc -ne 0 ]; then tail -5 gpurun_out/$TAG/sort_bench.log; exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench.log | cut -c1-1500
exit $rc
