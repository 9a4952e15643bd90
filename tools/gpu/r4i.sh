#!/bin/bash
# Round 4: the whole -m gpu suite, then the default bench line exactly as the driver runs it.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -n 4 $OUT/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -n 3 $OUT/bench.err; cat $OUT/bench.json; exit $rc
