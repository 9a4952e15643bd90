#!/bin/bash
# The whole -m gpu suite as the driver runs it (one process, prebuilt libraries), with per-test durations.
# Usage: tools/gpu/suite.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-suite}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum projects2014-metagenome_amd/libmtg_boss.so oracle/liboracle_boss.so > $OUT/build_sha.txt
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 900 --timeout-method thread --durations 40 > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -45 $OUT/pytest_gpu.log | grep -E "passed|failed|s call|s setup" | head -45
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -30; exit $rc; fi
if [ -n "$*" ]; then
  timeout -k 10 100 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.json | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
fi
exit 0
