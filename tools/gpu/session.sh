#!/bin/bash
# One GPU session on the prebuilt libraries of this tree (built here with __graft_entry__.build(); set
# REBUILD=1 to rebuild on the box first): the -m gpu tests matching an optional -k expression, then
# optional bench runs.  Every step has its own time limit; the first failure ends the session.
# Usage: tools/gpu/session.sh <tag> [pytest -k expr | none] [bench args ... ]
#        BENCH2="--config cfg5" adds a second bench line (its own log)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; KEXPR=${2:-}; shift 2 2>/dev/null; BARGS="$@"
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$REBUILD" ]; then
  timeout -k 10 300 make -B -s -C projects2014-metagenome_amd/csrc > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
  timeout -k 10 120 make -B -s -C oracle >> $OUT/build.log 2>&1 || { echo "oracle build failed"; exit 1; }
fi
sha256sum projects2014-metagenome_amd/libmtg_boss.so oracle/liboracle_boss.so > $OUT/build_sha.txt
if [ "$KEXPR" != "none" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 1200 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -30; exit $rc; fi
fi
if [ -n "$BARGS" ]; then
  timeout -k 10 600 python -u bench.py $BARGS > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.err; tail -1 $OUT/bench.json | cut -c1-3000
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$BENCH2" ]; then
  timeout -k 10 900 python -u bench.py $BENCH2 > $OUT/bench2.json 2> $OUT/bench2.err
  rc=$?; echo "bench2 rc=$rc"; tail -3 $OUT/bench2.err; tail -1 $OUT/bench2.json | cut -c1-3000
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
