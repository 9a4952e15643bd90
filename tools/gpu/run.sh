#!/bin/bash
# One GPU session: rebuild every native library from source (so the .so under test is the one
# this tree's sources make), the -m gpu parity tests, then the default bench line.
# Usage: tools/gpu/run.sh <tag> [pytest -k expr] [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; KEXPR=${2:-}; shift 2 2>/dev/null; BARGS="$@"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 make -B -s -j16 -C projects2014-metagenome_amd/csrc > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
timeout -k 10 120 make -B -s -C oracle >> $OUT/build.log 2>&1 || { echo "oracle build failed"; exit 1; }
sha256sum projects2014-metagenome_amd/libmtg_boss.so oracle/liboracle_boss.so > $OUT/build_sha.txt
if [ "$KEXPR" != "none" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -30; exit $rc; fi
fi
timeout -k 10 600 python -u bench.py $BARGS > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-3000
exit $rc
