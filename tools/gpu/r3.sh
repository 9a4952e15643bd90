#!/bin/bash
# Round-3 GPU session: rebuild from source, the whole -m gpu suite, the default bench line and a
# preset line.  Usage: tools/gpu/r3.sh <tag> [pytest -k expr|none|all] [preset]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; KEXPR=${2:-all}; PRESET=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 make -B -s -j16 -C projects2014-metagenome_amd/csrc > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
timeout -k 10 120 make -B -s -C oracle >> $OUT/build.log 2>&1 || { echo "oracle build failed"; exit 1; }
sha256sum projects2014-metagenome_amd/libmtg_boss.so oracle/liboracle_boss.so > $OUT/build_sha.txt
if [ "$KEXPR" != "none" ]; then
  K=(); [ "$KEXPR" != "all" ] && K=(-k "$KEXPR")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -30; exit $rc; fi
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-4000
[ $rc -ne 0 ] && exit $rc
if [ -n "$PRESET" ]; then
  timeout -k 10 400 python -u bench.py --config $PRESET > $OUT/bench_$PRESET.log 2>&1
  rc=$?; echo "bench $PRESET rc=$rc"; tail -1 $OUT/bench_$PRESET.log | cut -c1-4000
fi
exit $rc
