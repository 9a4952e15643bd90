#!/bin/bash
# The whole -m gpu suite on the prebuilt libraries, then the default bench line and optional presets.
# Usage: tools/gpu/full.sh <tag> [presets...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-full}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum projects2014-metagenome_amd/libmtg_boss.so oracle/liboracle_boss.so > $OUT/build_sha.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 1200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.json | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
for c in "$@"; do
  timeout -k 10 600 python -u bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; tail -1 $OUT/bench_$c.json | cut -c1-1200; [ $rc -ne 0 ] && exit $rc
done
exit 0
