#!/bin/bash
# The BASELINE preset lines on one GPU: configs[3] (cfg4: one 125 M-read share, key rounds),
# configs[4] (cfg5: counted build from a k=31 KMC1 database) and configs[2] (cfg3: k=63, 100 M
# reads, key ranges).  Usage: tools/gpu/presets.sh <tag> [presets...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-presets}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
P="$@"; [ -z "$P" ] && P="cfg4 cfg5 cfg3"
for c in $P; do
  timeout -k 10 420 python -u bench.py --config $c > $OUT/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -1 $OUT/bench_$c.log | cut -c1-1500
  [ $rc -ne 0 ] && exit $rc
done
exit 0
