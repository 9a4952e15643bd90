#!/bin/bash
# Multi-rank check on one GPU: the dist parity tests, then tools/dist_sim.py at P ranks (20 M reads
# in total, at most 10 M per rank) against the single build of the same reads.
# Usage: tools/gpu/dist_check.sh <tag> [ranks...]   (outputs under gpurun_out/<tag>)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-dist}; shift; RANKS=${@:-1 2 8}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for P in $RANKS; do
  R=$((20000000 / P)); [ $R -gt 10000000 ] && R=10000000
  timeout -k 10 150 python -u tools/dist_sim.py --ranks $P --reads $R --steps 3 > $OUT/p$P.json 2> $OUT/p$P.err || { echo "sim P=$P failed"; tail -5 $OUT/p$P.err; exit 1; }
done
python3 - $OUT $RANKS <<'PY'
import json, sys
out = sys.argv[1]
for P in map(int, sys.argv[2:]):
    d = json.load(open("%s/p%d.json" % (out, P)))
    print(P, d["reads_per_rank"], "single %.1f ms" % d["single_ms"], "dist wall %.1f ms" % d["dist_wall_ms"],
          "work ratio %.2f" % (d["dist_wall_ms"] / d["single_ms"]), "-> est. scaling %.2f" % (P * d["single_ms"] / d["dist_wall_ms"]))
PY
