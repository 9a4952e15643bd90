#!/bin/bash
# Multi-GPU cost model on one GPU: the dist parity tests, then tools/dist_sim.py (P serial ranks) for
# each collect route, then the per-rank kernel stats of the first route.
# Usage: tools/gpu/dist_sims.sh <tag> <ranks> <reads per rank> <collect>...   (e.g. r5m 8 2500000 superkmer routed)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; P=$2; READS=$3; shift 3; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -k "dist" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head; exit $rc; }
for col in "$@"; do
  timeout -k 10 400 python -u tools/dist_sim.py --ranks $P --reads $READS --steps 2 --serial --collect $col > $OUT/s${P}_$col.json 2> $OUT/s${P}_$col.err || { tail $OUT/s${P}_$col.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d[k] for k in ('single_ms','dist_wall_ms','work_ratio','max_rank_ratio') if k in d}, 'held', max(d.get('rank_held_ms',[0])), 'sent GB', max(d.get('sent_bytes',[0]))/1e9)" $OUT/s${P}_$col.json $col
done
bash tools/gpu/prof_rank.sh $TAG/p${P}_$1 $P $READS --collect $1 > /dev/null && head -20 gpurun_out/$TAG/p${P}_$1/kernel_stats.txt
