#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5l; mkdir -p $OUT
for env in "X=1" "MTG_SPEC_RC=0" "MTG_SPEC=0" "MTG_DEFER_GATHER=0"; do
  env $env timeout -k 10 200 python -u tools/dist_sim.py --ranks 8 --reads 1000000 --steps 1 --serial --collect superkmer --no-single > $OUT/s8.json 2> $OUT/s8.err || { tail -5 $OUT/s8.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'held', max(d.get('rank_held_ms',[0])), 'rc', [round(x['rc_ms'],1) for x in d['rank_stages']])" $OUT/s8.json "$env"
done
