#!/bin/bash
# super-k-mer collect after the run-packing rewrite: parity, then the P = 8 cost model of both collects
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5j; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -k "superkmer or collect_modes or dist_rounds or large_multi_tile" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head; exit $rc; }
for col in routed superkmer; do
  timeout -k 10 400 python -u tools/dist_sim.py --ranks 8 --reads 2500000 --steps 2 --serial --collect $col > $OUT/s8_$col.json 2> $OUT/s8_$col.err || { tail $OUT/s8_$col.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d[k] for k in ('single_ms','dist_wall_ms','work_ratio','max_rank_ratio') if k in d}, 'held', max(d.get('rank_held_ms',[0])))" $OUT/s8_$col.json $col
done
bash tools/gpu/prof_rank.sh r5j/p8_superkmer 8 2500000 --collect superkmer > /dev/null && head -25 $OUT/p8_superkmer/kernel_stats.txt
