#!/bin/bash
# Round 4: trace of the P = 1 distributed configs[3] share, then the A/B and bench legs of r4c.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4e; mkdir -p $OUT
MTG_TRACE=1 MTG_DEBUG=1 timeout -k 10 400 python -u tools/gpu/cfg4_dist_debug.py > $OUT/cfg4_dist_debug.txt 2>&1
echo "debug rc=$?"; tail -25 $OUT/cfg4_dist_debug.txt
for w in 1 0 1 0; do
  MTG_WIDE_B1=$w timeout -k 10 300 python -u tools/dist_sim.py --ranks 2 --reads 10000000 --only-single --steps 5 >> $OUT/single20m_wide$w.txt 2>&1 || exit 1
done
tail -n 2 $OUT/single20m_wide1.txt $OUT/single20m_wide0.txt
timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > $OUT/cfg4_bench.json 2> $OUT/cfg4_bench.err
rc=$?; tail -3 $OUT/cfg4_bench.err; cat $OUT/cfg4_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $OUT/cfg5_bench.json 2> $OUT/cfg5_bench.err
rc=$?; tail -3 $OUT/cfg5_bench.err; cat $OUT/cfg5_bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg.sh r4e/cfg4 cfg4
