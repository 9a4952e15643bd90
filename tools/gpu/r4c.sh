#!/bin/bash
# Round 4: the whole -m gpu suite (rounds, wide level 1, counted speculative levels, narrowed weights,
# pinned KMC reads), the 20 M-read single build A/B (wide level 1), the configs[3]-share and
# configs[4] bench lines, kernel stats of the configs[3] share.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4c; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
for w in 1 0 1 0; do
  MTG_WIDE_B1=$w timeout -k 10 300 python -u tools/dist_sim.py --ranks 2 --reads 10000000 --only-single --steps 5 >> $OUT/single20m_wide$w.txt 2>&1 || exit 1
done
tail -2 $OUT/single20m_wide1.txt $OUT/single20m_wide0.txt
timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > $OUT/cfg4_bench.json 2> $OUT/cfg4_bench.err
rc=$?; tail -3 $OUT/cfg4_bench.err; cat $OUT/cfg4_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $OUT/cfg5_bench.json 2> $OUT/cfg5_bench.err
rc=$?; tail -3 $OUT/cfg5_bench.err; cat $OUT/cfg5_bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg.sh r4c/cfg4 cfg4
