#!/bin/bash
# Round 4: canonical key rounds (single + routed multi-GPU), pinned KMC reads -- parity tests, the
# configs[3]-share and configs[4] bench lines, kernel stats of the configs[3] share.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4c; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_rounds.py \
  tests/test_gpu_dist.py -k "rounds or large_multi_tile" > $OUT/pytest.txt 2>&1
rc=$?; tail -5 $OUT/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_kmc.py > $OUT/pytest_kmc.txt 2>&1
rc=$?; tail -3 $OUT/pytest_kmc.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > $OUT/cfg4_bench.json 2> $OUT/cfg4_bench.err
rc=$?; tail -3 $OUT/cfg4_bench.err; cat $OUT/cfg4_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $OUT/cfg5_bench.json 2> $OUT/cfg5_bench.err
rc=$?; tail -3 $OUT/cfg5_bench.err; cat $OUT/cfg5_bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg.sh r4c/cfg4 cfg4
