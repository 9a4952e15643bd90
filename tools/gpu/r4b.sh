#!/bin/bash
# Round 4: canonical key rounds of the fused K1 -- parity tests, the configs[3]-share bench line, its kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_rounds.py \
  "tests/test_gpu_dist.py::test_dist_large_multi_tile" > $OUT/pytest.txt 2>&1
rc=$?; tail -15 $OUT/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > $OUT/cfg4_bench.json 2> $OUT/cfg4_bench.err
rc=$?; tail -3 $OUT/cfg4_bench.err; cat $OUT/cfg4_bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg.sh r4b/cfg4 cfg4
