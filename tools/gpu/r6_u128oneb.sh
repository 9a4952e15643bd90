#!/bin/bash
# u128 rounds tests with one pass B for both rounds, then the configs[2] preset line (traced).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6u1}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rounds.py \
  -k "u128" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
MTG_TRACE=1 timeout -k 10 480 python -u bench.py --config cfg3 > $OUT/cfg3.log 2> $OUT/cfg3.err
rc=$?; echo "cfg3 rc=$rc"; tail -1 $OUT/cfg3.log | cut -c1-1200; grep "rounds:" $OUT/cfg3.err | tail -8; exit $rc
