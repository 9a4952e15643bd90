#!/bin/bash
# Round 4: the sink join's staged bucket-index slice -- parity (single + multi-rank), then A/B vs the previous build
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4s2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "not rounds" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bench_generator_2m" > $OUT/pytest2.log 2>&1
rc=$?; tail -3 $OUT/pytest2.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_fast.sh r4s2/ab w8b4 sinkidx
