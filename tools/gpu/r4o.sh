#!/bin/bash
# Round 4: the sampled pass A / speculative level-1 layout -- its parity tests, then the default bench
# with it on and off (interleaved, 2 rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r4o}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "speculative_level1 or bench_generator_2m" > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
MTG_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --fasta-reads 0 > $OUT/debug.log 2>&1 || { echo "debug bench failed"; tail -20 $OUT/debug.log; exit 1; }
grep "speculative level 1\|fused extract" $OUT/debug.log | head -4
bash tools/gpu/ab_env.sh ${TAG:-r4o}/ab 2 "MTG_SPEC_L1=1" "MTG_SPEC_L1=0"
