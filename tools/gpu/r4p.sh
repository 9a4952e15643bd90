#!/bin/bash
# Round 4: the sampled pass A / speculative level-1 layout and the pulled multi-GPU sink join -- their
# parity tests, the default bench with the level-1 layout on and off, and the serial cost model.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r4p}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "speculative_level1 or bench_generator_2m" > $OUT/pytest_scale.log 2>&1
rc=$?; tail -12 $OUT/pytest_scale.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1
rc=$?; tail -5 $OUT/pytest_dist.log; [ $rc -ne 0 ] && exit $rc
MTG_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --fasta-reads 0 > $OUT/debug.log 2>&1 || { echo "debug bench failed"; tail -20 $OUT/debug.log; exit 1; }
grep "speculative level 1\|fused extract" $OUT/debug.log | head -4
bash tools/gpu/ab_env.sh ${TAG:-r4p}/ab 2 "MTG_SPEC_L1=1" "MTG_SPEC_L1=0" "MTG_KSPEC=0" || exit 1
TAG=${TAG:-r4p}/d bash -c 'R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
for cfg in "s2 2 10000000" "s8 8 2500000"; do set -- $cfg
  timeout -k 10 300 python3 -u tools/dist_sim.py --ranks $2 --reads $3 --serial > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "$1 failed"; tail -5 "$OUT/$1.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], \"single %.1f ms work ratio %s held %s sent GB max %.2f\" % (d[\"single_ms\"], d[\"work_ratio\"], d[\"rank_held_ms\"], max(d.get(\"sent_bytes\") or [0])/1e9))" "$OUT/$1.json" $1
done'
