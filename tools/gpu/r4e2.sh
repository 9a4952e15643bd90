#!/bin/bash
# Round 4: empty groups of the fused rc merge exit early -- parity, the serial P = 8 / P = 2 cost model, the bench
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4e2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_rounds.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "s8 8 2500000" "s2 2 10000000"; do set -- $cfg
  timeout -k 10 300 python3 -u tools/dist_sim.py --ranks $2 --reads $3 --serial > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "$1 failed"; tail -5 "$OUT/$1.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'single %.1f ms work ratio %s held %s sent GB max %.2f' % (d['single_ms'], d['work_ratio'], d['rank_held_ms'], max(d.get('sent_bytes') or [0])/1e9))" "$OUT/$1.json" $1
done
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > $OUT/b.log 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.2f ms' % d['ms_per_step'], ' '.join('%s=%.2f' % (k[:-3], v) for k, v in d['stages_ms'].items()), 'pass %.3f' % d['roofline']['pass_ms'])" $OUT/b.log
