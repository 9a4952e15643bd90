#!/bin/bash
# Round 4: parity of the speculative level-1 tests + 2 M-read generator tests, then the device-path bench (2 runs)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4y; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "speculative or bench_generator" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > $OUT/b$r.log 2>&1 || { tail -5 $OUT/b$r.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.2f ms' % d['ms_per_step'], ' '.join('%s=%.2f' % (k[:-3], v) for k, v in d['stages_ms'].items()), 'pass %.3f' % d['roofline']['pass_ms'])" $OUT/b$r.log
done
