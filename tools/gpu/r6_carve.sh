#!/bin/bash
# Round 6: the carving workspace + in-place speculative level 3 of the batched collect.  The rounds tests,
# then configs[3]'s share traced (default, and with one pass B for both rounds), then the default bench.
# Usage: tools/gpu/r6_carve.sh <tag> [skip-tests]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r6carve}; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -z "$2" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rounds.py -k "three_msd or random_reads or bench_generator" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
  tail -3 $OUT/pytest.txt
fi
MTG_TRACE=1 timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err || { echo "cfg4 rc=$?"; tail -20 $OUT/cfg4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg4 %.1f ms' % d['ms_per_step'], {k: round(v, 1) for k, v in d['stages_ms'].items()}, 'peak %.1f GB' % (d['counts']['peak_bytes'] / 1e9), 'parity', d.get('parity', {}).get('ok'))" $OUT/cfg4.json
grep -E "rounds:|msd n=|carved|speculative" $OUT/cfg4.err | tail -24
MTG_ROUNDS_ONE_B=1 MTG_TRACE=1 timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --parity-full-max 0 > $OUT/cfg4_oneb.json 2> $OUT/cfg4_oneb.err || { echo "cfg4 one-b rc=$?"; tail -20 $OUT/cfg4_oneb.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg4 one-b %.1f ms' % d['ms_per_step'], {k: round(v, 1) for k, v in d['stages_ms'].items()}, 'peak %.1f GB' % (d['counts']['peak_bytes'] / 1e9), 'parity', d.get('parity', {}).get('ok'))" $OUT/cfg4_oneb.json
grep -E "rounds:|carved|dropping" $OUT/cfg4_oneb.err | tail -16
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg1 %.2f ms' % d['ms_per_step'], {k: round(v, 2) for k, v in d['stages_ms'].items()}, 'peak %.1f GB' % (d['counts']['peak_bytes'] / 1e9))" $OUT/bench.json
