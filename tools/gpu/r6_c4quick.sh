#!/bin/bash
# The rounds tests, configs[3]'s share traced, and the default bench's device path.  Usage: r6_c4quick.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r6c4q}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rounds.py ${PYT_EXTRA} > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "Error|FAILED" $OUT/pytest.txt | head; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
MTG_TRACE=1 timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err || { echo "cfg4 rc=$?"; tail -20 $OUT/cfg4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg4 %.1f ms' % d['ms_per_step'], {k: round(v, 1) for k, v in d['stages_ms'].items()}, 'peak %.1f GB' % (d['counts']['peak_bytes'] / 1e9), d['counts']['n_real'], d['counts']['n_dummy'], d['counts']['n_rows'])" $OUT/cfg4.json
grep -E "rounds:|msd n=" $OUT/cfg4.err | tail -6
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg1 %.2f ms' % d['ms_per_step'], {k: round(v, 2) for k, v in d['stages_ms'].items()}, 'peak %.1f GB' % (d['counts']['peak_bytes'] / 1e9))" $OUT/bench.json
