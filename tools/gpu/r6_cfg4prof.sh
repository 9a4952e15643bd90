#!/bin/bash
# configs[3]'s share: the rounds tests, the preset traced, and one step's kernel statistics.
# Usage: tools/gpu/r6_cfg4prof.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r6c4}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rounds.py > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
MTG_TRACE=1 timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err || { echo "cfg4 rc=$?"; tail -20 $OUT/cfg4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg4 %.1f ms' % d['ms_per_step'], {k: round(v, 1) for k, v in d['stages_ms'].items()}, 'peak %.1f GB' % (d['counts']['peak_bytes'] / 1e9))" $OUT/cfg4.json
grep -E "rounds:|carved|dropping" $OUT/cfg4.err | tail -12
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cfg4 -- python3 bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
for cfg in cfg3 cfg5; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline > $OUT/$cfg.json 2> $OUT/$cfg.err || { echo "$cfg rc=$?"; tail -20 $OUT/$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.1f ms' % d['ms_per_step'], {k: round(v, 1) for k, v in d['stages_ms'].items()}, 'peak %.1f GB' % (d['counts']['peak_bytes'] / 1e9), 'parity', (d.get('parity') or {}).get('ok'))" $OUT/$cfg.json $cfg
done
