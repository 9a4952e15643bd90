#!/bin/bash
# pytest subset, then configs[1] (20 steps, no full parity) and configs[2] lines.  Usage: tools/gpu/r6_check.sh <tag> <pytest args...>
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in cfg1 cfg3; do
  if [ $cfg = cfg1 ]; then A="--steps 20 --warmup 3"; else A="--config cfg3 --steps 2 --warmup 1"; fi
  timeout -k 10 300 python -u bench.py $A --no-cpu-baseline --host-steps 0 --parity-full-max 0 > $OUT/$cfg.log 2> $OUT/$cfg.err
  rc=$?; echo "$cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$cfg.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$OUT/$cfg.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stages_ms'].items()})"
done
