#!/bin/bash
# A/B of one env knob on configs[1] (default bench, 20 steps) and configs[2] (cfg3), after a pytest subset.
# Usage: tools/gpu/r6_ab_both.sh <tag> <KNOB> <pytest args...>
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; KNOB=$2; shift 2; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in cfg1 cfg3; do for v in default 0 default; do
  if [ $v = default ]; then unset $KNOB; else export $KNOB=$v; fi
  if [ $cfg = cfg1 ]; then A="--steps 20 --warmup 3"; else A="--config cfg3 --steps 2 --warmup 1"; fi
  timeout -k 10 300 python -u bench.py $A --no-cpu-baseline --host-steps 0 --parity-full-max 0 > $OUT/${cfg}_$v.log 2> $OUT/${cfg}_$v.err
  rc=$?; echo "$cfg $KNOB=$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/${cfg}_$v.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$OUT/${cfg}_$v.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stages_ms'].items()})"
done; done
