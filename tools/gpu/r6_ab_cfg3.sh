#!/bin/bash
# configs[2] A/B of one env knob: u128 rounds tests, then bench cfg3 with the knob at its default and at "0".
# Usage: tools/gpu/r6_ab_cfg3.sh <tag> <KNOB> [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; KNOB=$2; KX=${3:-u128}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rounds.py -k "$KX" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in default 0; do
  if [ $v = default ]; then unset $KNOB; else export $KNOB=$v; fi
  timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline --host-steps 0 > $OUT/cfg3_$v.log 2> $OUT/cfg3_$v.err
  rc=$?; echo "cfg3 $KNOB=$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/cfg3_$v.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/cfg3_$v.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'])"
done
