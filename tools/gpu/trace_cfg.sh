#!/bin/bash
# Build traces (MTG_TRACE=1: per-stage times and every workspace allocation of 256 MiB or more) of
# bench presets, two timed steps after one warmup each, stage times printed.
# Usage: tools/gpu/trace_cfg.sh <tag> <config>...   (e.g. cfg4 cfg3; outputs under gpurun_out/<tag>)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-trace}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for cfg in "$@"; do
  MTG_TRACE=1 timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 > $OUT/$cfg.json 2> $OUT/$cfg.err
  rc=$?; grep "mtg trace" $OUT/$cfg.err | grep -v workspace | tail -12
  [ $rc -ne 0 ] && { tail -3 $OUT/$cfg.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['stages_ms'])" $OUT/$cfg.json $cfg
done
exit 0
