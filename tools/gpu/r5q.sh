#!/bin/bash
# configs[3]'s share and configs[2] with the wider bucket index for huge edge sets (build traces)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5q; mkdir -p $OUT
for cfg in cfg4 cfg3; do
  MTG_TRACE=1 timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 > $OUT/$cfg.json 2> $OUT/$cfg.err
  rc=$?; grep "mtg trace" $OUT/$cfg.err | grep -v workspace | tail -8
  [ $rc -ne 0 ] && { tail -3 $OUT/$cfg.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['stages_ms'])" $OUT/$cfg.json $cfg
done
exit 0
