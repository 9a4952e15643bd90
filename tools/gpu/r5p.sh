#!/bin/bash
# collect rounds sharing one pass B, wider bucket index for huge edge sets, dummy_sink staging loads:
# sink A/B, the rounds tests, configs[3]'s share with the build trace, the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5p; mkdir -p $OUT
true
timeout -k 10 900 python -u -m pytest tests/test_gpu_rounds.py -m gpu -x -q -k "not 20m and not 10m" -p no:cacheprovider --timeout 900 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head; exit $rc; }
MTG_TRACE=1 timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/cfg4.json 2> $OUT/cfg4.err
rc=$?; grep "mtg trace" $OUT/cfg4.err | grep -v workspace | tail -16
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'])" $OUT/cfg4.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'])" $OUT/bench.json
exit $rc
