#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5o; mkdir -p $OUT
timeout -k 10 180 tools/sink_bench > $OUT/sink_bench.txt 2>&1; rc=$?; cat $OUT/sink_bench.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread -k "parity or dummy or dist" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; rc=$?
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'])" $OUT/bench.json
exit $rc
