#!/bin/bash
# A -m gpu test subset (pytest -k expression), then optional build traces of presets (trace_cfg.sh).
# Usage: tools/gpu/check.sh <tag> "<pytest -k expr>" [config...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; KEXPR=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread -k "$KEXPR" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head; exit $rc; }
[ $# -gt 0 ] && { bash tools/gpu/trace_cfg.sh $TAG "$@" || exit 1; }
exit 0
