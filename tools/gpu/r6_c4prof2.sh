#!/bin/bash
# One configs[3]-share step under rocprofv3 --kernel-trace (rocpd database).  Usage: r6_c4prof2.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r6c4p}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof -o cfg4 -- python3 bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $OUT/prof.log; exit 1; }
ls $OUT/prof
