#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5n; mkdir -p $OUT
MTG_TRACE=1 MTG_DEBUG_LITE=1 timeout -k 10 600 python -u bench.py --config cfg4 --fasta-reads 0 --no-cpu-baseline --steps 1 --warmup 1 > $OUT/cfg4.json 2> $OUT/cfg4.err
rc=$?; grep "mtg trace" $OUT/cfg4.err | tail -40; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg_launches.sh r5n/cfg4 cfg4 extract_hist_fast --fasta-reads 0
