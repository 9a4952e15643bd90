#!/bin/bash
# Round 4: the configs[3]-share and configs[4] bench lines, kernel stats of the former.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-r4h}; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > $OUT/cfg4_bench.json 2> $OUT/cfg4_bench.err
rc=$?; tail -n 3 $OUT/cfg4_bench.err; cat $OUT/cfg4_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $OUT/cfg5_bench.json 2> $OUT/cfg5_bench.err
rc=$?; tail -n 3 $OUT/cfg5_bench.err; cat $OUT/cfg5_bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg.sh ${TAG:-r4h}/cfg4 cfg4
