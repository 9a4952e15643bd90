#!/bin/bash
# Round 4: the configs[3] share through the single build and the P = 1 distributed build with the debug
# trace; its two full-size tests; then the configs[3]-share and configs[4] bench lines and the kernel
# stats of the former.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4f; mkdir -p $OUT
MTG_TRACE=1 MTG_DEBUG=1 timeout -k 10 500 python -u tools/gpu/cfg4_dist_debug.py 125000000 both > $OUT/cfg4_debug.txt 2>&1
rc=$?; echo "debug rc=$rc"; grep -v "order violations" $OUT/cfg4_debug.txt | grep -v amdgpu | tail -n 30; grep "order violations" $OUT/cfg4_debug.txt | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_scale.py -k "cfg4_share or config3_share" > $OUT/pytest.txt 2>&1
rc=$?; tail -n 4 $OUT/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > $OUT/cfg4_bench.json 2> $OUT/cfg4_bench.err
rc=$?; tail -n 3 $OUT/cfg4_bench.err; cat $OUT/cfg4_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $OUT/cfg5_bench.json 2> $OUT/cfg5_bench.err
rc=$?; tail -n 3 $OUT/cfg5_bench.err; cat $OUT/cfg5_bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg.sh r4f/cfg4 cfg4
