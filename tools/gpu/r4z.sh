#!/bin/bash
# Round 4: the dummy-source bitmap -- parity (every k, the alternate paths incl. MTG_DUMMY_BITMAP=0, 2 M reads),
# then the device-path bench with the bitmap on and off (interleaved, 2 rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4z; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "not full_bench and not cfg3 and not cfg4 and not config3" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
MTG_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 2>&1 | grep "dummies:" | head -2
bash tools/gpu/ab_env.sh r4z/ab 2 "MTG_DUMMY_BITMAP=1" "MTG_DUMMY_BITMAP=0"
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r4z/prof && cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4z/prof/stats -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > $GRAFT_REPO_ROOT/gpurun_out/r4z/prof/b.log 2>&1 && python3 $GRAFT_REPO_ROOT/tools/klaunch.py $GRAFT_REPO_ROOT/gpurun_out/r4z/prof/stats > $GRAFT_REPO_ROOT/gpurun_out/r4z/prof/launches.txt && grep -E "dummy|onesweep|unique_kernel<1, false>|radix_hist" $GRAFT_REPO_ROOT/gpurun_out/r4z/prof/launches.txt
