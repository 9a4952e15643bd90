#!/bin/bash
# Round 4: the 3-level rounds parity tests, then the configs[3] share with the exact rc level (trace).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4g; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rounds.py -k "three_msd or bench_generator" > $OUT/pytest.txt 2>&1
rc=$?; tail -n 8 $OUT/pytest.txt
MTG_SPEC_RC=0 MTG_DEBUG=1 timeout -k 10 400 python -u tools/gpu/cfg4_dist_debug.py 125000000 single > $OUT/cfg4_specrc0.txt 2>&1
echo "specrc0 rc=$?"; grep -v "order violations" $OUT/cfg4_specrc0.txt | grep -v amdgpu | tail -12; grep "order violations" $OUT/cfg4_specrc0.txt | cut -c1-200
