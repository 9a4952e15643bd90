#!/bin/bash
# Round-4 first GPU pass: the changed parity tests, then kernel stats of the configs[3] share.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_scale.py::test_bench_generator_2m_reads_k31" \
  "tests/test_gpu_scale.py::test_bench_generator_three_msd_levels" \
  "tests/test_gpu_scale.py::test_bench_generator_speculative_overflow" \
  "tests/test_gpu_dist.py::test_dist_large_multi_tile" > $OUT/pytest.txt 2>&1
rc=$?; tail -15 $OUT/pytest.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_cfg.sh r4a/cfg4 cfg4 --fasta-reads 0
