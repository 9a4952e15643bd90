#!/bin/bash
# run_gpu6 (checker, microbench, tests, bench, stats) then the bench under env variants.
# Usage: run_gpu8.sh <tag> "<ENV=V ...>" ["<ENV=V ...>" ...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; shift
bash tools/gpu/run_gpu6.sh $TAG || exit $?
for v in "$@"; do
  (export $v; timeout -k 10 300 python bench.py --no-cpu-baseline > "gpurun_out/$TAG/bench_$(echo $v | tr ' =' '__').log" 2>&1) || exit 1
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$TAG/bench_$(echo $v | tr ' =' '__').log)"
done
