#!/bin/bash
# bench under env variants, kernel trace of each.  Usage: run_gpu7.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for v in "A" "MTG_PART_VEC=0" "MTG_DIGIT_BITS=8" "MTG_PART_VEC=0 MTG_DIGIT_BITS=8"; do
  name=$(echo "$v" | tr ' =' '__')
  (export $v 2>/dev/null; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/$name" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/$name.log" 2>&1) || exit 1
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' $GRAFT_REPO_ROOT/gpurun_out/$TAG/$name.log)"
done
