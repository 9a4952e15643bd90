#!/bin/bash
# A/B of environment switches on one box: the default bench (device path only) under each setting,
# interleaved for ROUNDS rounds; prints ms/step and the stage times per run.
# Usage: tools/gpu/ab_env.sh <tag> <rounds> "<ENV=a>" "<ENV=b>" ...
R="$GRAFT_REPO_ROOT"; TAG=${1:-ab}; ROUNDS=${2:-2}; shift 2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
for r in $(seq 1 $ROUNDS); do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --fasta-reads 0 > "$OUT/run.log" 2>&1 || { echo "bench failed: $setting"; tail -5 "$OUT/run.log"; exit 1; }
    python3 - "$setting" "$OUT/run.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = d["stages_ms"]
print("%-28s %7.3f ms/step  %s" % (sys.argv[1], d["ms_per_step"], "  ".join("%s=%.3f" % (k[:-3], v) for k, v in s.items())))
PY
  done
done
