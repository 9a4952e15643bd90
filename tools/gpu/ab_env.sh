#!/bin/bash
# A/B of environment settings on the default bench's device path only (no host legs, no parity, no CPU
# baseline), interleaved for 2 rounds.  Usage: tools/gpu/ab_env.sh <tag> "<VAR=v ...>" ...  ("-" = no setting)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1)); [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > $OUT/v$i.$rep.log 2>&1 || { echo "bench [$e] failed"; tail -5 $OUT/v$i.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-24s %.2f ms' % (sys.argv[2], d['ms_per_step']), ' '.join('%s=%.2f' % (k[:-3], v) for k, v in d['stages_ms'].items()))" $OUT/v$i.$rep.log "[$e]"
  done
done
