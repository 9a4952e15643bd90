#!/bin/bash
# A/B of prebuilt library variants ab/<variant>/libmtg_boss.so on the default bench's device path only
# (no host legs, no parity, no CPU baseline), interleaved for 2 rounds; the package library is restored.
# Usage: tools/gpu/ab_fast.sh <tag> <variant>...   (outputs under gpurun_out/<tag>)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
LIB=projects2014-metagenome_amd/libmtg_boss.so
cp $LIB $OUT/keep.so
for rep in 1 2; do
  for v in "$@"; do
    cp ab/$v/libmtg_boss.so $LIB || exit 1
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --fasta-reads 0 --parity-full-max 0 > $OUT/$v.$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/$v.$rep.log; cp $OUT/keep.so $LIB; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-6s %.2f ms' % (sys.argv[2], d['ms_per_step']), ' '.join('%s=%.2f' % (k[:-3], v) for k, v in d['stages_ms'].items()), 'pass %.3f' % d['roofline']['pass_ms'])" $OUT/$v.$rep.log $v
  done
done
cp $OUT/keep.so $LIB; rm -f $OUT/keep.so
