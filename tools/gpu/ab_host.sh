#!/bin/bash
# A/B of prebuilt library variants on the bench's host-ABI leg (add_packed + build_chunk):
# ab/<variant>/libmtg_boss.so copied over the package library in turn, interleaved, 3 rounds.
# Usage: tools/gpu/ab_host.sh <tag> <variant>...   (outputs under gpurun_out/<tag>)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
LIB=projects2014-metagenome_amd/libmtg_boss.so
for rep in 1 2 3; do
  for v in "$@"; do
    cp ab/$v/libmtg_boss.so $LIB || exit 1
    timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-steps 4 --fasta-reads 0 > $OUT/$v.$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_path']; print(sys.argv[2], '%.2f ms' % h['ms_per_step'], {k: round(v, 2) for k, v in h['stages_ms'].items()})" $OUT/$v.$rep.log $v
  done
done
