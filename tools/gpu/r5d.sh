#!/bin/bash
# cfg3 (k=63) preset line on the u128 rounds, then an A/B of the lean local-unique kernel
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5d; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --config cfg3 --fasta-reads 0 > $OUT/cfg3.json 2> $OUT/cfg3.err
rc=$?; tail -3 $OUT/cfg3.err; tail -1 $OUT/cfg3.json | cut -c1-2500; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_env.sh r5d/ab 3 "MTG_LU_LEAN=0" "MTG_LU_LEAN=1"
