#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5f; mkdir -p $OUT
MTG_TRACE=1 timeout -k 10 600 python -u bench.py --config cfg3 --fasta-reads 0 --no-cpu-baseline --steps 1 --warmup 1 > $OUT/cfg3.json 2> $OUT/cfg3.err
rc=$?; grep -v amdgpu.ids $OUT/cfg3.err | tail -60; tail -1 $OUT/cfg3.json | cut -c1-1500; exit $rc
